# round-4 session 1: VALU issue micro-benchmark, GPU tests (linear mask windows in the product build),
# C5 parity A/B (linear mask windows vs the 9-VALU evaluation), C3 A/B of the REJ32 sign test
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 60 tools/ubench_valu > gpurun_out/ubench_valu.json 2>&1 || { cat gpurun_out/ubench_valu.json; exit 1; }
cat gpurun_out/ubench_valu.json
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
LIBS="lidar_slam_amd/variants/lib_masklin0.so lidar_slam_amd/liblidarslam.so" REPS=2 bash tools/c5_libs.sh || exit 1
LIBS="lidar_slam_amd/liblidarslam.so lidar_slam_amd/variants/lib_rej32.so" REPS=2 bash tools/ab_multi.sh
