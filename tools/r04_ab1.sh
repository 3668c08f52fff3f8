# round-4 session 1: VALU issue micro-benchmark, GPU tests, C3 A/B of the REJ32 sign test
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 60 tools/ubench_valu > gpurun_out/ubench_valu.json 2>&1 || { cat gpurun_out/ubench_valu.json; exit 1; }
cat gpurun_out/ubench_valu.json
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
LIBS="lidar_slam_amd/liblidarslam.so lidar_slam_amd/variants/lib_rej32.so" REPS=3 bash tools/ab_multi.sh
ENVS="LSLAM_RESOLVE_STREAM=0|LSLAM_RESOLVE_STREAM=1|LSLAM_SLOTS=3" REPS=2 bash tools/ab_envs.sh
