# round-4 session 8: parity of the asm window without its trailing s_nop (GPU tests on it), then C3 A/B
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
LSLAM_LIB=$PWD/lidar_slam_amd/variants/lib_nonop.so LSLAM_ALLOW_STALE=1 timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_nonop.log 2>&1 || { tail -30 gpurun_out/gpu_tests_nonop.log; exit 1; }
tail -1 gpurun_out/gpu_tests_nonop.log
LIBS="lidar_slam_amd/liblidarslam.so lidar_slam_amd/variants/lib_nonop.so" REPS=4 bash tools/ab_multi.sh
