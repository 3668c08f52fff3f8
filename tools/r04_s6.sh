# round-4 session 6: parity of the hand-scheduled evaluation + temper variant (GPU tests on it), then C3 A/B
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
LSLAM_LIB=$PWD/lidar_slam_amd/variants/lib_ahead2.so LSLAM_ALLOW_STALE=1 timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_ahead2.log 2>&1 || { tail -30 gpurun_out/gpu_tests_ahead2.log; exit 1; }
tail -1 gpurun_out/gpu_tests_ahead2.log
LIBS="lidar_slam_amd/liblidarslam.so lidar_slam_amd/variants/lib_ahead2.so lidar_slam_amd/variants/lib_ahead2s.so lidar_slam_amd/variants/lib_sbase.so" REPS=3 bash tools/ab_multi.sh
