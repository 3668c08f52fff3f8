cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { tail -30 gpurun_out/t_all.log; exit 1; }
tail -1 gpurun_out/t_all.log
timeout -k 10 120 python -u tools/wstamps.py > gpurun_out/wstamps.json 2> gpurun_out/wstamps.err || { tail -20 gpurun_out/wstamps.err; exit 1; }
cat gpurun_out/wstamps.json
LIBS="lidar_slam_amd/variants/lib_mix7.so lidar_slam_amd/liblidarslam.so lidar_slam_amd/variants/lib_u2.so" REPS=3 bash tools/ab_multi.sh
