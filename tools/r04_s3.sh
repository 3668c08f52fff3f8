# round-4 session 3: GPU tests, C3 A/B of the late convergence check (LSLAM_TBL_LATECHECK), window stamps of both
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for v in wstamps wstamps_late; do
  LSLAM_LIB=$PWD/lidar_slam_amd/variants/lib_$v.so timeout -k 10 120 python -u tools/wstamps.py > gpurun_out/wstamps_$v.json 2> gpurun_out/wstamps.err || { tail -20 gpurun_out/wstamps.err; exit 1; }
  echo "$v $(cat gpurun_out/wstamps_$v.json)"
done
LIBS="lidar_slam_amd/liblidarslam.so lidar_slam_amd/variants/lib_latecheck.so" REPS=3 bash tools/ab_multi.sh
