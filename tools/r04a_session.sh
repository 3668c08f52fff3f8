# round-4 A/B session: GPU tests on the in-tree build, window stamps, C3 A/B of variant builds
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { tail -30 gpurun_out/t_all.log; exit 1; }
tail -1 gpurun_out/t_all.log
for v in ${WST:-wstamps}; do
  LSLAM_LIB=$PWD/lidar_slam_amd/variants/lib_$v.so timeout -k 10 120 python -u tools/wstamps.py > gpurun_out/wstamps_$v.json 2> gpurun_out/wstamps.err || { tail -20 gpurun_out/wstamps.err; exit 1; }
  echo "$v $(cat gpurun_out/wstamps_$v.json)"
done
LIBS="$LIBS" REPS=${REPS:-2} bash tools/ab_multi.sh
