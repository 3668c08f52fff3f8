# A/B: GPU parity tests on the in-tree build (B), then tools/microbench.py on build A and B, twice
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
A=${A:-lidar_slam_amd/liblidarslam_prev.so}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for rep in 1 2; do
for lib in $A lidar_slam_amd/liblidarslam.so; do
  echo "$lib $(LSLAM_LIB=$PWD/$lib timeout -k 10 180 python -u tools/microbench.py --reps 10)" || exit 1
done; done
