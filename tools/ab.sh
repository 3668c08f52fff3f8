# A/B: the in-tree build (B, also runs the GPU parity tests) against another build A
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
A=${A:-lidar_slam_amd/liblidarslam_prev.so}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for rep in 1 2; do
for lib in $A lidar_slam_amd/liblidarslam.so; do
  echo "$lib $(LSLAM_LIB=$PWD/$lib timeout -k 10 120 python -u tools/drawsbench.py 1024 4096 | tail -1) $(LSLAM_LIB=$PWD/$lib timeout -k 10 60 python -u tools/hostprobe.py 2>&1 | sed -n 1p | sed 's/.*step/step/')" || exit 1
done; done
