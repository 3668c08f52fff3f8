# A/B of two builds: producer alone (drawsbench) and the C3 step (hostprobe); B also runs the GPU parity tests
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
B=${B:-lidar_slam_amd/liblidarslam_fp2.so}
LSLAM_LIB=$PWD/$B timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_b.log 2>&1 || { tail -30 gpurun_out/gpu_tests_b.log; exit 1; }
tail -1 gpurun_out/gpu_tests_b.log
for rep in 1 2; do
for lib in lidar_slam_amd/liblidarslam.so $B; do
  echo "$lib $(LSLAM_LIB=$PWD/$lib timeout -k 10 120 python -u tools/drawsbench.py 1024 4096 | tail -1) $(LSLAM_LIB=$PWD/$lib timeout -k 10 60 python -u tools/hostprobe.py 2>&1 | sed -n 1p | sed 's/.*step/step/')" || exit 1
done; done
