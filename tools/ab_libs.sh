# GPU parity tests on the in-tree build, then bench.py (C3) A/B of two builds, REPS rounds:
# A = ${A:-lidar_slam_amd/liblidarslam_prev.so} vs the in-tree lidar_slam_amd/liblidarslam.so
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
A=${A:-lidar_slam_amd/liblidarslam_prev.so}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for rep in $(seq ${REPS:-3}); do for lib in $A lidar_slam_amd/liblidarslam.so; do
  LSLAM_ALLOW_STALE=1 LSLAM_LIB=$PWD/$lib timeout -k 10 200 python -u bench.py --steps 40 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab_bench.json 2> gpurun_out/ab_bench.err || { tail -5 gpurun_out/ab_bench.err; exit 1; }
  echo "$lib $(python3 -c "import json; d=json.load(open('gpurun_out/ab_bench.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], r.get('kernel_ms'), r.get('kernel_alone_ms'), r.get('consensus', {}).get('ms'))")"
done; done
