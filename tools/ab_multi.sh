# C3 bench A/B over several library builds, REPS rounds round-robin; every step time-limited.
# LIBS="lidar_slam_amd/variants/lib_a.so lidar_slam_amd/liblidarslam.so" REPS=3 bash tools/ab_multi.sh
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for rep in $(seq ${REPS:-3}); do for lib in $LIBS; do
  LSLAM_ALLOW_STALE=1 LSLAM_LIB=$PWD/$lib timeout -k 10 200 python -u bench.py --steps ${STEPS:-40} --warmup 3 --no-cpu-baseline --no-alone ${BENCH_ARGS:-} > gpurun_out/ab_bench.json 2> gpurun_out/ab_bench.err || { tail -5 gpurun_out/ab_bench.err; exit 1; }
  echo "$lib $(python3 -c "import json; d=json.load(open('gpurun_out/ab_bench.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], r.get('kernel_ms'), r.get('consensus', {}).get('ms'))")"
done; done
