# bench.py (C3) under several environments, REPS rounds (no tests):
# ENVS="LSLAM_POST_W4=0|LSLAM_POST_W4=1 LSLAM_CONS_PRIO=000" bash tools/ab_envs.sh
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
IFS='|' read -ra LIST <<< "$ENVS"
for rep in $(seq ${REPS:-2}); do for ev in "${LIST[@]}"; do
  env $ev timeout -k 10 200 python -u bench.py --steps 40 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab_bench.json 2> gpurun_out/ab_bench.err || { tail -5 gpurun_out/ab_bench.err; exit 1; }
  echo "$ev: $(python3 -c "import json; d=json.load(open('gpurun_out/ab_bench.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], r.get('kernel_ms'), r.get('consensus', {}).get('ms'))")"
done; done
