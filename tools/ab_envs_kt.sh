# bench.py (C3) under several environments, REPS rounds, then one kernel trace per environment
# (timeline of the last kernels: which queue each ran on, and how long each took beside the others):
# ENVS="LSLAM_CONS_PRIO=0000|LSLAM_CONS_PRIO=3000" bash tools/ab_envs_kt.sh
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export TMPDIR=/tmp
IFS='|' read -ra LIST <<< "$ENVS"
for rep in $(seq ${REPS:-2}); do for ev in "${LIST[@]}"; do
  env $ev timeout -k 10 200 python -u bench.py --steps 40 --warmup 3 --no-cpu-baseline --no-alone ${BENCH_ARGS:-} > gpurun_out/ab_bench.json 2> gpurun_out/ab_bench.err || { tail -5 gpurun_out/ab_bench.err; exit 1; }
  echo "$ev: $(python3 -c "import json; d=json.load(open('gpurun_out/ab_bench.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], r.get('kernel_ms'), r.get('consensus', {}).get('ms'))")"
done; done
[ -n "${NO_KT:-}" ] && exit 0
i=0
for ev in "${LIST[@]}"; do
  i=$((i+1))
  env $ev timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/abkt_$i -o kt --output-format csv -- python3 bench.py --no-cpu-baseline --no-alone --steps 10 --warmup 2 > gpurun_out/abkt_$i.log 2>&1 || { tail -5 gpurun_out/abkt_$i.log; exit 1; }
  echo "== $ev"
  python3 tools/trace_timeline.py $(find gpurun_out/abkt_$i -name "kt_kernel_trace.csv") 14
done
