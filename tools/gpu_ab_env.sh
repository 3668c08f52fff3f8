# GPU parity tests, then bench.py (C3) for each value of one env knob, REPS rounds:
# VAR=LSLAM_RNG_TABLE VALS="0 1" bash tools/gpu_ab_env.sh
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for rep in $(seq ${REPS:-2}); do for v in $VALS; do
  env $VAR=$v timeout -k 10 200 python -u bench.py --steps 40 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab_bench.json 2> gpurun_out/ab_bench.err || { tail -5 gpurun_out/ab_bench.err; exit 1; }
  echo "$VAR=$v $(python3 -c "import json; d=json.load(open('gpurun_out/ab_bench.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], r.get('kernel_ms'), r.get('consensus', {}).get('ms'))")"
done; done
