# bench.py (C3, parity mode) A/B of an environment knob: VAR=name VALS="a b" [REPS=3]
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for rep in $(seq ${REPS:-3}); do for v in $VALS; do
  env $VAR=$v timeout -k 10 200 python -u bench.py --steps 40 --warmup 3 --no-cpu-baseline > gpurun_out/ab_bench.json 2> gpurun_out/ab_bench.err || { tail -5 gpurun_out/ab_bench.err; exit 1; }
  echo "$VAR=$v $(python3 -c "import json; d=json.load(open('gpurun_out/ab_bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])")"
done; done
