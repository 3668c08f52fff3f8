# GPU tests, then C3 A/B of one env knob and map-mode A/B of another; every step time-limited.
# VAR=LSLAM_RESOLVE_REG VALS="1 2" MVAR=LSLAM_MT_SPECULATE MVALS="0 1" bash tools/round_ab.sh
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for rep in $(seq ${REPS:-2}); do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 200 python -u bench.py --steps 40 --warmup 3 --no-cpu-baseline --no-alone > gpurun_out/ab_bench.json 2> gpurun_out/ab_bench.err || { tail -5 gpurun_out/ab_bench.err; exit 1; }
    echo "$VAR=$v $(python3 -c "import json; d=json.load(open('gpurun_out/ab_bench.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], r.get('kernel_ms'), r.get('consensus', {}).get('ms'))")"
  done
  for v in $MVALS; do
    env $MVAR=$v timeout -k 10 200 python -u tools/mapbench.py > gpurun_out/ab_map.json 2> gpurun_out/ab_map.err || { tail -5 gpurun_out/ab_map.err; exit 1; }
    echo "map $MVAR=$v $(python3 -c "import json; d=json.load(open('gpurun_out/ab_map.json')); print(d['value'], d['ms_per_step'])")"
  done
done
