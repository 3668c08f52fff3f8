# per-step time vs the number of timed steps (fixed pipeline fill/drain cost), one box
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for k in 20 50 100 20; do
  timeout -k 10 200 python -u bench.py --steps $k --warmup 3 --no-cpu-baseline --no-alone > gpurun_out/ks.json 2> gpurun_out/ks.err || { tail -5 gpurun_out/ks.err; exit 1; }
  echo "K=$k $(python3 -c "import json; d=json.load(open('gpurun_out/ks.json')); print(d['ms_per_step'], d['roofline']['kernel_ms'])")"
done
