# GPU tests + C3 bench (parity + Philox) + map bench; every step time-limited, stop at the first failure
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --also-philox --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench.json')); print('C3', d['value'], d['ms_per_step'], 'rng', d['roofline']['kernel_ms'], 'philox', d.get('philox_scans_per_s'))"
timeout -k 10 300 python -u tools/mapbench.py > gpurun_out/mapbench.json 2> gpurun_out/mapbench.err || { tail -20 gpurun_out/mapbench.err; exit 1; }
cat gpurun_out/mapbench.json
