cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
LSLAM_POST_STREAM=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_dropin.py tests/test_gpu_map.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_ps.log 2>&1 || { tail -30 gpurun_out/gpu_tests_ps.log; exit 1; }
echo "post-stream: $(tail -1 gpurun_out/gpu_tests_ps.log)"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --also-philox --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench.json')); print('C3', d['value'], d['ms_per_step'], 'rng', d['roofline']['kernel_ms'], 'philox', d.get('philox_scans_per_s'))"
