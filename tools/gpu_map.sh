set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_map.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/map_tests.log 2>&1 || { tail -30 gpurun_out/map_tests.log; exit 1; }
tail -2 gpurun_out/map_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -30 gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 300 python -u tools/mapbench.py > gpurun_out/mapbench.json 2> gpurun_out/mapbench.err || { tail -20 gpurun_out/mapbench.err; exit 1; }
cat gpurun_out/mapbench.json
timeout -k 10 300 python -u tools/mapbench.py --hyp philox > gpurun_out/mapbench_philox.json 2>> gpurun_out/mapbench.err || { tail -20 gpurun_out/mapbench.err; exit 1; }
cat gpurun_out/mapbench_philox.json
