cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for rep in 1 2; do for ps in 0 1; do
  echo "post_stream=$ps $(LSLAM_POST_STREAM=$ps timeout -k 10 60 python -u tools/hostprobe.py 2>&1 | sed -n 1p | sed 's/.*step/step/') map $(LSLAM_POST_STREAM=$ps timeout -k 10 120 python -u tools/mapbench.py 2>/dev/null | python3 -c 'import json,sys; print(json.load(sys.stdin)["ms_per_step"])')" || exit 1
done; done
