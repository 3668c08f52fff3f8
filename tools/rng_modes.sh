# producer alone (tools/drawsbench.py) for each LSLAM_RNG_TABLE value in VALS, twice
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for rep in 1 2; do for m in ${VALS:-0 1 2 3 4 5 6 7 8}; do
  echo "mode $m $(LSLAM_RNG_TABLE=$m timeout -k 10 120 python -u tools/drawsbench.py 1024 4096 | tail -1)" || exit 1
done; done
