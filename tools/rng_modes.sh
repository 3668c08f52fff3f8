# producer alone (tools/drawsbench.py) with the table-mode parse off (0) and on (1), twice
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for rep in 1 2; do for m in ${VALS:-0 1}; do
  echo "mode $m $(LSLAM_RNG_TABLE=$m timeout -k 10 120 python -u tools/drawsbench.py 1024 4096 | tail -1)" || exit 1
done; done
