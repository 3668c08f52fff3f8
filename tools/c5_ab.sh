# C5 parity A/B of an environment switch: VAR (default LSLAM_EPOCH_SERIAL) over VALS, REPS rounds
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
VAR=${VAR:-LSLAM_EPOCH_SERIAL}
for rep in $(seq ${REPS:-2}); do for v in ${VALS:-0 1}; do
  env $VAR=$v timeout -k 10 200 python -u tools/c5bench.py --scans 4096 --hyp mt19937 --reps 2 > gpurun_out/c5_$v.json 2> gpurun_out/c5.err || { tail -5 gpurun_out/c5.err; exit 1; }
  echo "$VAR=$v $(cat gpurun_out/c5_$v.json)"
done; done
