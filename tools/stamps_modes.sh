cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for m in 0 1 2; do
  echo "mode $m draws $(LSLAM_RNG_TABLE=$m timeout -k 10 120 python -u tools/drawsbench.py 1024 4096 | tail -1)" || exit 1
  LSLAM_RNG_TABLE=$m timeout -k 10 120 python -u tools/stamps.py 4096 > gpurun_out/stamps_$m.json || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/stamps_$m.json')); print({k: d[k] for k in ('shares','cycles_per_window','iterations_per_window','parser_us_p50_max','parser_us_by_age_rank')})"
done
