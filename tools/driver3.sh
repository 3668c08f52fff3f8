cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/drv_$i.json 2> gpurun_out/drv_$i.err || { tail -5 gpurun_out/drv_$i.err; exit 1; }
  tail -1 gpurun_out/drv_$i.json | cut -c1-200
done
