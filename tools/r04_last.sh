# round-4 final: the round profile of HEAD plus smoke()
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
bash tools/round_profile.sh r04f || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
