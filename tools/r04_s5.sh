# round-4 session 5: SALU issue rate (micro-benchmark)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 90 tools/ubench_valu > gpurun_out/ubench_valu3.json 2>&1 || { cat gpurun_out/ubench_valu3.json; exit 1; }
cat gpurun_out/ubench_valu3.json
