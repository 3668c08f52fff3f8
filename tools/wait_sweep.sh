cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for w in 3 2 1 0; do
  echo "wait=$w $(LSLAM_DBG_WAIT=$w timeout -k 10 60 python -u tools/hostprobe.py 2>&1 | sed -n 1p | sed 's/.*step/step/')" || exit 1
done
