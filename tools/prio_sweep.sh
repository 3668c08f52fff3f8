cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for w in 033 133 233 333 022 011 000; do
  echo "prio(post,chunk,resolve)=$w $(LSLAM_CONS_PRIO=$w timeout -k 10 60 python -u tools/hostprobe.py 2>&1 | sed -n 1p | sed 's/.*step/step/')" || exit 1
done
