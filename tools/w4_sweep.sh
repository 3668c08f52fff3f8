cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for rep in 1 2; do for w4 in 0 1; do for pr in 033 133 233 333; do
  echo "w4=$w4 prio=$pr $(LSLAM_POST_W4=$w4 LSLAM_CONS_PRIO=$pr timeout -k 10 60 python -u tools/hostprobe.py 2>&1 | sed -n 1p | sed 's/.*step/step/')" || exit 1
done; done; done
