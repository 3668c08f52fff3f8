cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for w in 0 256 512 1024 2048 4096; do
  if [ $w = 0 ]; then unset LSLAM_CONSUMER_WGS; else export LSLAM_CONSUMER_WGS=$w; fi
  echo "wgs=$w $(timeout -k 10 60 python -u tools/hostprobe.py 2>&1 | sed -n 1p | sed 's/.*step/step/')" || exit 1
done
