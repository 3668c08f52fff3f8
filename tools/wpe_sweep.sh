cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for rep in 1 2; do
for w in 1 4; do
  export LSLAM_LIB=$PWD/lidar_slam_amd/liblidarslam_wpe$w.so
  for side in 0 1; do
  for pr in 000 033; do
  echo "rep=$rep wpe=$w side=$side prio=$pr $(LSLAM_UKF_SIDE=$side LSLAM_CONS_PRIO=$pr timeout -k 10 60 python -u tools/hostprobe.py 2>&1 | sed -n 1p | sed 's/.*step/step/')" || exit 1
  done; done
done; done
