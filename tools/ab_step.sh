# A/B of the C3 step time only: another build A against the in-tree build, interleaved in both orders
cd $GRAFT_REPO_ROOT
A=${A:-lidar_slam_amd/liblidarslam_prev.so}
B=lidar_slam_amd/liblidarslam.so
for pair in "$A $B" "$B $A" "$A $B" "$B $A"; do for lib in $pair; do
  echo "$lib $(LSLAM_LIB=$PWD/$lib timeout -k 10 60 python -u tools/hostprobe.py 2>&1 | sed -n 1p | sed 's/.*step/step/')" || exit 1
done; done
