# round-4 session 2: C5 parity A/B (linear mask windows with the sensitivity shortcut vs the
# 9-VALU evaluation), then the round profile of the product build (GPU tests, bench, rocprof, C5, map, stamps)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
LIBS="lidar_slam_amd/variants/lib_masklin0.so lidar_slam_amd/liblidarslam.so" REPS=2 bash tools/c5_libs.sh || exit 1
bash tools/round_profile.sh ${TAG:-r04a}
