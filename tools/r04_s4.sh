# round-4 session 4: VALU encoding micro-benchmark; C3 A/B of the unchecked evaluations per table window (1 / 2 / 3)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 90 tools/ubench_valu > gpurun_out/ubench_valu2.json 2>&1 || { cat gpurun_out/ubench_valu2.json; exit 1; }
cat gpurun_out/ubench_valu2.json
LIBS="lidar_slam_amd/liblidarslam.so lidar_slam_amd/variants/lib_unch1.so lidar_slam_amd/variants/lib_unch3.so" REPS=3 bash tools/ab_multi.sh
ENVS="LSLAM_RESOLVE_STREAM=0|LSLAM_RESOLVE_STREAM=1|LSLAM_SLOTS=3" REPS=2 bash tools/ab_envs.sh
