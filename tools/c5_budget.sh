# C5 parity over producer slot budgets (epoch sizes): LIB=x.so BUDGETS="2 8 16" bash tools/c5_budget.sh
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for b in ${BUDGETS:-2 8 16}; do
  LSLAM_ALLOW_STALE=1 LSLAM_LIB=$PWD/${LIB:-lidar_slam_amd/liblidarslam.so} timeout -k 10 200 python -u tools/c5bench.py --scans 4096 --hyp mt19937 --reps 2 --budget-gib $b > gpurun_out/c5_b.json 2> gpurun_out/c5_b.err || { tail -5 gpurun_out/c5_b.err; exit 1; }
  echo "budget $b GiB $(cat gpurun_out/c5_b.json)"
done
