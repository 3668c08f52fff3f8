# C5 parity A/B over library builds: LIBS="a.so b.so" REPS=2 bash tools/c5_libs.sh
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for rep in $(seq ${REPS:-2}); do for lib in $LIBS; do
  LSLAM_ALLOW_STALE=1 LSLAM_LIB=$PWD/$lib timeout -k 10 200 python -u tools/c5bench.py --scans 4096 --hyp mt19937 --reps 2 > gpurun_out/c5_ab.json 2> gpurun_out/c5.err || { tail -5 gpurun_out/c5.err; exit 1; }
  echo "$lib $(cat gpurun_out/c5_ab.json)"
done; done
