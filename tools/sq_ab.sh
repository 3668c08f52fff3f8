# Counted instructions per scan for several library builds (every perf change
# with the SQ instruction delta of the kernels it touches).  One rocprofv3 --pmc pass per build,
# each time-limited; stop at the first failure.
# LIBS="lidar_slam_amd/variants/lib_a.so lidar_slam_amd/liblidarslam.so" bash tools/sq_ab.sh
# then: python tools/sq_ab.py gpurun_out/sqab_*
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}; mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in $LIBS; do
  name=$(basename $lib .so)
  out=gpurun_out/sqab_$name
  rm -rf $out; mkdir -p $out
  LSLAM_ALLOW_STALE=1 LSLAM_LIB=$PWD/$lib timeout -k 10 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH -d $out/sq1 -o sq1 --output-format csv -- python3 bench.py --no-cpu-baseline --no-alone --no-coupled --steps 3 --warmup 1 > $out/sq1.log 2>&1 || { echo "sq pass failed: $lib"; tail -5 $out/sq1.log; exit 1; }
  echo "$lib ok"
done
