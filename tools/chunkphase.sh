# Per-phase instruction counts of chunk_kernel: one rocprofv3 SQ pass per
# LSLAM_CHUNK_EXIT variant (built beforehand: python tools/build_variants.py cx0=-DLSLAM_CHUNK_EXIT=0 ...),
# then python tools/chunkphase_summary.py.  Every pass time-limited; stop at the first failure.
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}; mkdir -p gpurun_out/chunkphase; export TMPDIR=/tmp
for v in cx0 cx6 cx1 cx2 cx3 cx4 full; do
  if [ $v = full ]; then lib=lidar_slam_amd/liblidarslam.so; else lib=lidar_slam_amd/variants/lib_$v.so; fi
  export LSLAM_LIB=$PWD/$lib LSLAM_ALLOW_STALE=1
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_INSTS_SMEM \
    -d gpurun_out/chunkphase/$v -o $v --output-format csv -- python3 tools/chunkphase.py > gpurun_out/chunkphase/$v.log 2>&1 \
    || { echo "pass $v failed"; tail -5 gpurun_out/chunkphase/$v.log; exit 1; }
  echo "$v ok"
done
