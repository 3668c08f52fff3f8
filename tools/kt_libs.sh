# Kernel traces of bench.py over several library builds (per-kernel average durations):
# LIBS="lidar_slam_amd/variants/lib_a.so lidar_slam_amd/liblidarslam.so" bash tools/kt_libs.sh
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for lib in $LIBS; do
  i=$((i+1))
  export LSLAM_ALLOW_STALE=1 LSLAM_LIB=$PWD/$lib
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_$i -o kt --output-format csv -- python3 bench.py --no-cpu-baseline --no-alone --steps 20 --warmup 3 > gpurun_out/kt_$i.log 2>&1 || { tail -5 gpurun_out/kt_$i.log; exit 1; }
  echo "== $lib"
  cut -d, -f1-4 gpurun_out/kt_$i/kt_kernel_stats.csv | head -12
done
