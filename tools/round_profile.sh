# Everything profiles/<tag>_* holds, in one GPU call; each step time-limited, stop at the first failure.
# Usage: tools/round_profile.sh <tag>   (then: python tools/profile_summary.py <tag>)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
TAG=${1:?tag}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
tail -1 gpurun_out/bench.log
bash tools/profile_session.sh $TAG || exit 1
timeout -k 10 300 python -u tools/c5bench.py --scans 4096 --reps 2 > gpurun_out/c5.json 2> gpurun_out/c5.err || { tail -20 gpurun_out/c5.err; exit 1; }
cat gpurun_out/c5.json
timeout -k 10 300 python -u tools/mapbench.py > gpurun_out/mapbench.json 2> gpurun_out/mapbench.err || { tail -20 gpurun_out/mapbench.err; exit 1; }
cat gpurun_out/mapbench.json
# producer window segments (diagnostic variant lib_wstamps.so) and consensus phases (liblidarslam_stamps.so;
# Philox hypotheses: in mt19937 mode the producer's own stamps share the debug buffer)
if [ -f lidar_slam_amd/variants/lib_wstamps.so ]; then
  LSLAM_LIB=$PWD/lidar_slam_amd/variants/lib_wstamps.so timeout -k 10 120 python -u tools/wstamps.py > gpurun_out/${TAG}_wstamps.json 2> gpurun_out/ws.err || { tail -5 gpurun_out/ws.err; exit 1; }
  cat gpurun_out/${TAG}_wstamps.json
fi
if [ -f lidar_slam_amd/liblidarslam_stamps.so ]; then
  timeout -k 10 120 python -u tools/chunkstamps.py 4096 philox > gpurun_out/${TAG}_chunkstamps.json 2> gpurun_out/cs.err || { tail -5 gpurun_out/cs.err; exit 1; }
  cat gpurun_out/${TAG}_chunkstamps.json
fi
