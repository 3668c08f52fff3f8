# GPU parity tests, bench.py A/B of one env knob, then a kernel trace of the default: one GPU call.
# VAR=LSLAM_RESOLVE_REG VALS="2 1" TAG=rr bash tools/ab_kt.sh
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_ab_env.sh || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG:-ab} -o kt --output-format csv -- python3 bench.py --no-cpu-baseline --no-alone --steps 10 --warmup 2 > gpurun_out/prof_${TAG:-ab}.log 2>&1 || exit 1
cat gpurun_out/prof_${TAG:-ab}/kt_kernel_stats.csv | cut -d, -f1-4,6,7
python3 tools/trace_timeline.py gpurun_out/prof_${TAG:-ab}/kt_kernel_trace.csv 14
