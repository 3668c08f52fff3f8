# C5 (4096 x 4096-point one-chunk scans, 2048 trials, mt19937) counted instructions per scan by kernel:
# one rocprofv3 --pmc pass over tools/c5bench.py (2 calls: the untimed first + 1 timed), then
#   python tools/c5_sq.py gpurun_out/c5sq/c5sq_counter_collection.csv
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}; mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/c5sq
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH -d gpurun_out/c5sq -o c5sq --output-format csv -- python3 tools/c5bench.py --scans 4096 --hyp mt19937 --reps 1 > gpurun_out/c5sq.log 2>&1 || { tail -5 gpurun_out/c5sq.log; exit 1; }
ls gpurun_out/c5sq
