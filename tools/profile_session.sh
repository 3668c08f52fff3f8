#!/bin/bash
# rocprofv3 session on the C3 bench: kernel trace + stats, HBM passes (FETCH_SIZE, WRITE_SIZE),
# SQ instruction-mix passes.  Each pass is its own time-limited run; stop at the first failure.
# Usage: tools/profile_session.sh <tag> [bench args...]
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=${1:?tag}; shift
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
B="bench.py --no-cpu-baseline --no-alone --no-coupled $*"
run() { local t=$1; shift; echo "== $*" >&2; timeout -k 10 "$t" "$@"; local rc=$?; echo "rc=$rc" >&2; return $rc; }
run 240 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 $B --steps 10 --warmup 2 > $OUT/kt.log 2>&1 || exit 1
run 180 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o fetch --output-format csv -- python3 $B --steps 3 --warmup 1 > $OUT/fetch.log 2>&1 || exit 1
run 180 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o write --output-format csv -- python3 $B --steps 3 --warmup 1 > $OUT/write.log 2>&1 || exit 1
run 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH -d $OUT/sq1 -o sq1 --output-format csv -- python3 $B --steps 3 --warmup 1 > $OUT/sq1.log 2>&1 || exit 1
run 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY -d $OUT/sq2 -o sq2 --output-format csv -- python3 $B --steps 3 --warmup 1 > $OUT/sq2.log 2>&1 || exit 1
find $OUT -name "*.csv" | sort
