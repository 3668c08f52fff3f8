#!/bin/bash
# One GPU session: parity tests, bench, rocprofv3 kernel trace + PMC passes.
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
STEPS=${STEPS:-20}
run() { local t=$1; shift; echo "== $*" >&2; timeout -k 10 "$t" "$@"; local rc=$?; echo "rc=$rc" >&2; return $rc; }
run 400 python -m pytest tests -m gpu -x -q > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
run 300 python bench.py --steps $STEPS --warmup 3 --also-philox > $OUT/bench.json 2> $OUT/bench.err || { cat $OUT/bench.err | tail -20; exit 1; }
cat $OUT/bench.json
run 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_kt -o kt --output-format csv -- python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 > $OUT/prof_kt.log 2>&1 || { tail -20 $OUT/prof_kt.log; exit 1; }
run 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/prof_fetch -o fetch --output-format csv -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > $OUT/prof_fetch.log 2>&1 || { tail -20 $OUT/prof_fetch.log; exit 1; }
run 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/prof_write -o write --output-format csv -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > $OUT/prof_write.log 2>&1 || { tail -20 $OUT/prof_write.log; exit 1; }
find $OUT -name "*.csv" | head -20
