#!/bin/bash
# SQ counters of the parity-stream producer at 4096 scans (one pass per group).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/pmc_rng
mkdir -p $OUT
rocprofv3 -L > $OUT/counters.txt 2>&1 || true
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU" \
           "SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --pmc $grp -d $OUT/p$i -o p$i --output-format csv -- python3 tools/drawsbench.py 4096 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; }
done
find $OUT -name "*counter_collection.csv" | head
