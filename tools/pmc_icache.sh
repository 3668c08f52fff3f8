# Instruction-cache counters per kernel: the C3 pipeline and the producer alone
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; OUT=gpurun_out/pmc_ic; mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE -d $OUT/pipe -o pipe --output-format csv -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > $OUT/pipe.log 2>&1 || { tail -5 $OUT/pipe.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE -d $OUT/alone -o alone --output-format csv -- python3 tools/drawsbench.py 4096 > $OUT/alone.log 2>&1 || { tail -5 $OUT/alone.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
for tag in ("pipe", "alone"):
    f = glob.glob("gpurun_out/pmc_ic/%s/*counter_collection.csv" % tag)[0]
    per = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.defaultdict(set)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"][:28]
        per[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[k].add(r["Dispatch_Id"])
    for k, v in per.items():
        d = len(n[k])
        print(tag, k, {c: round(x / d) for c, x in v.items()})
PY
