"""Average SQ counters per dispatch of one kernel from tools/pmc_rng.sh output."""
import collections
import csv
import glob
import sys

kern = sys.argv[1] if len(sys.argv) > 1 else "rng_kernel"
units = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
tot = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/pmc_rng/p*/p*_counter_collection.csv")):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if kern not in r["Kernel_Name"]:
            continue
        per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (d, n), v in per.items():
        tot[n].append(v)
for n, v in sorted(tot.items()):
    m = sum(v) / len(v)
    print("%-22s %12.4g   per unit %10.4g" % (n, m, m / units))
