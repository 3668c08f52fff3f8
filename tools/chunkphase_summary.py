"""Summarise tools/chunkphase.sh: instructions per C3 chunk of each chunk_kernel phase (the
difference of consecutive LSLAM_CHUNK_EXIT variants; Philox hypotheses, so phase 0 generates
the draws instead of reading the resolve's).  python tools/chunkphase_summary.py > profiles/<tag>_chunkphase.md"""
import csv
import glob
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
D = os.path.join(ROOT, "gpurun_out", "chunkphase")
ORDER = [("cx0", "owning scan, record init, Philox draws"), ("cx6", "point staging"),
         ("cx1", "bounding box + cutoffs"), ("cx2", "count pass"), ("cx3", "ties + selection"),
         ("cx4", "winner mask + refit"), ("full", "line record, mask / y_proj stores")]
CTRS = ["SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_BRANCH", "SQ_INSTS_LDS", "SQ_INSTS_SMEM"]


def per_chunk(v):
    f = glob.glob(os.path.join(D, v, "**", "*counter_collection.csv"), recursive=True)[0]
    per = {}
    for r in csv.DictReader(open(f)):
        if "chunk_kernel" not in r["Kernel_Name"]:
            continue
        per.setdefault(r["Dispatch_Id"], {}).setdefault(r["Counter_Name"], 0.0)
        per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    last = per[sorted(per, key=int)[-1]]  # the second launch
    nch = last["SQ_WAVES"]
    return {c: last[c] / nch for c in CTRS}, nch


rows, prev = [], {c: 0.0 for c in CTRS}
for v, name in ORDER:
    cur, nch = per_chunk(v)
    rows.append((name, {c: cur[c] - prev[c] for c in CTRS}))
    prev = cur
print("# chunk_kernel instructions per C3 chunk by phase (%d waves = chunks per launch)" % nch)
print()
print("| phase | VALU | SALU | branch | LDS | SMEM | total |")
print("|---|---|---|---|---|---|---|")
tot = {c: 0.0 for c in CTRS}
for name, d in rows:
    print("| %s | %s | %.0f |" % (name, " | ".join("%.0f" % d[c] for c in CTRS), sum(d.values())))
    for c in CTRS:
        tot[c] += d[c]
print("| **all** | %s | %.0f |" % (" | ".join("%.0f" % tot[c] for c in CTRS), sum(tot.values())))
