"""Per-scan counted instructions (SQ_INSTS_*) per kernel for the arms of tools/sq_ab.sh.

    python tools/sq_ab.py gpurun_out/sqab_A gpurun_out/sqab_B ...

Prints one table: kernel x class, a column per arm (per scan, 4096-scan C3 step), and the
total over VALU + SALU + branch + LDS + SMEM (s_nop / s_waitcnt are not counted by the SQ)."""
import csv
import os
import sys

KERNELS = {"seed_kernel": "seed_kernel", "cut_lane_kernel": "cut_lane_kernel", "rng_kernel": "rng_kernel", "resolve_reg": "resolve_reg",
           "chunk_kernel": "chunk_kernel", "ukf_group_kernel": "ukf_group_kernel", "fixup": "scan_kernel<0, 1>",
           "post": "post_reg_kernel"}
KINDS = ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_BRANCH", "SQ_INSTS_LDS", "SQ_INSTS_SMEM")


def per_scan(d, scans=4096):
    f = os.path.join(d, "sq1", "sq1_counter_collection.csv")
    rows = list(csv.DictReader(open(f)))
    out = {}
    for k, sub in KERNELS.items():
        for n in KINDS:
            per = {}
            for r in rows:
                if sub in r["Kernel_Name"] and r["Counter_Name"] == n:
                    per[r["Dispatch_Id"]] = per.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
            if per:
                out.setdefault(k, {})[n] = sum(per.values()) / len(per) / scans
    return out


def main(dirs):
    arms = [(os.path.basename(d.rstrip("/")), per_scan(d)) for d in dirs]
    print("| kernel | class | " + " | ".join(a for a, _ in arms) + " |")
    print("|---|---|" + "---|" * len(arms))
    tot = [0.0] * len(arms)
    for k in KERNELS:
        if not any(k in a for _, a in arms):
            continue
        ksum = [0.0] * len(arms)
        for n in KINDS:
            vals = [a.get(k, {}).get(n, 0.0) for _, a in arms]
            ksum = [x + y for x, y in zip(ksum, vals)]
            print("| %s | %s | " % (k, n[9:]) + " | ".join("%.0f" % v for v in vals) + " |")
        print("| %s | **all** | " % k + " | ".join("**%.0f**" % v for v in ksum) + " |")
        tot = [x + y for x, y in zip(tot, ksum)]
    print("| **step** | **all** | " + " | ".join("**%.0f**" % v for v in tot) + " |")


if __name__ == "__main__":
    main(sys.argv[1:])
