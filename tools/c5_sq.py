"""C5 counted instructions per scan and per call, by kernel (tools/c5_sq.sh), and the producer's
per-window figure against the expected MT19937 words of a C5 scan.

    python tools/c5_sq.py gpurun_out/c5sq/c5sq_counter_collection.csv [calls=2]

C5: 4096 one-chunk scans of 4096 points, 2048 trials (2049 draws, numpy's choice via Fisher-Yates
steps i = 4095..1, each step random_interval(i): a word accepted with probability
(i + 1) / (mask(i) + 1)).  The producer runs in epoch launches; the counters of every launch of
the profiled calls are summed and divided by calls x scans."""
import csv
import sys

KINDS = ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_BRANCH", "SQ_INSTS_LDS", "SQ_INSTS_SMEM")
KERNELS = (("rng_kernel", "rng_kernel"), ("resolve_walk", "resolve_walk"), ("model_kernel", "model_kernel"),
           ("count_kernel", "count_kernel"), ("select_kernel", "select_kernel"), ("fixup", "scan_kernel<0, 1>"),
           ("ukf_group_kernel", "ukf_group_kernel"), ("post", "post_reg_kernel"), ("seed_kernel", "seed_kernel"))


def expected_words(K=4095, draws=2049):
    def mask(i):
        m = i
        for s in (1, 2, 4, 8, 16):
            m |= m >> s
        return m
    return draws * sum((mask(i) + 1) / (i + 1) for i in range(1, K + 1))


def main(path, calls=2, scans=4096):
    rows = list(csv.DictReader(open(path)))
    tab = {}
    for name, sub in KERNELS:
        for r in rows:
            if sub in r["Kernel_Name"] and r["Counter_Name"] in KINDS:
                d = tab.setdefault(name, {})
                d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    print("| kernel | VALU | SALU | branch | LDS | SMEM | total per scan |")
    print("|---|---|---|---|---|---|---|")
    tot = 0.0
    for name, _ in KERNELS:
        if name not in tab:
            continue
        v = [tab[name].get(k, 0.0) / calls / scans for k in KINDS]
        tot += sum(v)
        print("| `%s` | %s | %.0f |" % (name, " | ".join("%.0f" % x for x in v), sum(v)))
    print("| **call** | | | | | | **%.0f** |" % tot)
    if "rng_kernel" in tab:
        words = expected_words()
        win = words / 64.0
        pr = sum(tab["rng_kernel"].get(k, 0.0) for k in KINDS) / calls / scans
        print()
        print("Producer: %.0f counted instructions per scan over %.0f expected words (%.0f 64-word windows, "
              "%.0f blocks): %.1f per window, %.3f per word." % (pr, words, win, words / 624.0, pr / win, pr / words))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 2)
