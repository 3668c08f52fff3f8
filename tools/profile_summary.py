"""Summarise a tools/profile_session.sh run into profiles/.

  python tools/profile_summary.py <tag> [bench_log]
      reads gpurun_out/prof_<tag>/{kt,fetch,write,sq1,sq2} and the bench line of the
      same build (default gpurun_out/bench.log); writes profiles/<tag>_*

Kernel time comes from --kernel-trace --stats; HBM traffic from separate
--pmc FETCH_SIZE and --pmc WRITE_SIZE passes (MI355X_MICROARCH.md §HBM:
FETCH_SIZE/WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reads 1/2 of the bytes
of a wide coalesced stream, so the read side is doubled).
"""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
PROF = os.path.join(ROOT, "profiles")


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def counter(path, name, kernel_sub="scan_kernel"):
    """Per-dispatch sums (rows may be split per XCD/instance) of one counter."""
    per = {}
    for r in rows(path):
        if kernel_sub in r["Kernel_Name"] and r["Counter_Name"] == name:
            per[r["Dispatch_Id"]] = per.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return list(per.values())


# kernel-name substrings: producer, consensus, fix-up (scan_kernel<MT, RANSAC>), post pass (post_reg_kernel: the
# association-only pass with the list in registers; scan_kernel<EXPLICIT, ...> for the other post modes)
KERNELS = {"seed_kernel": "seed_kernel", "cut_lane_kernel": "cut_lane_kernel", "rng_kernel": "rng_kernel",
           "resolve_reg": "resolve_reg", "resolve_kernel": "resolve_kernel<",
           "chunk_kernel": "chunk_kernel", "ukf_group_kernel": "ukf_group_kernel", "fixup": "scan_kernel<0, 1>",
           "post": "post_reg_kernel", "post_scan": "scan_kernel<2, "}


def resolve_alg_bytes(beams, scans, trials):
    """The resolve's algorithmic bytes per launch: every Fisher-Yates step of a resolved draw read
    once (u8, chunks <= 256 points: K = N - 1 steps per draw) + the draws written (2 x int32 per
    draw).  The bench passes no draws_out, so the resolve skips draw T (the one skimage makes
    after the last trial): D = trials draws per chunk (D = 1 when trials = 0)."""
    sys.path.insert(0, ROOT)
    from lidar_slam_amd import synth
    sizes = synth.chunk_sizes(beams)
    D = max(trials, 1)
    steps = sum(D * (n - 1) for n in sizes if n >= 3)
    draws = sum(D * 8 for n in sizes if n >= 3)
    return scans * steps, scans * draws


def main(tag, bench_log=None):
    os.makedirs(PROF, exist_ok=True)
    S = os.path.join(OUT, "prof_" + tag)
    stats = rows(os.path.join(S, "kt", "kt_kernel_stats.csv"))
    bench = [json.loads(l) for l in open(bench_log or os.path.join(OUT, "bench.log")) if l.startswith("{")][-1]
    per = {}
    for k, sub in KERNELS.items():
        fetch = counter(os.path.join(S, "fetch", "fetch_counter_collection.csv"), "FETCH_SIZE", sub)
        write = counter(os.path.join(S, "write", "write_counter_collection.csv"), "WRITE_SIZE", sub)
        if not fetch or not write:
            continue
        f_kib = sum(fetch) / len(fetch)
        w_kib = sum(write) / len(write)
        per[k] = {"fetch_kib": f_kib, "write_kib": w_kib, "bytes_per_launch": int(2 * f_kib * 1024 + w_kib * 1024),
                  "avg_us": [float(r["AverageNs"]) / 1e3 for r in stats if sub in r["Name"]]}
    lines = ["# rocprofv3 summary: %s" % tag, "",
             "Command: `rocprofv3 --kernel-trace --stats -- python3 bench.py --no-cpu-baseline --steps 10 --warmup 2`",
             "(PMC: separate `--pmc FETCH_SIZE` and `--pmc WRITE_SIZE` passes, --steps 3 --warmup 1)", "",
             "| kernel | calls | avg us | min us | max us | % |", "|---|---|---|---|---|---|"]
    for r in stats:
        lines.append("| `%s` | %s | %.1f | %.1f | %.1f | %s |" % (
            r["Name"], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["MinNs"]) / 1e3,
            float(r["MaxNs"]) / 1e3, r["Percentage"]))
    lines += ["", "PMC HBM traffic per launch (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE):", ""]
    for k, v in per.items():
        lines.append("- `%s`: FETCH_SIZE %.1f KiB, WRITE_SIZE %.1f KiB -> %d bytes/launch"
                     % (k, v["fetch_kib"], v["write_kib"], v["bytes_per_launch"]))
    cfg = bench["config"]
    st, dr = resolve_alg_bytes(cfg["points_per_scan"], cfg["scans_per_gpu"], cfg["trials"])
    if "resolve_reg" in per:  # resolve_reg_kernel or resolve_reg8_kernel
        v = per["resolve_reg"]
        lines += ["", "Resolve, algorithmic vs PMC: steps read %d B + draws written %d B = %d B per launch; PMC read "
                  "%d B (x2 corrected), written %d B." % (st, dr, st + dr, int(2 * v["fetch_kib"] * 1024),
                                                         int(v["write_kib"] * 1024))]
    # the profiled process's own bench line: its HIP-event kernel time must agree with rocprof's
    scans = bench["config"]["scans_per_gpu"]
    sq = {}
    for p in ("sq1", "sq2"):
        f = os.path.join(S, p, p + "_counter_collection.csv")
        if not os.path.exists(f):
            continue
        for k, sub in KERNELS.items():
            names = {r["Counter_Name"] for r in rows(f)}
            for n in sorted(names):
                v = counter(f, n, sub)
                if v:
                    sq.setdefault(k, {})[n] = sum(v) / len(v)
    if sq:
        lines += ["", "SQ counters per launch (separate --pmc passes), and per scan (%d scans):" % scans, "",
                  "| kernel | counter | per launch | per scan |", "|---|---|---|---|"]
        for k, d in sq.items():
            for n, v in d.items():
                lines.append("| `%s` | %s | %.4g | %.4g |" % (k, n, v, v / scans))
        # Issue view of the whole step: wave-instructions per scan over every kernel,
        # per SIMD per step (4 scans per SIMD at 4096 scans on 1024 SIMDs), and the cycles per
        # instruction that leaves at the producer's own clock (SQ_WAVE_CYCLES are quad-cycles).
        kinds = ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_BRANCH", "SQ_INSTS_LDS", "SQ_INSTS_SMEM")
        tot = sum(d.get(n, 0.0) for d in sq.values() for n in kinds) / scans
        rng = sq.get("rng_kernel", {})
        roc = [float(r["AverageNs"]) / 1e3 for r in stats if "rng_kernel" in r["Name"]]
        if tot and rng.get("SQ_WAVE_CYCLES") and roc:
            ghz = 4.0 * rng["SQ_WAVE_CYCLES"] / scans / (roc[0] * 1e3)
            simds = 1024.0
            per_simd = tot * scans / simds
            step_cyc = bench["ms_per_step"] * 1e6 * ghz
            lines += ["", "Issue: %.0f wave-instructions per scan (VALU + SALU + branch + LDS + SMEM, all kernels), "
                      "%.0f per SIMD per step; at the producer's clock under the profiler (%.2f GHz: SQ_WAVE_CYCLES x 4 "
                      "per wave / rocprof average) the bench line's %.4f ms step is %.0f cycles = %.2f cycles per "
                      "instruction per SIMD (micro-benchmark: 2.0 for simple ops, 3.3 for v_bitop3/v_mbcnt/64-bit ops)."
                      % (tot, per_simd, ghz, bench["ms_per_step"], step_cyc, step_cyc / per_simd)]
    prof_line = [l for l in open(os.path.join(S, "kt.log")) if l.startswith('{"metric"')]
    if prof_line:
        pb = json.loads(prof_line[-1])
        roc = [float(r["AverageNs"]) / 1e3 for r in stats if "rng_kernel" in r["Name"]]
        lines += ["", "Dominant kernel, the profiled run itself: bench.py HIP events %.1f us per launch "
                  "(rng_kernel), rocprofv3 average %.1f us (%+.1f %%); step %.4f ms under the profiler."
                  % (1e3 * pb["roofline"]["kernel_ms"], roc[0] if roc else float("nan"),
                     100.0 * ((roc[0] if roc else 0) / (1e3 * pb["roofline"]["kernel_ms"]) - 1.0), pb["ms_per_step"])]
    lines += ["", "bench.py line of the same build (separate run, no profiler):", "", "```", json.dumps(bench), "```"]
    open(os.path.join(PROF, "%s_rocprof.md" % tag), "w").write("\n".join(lines) + "\n")
    for src in ("kt/kt_kernel_stats.csv",):
        data = open(os.path.join(S, src)).read()
        open(os.path.join(PROF, "%s_%s" % (tag, os.path.basename(src))), "w").write(data)
    t = {"tag": tag, "scans": scans, "hyp": bench["config"]["hyp"], "kernels": per,
         "sq_per_scan": {k: {n: v / scans for n, v in d.items()} for k, d in sq.items()}}
    json.dump(t, open(os.path.join(PROF, "traffic_latest.json"), "w"), indent=1)
    json.dump(bench, open(os.path.join(PROF, "%s_bench.json" % tag), "w"))
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
