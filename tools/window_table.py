"""Per-window instruction classes of the producer's table-mode parse.

    python tools/window_table.py [wstamps.json] [traffic.json]  > profiles/<tag>_window_table.md

Static part (CPU, from the built library): disassembles rng_kernel<u8> and, for every inlined
table window (the asm block's TBLA_n/TBLX_n labels), takes the loop around it -- from the loop
header the back-edge jumps to, through the back-edge -- and sorts its instructions into
classes.  The checked-turn loop (TBLA_n .. TBLX_n holds two turns) is counted per turn;
everything else in the run loop once, divided by the windows one loop turn holds (two since
r05: `windows()`).

Dynamic part (GPU numbers already measured): the checked turns per window and windows per
scan from tools/wstamps.py, the SQ_INSTS_* per scan from profile_summary.py's
traffic_latest.json.  In-run windows x the static window give the in-run share; the rest of
the SQ counts are the parser's other work (twists of the next block, block switches and their
checked crossing windows, chunk-end windows, table copies, the epilogue)."""
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
SYM = "_Z10rng_kernelIhEv5KArgs"
CLASSES = ("VALU", "SALU", "s_nop", "s_waitcnt", "branch", "LDS", "VMEM", "SMEM")


def klass(m):
    if m.startswith("v_"):
        return "VALU"
    if m.startswith("ds_"):
        return "LDS"
    if m.startswith(("global_", "buffer_", "flat_")):
        return "VMEM"
    if m.startswith(("s_load", "s_buffer_load")):
        return "SMEM"
    if m.startswith("s_nop"):
        return "s_nop"
    if m.startswith("s_waitcnt"):
        return "s_waitcnt"
    if m.startswith(("s_cbranch", "s_branch")):
        return "branch"
    return "SALU"


def disassemble(lib):
    d = tempfile.mkdtemp(prefix="wtab_")
    so = os.path.join(d, "lib.so")
    shutil.copy(lib, so)
    subprocess.check_call([os.path.join(LLVM, "llvm-objdump"), "--offloading", so], cwd=d,
                          stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    co = [f for f in os.listdir(d) if "gfx950" in f][0]
    text = subprocess.check_output([os.path.join(LLVM, "llvm-objdump"), "-d", "--mcpu=gfx950",
                                    os.path.join(d, co)], text=True)
    shutil.rmtree(d)
    return text


def function(text, symbol):
    """[(addr, mnemonic, text, target or None)], labels {name: addr} of one function."""
    syms = {}
    for ln in text.splitlines():
        m = re.match(r"^([0-9a-f]+) <(.+)>:$", ln)
        if m:
            syms[m.group(2)] = int(m.group(1), 16)
    lines = text.splitlines()
    start = next(i for i, ln in enumerate(lines) if ln.endswith("<%s>:" % symbol))
    out, labels = [], {}
    for ln in lines[start + 1:]:
        m = re.match(r"^([0-9a-f]+) <(.+)>:$", ln)
        if m:
            if not m.group(2).startswith("TBL"):
                break
            labels[m.group(2)] = int(m.group(1), 16)
            continue
        m = re.match(r"^\s+(\S+)\s*(.*?)\s*//\s*([0-9A-F]+):", ln)
        if not m:
            continue
        tgt = None
        if m.group(1).startswith(("s_cbranch", "s_branch")):
            t = re.search(r"<([^+>]+)(?:\+0x([0-9a-f]+))?>", ln)
            if t:
                tgt = syms[t.group(1)] + (int(t.group(2), 16) if t.group(2) else 0)
        out.append((int(m.group(3), 16), m.group(1), m.group(2), tgt))
    return out, labels


def windows(ins, labels):
    """One entry per run loop that holds inlined table windows: the loop is the innermost
    back-edge around a window's asm block (the checked-turn branches back to TBLA_n itself are
    not loops of the run).  Since r05 a loop turn holds two windows (`parse_chunk_tbl`: one
    loop test and one address step per pair), so the loop's instructions outside the windows'
    checked-turn spans are divided by the windows it holds; each span (TBLA_n .. TBLX_n, two
    turns) is counted per turn.  A window outside every loop (the odd window of a run with an
    odd count, ahead of the loop) is listed by itself and not used for the per-window figure."""
    addrs = [a for a, *_ in ins]
    tbla = sorted((a, n) for n, a in labels.items() if n.startswith("TBLA"))
    spans = {n: (addrs.index(a), addrs.index(labels["TBLX" + n[4:]])) for a, n in tbla}
    loops = []  # (i_header, i_back) of back-edges that are not a checked-turn branch
    tbla_addrs = {a for a, _ in tbla}
    for j, (a, m, _, t) in enumerate(ins):
        if t is not None and t < a and m.startswith(("s_cbranch", "s_branch")) and t not in tbla_addrs:
            loops.append((addrs.index(t), j))
    res = []
    seen = {}
    for a, name in tbla:
        i_a, i_x = spans[name]
        around = [(h, b) for h, b in loops if h <= i_a and i_x < b and b - h < 300]
        if not around:
            res.append({"label": name, "loop": None, "windows": 1})
            continue
        h, b = min(around, key=lambda hb: hb[1] - hb[0])
        seen.setdefault((h, b), []).append(name)
    for (h, b), names in seen.items():
        inside = {c: 0 for c in CLASSES}
        turn2 = {c: 0 for c in CLASSES}
        in_span = set()
        for n in names:
            i_a, i_x = spans[n]
            in_span.update(range(i_a, i_x))
        for j in range(h, b + 1):
            c = klass(ins[j][1])
            if j in in_span:
                turn2[c] += 1
            else:
                inside[c] += 1
        nw = len(names)
        res.append({"label": "+".join(names), "loop": (ins[h][0], ins[b][0]), "windows": nw, "loop_len": b + 1 - h,
                    "fixed": {c: v / nw for c, v in inside.items()},
                    "per_turn": {c: v / (2.0 * nw) for c, v in turn2.items()}})
    return res


def main():
    from lidar_slam_amd import build
    lib = build.build(verbose=False)
    ins, labels = function(disassemble(lib), SYM)
    wins = windows(ins, labels)
    ws = json.load(open(sys.argv[1])) if len(sys.argv) > 1 else None
    tr = json.load(open(sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "profiles", "traffic_latest.json")))
    sq = tr["sq_per_scan"]["rng_kernel"]
    turns = ws["checked_turns_per_window"] if ws else 2.85
    nwin = ws["windows_per_scan"] if ws else None
    L = ["# Producer table window: instruction classes", "",
         "Static: `rng_kernel<u8>` of the built library (`tools/window_table.py`), every inlined run-loop window "
         "(asm block `TBLA_n`); the checked-turn loop counted per turn. `s_nop` and `s_waitcnt` are shown apart "
         "from the other SALU.", "",
         "| window | loop instructions | " + " | ".join(CLASSES) + " |", "|---|---|" + "---|" * len(CLASSES)]
    for w in wins:
        if w["loop"] is None:
            L.append("| `%s` (outside a loop: a run's odd first window) | | %s |" % (w["label"], " | ".join("" for _ in CLASSES)))
            continue
        L.append("| `%s` fixed, per window (loop %#x-%#x: %d instructions, %d windows) | %d | "
                 % (w["label"], w["loop"][0], w["loop"][1], w["loop_len"], w["windows"], w["loop_len"]) +
                 " | ".join("%g" % w["fixed"][c] for c in CLASSES) + " |")
        L.append("| `%s` per checked turn | | " % w["label"] + " | ".join("%g" % w["per_turn"][c] for c in CLASSES) + " |")
    looped = [w for w in wins if w["loop"] is not None]
    if looped and nwin:
        # the dominant in-run window: C3's 100-point chunks (K = 99 >= 64: rt_wrap is one
        # subtract-and-min, no loop), the shortest run loop per window
        w = min(looped, key=lambda w: w["loop_len"] / w["windows"])
        per = {c: w["fixed"][c] + turns * w["per_turn"][c] for c in CLASSES}
        L += ["", "Per in-run window at %.3f checked turns (wstamps, C3), window `%s`: " % (turns, w["label"]) +
              ", ".join("%s %.1f" % (c, per[c]) for c in CLASSES) + " = %.1f instructions." % sum(per.values()), ""]
        L += ["Per scan (%.1f in-run windows, wstamps) against the SQ counters of the profiled bench:" % nwin, "",
              "| class | in-run windows | SQ counter per scan | rest of the parser |", "|---|---|---|---|"]
        pairs = [("VALU", ["VALU"], "SQ_INSTS_VALU"), ("SALU (s_nop, s_waitcnt not counted)", ["SALU"], "SQ_INSTS_SALU"),
                 ("branch", ["branch"], "SQ_INSTS_BRANCH"), ("LDS", ["LDS"], "SQ_INSTS_LDS"), ("SMEM", ["SMEM"], "SQ_INSTS_SMEM")]
        for name, cs, ctr in pairs:
            a = nwin * sum(per[c] for c in cs)
            L.append("| %s | %.0f | %.0f | %.0f |" % (name, a, sq.get(ctr, 0.0), sq.get(ctr, 0.0) - a))
        L.append("| VMEM (the steps' stores) | %.0f | | |" % (nwin * per["VMEM"]))
        L += ["", "SQ_INSTS_SALU counts neither `s_nop` nor `s_waitcnt` (`tools/ubench_nopcount.hip`, "
              "`profiles/r05_ubench_nopcount.txt`): the in-run window's %.1f `s_nop` (the hazard wait states of "
              "tools/hazard_probe.hip) and %.1f `s_waitcnt`, %.0f and %.0f per scan, are issued on top of the "
              "counters' total." % (per["s_nop"], per["s_waitcnt"], nwin * per["s_nop"], nwin * per["s_waitcnt"])]
    print("\n".join(L))


if __name__ == "__main__":
    sys.path.insert(0, ROOT)
    main()
