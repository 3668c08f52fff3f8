"""Per-window instruction classes of the producer's table-mode parse.

    python tools/window_table.py [wstamps.json] [traffic.json]  > profiles/<tag>_window_table.md

Static part (CPU, from the built library): disassembles rng_kernel<u8> and, for every inlined
table window (the asm block's TBLA_n/TBLX_n labels), takes the loop around it -- from the loop
header the back-edge jumps to, through the back-edge -- and sorts its instructions into
classes.  The checked-turn loop (TBLA_n .. TBLX_n holds two turns) is counted per turn;
everything else in the window loop once.

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
    """One entry per inlined window: the static counts of its loop outside the checked turns,
    per checked turn, and whether it is a run loop (has a back-edge around the block)."""
    res = []
    addrs = [a for a, *_ in ins]
    for name, a_tbla in sorted(labels.items(), key=lambda kv: kv[1]):
        if not name.startswith("TBLA"):
            continue
        a_tblx = labels["TBLX" + name[4:]]
        i_a, i_x = addrs.index(a_tbla), addrs.index(a_tblx)
        # the run loop: the first backward branch after TBLX whose target lies before TBLA
        back = None
        for j in range(i_x, min(i_x + 80, len(ins))):
            t = ins[j][3]
            if t is not None and t < a_tbla and ins[j][1].startswith("s_cbranch"):
                back = j
                break
        if back is None:
            continue
        i_h = addrs.index(ins[back][3])
        if a_tbla - ins[i_h][0] > 1024:  # not this window's loop
            continue
        fixed = {c: 0 for c in CLASSES}
        turn2 = {c: 0 for c in CLASSES}
        for j in range(i_h, back + 1):
            c = klass(ins[j][1])
            if i_a <= j < i_x:
                turn2[c] += 1
            else:
                fixed[c] += 1
        turn = {c: v / 2.0 for c, v in turn2.items()}
        res.append({"label": name, "fixed": fixed, "per_turn": turn, "loop_len": back + 1 - i_h})
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
        L.append("| `%s` fixed | %d | " % (w["label"], w["loop_len"]) + " | ".join("%g" % w["fixed"][c] for c in CLASSES) + " |")
        L.append("| `%s` per checked turn | | " % w["label"] + " | ".join("%g" % w["per_turn"][c] for c in CLASSES) + " |")
    if wins and nwin:
        # the dominant in-run window: C3's 100-point chunks (K = 99 >= 64: rt_wrap is one
        # subtract-and-min, no loop), the shortest run loop
        w = min(wins, key=lambda w: w["loop_len"])
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
