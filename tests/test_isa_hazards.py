"""The hand-placed wait states of the producer's asm table window, pinned to the compiler's own
gfx950 hazard model (CPU test: needs hipcc and llvm-objdump, no GPU).

``lslam_rng_pipe.h`` tbl_window issues the fixed-point evaluations of the table-mode parse
(fit.py:819-826 behind ransac_functions.py:23-24: numpy's random_interval rejection) as one
asm block, so the compiler's hazard recognizer does not see them; the block places its wait
states by hand:

  (A) one between ``v_lshlrev_b64 v[28:29]`` and the v_cmp that reads v29;
  (B) two between a v_cmp writing VCC or s[40:41] and the v_mbcnt that reads it as a lane mask
      (an ``s_nop 1``, or the ``s_cmp`` + ``s_cbranch`` of a checked turn).

``tools/hazard_probe.hip`` writes the same evaluation chain in plain HIP (dependent and
unrolled, so the scheduler has nothing to fill the gaps with): the wait states the compiler puts
there are its requirement for gfx950.  This test reads them from the probe's assembly and then
walks every control-flow path of the built library's ``rng_kernel`` (both step widths) from
each such writer to its first VALU reader, checking that no path has fewer.

The resolve's full groups (``lidarslam.hip`` rr_group_sdwa) are hand-scheduled the same way:

  (C) two wait states between a v_cmp writing its mask SGPR pair and the v_cndmask reading it
      (the probe's second kernel, SDWA byte compares and selects of two dependent trackers,
      gives the compiler's requirement);
  (D) one between a VALU write of a VGPR and an SDWA compare reading it (the trackers and the
      pre-masked dwords), and one between a v_cndmask and the next SDWA instruction.  The
      compiler's own SDWA chains put an ``s_nop 0`` in those places in most but not all cases
      (a tight pair appears in the probe too), so (D) is a conservative rule of ours rather than
      one read off the probe.

The consensus count loop's four-point blocks (``lidarslam.hip`` count_four) likewise:

  (E) a v_fma_f64 and the first VALU reading its result: the compiler needs none (so the block
      may chain its FMAs freely);
  (F) two wait states between a v_cmp writing its mask SGPR pair and the v_addc reading it as
      the carry-in (the probe's third kernel).

A toolchain or firmware change to these hazard rules then fails here, on the CPU, instead of as
a rare wrong draw or count on the GPU.
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

pytestmark = pytest.mark.skipif(not (os.path.exists(HIPCC) and os.path.exists(os.path.join(LLVM, "llvm-objdump"))),
                                reason="needs hipcc and llvm-objdump")

_REG = re.compile(r"(?<!\w)(v\[\d+:\d+\]|s\[\d+:\d+\]|[vs]\d+\b|vcc_lo\b|vcc_hi\b|vcc\b|exec\b)")


def _regs(text):
    """Registers named in an operand list, ranges expanded (vcc -> vcc_lo, vcc_hi)."""
    out = set()
    for r in _REG.findall(text):
        m = re.match(r"([vs])\[(\d+):(\d+)\]", r)
        if m:
            out.update("%s%d" % (m.group(1), i) for i in range(int(m.group(2)), int(m.group(3)) + 1))
        elif r == "vcc":
            out.update(("vcc_lo", "vcc_hi"))
        else:
            out.add(r)
    return out


class Insn:
    def __init__(self, addr, mnem, ops, target=None):
        self.addr, self.mnem, self.ops, self.target = addr, mnem, ops, target
        parts = [p.strip() for p in ops.split(",")] if ops else []
        self.dst = _regs(parts[0]) if parts else set()
        self.src = set().union(*[_regs(p) for p in parts[1:]]) if len(parts) > 1 else set()
        if mnem.startswith("v_cmp") and mnem.endswith("_e32"):  # VOPC: vcc is the implicit destination
            self.src |= self.dst
            self.dst = {"vcc_lo", "vcc_hi"}

    @property
    def wait(self):
        m = re.match(r"s_nop\s+(\d+)", self.mnem + " " + self.ops)
        return int(m.group(1)) + 1 if m else 1


def _parse_s(text):
    """Instructions of a compiler .s file, in order (labels and directives dropped)."""
    out = []
    for ln in text.splitlines():
        ln = ln.split(";")[0].rstrip()
        if not re.match(r"^\s+[sv]_", ln):
            continue
        f = ln.strip().split(None, 1)
        out.append(Insn(len(out), f[0], f[1] if len(f) > 1 else ""))
    return out


def _parse_objdump(text, symbol):
    """Instructions of one function of llvm-objdump -d output, with addresses and branch targets.
    The asm block's local labels (TBLA_n / TBLX_n) appear as symbols inside the function."""
    syms = {}
    for ln in text.splitlines():
        m = re.match(r"^([0-9a-f]+) <(.+)>:$", ln)
        if m:
            syms[m.group(2)] = int(m.group(1), 16)
    lines = text.splitlines()
    start = next(i for i, ln in enumerate(lines) if ln.endswith("<%s>:" % symbol))
    out = []
    for ln in lines[start + 1:]:
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", ln)
        if m and not m.group(1).startswith("TBL"):
            break  # the next function
        m = re.match(r"^\s+(\S+)\s*(.*?)\s*//\s*([0-9A-F]+):", ln)
        if not m:
            continue
        mnem, ops, addr = m.group(1), m.group(2), int(m.group(3), 16)
        tgt = None
        if mnem.startswith("s_cbranch") or mnem == "s_branch":
            t = re.search(r"<([^+>]+)(?:\+0x([0-9a-f]+))?>", ln)
            tgt = syms[t.group(1)] + (int(t.group(2), 16) if t.group(2) else 0) if t else None
            ops = ""
        out.append(Insn(addr, mnem, ops, tgt))
    return out


def _min_wait(insns, is_writer, regs_of, is_reader, need=None):
    """Smallest number of wait states on any control-flow path from a writer to the first
    instruction reading what it wrote (is_reader), over all writers; paths stop where the
    registers are overwritten or `need` wait states have passed."""
    index = {x.addr: i for i, x in enumerate(insns)}
    best = None
    for i, w in enumerate(insns):
        if not is_writer(w):
            continue
        regs = regs_of(w)
        stack, seen = [(i + 1, 0)], set()
        while stack:
            j, ws = stack.pop()
            if j >= len(insns) or (j, ws) in seen:
                continue
            seen.add((j, ws))
            x = insns[j]
            if is_reader(x, regs):
                best = ws if best is None else min(best, ws)
                continue
            if x.dst & regs and not x.mnem.startswith("s_cbranch"):
                continue
            if need is not None and ws >= need:
                continue
            if x.mnem in ("s_endpgm", "s_setpc_b64"):
                continue
            nws = ws + x.wait
            if x.mnem == "s_branch":
                if x.target in index:
                    stack.append((index[x.target], nws))
                continue
            stack.append((j + 1, nws))
            if x.mnem.startswith("s_cbranch") and x.target in index:
                stack.append((index[x.target], nws))
    return best


def _shift_writer(x):
    return x.mnem == "v_lshlrev_b64"


def _shift_regs(x):
    return {max(x.dst, key=lambda r: int(r[1:]))}  # the high dword


def _valu_reads(x, regs):
    return x.mnem.startswith("v_") and bool(x.src & regs)


def _mbcnt_reads(x, regs):
    return x.mnem.startswith("v_mbcnt") and bool(x.src & regs)


def _mask_writer(x):
    return x.mnem.startswith("v_cmp") and bool(x.dst & {"vcc_lo", "vcc_hi"} or any(r.startswith("s") for r in x.dst))


def _mask_regs(x):
    return set(x.dst)


def _cndmask_reads(x, regs):
    return x.mnem.startswith("v_cndmask") and bool(x.src & regs)


def _addc_reads(x, regs):
    return x.mnem.startswith("v_addc") and bool(x.src & regs)


def _fma64_writer(x):
    return x.mnem in ("v_fma_f64", "v_fmac_f64_e32")


def _vgpr_writer(x):
    return x.mnem.startswith("v_") and any(r.startswith("v") and r[1:].isdigit() for r in x.dst)


def _vgpr_regs(x):
    return {r for r in x.dst if r.startswith("v") and r[1:].isdigit()}


def _sdwa_reads(x, regs):
    return x.mnem.endswith("_sdwa") and bool(x.src & regs)


@pytest.fixture(scope="module")
def probe_waits(tmp_path_factory):
    d = tmp_path_factory.mktemp("probe")
    out = str(d / "probe.s")
    subprocess.check_call([HIPCC, "--offload-arch=gfx950", "-O3", "--cuda-device-only", "-S", "-o", out,
                           os.path.join(ROOT, "tools", "hazard_probe.hip")], stderr=subprocess.DEVNULL)
    ins = _parse_s(open(out).read())
    a = _min_wait(ins, _shift_writer, _shift_regs, _valu_reads)
    b = _min_wait(ins, _mask_writer, _mask_regs, _mbcnt_reads)
    c = _min_wait(ins, _mask_writer, _mask_regs, _cndmask_reads)
    e = _min_wait(ins, _fma64_writer, _vgpr_regs, _valu_reads)
    f = _min_wait(ins, _mask_writer, _mask_regs, _addc_reads)
    assert None not in (a, b, c, e, f), "probe: a chain not found"
    assert any(x.mnem.endswith("_sdwa") for x in ins), "probe: no SDWA compare emitted"
    return a, b, c, e, f


@pytest.fixture(scope="module")
def library_code(tmp_path_factory):
    from lidar_slam_amd import build
    lib = build.build(verbose=False)
    d = tmp_path_factory.mktemp("lib")
    so = str(d / "lib.so")
    shutil.copy(lib, so)
    subprocess.check_call([os.path.join(LLVM, "llvm-objdump"), "--offloading", so], cwd=str(d),
                          stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    co = [f for f in os.listdir(str(d)) if "gfx950" in f]
    assert co, "no gfx950 code object in the library"
    return subprocess.check_output([os.path.join(LLVM, "llvm-objdump"), "-d", "--mcpu=gfx950", str(d / co[0])],
                                   text=True)


def test_probe_matches_the_documented_rules(probe_waits):
    """The compiler's requirement is what the sources' comments state: (A) 1, (B) 2 in
    lslam_rng_pipe.h; (C) 2 at rr_group_sdwa; (E) 0, (F) 2 at count_four."""
    assert probe_waits == (1, 2, 2, 0, 2)


@pytest.mark.parametrize("symbol", ["_Z10rng_kernelIhEv5KArgs", "_Z10rng_kernelItEv5KArgs"])
def test_rng_kernel_asm_window_wait_states(probe_waits, library_code, symbol):
    need_a, need_b = probe_waits[:2]
    ins = _parse_objdump(library_code, symbol)
    assert sum(x.mnem == "v_lshlrev_b64" for x in ins) >= 8, "asm table window not found"
    # (paths stop once `need` wait states have passed: a writer whose every path is padded that
    # far records nothing; the asm block's own pairs sit exactly at the bound)
    a = _min_wait(ins, _shift_writer, _shift_regs, _valu_reads, need=need_a)
    b = _min_wait(ins, _mask_writer, _mask_regs, _mbcnt_reads, need=need_b)
    assert a == need_a, ("v_lshlrev_b64 -> VALU reader", a, need_a)
    assert b == need_b, ("v_cmp mask -> v_mbcnt", b, need_b)


def test_resolve_sdwa_group_wait_states(probe_waits, library_code):
    need_c = probe_waits[2]
    ins = _parse_objdump(library_code, "_Z19resolve_reg8_kernel5KArgsi")
    assert sum(x.mnem == "v_cmp_eq_u32_sdwa" for x in ins) >= 2 * 15 * 7, "SDWA groups not found"
    c = _min_wait(ins, _mask_writer, _mask_regs, _cndmask_reads, need=need_c)
    assert c == need_c, ("v_cmp mask -> v_cndmask", c, need_c)
    # (D): paths stop after one wait state, so None = every pair has at least one
    d = _min_wait(ins, _vgpr_writer, _vgpr_regs, _sdwa_reads, need=1)
    assert d in (None, 1), ("VALU VGPR write -> SDWA read", d)
    e = _min_wait(ins, lambda x: x.mnem.startswith("v_cndmask"), lambda x: set(),
                  lambda x, regs: x.mnem.endswith("_sdwa"), need=1)
    assert e in (None, 1), ("v_cndmask -> SDWA", e)


@pytest.mark.parametrize("symbol", ["_Z12chunk_kernelILi0EEv5KArgs", "_Z12chunk_kernelILi1EEv5KArgs",
                                    "_Z12chunk_kernelILi2EEv5KArgs"])
def test_consensus_count_block_wait_states(probe_waits, library_code, symbol):
    need_f = probe_waits[4]
    ins = _parse_objdump(library_code, symbol)
    blocks = sum(x.mnem == "v_addc_co_u32_e64" and "s[80:81]" in x.ops for x in ins)
    assert blocks >= 2 * 5, "count_four blocks not found"
    # paths stop after need_f wait states: None or need_f = every mask -> carry-in pair has enough
    f = _min_wait(ins, _mask_writer, _mask_regs, _addc_reads, need=need_f)
    assert f is None or f >= need_f, ("v_cmp mask -> v_addc carry-in", f, need_f)


def _lgkm_zero(x):
    return x.mnem == "s_waitcnt" and re.search(r"lgkmcnt\(0\)", x.ops) is not None


def _pending_sload_touches(insns):
    """Every (s_load, instruction) pair where an instruction reads or writes the load's destination
    SGPRs on some control-flow path before an ``s_waitcnt lgkmcnt(0)``."""
    index = {x.addr: i for i, x in enumerate(insns)}
    bad = []
    for i, w in enumerate(insns):
        if not w.mnem.startswith("s_load"):
            continue
        regs = w.dst
        stack, seen = [i + 1], set()
        while stack:
            j = stack.pop()
            if j >= len(insns) or j in seen:
                continue
            seen.add(j)
            x = insns[j]
            if _lgkm_zero(x):
                continue
            if (x.src | x.dst) & regs:
                bad.append((hex(w.addr), w.ops, hex(x.addr), x.mnem, x.ops))
                continue
            if x.mnem in ("s_endpgm", "s_setpc_b64"):
                continue
            if x.mnem == "s_branch":
                if x.target in index:
                    stack.append(index[x.target])
                continue
            stack.append(j + 1)
            if x.mnem.startswith("s_cbranch") and x.target in index:
                stack.append(index[x.target])
    return bad


@pytest.mark.parametrize("symbol", ["_Z12chunk_kernelILi0EEv5KArgs", "_Z12chunk_kernelILi1EEv5KArgs",
                                    "_Z12chunk_kernelILi2EEv5KArgs"])
def test_consensus_pending_scalar_loads_untouched(library_code, symbol):
    """count_points_sgpr keeps the next group's s_load_dwordx16 in flight while count_four runs on
    the other buffer (its asm clobbers s[80:87]); scalar loads return out of order, so nothing may
    read, copy or overwrite a load's destination SGPRs before the s_waitcnt lgkmcnt(0) that
    swait() places ahead of its first use.  A compiler copy or spill of the in-flight buffer
    would read stale points: checked on every control-flow path of the built code object."""
    ins = _parse_objdump(library_code, symbol)
    assert sum(x.mnem == "s_load_dwordx16" for x in ins) >= 4, "count loop's scalar loads not found"
    bad = _pending_sload_touches(ins)
    assert not bad, bad[:5]
