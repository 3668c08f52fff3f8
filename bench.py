"""Benchmark: scans/s of the fused RANSAC + landmark + UKF hot path (BASELINE.json).

python bench.py [--gpus N] [--steps K] [--warmup W]
  N > 1: launched by the driver as
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
         --master-port P bench.py --gpus N --steps K --warmup W

Main line (config C3 of BASELINE.json, per GPU): 4096 synthetic 720-point scans
(SURVEY §8d generator), chunked 7x100 + 20 as functions.py:64-76 does; per
chunk skimage-semantics RANSAC (100 trials, 20 mm, numpy legacy MT19937 stream
seeded per scan: results identical to the reference), landmark association
(ransac_functions.py:34-54), then one UKF predict+update per scan with
L = 20 landmarks (dim_z = 40).  One step = one pass over the batch = one launch
of lslam_scan_pipeline.  Inputs are resident in HBM before timing.  Multi-GPU:
each rank owns its own 4096 scans (ids rank*4096 ...), no data-path
collective; a host TCP group (lidar_slam_amd/hostgroup.py; no torch in the
process) gives the barrier and the max-over-ranks of the elapsed time.

C4 leg (configs[3]; at N > 1 by default, or --c4): one host batch of 65,536
scans in shared memory split across the ranks, H2D + pipeline + RCCL gather of
the results to rank 0 + D2H, timed end to end (the "c4" object of the line;
c4_leg below).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

os.environ.setdefault("OPENBLAS_NUM_THREADS", "1")  # the CPU baseline's twin is single-threaded per process

import numpy as np  # noqa: E402

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FP64_PEAK_TFLOPS = 78.6   # MI355X FP64 vector peak (AMD spec); the RANSAC residuals are FP64 VALU work
VALU_PEAK_TOPS = 78.6     # 32-bit integer VALU lane-ops/s: 256 CU x 4 SIMD x 32 lanes/clk x 2.4 GHz
HBM_PEAK_GBS = 8000.0     # MI355X HBM3E peak (MI355X_MICROARCH.md)
FLOPS_PER_EVAL = 12       # residual + inlier test per (point, hypothesis): SURVEY §8d
OPS_PER_WORD = 20         # MT19937: twist 8 + temper 10 + masked compare 2 (per 32-bit word)
OPS_PER_STEP = 5          # random_interval's mask for each Fisher-Yates step


def mt_stream_ops(chunk_sizes, trials):
    """Algorithmic 32-bit integer ops of the reference's sequential hypothesis
    stream: per chunk of N >= 3 points, trials+1 draws of choice(N, 2) =
    Fisher-Yates steps i = N-1..1, each consuming (m(i)+1)/(i+1) words on
    average (random_interval's masked rejection, m(i) = 2^bitlen(i) - 1)."""
    ops = 0.0
    D = trials + 1
    for n, cnt in zip(*np.unique(np.asarray(chunk_sizes), return_counts=True)):
        if n < 3:
            continue
        i = np.arange(1, n, dtype=np.float64)
        m = 2.0 ** np.floor(np.log2(i) + 1) - 1
        words = np.sum((m + 1) / (i + 1))
        ops += cnt * D * (OPS_PER_WORD * words + OPS_PER_STEP * (n - 1))
    return ops


def make_workload(scan_ids, n_beams, L, seed_base=0):
    from lidar_slam_amd import synth
    b = synth.make_batch(scan_ids, n_beams)
    S = len(scan_ids)
    rng = np.random.default_rng(424242 + seed_base)
    poses = b["poses"]
    lmk = rng.uniform(-3000.0, 3000.0, (S, L, 2))
    dx = lmk[:, :, 0] - poses[:, None, 0]
    dy = lmk[:, :, 1] - poses[:, None, 1]
    d = np.sqrt(dx * dx + dy * dy) + rng.normal(0, 0.5, (S, L))
    ph = np.arctan2(dy, dx) - poses[:, None, 2] + rng.normal(0, 0.3, (S, L))
    ph = (ph + np.pi) % (2 * np.pi) - np.pi
    z = np.stack([d, ph], -1).reshape(S, 2 * L)
    ukf = dict(n_landmarks=L, x=poses.copy(), P=np.tile(np.diag([.1, .1, .05]), (S, 1, 1)),
               u=np.tile([2.0, 2.5], (S, 1)), z=z, lmk=lmk, R_diag=np.array([0.25, 0.09] * L))
    return b, ukf


_TWIN_JOBS = None  # set before the pool forks: the workers inherit the sample, only indices travel


def _twin_run(job):
    xy, cpo, seed, ukf_in = job
    from oracle import numpy_twin as tw
    from oracle import ukf as oukf
    tw.process_scan(xy, cpo, seed)
    x, P, u, z, lmk, Rd = ukf_in
    oukf.ukf_batch(x[None], P[None], u[None], z[None], lmk[None], Rd)
    return 1


def _twin_worker(rng):
    return sum(_twin_run(_TWIN_JOBS[i]) for i in range(*rng))


def _twin_jobs(n_scans, n_beams, L):
    ids = list(range(n_scans))
    b, ukf = make_workload(ids, n_beams, L)
    sco, cpo = b["scan_chunk_off"], b["chunk_pt_off"]
    jobs = []
    for s in ids:
        c0, c1 = sco[s], sco[s + 1]
        jobs.append((b["xy"][cpo[c0]:cpo[c1]], cpo[c0:c1 + 1] - cpo[c0], s,
                     (ukf["x"][s], ukf["P"][s], ukf["u"][s], ukf["z"][s], ukf["lmk"][s], ukf["R_diag"])))
    return jobs


def cpu_baseline_1core(n_scans, n_beams, L):
    """The same twin in this process alone: one core (OPENBLAS_NUM_THREADS=1 is set at import)."""
    jobs = _twin_jobs(n_scans, n_beams, L)
    _twin_run(jobs[0])
    t0 = time.perf_counter()
    for j in jobs:
        _twin_run(j)
    dt = time.perf_counter() - t0
    return len(jobs) / dt, dt


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def usable_cpus():
    """CPUs this process may run on: the affinity mask, capped by a cgroup v2 CPU quota
    (cpu.max) if one is set.  Returns (cpus, quota_cpus or None)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = max(1, int(-(-int(q) // int(per))))
    except (OSError, ValueError):
        pass
    return (min(n, quota) if quota else n), quota


def capacity_overflows(models):
    """Chunks whose new landmark was dropped because the per-scan list was full (LSLAM_CAPACITY).
    The reference's list is unbounded (ransac_functions.py:75-76): a timed step is
    reference-exact only if this is 0."""
    return int(np.sum((models["flags"] & 256) != 0))


def cpu_baseline(n_scans, n_beams, L, procs):
    """The reference's CPU path (NumPy twin, per-trial skimage structure) + the NumPy UKF
    restatement, over a bounded sample, on ``procs`` host processes (one per core).  The
    sample is made once here; the forked workers inherit it and receive index ranges."""
    import multiprocessing as mp
    global _TWIN_JOBS
    _TWIN_JOBS = _twin_jobs(n_scans, n_beams, L)
    n = len(_TWIN_JOBS)
    per = max(1, n // (4 * procs))  # ~4 ranges per process: balances the tail
    ranges = [(i, min(n, i + per)) for i in range(0, n, per)]
    ctx = mp.get_context("fork")
    with ctx.Pool(procs) as pool:
        pool.map(_twin_worker, [(i % n, i % n + 1) for i in range(procs)], chunksize=1)  # warm imports
        t0 = time.perf_counter()
        done = sum(pool.map(_twin_worker, ranges, chunksize=1))
        dt = time.perf_counter() - t0
    _TWIN_JOBS = None
    return done / dt, dt


def shard_scan_ids(rank, per_rank):
    """Weak scaling: rank r owns scans [r*per_rank, (r+1)*per_rank)."""
    return list(range(rank * per_rank, (rank + 1) * per_rank))


def timed_region(step, steps, warmup, sync, barrier):
    """W untimed steps, then exactly K steps bracketed by barrier + sync."""
    for _ in range(warmup):
        step()
    sync()
    barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    barrier()
    return time.perf_counter() - t0


def reduce_max(x, group):
    """Max over ranks (group: lidar_slam_amd.hostgroup.HostGroup, None at one rank)."""
    return float(x) if group is None else group.allreduce_max(float(x))


def load_traffic(path):
    try:
        with open(path) as f:
            return json.load(f)
    except Exception:
        return None


C4_FIELDS = ("mask", "models", "ukf_x", "ukf_P", "lmk_count")


C4_TIMEOUT_RC = 3  # exit status of a rank whose C4 leg timed out


def run_guarded(leg, timeout, rank, line):
    """Run ``leg(segments)`` under a watchdog.  ``segments`` is a list the leg appends its
    shared-memory segments to.  If the leg has not returned after ``timeout`` seconds (a hung
    collective), rank 0 prints ``line`` with ``"c4": {"error": "timeout..."}``, unlinks the
    segments, and the process exits with ``C4_TIMEOUT_RC`` without running further Python
    (the hung thread cannot be joined).  A leg that raises is reported as ``{"error": ...}``."""
    import threading
    done, lock, segments = threading.Event(), threading.Lock(), []

    def watchdog():
        if done.wait(timeout):
            return
        with lock:
            if done.is_set():
                return
            if rank == 0:
                print(json.dumps(dict(line, c4={"error": "timeout: the C4 leg did not finish in %.0f s" % timeout})),
                      flush=True)
                for shm in segments:
                    try:
                        shm.unlink()
                    except Exception:  # already gone
                        pass
            sys.stderr.write("bench.py: the C4 leg timed out after %.0f s; exiting %d\n" % (timeout, C4_TIMEOUT_RC))
            sys.stderr.flush()
            sys.stdout.flush()
            os._exit(C4_TIMEOUT_RC)

    threading.Thread(target=watchdog, daemon=True).start()
    try:
        res = leg(segments)
    except Exception as e:
        res = {"error": "%s: %s" % (type(e).__name__, e)}
    with lock:
        done.set()
    return res


def c4_leg(args, rank, world, dist, ctx, L, segments=None, keep=None):
    """BASELINE configs[3] (C4): ONE host batch of ``--c4-scans`` scans split across the ranks,
    end to end.  The batch lives in one shared-memory segment of the node (the stand-in for
    the reference's mp.Queue hand-off, SLAM.py:13,18-23): rank 0 creates it, each rank fills
    its own shard (the generator is per scan) and page-locks the segment.  Per timed step,
    every rank H2Ds its shard's inputs, runs the fused pipeline on them, and the per-scan
    results (inlier masks, chunk records, UKF x / P, landmark counts) are gathered to rank 0's
    HBM over RCCL (lidar_slam_amd.collective: grouped send / recv on the context stream), then
    copied to rank 0's host.  Timed like the main line: barrier + sync on both sides, max over
    ranks.  After the timing, one more clean step (fresh inputs and empty landmark lists) is what
    the consistency check reads; with ``keep`` (a dict) rank 0 also leaves there the gathered
    results of that step as the single-GPU arrays, for tests/test_gpu_c4.py.  Returns the JSON
    object of the leg."""
    from multiprocessing import shared_memory

    from lidar_slam_amd import shard, synth
    total = int(args.c4_scans)
    sizes = synth.chunk_sizes(args.beams)
    nch, npt = len(sizes), int(sum(sizes))
    sco = (np.arange(total + 1) * nch).astype(np.int32)
    cpo = np.concatenate([[0], np.cumsum(np.tile(sizes, total))]).astype(np.int32)
    plan = shard.plan(sco, cpo, world)
    # the shared host batch: xy | seeds | x | P | u | z | lmk | R_diag, page-aligned parts
    layout, off = {}, 0
    for name, shape, dt in (("xy", (total * npt, 2), np.float64), ("seeds", (total,), np.uint32),
                            ("ukf_x", (total, 3), np.float64), ("ukf_P", (total, 3, 3), np.float64),
                            ("ukf_u", (total, 2), np.float64), ("ukf_z", (total, 2 * L), np.float64),
                            ("ukf_lmk", (total, L, 2), np.float64), ("ukf_R_diag", (2 * L,), np.float64)):
        nb = int(np.prod(shape)) * np.dtype(dt).itemsize
        layout[name] = (off, shape, dt)
        off = (off + nb + 4095) & ~4095
    seg_name = "lslam_c4_%d_%d" % (os.getpid(), int(time.time()))
    shm = None
    try:
        # every rank learns whether the segment exists on all of them before any collective
        err = None
        if rank == 0:
            try:
                shm = shared_memory.SharedMemory(name=seg_name, create=True, size=off)
                if segments is not None:
                    segments.append(shm)  # unlinked by run_guarded's watchdog on a timeout
            except Exception as e:  # e.g. /dev/shm smaller than the batch
                err = e
        if dist is not None:
            name = dist.broadcast((seg_name if err is None else "").encode()).decode()
            if rank != 0 and name:
                try:
                    shm = shared_memory.SharedMemory(name=name)
                    # attaching registers the segment with this process's resource tracker, which
                    # would unlink it again at exit (rank 0 owns and unlinks it)
                    from multiprocessing import resource_tracker
                    resource_tracker.unregister(shm._name, "shared_memory")
                except Exception as e:
                    err = e
            failed = dist.allreduce_max(0.0 if (name and err is None) else 1.0)
            if failed and err is None:
                err = RuntimeError("the C4 host batch segment could not be shared on every rank")
        if err is not None:
            raise err
        return _c4_run(args, rank, world, dist, ctx, L, shm, layout, off, sco, cpo, plan, keep)
    finally:
        if dist is not None:
            dist.barrier()
        if shm is not None:
            try:
                shm.close()
            except BufferError:  # views still referenced (an exception's traceback): the OS reclaims it
                pass
            if rank == 0:
                shm.unlink()


def _c4_run(args, rank, world, dist, ctx, L, shm, layout, off, sco, cpo, plan, keep=None):
    from lidar_slam_amd import collective, shard
    from lidar_slam_amd.device import DeviceArray, register_host, unregister_host
    from lidar_slam_amd.pipeline import ScanPipeline
    me = plan[rank]
    total = len(sco) - 1
    seg = np.ndarray((off,), np.uint8, buffer=shm.buf)
    host = {k: np.ndarray(shape, dt, buffer=shm.buf, offset=o) for k, (o, shape, dt) in layout.items()}
    ids = list(range(me.lo, me.hi))
    b, wk = make_workload(ids, args.beams, L, seed_base=1000 + rank)
    host["xy"][me.p0:me.p1] = b["xy"]
    host["seeds"][me.lo:me.hi] = ids
    for k in ("x", "P", "u", "z", "lmk"):
        host["ukf_" + k][me.lo:me.hi] = wk[k].reshape(host["ukf_" + k][me.lo:me.hi].shape)
    if rank == 0:
        host["ukf_R_diag"][:] = wk["R_diag"]
    del b, wk
    if dist is not None:
        dist.barrier()
    pinned = register_host(seg)
    mine = me.inputs(dict(host, scan_chunk_off=sco, chunk_pt_off=cpo))
    ukf = dict(n_landmarks=L, **{k: mine["ukf_" + k] for k in ("x", "P", "u", "z", "lmk", "R_diag")})
    pipe = ScanPipeline(ctx, mine["xy"], mine["scan_chunk_off"], mine["chunk_pt_off"], seeds=mine["seeds"],
                        max_trials=args.trials, lmk_capacity=args.lmk_capacity, want_yproj=False, ukf=ukf)
    if getattr(args, "c4_transport", "rccl") == "host":
        comm = collective.HostComm(ctx, dist)
    else:
        comm = collective.Comm.from_process_group(ctx, dist)
    local = {"mask": pipe.mask, "models": pipe.models, "ukf_x": pipe.ukf_x, "ukf_P": pipe.ukf_P,
             "lmk_count": pipe.lmk_count}
    recv, host_out = {}, {}
    if rank == 0:
        for k in C4_FIELDS:
            nb = sum(s.field_bytes(args.lmk_capacity)[k] for s in plan)
            recv[k] = DeviceArray(ctx, (nb,), np.uint8)
            host_out[k] = np.empty(nb, np.uint8)
            register_host(host_out[k])
    upload = {k: mine[k] for k in ("xy", "seeds", "ukf_u", "ukf_z", "ukf_lmk", "ukf_x", "ukf_P")}

    def h2d():
        pipe.upload_async(**upload)
        pipe.clear_lists_async()

    def compute():
        pipe.run(sync=False)

    def gather():
        shard.gather(plan, rank, local, comm.gatherv, lambda k, n: recv[k], lmk_capacity=args.lmk_capacity)

    def d2h():
        for k in (C4_FIELDS if rank == 0 else ()):
            recv[k].download_async(host_out[k])

    def step():
        h2d()
        compute()
        gather()
        d2h()

    def barrier():
        if dist is not None:
            dist.barrier()

    elapsed = reduce_max(timed_region(step, args.c4_steps, args.warmup, ctx.sync, barrier), dist)
    phases = {}
    for name, fn in (("h2d", h2d), ("pipeline", compute), ("gather", gather), ("d2h", d2h)):
        ts = [timed_region(fn, 1, 0, ctx.sync, barrier) for _ in range(3)]
        phases[name + "_ms"] = round(reduce_max(float(np.median(ts)), dist) * 1e3, 4)
    # the phases above chain the landmark lists and UKF state across calls: one clean step
    # from the shared batch's inputs is what rank 0 checks (and what a 1-GPU run would give)
    step()
    ctx.sync()
    res = {"workload": "C4: %d synthetic %d-pt scans in one shared host batch, %d shards of %d-%d scans; per step "
                       "H2D + fused RANSAC/association/UKF pipeline + gather (see transport) of masks, chunk records, "
                       "UKF x/P and landmark counts to rank 0 + D2H there"
                       % (total, args.beams, world, min(s.n_scans for s in plan), max(s.n_scans for s in plan)),
           "total_scans": total, "steps": args.c4_steps, "ms_per_step": round(elapsed / args.c4_steps * 1e3, 4),
           "e2e_scans_per_s": round(total * args.c4_steps / elapsed, 1), "phases_alone": phases,
           "gathered_bytes_per_step": int(sum(v.nbytes for v in host_out.values())) if rank == 0 else None,
           "host_batch": "shared memory, %s" % ("page-locked" if pinned else "pageable"),
           "rccl_version": collective.version(), "transport": comm.transport}
    if rank == 0:
        m = shard.host_view("models", host_out["models"], total)
        pop = np.add.reduceat(host_out["mask"].astype(np.int64), cpo[:-1])
        x = shard.host_view("ukf_x", host_out["ukf_x"], total)
        res["consistent"] = bool(np.all(m["flags"] & 1) and np.array_equal(pop, m["n_inliers"]) and
                                 np.all(np.isfinite(x)) and np.array_equal(m["n_points"], np.diff(cpo)))
        res["capacity_overflows"] = capacity_overflows(m)
        if keep is not None:
            for k in C4_FIELDS:
                keep[k] = shard.host_view(k, host_out[k], total).copy()
        for v in host_out.values():
            unregister_host(v)
    comm.close()
    del pipe, local, recv
    ctx.sync()
    if pinned:
        unregister_host(seg)
    return res


def coupled_leg(args, ctx, b, ukf, ids, L, sync_all, barrier, dist):
    """SURVEY §8(d)'s end-to-end step: the same batch with flags = PREDICT | UPDATE |
    LMK_FROM_RANSAC, so landmark slot j < 8 of scan s is chunk j's fitted origin (Landmark.pos,
    /root/reference/landmarking.py:17, ransac_functions.py:31) feeding hx (UKFMethods.py:26-34)
    in the same call; the remaining slots keep the uniform landmarks.  The UKF then depends on
    this call's RANSAC, so the library runs it after the consensus instead of beside it (the
    main line's independent UKF).  z is made for that landmark set: the origins come from one
    untimed call, the measurements are hx(pose) + N(0, R) on the host.  Timed with the main
    line's protocol (W warmup steps, K steps between barrier + sync, max over ranks)."""
    from lidar_slam_amd import _lib
    from lidar_slam_amd.pipeline import ScanPipeline
    flags = _lib.UKF_PREDICT | _lib.UKF_UPDATE | _lib.UKF_LMK_FROM_RANSAC
    pipe = ScanPipeline(ctx, b["xy"], b["scan_chunk_off"], b["chunk_pt_off"], seeds=np.array(ids, np.uint32),
                        max_trials=args.trials, lmk_capacity=args.lmk_capacity, want_yproj=True,
                        ukf=dict(ukf, flags=flags))
    pipe.run()
    m = pipe.results()["models"]
    sco = b["scan_chunk_off"]
    nch = np.diff(sco)
    lmk = ukf["lmk"].copy()
    fused = 0
    for j in range(min(L, int(nch.max()) if len(nch) else 0)):
        s = np.nonzero(nch > j)[0]
        c = sco[s] + j
        ok = (m["flags"][c] & 1) != 0
        lmk[s[ok], j, 0] = m["ox"][c[ok]]
        lmk[s[ok], j, 1] = m["oy"][c[ok]]
        fused += int(ok.sum())
    poses = b["poses"]
    rng = np.random.default_rng(515151 + int(ids[0]) if len(ids) else 515151)
    dx = lmk[:, :, 0] - poses[:, None, 0]
    dy = lmk[:, :, 1] - poses[:, None, 1]
    S = len(ids)
    d = np.sqrt(dx * dx + dy * dy) + rng.normal(0, 0.5, (S, L))
    ph = np.arctan2(dy, dx) - poses[:, None, 2] + rng.normal(0, 0.3, (S, L))
    ph = (ph + np.pi) % (2 * np.pi) - np.pi
    pipe.reset_state()
    pipe.upload_async(ukf_z=np.stack([d, ph], -1).reshape(S, 2 * L))
    sync_all()
    elapsed = reduce_max(timed_region(lambda: pipe.run(sync=False), args.steps, args.warmup, sync_all, barrier),
                         dist)
    r = pipe.results()
    del pipe
    return {"flags": "PREDICT|UPDATE|LMK_FROM_RANSAC", "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "scans_per_s": round(S * args.steps / elapsed * (dist.world if dist is not None else 1), 1),
            "fused_slots_per_scan": round(fused / max(S, 1), 3), "valid_chunks": int(np.sum(r["models"]["flags"] & 1)),
            "capacity_overflows": capacity_overflows(r["models"]),
            "all_finite": bool(np.all(np.isfinite(r["ukf_x"])))}


def rank_device(local_rank):
    """The HIP device of this rank: LOCAL_RANK, or LSLAM_RANK_DEVICE for every rank when set (a
    multi-rank rehearsal of the driver's N > 1 launch on a one-GPU box: all ranks on device 0).
    Read before any HIP call."""
    v = os.environ.get("LSLAM_RANK_DEVICE")
    return int(v) if v not in (None, "") else int(local_rank)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 50 steps of ~1 ms: the two-stream pipeline's fill and drain (the first producer has no
    # consumers beside it, the last consumers no producer) amortised to ~1 % of the step
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--scans", type=int, default=4096, help="scans per GPU")
    ap.add_argument("--beams", type=int, default=720)
    ap.add_argument("--landmarks", type=int, default=20)
    ap.add_argument("--trials", type=int, default=100)
    ap.add_argument("--hyp", default="mt19937", choices=["mt19937", "philox"])
    ap.add_argument("--no-ukf", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=2048, help="CPU baseline: at least this many scans")
    ap.add_argument("--cpu-per-proc", type=int, default=16, help="CPU baseline: at least this many scans per process")
    ap.add_argument("--cpu-sample-1core", type=int, default=96)
    ap.add_argument("--cpu-procs", type=int, default=0, help="CPU baseline processes (default: every usable core)")
    ap.add_argument("--lmk-capacity", type=int, default=64,
                    help="per-scan landmark list capacity (>= the steady-state list, ~42 on C3)")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "traffic_latest.json"))
    ap.add_argument("--also-philox", action="store_true", help="also time the Philox (throughput) mode")
    ap.add_argument("--c4", action="store_true", help="run the C4 leg (also at one GPU; default: only N > 1)")
    ap.add_argument("--no-c4", action="store_true", help="skip the C4 leg at N > 1")
    ap.add_argument("--c4-scans", type=int, default=65536, help="C4: scans of the one shared batch")
    ap.add_argument("--c4-steps", type=int, default=5)
    ap.add_argument("--c4-transport", default="rccl", choices=["rccl", "host"],
                    help="C4 gather: RCCL (the product), or host TCP for a rehearsal whose ranks share one device")
    ap.add_argument("--c4-timeout", type=float, default=240.0, help="seconds before the C4 leg is abandoned")
    ap.add_argument("--no-alone", action="store_true", help="skip the producer-alone timing (profiled runs)")
    ap.add_argument("--no-coupled", action="store_true",
                    help="skip the coupled RANSAC->UKF step (LMK_FROM_RANSAC) of SURVEY 8(d)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    L = args.landmarks

    # CPU baseline first: before anything touches the GPU (the pool forks)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        usable, quota = usable_cpus()
        procs = args.cpu_procs or usable
        sample = max(args.cpu_sample, args.cpu_per_proc * procs)
        rate1, dt1 = cpu_baseline_1core(args.cpu_sample_1core, args.beams, L)
        rate, dt = cpu_baseline(sample, args.beams, L, procs)
        cpu = {"value": round(rate, 2), "unit": "scans/s", "cores": procs, "kind": "port",
               "value_1core": round(rate1, 2), "host_cpus": os.cpu_count(), "usable_cpus": usable,
               "cgroup_cpu_quota": quota, "cpu_model": cpu_model(),
               "sample": "%d synthetic %d-pt scans (same generator, per-scan seeds) through the NumPy twin of "
                         "the reference (skimage-structured ransac + landmark association, oracle/numpy_twin.py) "
                         "+ the NumPy UKF restatement (oracle/ukf.py), %d processes (one per usable core), %.2f s "
                         "wall; 1 core: %d scans in %.1f s; twin/reference calibration in BASELINE.md"
                         % (sample, args.beams, procs, dt, args.cpu_sample_1core, dt1)}

    dist = None
    if world > 1:
        # the ranks' barrier / max-reduce over TCP (lidar_slam_amd.hostgroup): no torch in this
        # process, whose bundled HIP runtime would sit beside /opt/rocm's and break RCCL
        from lidar_slam_amd.hostgroup import HostGroup
        dist = HostGroup(rank, world)

    from lidar_slam_amd import _lib
    from lidar_slam_amd.device import Context
    from lidar_slam_amd.pipeline import ScanPipeline

    ctx = Context(rank_device(local))
    S = args.scans
    ids = shard_scan_ids(rank, S)
    b, ukf = make_workload(ids, args.beams, L, seed_base=rank)
    pipe = ScanPipeline(ctx, b["xy"], b["scan_chunk_off"], b["chunk_pt_off"], seeds=np.array(ids, np.uint32),
                        max_trials=args.trials, hyp=args.hyp, lmk_capacity=args.lmk_capacity, want_yproj=True,
                        ukf=None if args.no_ukf else ukf)
    def sync_all():
        ctx.sync()

    def barrier():
        if dist is not None:
            dist.barrier()

    def step():
        pipe.run(sync=False)

    # warmup outside the HIP-event window, then the timed region with the dominant kernel's
    # events on (they sit on the producer's stream).  Every event recorded on the ctx stream is
    # a marker packet that drains it (~7 us between two kernels on the MI355X), so
    # the consensus / whole-call events run in a separate instrumented pass after the timed one.
    for _ in range(args.warmup):
        step()
    sync_all()
    ctx.set_timing(True, kernels=[_lib.K_RNG])
    ctx.timing_reset()
    elapsed = timed_region(step, args.steps, 0, sync_all, barrier)
    rms, rl = ctx.timing(_lib.K_RNG)
    ctx.set_timing(True)
    ctx.timing_reset()
    for _ in range(max(3, min(args.steps, 10))):
        step()
    sync_all()
    kms, klaunch = ctx.timing(_lib.K_PIPELINE)
    cms, cl = ctx.timing(_lib.K_CONSENSUS)
    ctx.set_timing(False)
    elapsed = reduce_max(elapsed, dist)
    kavg = reduce_max(kms / max(klaunch, 1), dist)
    ravg = reduce_max(rms / rl, dist) if rl else None
    cavg = reduce_max(cms / max(cl, 1), dist)

    coupled = None
    if not args.no_coupled and not args.no_ukf:
        coupled = coupled_leg(args, ctx, b, ukf, ids, L, sync_all, barrier, dist)
        coupled["vs_main_step"] = round(coupled["ms_per_step"] / (elapsed / args.steps * 1e3), 4)

    # the producer alone (no consumers beside it), for the record: lslam_hyp_mt19937 over the same batch
    alone = None
    if args.hyp == "mt19937" and not args.no_alone:
        from lidar_slam_amd import pipeline as pl
        pl.hyp_mt19937(ctx, b["scan_chunk_off"], b["chunk_pt_off"], seeds=np.array(ids, np.uint32),
                       max_trials=args.trials)
        ctx.set_timing(True, kernels=[_lib.K_RNG])
        ctx.timing_reset()
        for _ in range(3):
            pl.hyp_mt19937(ctx, b["scan_chunk_off"], b["chunk_pt_off"], seeds=np.array(ids, np.uint32),
                           max_trials=args.trials)
        ams, al = ctx.timing(_lib.K_RNG)
        ctx.set_timing(False)
        alone = reduce_max(ams / max(al, 1), dist)

    # sanity: results are well-formed (every chunk fitted or flagged)
    r = pipe.results()
    valid = int(np.sum((r["models"]["flags"] & 1) != 0))
    overflows = capacity_overflows(r["models"])  # of the last timed step (the lists chain across steps)

    total_scans = S * world * args.steps
    value = total_scans / elapsed
    sizes = np.diff(b["chunk_pt_off"])
    evals = int(np.sum(sizes) * args.trials)   # (point, hypothesis) pairs per step
    flops = FLOPS_PER_EVAL * evals
    cons_tf = flops / (cavg * 1e-3) / 1e12
    n_pts = int(b["chunk_pt_off"][-1])
    n_chunks = int(b["scan_chunk_off"][-1])
    # algorithmic HBM bytes of the whole pipeline per step: points in (16 B), mask (1 B) + projected y
    # (8 B) out, chunk CSR (4 B) + model record (112 B) per chunk, the draws handed from the producer to
    # the consensus kernel (written + read), per scan: seed, CSR, landmark count in/out + the list written
    alg_bytes = n_pts * (16 + 1 + 8) + n_chunks * (4 + 112) + S * (4 + 4 + 8) + int(np.sum(r["lmk_count"])) * 56
    if args.hyp == "mt19937":
        alg_bytes += n_chunks * (args.trials + 1) * 8 * 2
    if not args.no_ukf:
        alg_bytes += S * (3 * 8 * 2 + 9 * 8 * 2 + 2 * 8 + 2 * L * 8 + 2 * L * 8)
    hbm_gbs = alg_bytes / (kavg * 1e-3) / 1e9
    traffic = load_traffic(args.traffic)

    def traffic_of(kernel):
        if traffic and traffic.get("scans") == S and traffic.get("hyp") == args.hyp:
            return (traffic.get("kernels") or {}).get(kernel, {}).get("bytes_per_launch")
        return None

    if args.hyp == "mt19937" and ravg:
        # dominant kernel: the parity-stream producer (integer VALU, one serial chain per scan)
        ops = mt_stream_ops(sizes, args.trials)
        achieved = ops / (ravg * 1e-3) / 1e12
        roof = {"bound": "valu", "achieved": round(achieved, 4), "peak": VALU_PEAK_TOPS, "unit": "TOPS (int32)",
                "frac": round(achieved / VALU_PEAK_TOPS, 5), "traffic": traffic_of("rng_kernel"),
                "kernel": "rng_kernel (MT19937 parse, lslam_rng_pipe.h)", "kernel_ms": round(ravg, 4),
                "kernel_alone_ms": round(alone, 4) if alone else None,
                "ops_per_launch": round(ops), "ops_def": "%d per MT word (expected words from random_interval's "
                "acceptance) + %d per Fisher-Yates step" % (OPS_PER_WORD, OPS_PER_STEP),
                "not_in_kernel_ms": "seed_kernel (numpy init_genrand of every scan, lane per scan, on its own "
                                    "stream beside the previous call; ~20 us per call in rocprof, DESIGN.md §4.1)"}
    else:
        roof = {"bound": "fp64-valu", "achieved": round(cons_tf, 4), "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": round(cons_tf / FP64_PEAK_TFLOPS, 5), "traffic": traffic_of("chunk_kernel"),
                "kernel": "chunk_kernel (consensus A4-A8)", "kernel_ms": round(cavg, 4), "flops_per_launch": flops}
    step_tf = flops / (elapsed / args.steps) / 1e12
    roof.update({
        # SURVEY §8(d)'s definition over the whole step: algorithmic FP64 flops per step (12 per
        # point-hypothesis evaluation) / the timed ms_per_step / the FP64 vector peak
        "step_fp64_tflops": round(step_tf, 4),
        "step_fp64_frac": round(step_tf / FP64_PEAK_TFLOPS, 5),
        "consensus": {"kernel": "chunk_kernel", "ms": round(cavg, 4), "fp64_tflops": round(cons_tf, 4),
                      "frac": round(cons_tf / FP64_PEAK_TFLOPS, 5), "flops_per_launch": flops,
                      "not_in_kernel_ms": "cut_lane_kernel (the chunks' box terms and cutoffs, lane per chunk, "
                                          "launched with seed_kernel on the seeding stream, DESIGN.md §4.2)"},
        "pipeline": {"ms": round(kavg, 4), "alg_bytes_per_launch": alg_bytes, "hbm_alg_gbs": round(hbm_gbs, 2),
                     "hbm_frac": round(hbm_gbs / HBM_PEAK_GBS, 5)},
    })

    out = {
        "metric": "scans/sec (RANSAC+UKF, 720-pt scans) at 1/2/4/8 MI355X + HBM GB/s vs peak",
        "value": round(value, 1),
        "unit": "scans/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (SURVEY 8d room-scan generator; per-scan seeds)",
        "config": {
            "workload": "C3: %d synthetic %d-pt scans per GPU, chunked 7x100+20; RANSAC (%d trials, 20 mm, %s "
                        "hypotheses) + landmark association + UKF predict/update (n=3, L=%d)%s"
                        % (S, args.beams, args.trials, args.hyp, L, " [UKF off]" if args.no_ukf else ""),
            "scans_per_gpu": S, "points_per_scan": args.beams, "trials": args.trials, "landmarks": L,
            "hyp": args.hyp, "parallelism": "dp%d (scan shards, no collective)" % world,
        },
        "roofline": roof,
        "cpu_baseline": cpu,
        "valid_chunks": valid,
        "capacity_overflows": overflows,
        "max_landmark_list": int(np.max(r["lmk_count"])),
        "coupled": coupled,
    }
    if args.also_philox and world == 1:
        pipe2 = ScanPipeline(ctx, b["xy"], b["scan_chunk_off"], b["chunk_pt_off"], max_trials=args.trials,
                             hyp="philox", lmk_capacity=args.lmk_capacity, ukf=None if args.no_ukf else ukf)
        for _ in range(args.warmup):
            pipe2.run(sync=False)
        ctx.sync()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            pipe2.run(sync=False)
        ctx.sync()
        out["philox_scans_per_s"] = round(S * args.steps / (time.perf_counter() - t0), 1)
    if args.c4 or (world > 1 and not args.no_c4):
        # The main line stands on its own: a C4 leg that fails is reported in it; one that does
        # not finish in --c4-timeout seconds (a collective that never completes on some node)
        # ends every rank non-zero, with the main line printed and the leg marked as timed out.
        out["c4"] = run_guarded(lambda segs: c4_leg(args, rank, world, dist, ctx, L, segs), args.c4_timeout,
                                rank, out)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.close()
    if overflows:
        sys.exit("capacity_overflows = %d: raise --lmk-capacity (the timed step was not reference-exact)"
                 % overflows)


if __name__ == "__main__":
    main()
