"""The C4 split / gather bookkeeping (lidar_slam_amd/shard.py) on CPU: a batch split
across ranks, each rank's results gathered to the root in rank order, equals the
single-process run bit for bit.  world_size 2 over gloo (127.0.0.1); the per-rank
compute is the CPU oracle.  The gather runs collective.gatherv_plan's per-peer
operations over gloo point-to-point, the same plan Comm.gatherv issues as grouped
ncclSend / ncclRecv (the multi-rank RCCL execution itself needs >= 2 GPUs; RCCL
refuses two ranks on one device, so it has not run on this builder's hardware)."""
import os
import socket

import numpy as np
import pytest

from lidar_slam_amd import shard
from lidar_slam_amd.pipeline import LANDMARK_DTYPE, MODEL_DTYPE


def test_shard_ranges_cover_and_balance():
    for n, w in ((65536, 8), (10, 3), (3, 4), (0, 2), (7, 1)):
        rs = [shard.shard_range(n, w, r) for r in range(w)]
        assert rs[0][0] == 0 and rs[-1][1] == n
        assert all(rs[i][1] == rs[i + 1][0] for i in range(w - 1))
        sizes = [hi - lo for lo, hi in rs]
        assert max(sizes) - min(sizes) <= 1
    assert shard.shard_range(65536, 8, 3) == (24576, 32768)


def test_plan_inputs_rebase():
    import bench
    ids = list(range(7))
    b, ukf = bench.make_workload(ids, 720, 4)
    batch = dict(b, seeds=np.array(ids, np.uint32), **{"ukf_" + k: v for k, v in ukf.items() if k != "n_landmarks"})
    plan = shard.plan(b["scan_chunk_off"], b["chunk_pt_off"], 3)
    for sh in plan:
        sub = sh.inputs(batch)
        ref, ukr = bench.make_workload(ids[sh.lo:sh.hi], 720, 4)
        assert np.array_equal(sub["xy"], ref["xy"])
        assert np.array_equal(sub["scan_chunk_off"], ref["scan_chunk_off"])
        assert np.array_equal(sub["chunk_pt_off"], ref["chunk_pt_off"])
        assert np.array_equal(sub["seeds"], np.array(ids[sh.lo:sh.hi], np.uint32))
        assert np.array_equal(sub["ukf_x"], batch["ukf_x"][sh.lo:sh.hi])
        assert np.array_equal(sub["ukf_R_diag"], batch["ukf_R_diag"])  # not per scan


def test_inputs_do_not_slice_r_diag_when_2l_equals_scans():
    """R_diag has 2L entries; with 2L == the scan count it must still pass through whole."""
    import bench
    ids = list(range(8))
    b, ukf = bench.make_workload(ids, 720, 4)   # L = 4 -> R_diag has 8 = n_scans entries
    batch = dict(b, seeds=np.array(ids, np.uint32), **{"ukf_" + k: v for k, v in ukf.items() if k != "n_landmarks"})
    assert batch["ukf_R_diag"].shape[0] == len(ids)
    for sh in shard.plan(b["scan_chunk_off"], b["chunk_pt_off"], 3):
        sub = sh.inputs(batch)
        assert np.array_equal(sub["ukf_R_diag"], batch["ukf_R_diag"])
        assert np.array_equal(sub["ukf_z"], batch["ukf_z"][sh.lo:sh.hi])
    bad = dict(batch, seeds=np.arange(5, dtype=np.uint32))
    with pytest.raises(ValueError, match="per-scan input 'seeds'"):
        shard.plan(b["scan_chunk_off"], b["chunk_pt_off"], 2)[0].inputs(bad)


def _oracle_results(b, ids, ukf, cap):
    from oracle import cpu as orc
    from oracle import ukf as oukf
    mask, _, models, lists = orc.run_batch(b["xy"], b["scan_chunk_off"], b["chunk_pt_off"], ids)
    m = np.zeros(len(models), MODEL_DTYPE)
    for i, d in enumerate(models):
        for f in MODEL_DTYPE.names:
            m[f][i] = d[f]
    lm = np.zeros((len(ids), cap), LANDMARK_DTYPE)
    cnt = np.zeros(len(ids), np.int32)
    for s, lst in enumerate(lists):
        cnt[s] = len(lst)
        for i, L in enumerate(lst):
            lm[s, i] = (L["a"], L["b"], L["pos"][0], L["pos"][1], L["end"][0], L["end"][1], L["id"], L["life"])
    x, P = oukf.ukf_batch(ukf["x"], ukf["P"], ukf["u"], ukf["z"], ukf["lmk"], ukf["R_diag"])
    return {"mask": mask, "models": m, "ukf_x": x, "ukf_P": P, "lmk_count": cnt, "landmarks": lm}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gloo_gatherv(dist, rank):
    """collective.gatherv_plan executed over gloo point-to-point (the RCCL path runs the same
    ops as grouped ncclSend / ncclRecv): checks the plan's peers, offsets, counts and
    directions, not just shard.gather's bookkeeping."""
    import torch

    from lidar_slam_amd.collective import gatherv_plan

    def gatherv(send, recv, counts, root):
        src = np.ascontiguousarray(send).view(np.uint8).ravel()
        for kind, peer, off, n in gatherv_plan(rank, dist.get_world_size(), counts, root):
            if kind == "copy":
                recv[off:off + n] = src[:n]
            elif kind == "send":
                dist.send(torch.from_numpy(src[off:off + n].copy()), dst=peer)
            else:
                buf = torch.empty(n, dtype=torch.uint8)
                dist.recv(buf, src=peer)
                recv[off:off + n] = buf.numpy()
    return gatherv


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist

    import bench
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ids = list(range(5))           # ragged over 2 ranks: 3 + 2 scans
    cap = 16
    b, ukf = bench.make_workload(ids, 720, 6)
    batch = dict(b, **{"ukf_" + k: v for k, v in ukf.items() if k != "n_landmarks"})
    plan = shard.plan(b["scan_chunk_off"], b["chunk_pt_off"], world)
    me = plan[rank]
    sub = me.inputs(batch)
    my_ids = ids[me.lo:me.hi]
    uk = {k: sub["ukf_" + k] for k in ("x", "P", "u", "z", "lmk", "R_diag")}
    local = _oracle_results(sub, my_ids, uk, cap)
    got = shard.gather(plan, rank, local, _gloo_gatherv(dist, rank), lambda f, n: np.zeros(n, np.uint8),
                       lmk_capacity=cap)
    if rank == 0:
        out["got"] = {k: shard.host_view(k, v, len(ids), cap).tobytes() for k, v in got.items()}
    # ragged transfers with a zero-count rank on either side, and a non-zero root
    gv = _gloo_gatherv(dist, rank)
    for counts, root in (([37, 0], 0), ([0, 29], 0), ([0, 29], 1), ([11, 5], 1), ([0, 0], 0)):
        send = (np.arange(64) + 100 * rank).astype(np.uint8)
        recv = np.full(sum(counts), 255, np.uint8) if rank == root else None
        gv(send, recv, counts, root)
        if rank == root:
            out["gv%s_%d" % (counts, root)] = recv.tobytes()
    dist.destroy_process_group()


def test_two_rank_gloo_split_gather_equals_single_run():
    import torch.multiprocessing as mp  # CPU-only test: torch stays out of GPU test sessions

    import bench
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    ids = list(range(5))
    b, ukf = bench.make_workload(ids, 720, 6)
    ref = _oracle_results(b, ids, ukf, 16)
    got = out["got"]
    assert set(got) == set(shard.FIELDS)
    for k in shard.FIELDS:
        assert got[k] == np.ascontiguousarray(ref[k]).tobytes(), k
    for counts, root in (([37, 0], 0), ([0, 29], 0), ([0, 29], 1), ([11, 5], 1), ([0, 0], 0)):
        want = b"".join((np.arange(64) + 100 * r).astype(np.uint8)[:n].tobytes() for r, n in enumerate(counts))
        assert out["gv%s_%d" % (counts, root)] == want, (counts, root)


def test_gatherv_plan():
    from lidar_slam_amd.collective import gatherv_plan
    counts = [5, 0, 7, 3]
    assert gatherv_plan(0, 4, counts) == [("copy", 0, 0, 5), ("recv", 2, 5, 7), ("recv", 3, 12, 3)]
    assert gatherv_plan(1, 4, counts) == []                       # zero-count rank: nothing
    assert gatherv_plan(2, 4, counts) == [("send", 0, 0, 7)]
    assert gatherv_plan(2, 4, counts, root=2) == [("copy", 2, 5, 7), ("recv", 0, 0, 5), ("recv", 3, 12, 3)]
    assert gatherv_plan(0, 1, [9]) == [("copy", 0, 0, 9)]
    # the root's receives tile recv exactly: every rank's bytes at sum(counts[:r])
    for root in range(4):
        ops = gatherv_plan(root, 4, counts, root)
        spans = sorted((off, off + n) for _, _, off, n in ops)
        assert spans[0][0] == 0 and spans[-1][1] == sum(counts)
        assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
    for bad in (dict(rank=0, world=2, counts=[1]), dict(rank=0, world=2, counts=[1, -1]),
                dict(rank=2, world=2, counts=[1, 1]), dict(rank=0, world=2, counts=[1, 1], root=2)):
        with pytest.raises(ValueError):
            gatherv_plan(**bad)
