"""The multi-rank bench path on CPU (world_size 2, 127.0.0.1): scan sharding is a disjoint
cover, the timed region is barrier-bracketed, and the elapsed time is the max over ranks.
The ranks talk through bench.py's host group (lidar_slam_amd/hostgroup.py: TCP, no torch
in the rank processes).  The per-rank work here is the CPU oracle on each rank's shard,
and the union of the shards' results equals the single-process run (the main line has
no exchange step; the C4 gather is tested in tests/test_shard.py)."""
import multiprocessing as mp
import os
import socket

import numpy as np


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import bench
    from lidar_slam_amd import synth
    from lidar_slam_amd.hostgroup import HostGroup
    from oracle import cpu as orc
    g = HostGroup.from_env()
    ids = bench.shard_scan_ids(rank, 3)
    b = synth.make_batch(ids)
    res = {}

    def step():
        res["mask"] = orc.run_batch(b["xy"], b["scan_chunk_off"], b["chunk_pt_off"], ids)[0]

    el = bench.timed_region(step, 2, 1, lambda: None, g.barrier)
    # rank 1 pretends to be slower: the reported time must be the max
    el_max = bench.reduce_max(el + (5.0 if rank == 1 else 0.0), g)
    word = g.broadcast(b"from rank 0" if rank == 0 else None)
    out[rank] = (ids, res["mask"].tobytes(), el_max, word)
    g.barrier()
    g.close()


def test_two_rank_sharding_barrier_and_max():
    world = 2
    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    out = mgr.dict()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, out)) for r in range(world)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(120)
        assert p.exitcode == 0
    ids0, m0, e0, w0 = out[0]
    ids1, m1, e1, w1 = out[1]
    assert set(ids0).isdisjoint(ids1) and sorted(ids0 + ids1) == list(range(6))
    assert e0 == e1 and e0 >= 5.0
    assert w0 == w1 == b"from rank 0"
    from lidar_slam_amd import synth
    from oracle import cpu as orc
    b = synth.make_batch(list(range(6)))
    full = orc.run_batch(b["xy"], b["scan_chunk_off"], b["chunk_pt_off"], list(range(6)))[0]
    both = np.concatenate([np.frombuffer(m0, np.uint8), np.frombuffer(m1, np.uint8)])
    assert np.array_equal(both, full)


def test_rank_device_override(monkeypatch):
    """bench.py's device per rank: LOCAL_RANK, or LSLAM_RANK_DEVICE for every rank (the one-GPU
    rehearsal of the driver's multi-rank launch, profiles/r05_rehearsal_2ranks.log)."""
    import bench
    monkeypatch.delenv("LSLAM_RANK_DEVICE", raising=False)
    assert bench.rank_device(3) == 3
    monkeypatch.setenv("LSLAM_RANK_DEVICE", "0")
    assert bench.rank_device(3) == 0
