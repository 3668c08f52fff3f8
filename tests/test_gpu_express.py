"""GPU parity of the express-scan codec (lslam_express_decode / lslam_express_scans)
against the reference's own outputs (tests/golden/express.npz: ExpressPacket.decode,
the Lidar.scan('express') measure stream and functions.scanning's rawPoints puts)
and the CPU oracle (oracle/express.py) on larger synthetic streams.

Bit-exact: packet validity, new-scan flags, distances, angles (degrees), CSR
revolution/chunk offsets, resume packet.  xy: device cos/sin against glibc,
|dxy| <= 1e-9 mm (the measured gap is a few ulp of a <= 16383 mm distance).
"""
import numpy as np
import pytest

from oracle import express as ox

pytestmark = pytest.mark.gpu

XY_TOL = 1e-9


@pytest.fixture(scope="module")
def ctx():
    from lidar_slam_amd.device import Context
    if Context.device_count() < 1:
        pytest.skip("no HIP device")
    return Context(0)


@pytest.mark.parametrize("name", ["clean", "dirty"])
def test_decode_matches_reference(ctx, golden, name):
    from lidar_slam_amd.express import express_measures
    g = golden("express.npz")
    m = express_measures(ctx, g[name + "_packets"])
    assert np.array_equal(m["pkt_valid"], g[name + "_valid"])
    assert np.array_equal(m["valid"], g[name + "_m_ok"])
    assert np.array_equal(m["new_scan"], g[name + "_m_new"])
    assert np.array_equal(m["dist_mm"], g[name + "_m_dist"].astype(np.float64))
    assert np.array_equal(m["angle_deg"], g[name + "_m_ang"])
    a, d = g[name + "_m_ang"], g[name + "_m_dist"].astype(np.float64)
    ref = np.stack([d * np.cos(-a * (np.pi / 180) + np.pi / 2), d * np.sin(-a * (np.pi / 180) + np.pi / 2)], -1)
    assert np.max(np.abs(m["xy"] - ref)) <= XY_TOL


def test_decode_large_stream_matches_oracle(ctx):
    from lidar_slam_amd import synth
    from lidar_slam_amd.express import express_measures
    pk = synth.express_packets(20011, seed=3, corrupt=0.003)
    m = express_measures(ctx, pk, want_xy=False)
    o = ox.measures(ox.decode_packets(pk))
    assert np.array_equal(m["pkt_valid"], ox.decode_packets(pk)["valid"])
    for k, ko in (("valid", "m_ok"), ("new_scan", "m_new"), ("angle_deg", "m_ang")):
        assert np.array_equal(m[k], o[ko]), k
    assert np.array_equal(m["dist_mm"], o["m_dist"].astype(np.float64))


@pytest.mark.parametrize("name", ["capA", "capB"])
def test_revolutions_match_reference_capture(ctx, golden, name):
    from lidar_slam_amd.express import ExpressRevolutions
    g = golden("express.npz")
    pk, drop = g[name + "_packets"], int(g[name + "_drop"])
    q, r = divmod(drop, 32)  # the warm-up: whole packets, then r measures of the next
    rv = ExpressRevolutions(ctx, len(pk)).run(pk[q:], skip=r)
    delim, sizes = g[name + "_delim"], g[name + "_chunk_sizes"]
    assert rv.n_scans == len(delim)
    assert np.array_equal(rv.scan_chunk_off, np.concatenate([[0], delim]))
    assert np.array_equal(np.diff(rv.chunk_pt_off), sizes[:delim[-1]])
    xy = rv.xy_host()
    ref = g[name + "_xy"][:rv.n_points]
    assert xy.shape == ref.shape and np.max(np.abs(xy - ref)) <= XY_TOL
    assert rv.resume == ox.revolutions(pk[q:], skip=r)["resume"]


@pytest.mark.parametrize("seed,corrupt,skip", [(1, 0.0, 0), (2, 0.01, 5), (4, 0.05, 31)])
def test_revolutions_large_stream_match_oracle(ctx, seed, corrupt, skip):
    from lidar_slam_amd import synth
    from lidar_slam_amd.express import ExpressRevolutions
    pk = synth.express_packets(3001, per_rev=22.5 + seed, seed=seed, corrupt=corrupt, scan_id=seed)
    rv = ExpressRevolutions(ctx, len(pk)).run(pk, skip=skip)
    o = ox.revolutions(pk, skip=skip)
    assert np.array_equal(rv.scan_chunk_off, o["scan_chunk_off"])
    assert np.array_equal(rv.chunk_pt_off, o["chunk_pt_off"])
    assert rv.resume == o["resume"]
    assert np.max(np.abs(rv.xy_host() - o["xy"])) <= XY_TOL


def test_revolution_edge_cases(ctx):
    from lidar_slam_amd import synth
    from lidar_slam_amd.express import ExpressRevolutions
    rv = ExpressRevolutions(ctx, 64)
    # 0 and 1 packets: no measures at all; 2 packets: one packet of measures
    for M in (0, 1, 2):
        pk = synth.express_packets(M, seed=9)
        r = rv.run(pk)
        assert (r.n_scans, r.n_chunks, r.n_points) == (0, 0, 0) and r.resume == -1
        assert np.array_equal(r.scan_chunk_off, [0]) and np.array_equal(r.chunk_pt_off, [0])
    # every packet wraps: 32-point revolutions (one chunk each) after a 1-point one
    pk = synth.express_packets(40, per_rev=1.001, seed=9)
    assert np.diff(ox.revolutions(pk)["scan_chunk_off"]).tolist() == [0] + [1] * 38  # rev 0: one point
    o = ox.revolutions(pk)
    r = rv.run(pk)
    assert np.array_equal(r.scan_chunk_off, o["scan_chunk_off"]) and np.array_equal(r.chunk_pt_off, o["chunk_pt_off"])
    # every packet corrupt: nothing
    bad = synth.express_packets(50, seed=9)
    bad[:, 0] ^= 0x40
    r = rv.run(bad)
    assert (r.n_scans, r.n_points, r.resume) == (0, 0, -1)
    with pytest.raises(ValueError):
        rv.run(synth.express_packets(65, seed=9))  # over max_packets


def test_unaligned_stream_is_rejected(ctx):
    import ctypes as C
    from lidar_slam_amd import _lib
    from lidar_slam_amd.express import ExpressRevolutions
    rv = ExpressRevolutions(ctx, 8)
    rv.upload(np.zeros((8, 84), np.uint8))
    with pytest.raises(ValueError):
        rv.launch(n_packets=4, packets_addr=rv.d_packets.addr + 2)
    with pytest.raises(ValueError):
        rv.launch(skip=32)
    m = _lib.ExpressMeasures()
    with pytest.raises(ValueError):
        _lib.check(_lib.load().lslam_express_decode(ctx.handle, rv.d_packets.addr + 1, 2, C.byref(m)), "decode")


def test_capture_in_pieces_equals_reference_loop(ctx):
    # ExpressCapture fed in ragged byte slices puts what functions.scanning puts
    # for every completed revolution
    from lidar_slam_amd import synth
    from lidar_slam_amd.express import ExpressCapture

    class Q:
        def __init__(self):
            self.items = []

        def put(self, x):
            self.items.append(x)

    pk = synth.express_packets(700, seed=5, scan_id=5)
    drop = 45
    q = Q()
    cap = ExpressCapture(q, ctx=ctx, drop=drop, max_packets=128)
    raw = pk.tobytes()
    rng = np.random.default_rng(0)
    pos = 0
    while pos < len(raw):
        n = int(rng.integers(1, 3000))
        cap.feed(raw[pos:pos + n])
        pos += n
    ref = ox.capture(pk, drop=drop)
    n_rev = sum(1 for x in q.items if isinstance(x, int))
    assert n_rev == len(ref["delim"])
    sizes = [len(x) for x in q.items if not isinstance(x, int)]
    assert np.array_equal(sizes, ref["chunk_sizes"][:ref["delim"][-1]])
    xy = np.concatenate([np.asarray(x) for x in q.items if not isinstance(x, int)])
    assert np.max(np.abs(xy - ref["xy"][:len(xy)])) <= XY_TOL
    # delimiters after the same chunk counts
    seen, delim = 0, []
    for x in q.items:
        if isinstance(x, int):
            delim.append(seen)
        else:
            seen += 1
    assert np.array_equal(delim, ref["delim"])


def test_revolutions_feed_the_scan_pipeline_on_device(ctx):
    # packets -> revolutions (device xy) -> RANSAC + landmarks without a host
    # round trip equals the same pipeline on the downloaded points
    from lidar_slam_amd import synth
    from lidar_slam_amd.express import ExpressRevolutions
    from lidar_slam_amd.pipeline import ScanPipeline
    pk = synth.express_packets(1200, seed=8, scan_id=8)
    rv = ExpressRevolutions(ctx, len(pk)).run(pk)
    seeds = np.arange(rv.n_scans)
    a = ScanPipeline(ctx, rv.xy, rv.scan_chunk_off, rv.chunk_pt_off, seeds=seeds, lmk_capacity=32)
    a.run()
    b = ScanPipeline(ctx, rv.xy_host(), rv.scan_chunk_off, rv.chunk_pt_off, seeds=seeds, lmk_capacity=32)
    b.run()
    ra, rb = a.results(), b.results()
    assert np.array_equal(ra["mask"], rb["mask"])
    assert ra["models"].tobytes() == rb["models"].tobytes()
    assert ra["landmarks"].tobytes() == rb["landmarks"].tobytes()
