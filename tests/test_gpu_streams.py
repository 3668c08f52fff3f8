"""Stream ordering across entry points (include/lidarslam.h: every call is async on the
context, later calls see earlier calls' outputs).  The MT producer runs on its own
stream and the Philox-mode UKF on a side stream, so a call that reads what a
previous, different entry point wrote must wait for it although nothing syncs
the host in between.  Each chain is compared with the same calls run with a
host sync after each one."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from lidar_slam_amd.device import Context
    if Context.device_count() < 1:
        pytest.skip("no HIP device")
    return Context(0)


def _hyp_batch(ctx, sco, cpo, seeds, draws, state_out, keep):
    from lidar_slam_amd import _lib
    hb = _lib.ScanBatch()
    hb.n_scans, hb.n_chunks, hb.n_points = len(sco) - 1, int(sco[-1]), int(cpo[-1])
    hb.max_chunk_points = int(np.diff(cpo).max())
    hb.max_scan_chunks = int(np.diff(sco).max())
    for name, arr in (("scan_chunk_off", sco), ("chunk_pt_off", cpo), ("seeds", seeds)):
        d = ctx.to_device(arr)
        keep.append(d)
        setattr(hb, name, d.addr)
    hb.draws_out, hb.mt_state_out = draws.addr, state_out.addr
    return hb


def test_hyp_mt19937_then_pipeline_chained_on_its_state(ctx):
    """lslam_hyp_mt19937 writes mt_state_out; a pipeline call whose mt_state_in IS that buffer
    follows with no sync: its producer must wait for the hyp call's stream position."""
    from lidar_slam_amd import _lib, synth
    from lidar_slam_amd.pipeline import ScanPipeline, mt_seed_state
    S = 2048
    ids = list(range(S))
    b = synth.make_batch(ids)
    sco, cpo = b["scan_chunk_off"], b["chunk_pt_off"]
    state = ctx.to_device(np.tile(mt_seed_state(99999), (S, 1)))  # valid but wrong if read too early
    p = ScanPipeline(ctx, b["xy"], sco, cpo, mt_state=state, want_state=True)
    keep = []
    draws = ctx.empty((int(sco[-1]), 101, 2), np.int32)
    hb = _hyp_batch(ctx, sco, cpo, np.array(ids, np.uint32), draws, state, keep)
    _lib.check(_lib.load().lslam_hyp_mt19937(ctx.handle, C.byref(hb), 100), "lslam_hyp_mt19937")
    p.run(sync=False)
    ctx.sync()
    r = p.results()
    st_after_hyp = state.download()
    q = ScanPipeline(ctx, b["xy"], sco, cpo, mt_state=st_after_hyp, want_state=True)
    q.run()
    rq = q.results()
    assert np.array_equal(r["mask"], rq["mask"])
    assert r["models"].tobytes() == rq["models"].tobytes()
    assert np.array_equal(r["mt_state"], rq["mt_state"])
    # and the hyp call itself continued each scan's seed stream
    st0 = np.stack([mt_seed_state(s) for s in ids])
    assert not np.array_equal(st_after_hyp, st0)


def test_ukf_step_then_philox_pipeline_side_ukf(ctx):
    """lslam_ukf_step (main stream) updates x, P; a Philox pipeline call follows with no sync and
    runs its UKF on the side stream, reading the same x, P: it must see the first step."""
    from lidar_slam_amd import synth
    from lidar_slam_amd.pipeline import ScanPipeline
    from oracle import ukf as oukf
    S, L = 4096, 20
    ids = list(range(S))
    b = synth.make_batch(ids)
    rng = np.random.default_rng(8)
    x = b["poses"].copy()
    lmk = rng.uniform(-3000, 3000, (S, L, 2))
    z = np.stack([oukf.transfer_function(x[s], lmk[s]) for s in range(S)]) + rng.normal(0, 0.3, (S, 2 * L))
    ukf = dict(n_landmarks=L, x=x, P=np.tile(np.diag([.1, .1, .05]), (S, 1, 1)), u=np.tile([2.0, 2.5], (S, 1)),
               z=z, lmk=lmk, R_diag=np.array([oukf.VAR_DIST, oukf.VAR_ANGLE] * L))

    def make():
        return ScanPipeline(ctx, b["xy"], b["scan_chunk_off"], b["chunk_pt_off"], hyp="philox", lmk_capacity=64,
                            ukf=ukf)

    p = make()
    p.run_ukf_only(sync=False)
    p.run(sync=False)
    ctx.sync()
    r = p.results()
    q = make()
    q.run_ukf_only()
    q.run()
    rq = q.results()
    assert np.array_equal(r["ukf_x"], rq["ukf_x"]) and np.array_equal(r["ukf_P"], rq["ukf_P"])
    assert np.array_equal(r["mask"], rq["mask"])
    one = make()
    one.run()
    assert not np.array_equal(one.results()["ukf_x"], rq["ukf_x"])  # two steps differ from one


def test_pipeline_chain_through_mt_state_union(ctx):
    """MT -> Philox -> MT: the third call's producer reads the FIRST call's mt_state_out (the
    union of outputs, not only the latest call's, decides the wait)."""
    from lidar_slam_amd import synth
    from lidar_slam_amd.pipeline import ScanPipeline, mt_seed_state
    S = 2048
    ids = list(range(S))
    b = synth.make_batch(ids)
    sco, cpo = b["scan_chunk_off"], b["chunk_pt_off"]
    a = ScanPipeline(ctx, b["xy"], sco, cpo, seeds=np.array(ids, np.uint32), want_state=True)
    a.state_out.upload(np.tile(mt_seed_state(12345), (S, 1)))  # valid but wrong if read too early
    mid = ScanPipeline(ctx, b["xy"], sco, cpo, hyp="philox")
    c = ScanPipeline(ctx, b["xy"], sco, cpo, mt_state=a.state_out, want_state=True)
    a.run(sync=False)
    mid.run(sync=False)
    c.run(sync=False)
    ctx.sync()
    rc = c.results()
    ref = ScanPipeline(ctx, b["xy"], sco, cpo, mt_state=a.state_out.download(), want_state=True)
    ref.run()
    rr = ref.results()
    assert np.array_equal(rc["mask"], rr["mask"])
    assert np.array_equal(rc["mt_state"], rr["mt_state"])
