"""Speculative producer for chained MT streams (lidarslam.hip run_split, map mode's pattern):
a call whose mt_state_in is the previous call's mt_state_out parses from the previous
producer's end state without waiting for that call's fix-up, and its fix-up replays the
scans the previous fix-up replayed.  Chained calls with early-stopping scans (every point
of a chunk on y = 7: the zero-sum stop at trial 0, fit.py:866-867) must equal the same
chain on a context that waits for each fix-up (LSLAM_MT_SPECULATE=0)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _contexts():
    from lidar_slam_amd.device import Context
    if Context.device_count() < 1:
        pytest.skip("no HIP device")
    spec = Context(0)
    old = os.environ.get("LSLAM_MT_SPECULATE")
    os.environ["LSLAM_MT_SPECULATE"] = "0"
    try:
        wait = Context(0)
    finally:
        if old is None:
            del os.environ["LSLAM_MT_SPECULATE"]
        else:
            os.environ["LSLAM_MT_SPECULATE"] = old
    return spec, wait


def _batch(S, stoppers):
    """synthetic scans; chunk 2 of the `stoppers` scans collinear on y = 7"""
    from lidar_slam_amd import synth
    b = synth.make_batch(list(range(S)))
    xy = b["xy"].copy()
    sco, cpo = b["scan_chunk_off"], b["chunk_pt_off"]
    for s in stoppers:
        c = sco[s] + 2
        p0, p1 = cpo[c], cpo[c + 1]
        xy[p0:p1, 0] = np.arange(p1 - p0) * 1.5
        xy[p0:p1, 1] = 7.0
    return xy, sco, cpo


def _chain(ctx, xy, sco, cpo, K):
    """K calls, call k+1's mt_state_in = call k's mt_state_out, no host sync in between"""
    from lidar_slam_amd.pipeline import ScanPipeline
    S = len(sco) - 1
    first = ScanPipeline(ctx, xy, sco, cpo, seeds=np.arange(S, dtype=np.uint32), lmk_capacity=64,
                         want_draws=True, want_state=True)
    pipes = [first]
    for _ in range(K - 1):
        pipes.append(ScanPipeline(ctx, xy, sco, cpo, mt_state=pipes[-1].state_out, lmk_capacity=64,
                                  want_draws=True, want_state=True))
    for p in pipes:
        p.run(sync=False)
    ctx.sync()
    return [p.results() for p in pipes]


@pytest.mark.parametrize("stoppers", [(), (5, 77, 200), tuple(range(0, 256, 3))])
def test_speculative_chain_equals_waiting_chain(stoppers):
    spec, wait = _contexts()
    xy, sco, cpo = _batch(256, stoppers)
    a = _chain(spec, xy, sco, cpo, 4)
    b = _chain(wait, xy, sco, cpo, 4)
    for k, (ra, rb) in enumerate(zip(a, b)):
        assert np.array_equal(ra["mt_state"], rb["mt_state"]), "call %d end states" % k
        assert np.array_equal(ra["draws"], rb["draws"]), "call %d draws" % k
        assert np.array_equal(ra["mask"], rb["mask"]), "call %d masks" % k
        assert ra["models"].tobytes() == rb["models"].tobytes(), "call %d models" % k
        assert np.array_equal(ra["lmk_count"], rb["lmk_count"]), "call %d lists" % k
    if stoppers:
        stop = (a[1]["models"]["flags"] & 16) != 0
        assert stop[np.array([sco[s] + 2 for s in stoppers])].all()  # the replay path ran


def test_state_upload_between_chained_calls_disables_speculation():
    """A caller writing the previous call's mt_state_out between two chained calls (here a
    DeviceArray.upload of other streams' states) must be what the next call parses from: the
    speculative context equals the waiting one and a fresh pipeline seeded from that state."""
    from lidar_slam_amd.pipeline import ScanPipeline, mt_seed_state
    spec, wait = _contexts()
    xy, sco, cpo = _batch(128, (3, 40))
    S = len(sco) - 1
    new_state = np.stack([mt_seed_state(1000 + s) for s in range(S)])
    outs = []
    for ctx in (spec, wait):
        p0 = ScanPipeline(ctx, xy, sco, cpo, seeds=np.arange(S, dtype=np.uint32), lmk_capacity=64, want_state=True)
        p1 = ScanPipeline(ctx, xy, sco, cpo, mt_state=p0.state_out, lmk_capacity=64, want_draws=True,
                          want_state=True)
        p0.run(sync=False)
        p0.state_out.upload(new_state)
        p1.run(sync=False)
        ctx.sync()
        outs.append(p1.results())
    fresh = ScanPipeline(spec, xy, sco, cpo, mt_state=new_state, lmk_capacity=64, want_draws=True, want_state=True)
    fresh.run()
    rf = fresh.results()
    for r in outs:
        assert np.array_equal(r["draws"], rf["draws"])
        assert np.array_equal(r["mt_state"], rf["mt_state"])
        assert np.array_equal(r["mask"], rf["mask"])


def test_long_speculative_chain_resyncs():
    """40 chained calls with early-stopping scans (past the LSLAM_SPEC_RESYNC bound of 32, where
    one call waits for the previous fix-up and the replay flags clear) equal the waiting chain."""
    spec, wait = _contexts()
    xy, sco, cpo = _batch(64, (1, 9, 30))
    a = _chain(spec, xy, sco, cpo, 40)
    b = _chain(wait, xy, sco, cpo, 40)
    for k, (ra, rb) in enumerate(zip(a, b)):
        assert np.array_equal(ra["mt_state"], rb["mt_state"]), "call %d end states" % k
        assert np.array_equal(ra["draws"], rb["draws"]), "call %d draws" % k
