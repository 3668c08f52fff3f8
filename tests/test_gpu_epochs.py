"""GPU: the parity producer in epochs (lslam_set_steps_budget).

One-chunk scans whose Fisher-Yates steps exceed the slot budget run the MT19937
producer in launches of as many draws as fit, each resolved before its slot is
reused, the stream state chained between launches (C5: 68.7 GB of steps per call
otherwise).  The draws, the end state and every pipeline output must equal the
single-launch run byte for byte, and the oracle's choice(N, 2) sequence.
Reference semantics: fit.py:819-826 (numpy legacy choice on the global stream).
"""
import numpy as np
import pytest

from oracle import cpu as orc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from lidar_slam_amd.device import Context
    if Context.device_count() < 1:
        pytest.skip("no HIP device")
    c = Context(0)
    yield c
    c.set_steps_budget(0)


def _one_chunk_batch(n, S):
    sco = np.arange(S + 1, dtype=np.int32)
    cpo = (np.arange(S + 1) * n).astype(np.int32)
    return sco, cpo


@pytest.mark.parametrize("n,trials,budget_draws", [(100, 150, 7), (100, 100, 64), (300, 120, 13), (1000, 60, 1)])
def test_hyp_epochs_equal_single_launch(ctx, n, trials, budget_draws):
    """u8 (table-mode parse) and u16 steps, LDS-staged and tiled resolves, 1..64 draws per epoch."""
    from lidar_slam_amd import pipeline as pl
    S = 20
    seeds = np.arange(S, dtype=np.uint32) + 500
    sco, cpo = _one_chunk_batch(n, S)
    ctx.set_steps_budget(0)
    d1, s1 = pl.hyp_mt19937(ctx, sco, cpo, seeds=seeds, max_trials=trials)
    esz = 1 if n <= 256 else 2
    ctx.set_steps_budget(budget_draws * S * n * esz)  # budget_draws draws per epoch
    try:
        d2, s2 = pl.hyp_mt19937(ctx, sco, cpo, seeds=seeds, max_trials=trials)
    finally:
        ctx.set_steps_budget(0)
    assert np.array_equal(d1, d2)
    assert np.array_equal(s1, s2)
    for s in (0, S - 1):
        st = orc.MTState(seed=int(seeds[s]))
        ref = np.array([st.choice2(n) for _ in range(trials + 1)])
        assert np.array_equal(d2[s], ref)
        assert np.array_equal(s2[s, :624], st.key) and s2[s, 624] == st.pos.value


def test_pipeline_epochs_chained_state(ctx):
    """The fused pipeline in epochs, from an explicit MT state, twice in a row (the second call
    chains from the first's end state): masks, models, draws and states equal the single-launch
    run, and the oracle."""
    from lidar_slam_amd import synth
    from lidar_slam_amd.pipeline import ScanPipeline
    S, n, trials = 12, 600, 90
    xys = [synth.polar_to_xy_ref(*synth.scan_polar(700 + s, n_beams=n, cfg=5)[:2]) for s in range(S)]
    xy = np.concatenate(xys)
    sco, cpo = _one_chunk_batch(n, S)
    st0 = np.stack([np.append(orc.MTState(seed=40 + s).key, 624) for s in range(S)]).astype(np.uint32)

    def two_calls():
        p = ScanPipeline(ctx, xy, sco, cpo, mt_state=st0, max_trials=trials, want_draws=True, want_state=True)
        p.run()
        r1 = p.results()
        p2 = ScanPipeline(ctx, xy, sco, cpo, mt_state=r1["mt_state"], max_trials=trials, want_draws=True,
                          want_state=True)
        p2.run()
        return r1, p2.results()

    ctx.set_steps_budget(0)
    a1, a2 = two_calls()
    ctx.set_steps_budget(5 * S * n * 2)  # 5 draws per epoch: 19 launches per call
    try:
        b1, b2 = two_calls()
    finally:
        ctx.set_steps_budget(0)
    for ra, rb in ((a1, b1), (a2, b2)):
        for k in ("mask", "draws", "mt_state"):
            assert np.array_equal(ra[k], rb[k]), k
        assert ra["models"].tobytes() == rb["models"].tobytes()
    for s in (0, 5):
        st = orc.MTState(seed=40 + s)
        mo, md, _ = orc.ransac(xys[s], 20.0, trials, state=st)
        assert np.array_equal(b1["mask"][s * n:(s + 1) * n], mo)
        assert b1["models"]["best_trial"][s] == md["best_trial"]
        assert np.array_equal(b1["mt_state"][s, :624], st.key)


@pytest.mark.parametrize("n", [20, 65, 100, 128])
def test_table_parse_windows_across_block_ends(ctx, n):
    """Table-mode parse (chunks of <= 128 points) from states whose position sits just before,
    at and after the 624-word block end, and one- to three-chunk scans: draws and end states
    (key + pos, numpy's lazy twist at pos == 624 included) equal the oracle's."""
    from lidar_slam_amd import pipeline as pl
    starts = [0, 100, 560, 600, 620, 623, 624]
    S = len(starts) * 3
    sizes, states, chunks = [], [], []
    for k, p0 in enumerate(starts):
        for nch in (1, 2, 3):
            st = orc.MTState(seed=3000 + 10 * k + nch)
            st.pos.value = p0
            states.append(np.append(st.key, p0))
            chunks.append(nch)
            sizes += [n - (c % 2) for c in range(nch)]
    sco = np.concatenate([[0], np.cumsum(chunks)]).astype(np.int32)
    cpo = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int32)
    trials = 37
    draws, state = pl.hyp_mt19937(ctx, sco, cpo, mt_state=np.array(states, np.uint32), max_trials=trials)
    for s in range(S):
        st = orc.MTState(key=states[s][:624], pos=int(states[s][624]))
        for c in range(sco[s], sco[s + 1]):
            nc = int(cpo[c + 1] - cpo[c])
            ref = np.array([st.choice2(nc) for _ in range(trials + 1)])
            assert np.array_equal(draws[c], ref), (n, s, c)
        assert np.array_equal(state[s, :624], st.key), (n, s)
        assert state[s, 624] == st.pos.value, (n, s)


def test_epochs_with_an_early_stop(ctx):
    """A one-chunk scan whose points are all on one line stops at the first trial (residual sum
    exactly 0, fit.py:866-869); the fix-up replays it from the input state.  In epochs the other
    scans' draws and end states come from the chained launches: every output equals the
    single-launch run, and the collinear scan's end state the oracle's."""
    from lidar_slam_amd import synth
    from lidar_slam_amd.pipeline import ScanPipeline
    S, n, trials = 6, 300, 80
    xys = [synth.polar_to_xy_ref(*synth.scan_polar(900 + s, n_beams=n, cfg=5)[:2]) for s in range(S)]
    xys[2] = np.stack([np.linspace(-900.0, 1500.0, n), np.full(n, 7.0)], 1)
    xy = np.concatenate(xys)
    sco, cpo = _one_chunk_batch(n, S)
    seeds = np.arange(S) + 77

    def run():
        p = ScanPipeline(ctx, xy, sco, cpo, seeds=seeds, max_trials=trials, want_draws=True, want_state=True)
        p.run()
        return p.results()

    ctx.set_steps_budget(0)
    a = run()
    ctx.set_steps_budget(9 * S * n * 2)  # 9 draws per epoch
    try:
        b = run()
    finally:
        ctx.set_steps_budget(0)
    assert b["models"]["flags"][2] & 16 and b["models"]["n_draws"][2] < trials + 1
    for k in ("mask", "draws", "mt_state"):
        assert np.array_equal(a[k], b[k]), k
    assert a["models"].tobytes() == b["models"].tobytes()
    st = orc.MTState(seed=int(seeds[2]))
    mo, md, _ = orc.ransac(xys[2], 20.0, trials, state=st)
    assert np.array_equal(b["mask"][2 * n:3 * n], mo)
    assert np.array_equal(b["mt_state"][2, :624], st.key) and b["mt_state"][2, 624] == st.pos.value


@pytest.mark.parametrize("top", [200, 300])
def test_walk_resolve_ragged_chunks(ctx, top):
    """Unstaged resolves (a chunk's steps over the 16 KiB stage): one wave per (chunk, draw),
    lanes = steps.  Chunks of 3..top points in one batch (K from 2, a single partial window with
    many tracker hops, to several 512-step groups), u8 (top 200) and u16 (top 300) steps: every
    draw and the end states equal the oracle's choice(N, 2) sequence.  Table-mode (N <= 128) and
    mask-mode chunks share the scans, both orders (the producer's reject table must exist whenever
    any chunk can use it, not only when the largest chunk does)."""
    from lidar_slam_amd import pipeline as pl
    sizes = [top, 3, 4, 5, 30, 64, 65, 66, 129, top]
    S = 3
    sco = (np.arange(S + 1) * len(sizes)).astype(np.int32)
    cpo = np.concatenate([[0], np.cumsum(sizes * S)]).astype(np.int32)
    trials = 120  # 121 draws x (top - 1) steps > 16 KiB
    seeds = np.arange(S, dtype=np.uint32) + 7100
    draws, state = pl.hyp_mt19937(ctx, sco, cpo, seeds=seeds, max_trials=trials)
    for s in range(S):
        st = orc.MTState(seed=int(seeds[s]))
        for c in range(sco[s], sco[s + 1]):
            nc = int(cpo[c + 1] - cpo[c])
            ref = np.array([st.choice2(nc) for _ in range(trials + 1)])
            assert np.array_equal(draws[c], ref), (top, s, c, nc)
        assert np.array_equal(state[s, :624], st.key) and state[s, 624] == st.pos.value


def test_register_resolve_ragged_pipeline(ctx):
    """The pipeline's resolve from registers (u8 steps that would fit the 16 KiB stage, the next
    call's producer beside it): chunks of 3..256 points in one batch (K from 2, tail-only rows, to
    fifteen 16-step loads), random points (no early stop): every chunk's draws equal the oracle's
    choice(N, 2) sequence chained through the scan."""
    from lidar_slam_amd.pipeline import ScanPipeline
    sizes = [3, 4, 17, 18, 19, 33, 100, 128, 129, 200, 256]
    S, T = 3, 60  # 61 draws x 255 steps < 16 KiB
    sco = (np.arange(S + 1) * len(sizes)).astype(np.int32)
    cpo = np.concatenate([[0], np.cumsum(sizes * S)]).astype(np.int32)
    rng = np.random.default_rng(11)
    xy = rng.uniform(-5000.0, 5000.0, (int(cpo[-1]), 2))
    seeds = np.arange(S, dtype=np.uint32) + 9100
    p = ScanPipeline(ctx, xy, sco, cpo, seeds=seeds, max_trials=T, want_draws=True)
    p.run()
    r = p.results()
    assert not np.any(r["models"]["flags"] & 16)  # LSLAM_EARLY_STOP
    for s in range(S):
        st = orc.MTState(seed=int(seeds[s]))
        for c in range(sco[s], sco[s + 1]):
            nc = int(cpo[c + 1] - cpo[c])
            ref = np.array([st.choice2(nc) for _ in range(T + 1)])
            assert np.array_equal(r["draws"][c], ref), (s, c, nc)
