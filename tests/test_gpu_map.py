"""GPU parity of the landmark-map step (LSLAM_UKF_MAP, lidar_slam_amd/slam.py,
SURVEY §8f rank 4) through the C ABI.

* Pose held at 0, no filter steps: a map step per revolution is the
  reference's check_ransac over it, so 14 revolutions reproduce the golden live
  run (one np.random.seed, one landmark list) bit for bit: masks, ids, lives,
  the MT19937 state.
* Moving robots with predict + update: each step against oracle/slam.py started
  from the device's previous state (x, P, map, stream).  Bit-exact: masks,
  chunk flags and matches, map ids/lives/counts, the stream.  Tolerances: the
  world-frame map values follow the predicted pose, whose rounding noise is the
  UKF's own (alpha = 1e-4 weights of ~1e8: |dx| <= 1e-4 mm), so positions
  <= 1e-3 mm, slope angles atan(a) <= 1e-6 rad; the filter state per
  component as for the UKF (x, y relative, theta absolute, P relative: 1e-5).
"""
import numpy as np
import pytest

from lidar_slam_amd import synth
from oracle import cpu as orc
from oracle import slam as osl
from oracle import ukf_exact

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from lidar_slam_amd.device import Context
    if Context.device_count() < 1:
        pytest.skip("no HIP device")
    return Context(0)


def test_identity_pose_map_is_the_reference_live_run(ctx, golden):
    from lidar_slam_amd.slam import LandmarkMap
    g = golden("live.npz")
    lm = LandmarkMap(ctx, 1, lmk_capacity=128, seeds=g["seed"], predict=False, update=False)
    sco, cpo = g["scan_chunk_off"], g["chunk_pt_off"]
    for r in range(len(sco) - 1):
        c0, c1 = sco[r], sco[r + 1]
        lm.step(g["xy"][cpo[c0]:cpo[c1]], [0, c1 - c0], cpo[c0:c1 + 1] - cpo[c0])
        res = lm.results()
        assert np.array_equal(res["mask"], g["mask"][cpo[c0]:cpo[c1]]), r
        assert list(res["models"]["landmark_id"]) == list(g["landmark_number"][c0:c1])
        l0, l1 = g["lm_off"][c1 - 1], g["lm_off"][c1]
        lst = res["landmarks"][0, :res["lmk_count"][0]]
        assert list(lst["id"]) == list(g["lm_id"][l0:l1]), r
        assert list(lst["life"]) == list(g["lm_life"][l0:l1]), r
        assert np.array_equal(lst["pos_x"], g["lm_pos"][l0:l1, 0])  # origins: sequential mean, exact
        assert np.array_equal(res["x"], np.zeros((1, 3)))
    assert np.array_equal(res["mt_state"][0, :624], g["state_after_key"][-1])
    assert res["mt_state"][0, 624] == g["state_after_pos"][-1]
    objs = lm.robot_map(0)
    assert [L.id for L in objs] == list(lst["id"]) and [L.life for L in objs] == list(lst["life"])


@pytest.fixture
def loose():
    orc.set_tolerances(0.1, 100.0, 1000.0)
    yield dict(tol_a=0.1, tol_b=100.0, tol_dist=1000.0)
    orc.set_tolerances()


@pytest.mark.parametrize("steps", [4])
def test_moving_robots_map_and_filter_vs_oracle(ctx, loose, steps):
    from lidar_slam_amd.slam import LandmarkMap
    R = 24
    robots = list(range(100, 100 + R))
    poses = synth.trajectory(robots, steps)
    rng = np.random.default_rng(9)
    x0 = poses[0] + rng.normal(0, [3.0, 3.0, 0.01], (R, 3))
    # consistent tuning (mm / rad): the reference's P0 = diag(.1, .1, .05) with R = [.25, .09]
    # lets mm-level range innovations swing the heading by 0.1 rad per update (oracle too)
    P0, Rd = np.diag([25.0, 25.0, 1e-4]), [25.0, 1e-4] * 8
    lm = LandmarkMap(ctx, R, lmk_capacity=256, seeds=robots, x0=x0, P0=P0, R_diag=Rd, **loose)
    rs = [osl.RobotState(seed=s, x0=x0[i], P0=P0, cap=256) for i, s in enumerate(robots)]
    n_match = 0
    for k in range(steps):
        rev = synth.revolutions_at(poses[k + 1], k, robots)
        lm.step(rev["xy"], rev["scan_chunk_off"], rev["chunk_pt_off"], u=np.tile([2.0, 2.5], (R, 1)))
        res = lm.results()
        sco, cpo = rev["scan_chunk_off"], rev["chunk_pt_off"]
        for i in range(R):
            c0, c1 = sco[i], sco[i + 1]
            mask, models = osl.map_step(rs[i], rev["xy"][cpo[c0]:cpo[c1]], cpo[c0:c1 + 1] - cpo[c0], (2.0, 2.5), Rd)
            assert np.array_equal(res["mask"][cpo[c0]:cpo[c1]], mask), (k, i)
            dm = res["models"][c0:c1]
            assert list(dm["flags"]) == [m["flags"] for m in models], (k, i)
            assert list(dm["match_index"]) == [m["match_index"] for m in models], (k, i)
            assert list(dm["landmark_id"]) == [m["landmark_id"] for m in models]
            n_match += int(np.sum((dm["flags"] & orc.FLAG_MATCHED) != 0))
            lst = res["landmarks"][i, :res["lmk_count"][i]]
            assert list(lst["id"]) == [L["id"] for L in rs[i].lst], (k, i)
            assert list(lst["life"]) == [L["life"] for L in rs[i].lst], (k, i)
            ref = np.array([[L["pos"][0], L["pos"][1], L["end"][0], L["end"][1]] for L in rs[i].lst])
            got = np.stack([lst["pos_x"], lst["pos_y"], lst["end_x"], lst["end_y"]], -1)
            assert np.max(np.abs(got - ref)) <= 1e-3, (k, i)
            ra = np.array([L["a"] for L in rs[i].lst])
            # slope as an angle: a = u_y/u_x amplifies the pose's heading noise by 1 + a^2
            assert np.max(np.abs(np.arctan(lst["a"]) - np.arctan(ra)), initial=0.0) <= 1e-6, (k, i)
            err = ukf_exact.component_errors(res["x"][i:i + 1], res["P"][i:i + 1], rs[i].x[None], rs[i].P[None])
            assert max(err.values()) <= 1e-5, (k, i, err)
            assert np.array_equal(res["mt_state"][i, :624], rs[i].st.key), (k, i)
            assert res["mt_state"][i, 624] == rs[i].st.pos.value
            # next step starts the oracle from the device's filter state (no drift)
            rs[i].x, rs[i].P = res["x"][i].copy(), res["P"][i].copy()
    assert n_match >= 50, n_match  # the update path is exercised


def test_map_mode_arguments(ctx):
    from lidar_slam_amd import _lib
    from lidar_slam_amd.pipeline import ScanPipeline
    from lidar_slam_amd.slam import LandmarkMap
    b = synth.make_batch([1, 2])
    ukf = dict(n_landmarks=8, flags=_lib.UKF_MAP | 3, x=np.zeros((2, 3)), P=np.tile(np.eye(3) * .1, (2, 1, 1)),
               u=np.zeros((2, 2)), z=np.zeros((2, 16)), lmk=np.zeros((2, 8, 2)), R_diag=np.ones(16))
    p = ScanPipeline(ctx, b["xy"], b["scan_chunk_off"], b["chunk_pt_off"], seeds=[1, 2], ukf=ukf)
    with pytest.raises(ValueError):
        p.run()  # MAP mode needs the landmark lists
    lm = LandmarkMap(ctx, 2, slots=4)
    with pytest.raises(ValueError):
        lm.step(b["xy"], b["scan_chunk_off"], b["chunk_pt_off"])  # 8 chunks > 4 slots
