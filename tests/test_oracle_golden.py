"""Pin the CPU oracle (oracle/ransac_oracle.c) against golden vectors produced
by importing the reference itself (tests/golden/make_golden.py).

Bit-exact: RNG words/draws/state, per-trial inlier counts, the tie-break sums,
the winning trial, inlier masks, the final origin (sequential mean), the tip x,
landmark ids/lives and list evolution.  Within tolerance: the final direction
(LAPACK dgesdd vs the closed-form 2x2 eigenvector) and what derives from it
(a, b, tip y, projected y).
"""
import numpy as np

from oracle import cpu as orc

RTOL_DIR = 1e-11


def _close_dir(u, v, tol=RTOL_DIR):
    u = np.asarray(u)
    v = np.asarray(v)
    return min(np.max(np.abs(u - v)), np.max(np.abs(u + v))) <= tol


def _rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return np.abs(a - b) / np.maximum(np.abs(b), 1.0)


def test_mt_seed_words_and_choice(golden):
    g = golden("mt_choice.npz")
    for i, seed in enumerate(g["seeds"]):
        st = orc.MTState(seed=int(seed))
        assert np.array_equal(st.key, g["init_key"][i])
        words = np.array([st.next32() for _ in range(g["words"].shape[1])], np.uint32)
        assert np.array_equal(words, g["words"][i])
        for j, n in enumerate(g["ns"]):
            st = orc.MTState(seed=int(seed))
            d = np.array([st.choice2(int(n)) for _ in range(g["draws"].shape[2])])
            assert np.array_equal(d, g["draws"][i, j]), (seed, n)
            assert np.array_equal(st.key, g["after_key"][i, j])
            assert st.pos.value == g["after_pos"][i, j]


def _check_chunk_seq(g, st, per_scan_seed=None, fresh_list_per_scan=False):
    """Run the oracle's landmark_extraction over every chunk of fixture g and
    compare with the reference record."""
    sco, cpo, xy = g["scan_chunk_off"], g["chunk_pt_off"], g["xy"]
    lst = []
    number = 0
    for s in range(len(sco) - 1):
        if per_scan_seed is not None:
            st = orc.MTState(seed=int(per_scan_seed[s]))
        if fresh_list_per_scan:
            lst = []
            number = 0
        for c in range(sco[s], sco[s + 1]):
            p0, p1 = cpo[c], cpo[c + 1]
            assert np.array_equal(st.key, g["state_before_key"][c]) and st.pos.value == g["state_before_pos"][c]
            # per-trial detail from the same entry state
            _, mod_t, ex = orc.ransac(xy[p0:p1], 20.0, 100, state=st.copy(), want_trials=True)
            assert np.array_equal(ex["draws"], g["draws"][c]), c
            assert np.array_equal(ex["cnt"], g["trial_cnt"][c]), c
            M = g["trial_cnt"][c].max()
            tied = (g["trial_cnt"][c] == M) & (np.arange(100) <= g["stop_trial"][c])
            assert np.array_equal(ex["sum"][tied], g["trial_sum"][c][tied]), c
            assert mod_t["best_trial"] == g["best_trial"][c]
            assert mod_t["n_draws"] == g["draws_used"][c]
            # the full landmark_extraction
            mask, yproj, mod, lst = orc.landmark_extraction(xy[p0:p1], number, lst, st, cap=len(lst) + 1)
            assert np.array_equal(mask, g["mask"][p0:p1]), c
            assert np.array_equal(st.key, g["state_after_key"][c]) and st.pos.value == g["state_after_pos"][c]
            assert mod["ox"] == g["origin"][c][0] and mod["oy"] == g["origin"][c][1], c
            assert _close_dir((mod["ux"], mod["uy"]), g["direction"][c]), c
            assert _rel(mod["a"], g["a"][c]) < 1e-9 and _rel(mod["b"], g["b"][c]) < 1e-9, c
            assert mod["tip_x"] == g["tip"][c][0] and _rel(mod["tip_y"], g["tip"][c][1]) < 1e-9
            assert bool(mod["flags"] & orc.FLAG_NEW_LANDMARK) == bool(g["new_landmark"][c])
            q0, q1 = g["q_off"][c], g["q_off"][c + 1]
            assert np.array_equal(xy[p0:p1][mask.astype(bool), 0], g["q_x"][q0:q1])
            assert np.all(_rel(yproj[mask.astype(bool)], g["q_y"][q0:q1]) < 1e-9)
            l0, l1 = g["lm_off"][c], g["lm_off"][c + 1]
            assert [L["id"] for L in lst] == list(g["lm_id"][l0:l1]), c
            assert [L["life"] for L in lst] == list(g["lm_life"][l0:l1]), c
            assert np.all(_rel([L["a"] for L in lst], g["lm_a"][l0:l1]) < 1e-9)
            number += 1
    return st


def test_batch_golden(golden):
    g = golden("batch.npz")
    _check_chunk_seq(g, None, per_scan_seed=g["seeds"], fresh_list_per_scan=True)


def test_live_golden(golden):
    g = golden("live.npz")
    st = orc.MTState(seed=int(g["seed"][0]))
    _check_chunk_seq(g, st)


def test_edge_chain_early_stop(golden):
    g = golden("edge_chain.npz")
    st = orc.MTState(seed=int(g["seed"][0]))
    _check_chunk_seq(g, st)
    assert list(g["draws_used"]) == [101, 2, 101]


def test_edge_cases(golden):
    g = golden("edge.npz")
    for k, name in enumerate(g["names"]):
        xy = g["xy"][g["off"][k]:g["off"][k + 1]]
        st = orc.MTState(seed=int(g["seeds"][k]))
        mask, mod, ex = orc.ransac(xy, float(g["thr"][k]), int(g["trials"][k]), state=st)
        err = g["err"][k]
        if err == 1 and len(xy) <= 2:
            assert mod["flags"] & orc.FLAG_N_TOO_SMALL, name
        elif err == 1:
            assert mod["flags"] & orc.FLAG_EST_FAIL, name
        elif err == 2:
            assert mod["flags"] & orc.FLAG_NO_INLIERS, name
        else:
            assert mod["flags"] & orc.FLAG_VALID, name
            p = g["params"][k]
            assert np.array_equal(mask, g["mask"][g["off"][k]:g["off"][k + 1]]), name
            assert mod["ox"] == p[0] and mod["oy"] == p[1], name
            assert _close_dir((mod["ux"], mod["uy"]), p[2:4]), name
            if np.isfinite(p[4]):
                assert _rel(mod["a"], p[4]) < 1e-9 and _rel(mod["b"], p[5]) < 1e-9, name
            else:
                assert not np.isfinite(mod["a"]), name
        assert mod["n_draws"] == g["ndraw"][k] or (len(xy) <= 2 and g["ndraw"][k] == 0), name
        assert np.array_equal(st.key, g["after_key"][k]) and st.pos.value == g["after_pos"][k], name


def test_assoc_quirks(golden):
    g = golden("assoc.npz")
    xy = g["xy"]
    for k, name in enumerate(g["names"]):
        i0, i1 = g["lm_in_off"][k], g["lm_in_off"][k + 1]
        lst = [{"a": g["lm_in_a"][i], "b": g["lm_in_b"][i], "pos": tuple(g["lm_in_pos"][i]),
                "end": tuple(g["lm_in_end"][i]), "id": int(g["lm_in_id"][i]), "life": int(g["lm_in_life"][i])}
               for i in range(i0, i1)]
        st = orc.MTState(seed=int(g["seed"][0]))
        mask, yproj, mod, out = orc.landmark_extraction(xy, 99, lst, st, cap=len(lst) + 1)
        o0, o1 = g["lm_out_off"][k], g["lm_out_off"][k + 1]
        assert [L["id"] for L in out] == list(g["lm_out_id"][o0:o1]), name
        assert [L["life"] for L in out] == list(g["lm_out_life"][o0:o1]), name
        assert bool(mod["flags"] & orc.FLAG_NEW_LANDMARK) == bool(g["new_landmark"][k]), name
        q0, q1 = g["q_off"][k], g["q_off"][k + 1]
        assert np.all(_rel(yproj[mask.astype(bool)], g["q_y"][q0:q1]) < 1e-9), name


def test_big_c5_shape(golden):
    g = golden("big.npz")
    T = int(g["trials"])
    for k in range(len(g["seeds"])):
        xy = g["xy"][g["off"][k]:g["off"][k + 1]]
        st = orc.MTState(seed=int(g["seeds"][k]))
        mask, mod, _ = orc.ransac(xy, 20.0, T, state=st)
        assert np.array_equal(mask, g["mask"][g["off"][k]:g["off"][k + 1]])
        assert mod["best_trial"] == g["best_trial"][k]
        p = g["params"][k]
        assert mod["ox"] == p[0] and mod["oy"] == p[1]
        assert _close_dir((mod["ux"], mod["uy"]), p[2:4])
        assert np.array_equal(st.key, g["after_key"][k]) and st.pos.value == g["after_pos"][k]


def test_known_answers(golden):
    g = golden("known.npz")
    # fit.py:48-62 docstring example goes through the >2-point (SVD) branch
    st = orc.MTState(seed=0)
    mask, mod, _ = orc.ransac(g["doc_xy"], 1e9, 1, state=st)
    assert mod["n_inliers"] == 25
    assert np.allclose([mod["ox"], mod["oy"]], g["doc_origin"], rtol=0, atol=1e-14)
    assert _close_dir((mod["ux"], mod["uy"]), g["doc_direction"], 1e-14)
    assert np.allclose(np.round(g["doc_direction"], 5), [0.5547, 0.83205])


def test_ecut_threshold_semantics():
    e = orc.ecut(20.0)
    assert e == 399.99999999999994
    assert np.sqrt(np.nextafter(e, 0)) < 20.0 and not (np.sqrt(e) < 20.0)
    for thr in (1e-9, 0.5, 1.0, 3.0, 7.25, 20.0, 123.456, 1e150):
        e = orc.ecut(thr)
        assert not (np.sqrt(e) < thr) and np.sqrt(np.nextafter(e, 0)) < thr
    assert orc.ecut(0.0) == 0.0
