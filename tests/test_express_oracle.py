"""The express-scan codec oracle (oracle/express.py) against the golden
vectors recorded from the reference's lidar.py (tests/golden/express.npz)."""
import numpy as np
import pytest

from oracle import express as ox


@pytest.mark.parametrize("name", ["clean", "dirty"])
def test_decode_matches_reference(golden, name):
    g = golden("express.npz")
    d = ox.decode_packets(g[name + "_packets"])
    assert np.array_equal(d["valid"], g[name + "_valid"])
    ok = g[name + "_valid"].astype(bool)
    for k in ("dist", "corr", "new_scan_bit", "start"):
        assert np.array_equal(d[k][ok], g["%s_%s" % (name, k)][ok]), k


@pytest.mark.parametrize("name", ["clean", "dirty"])
def test_measure_stream_matches_reference(golden, name):
    g = golden("express.npz")
    m = ox.measures(ox.decode_packets(g[name + "_packets"]))
    for k in ("m_ok", "m_new", "m_ang", "m_dist"):
        assert np.array_equal(m[k], g["%s_%s" % (name, k)]), k


def test_dirty_stream_flags_the_corrupted_packets(golden):
    g = golden("express.npz")
    bad = g["bad_index"]
    assert not g["dirty_valid"][bad].any() and g["dirty_valid"].sum() == len(g["dirty_valid"]) - len(bad)
    m_ok = g["dirty_m_ok"]
    for p in bad:
        assert not m_ok[p].any() and not m_ok[p - 1].any()


def test_twos_comp_quirk():
    # bits above the sign bit are not masked (lidar.py:55-59 + the (b & 3) << 4 term)
    assert list(ox.twos_comp([0, 15, 16, 31, 32, 47, 48, 63], 5)) == [0, 15, -16, -1, 32, 47, 16, 31]


@pytest.mark.parametrize("name", ["capA", "capB"])
def test_capture_loop_matches_reference(golden, name):
    # functions.scanning over the reference's measure stream (warm-up drop included)
    g = golden("express.npz")
    r = ox.capture(g[name + "_packets"], int(g[name + "_drop"]))
    assert np.array_equal(r["chunk_sizes"], g[name + "_chunk_sizes"])
    assert np.array_equal(r["delim"], g[name + "_delim"])
    assert np.array_equal(r["xy"], g[name + "_xy"])


@pytest.mark.parametrize("name", ["capA", "capB"])
def test_revolutions_are_the_completed_part_of_the_capture(golden, name):
    g = golden("express.npz")
    pk, drop = g[name + "_packets"], int(g[name + "_drop"])
    # a warm-up drop of 32q + r measures = start at packet q with skip r
    q, r = divmod(drop, 32)
    rv = ox.revolutions(pk[q:], skip=r)
    delim, sizes = g[name + "_delim"], g[name + "_chunk_sizes"]
    assert np.array_equal(rv["scan_chunk_off"], np.concatenate([[0], delim]))
    assert np.array_equal(np.diff(rv["chunk_pt_off"]), sizes[:delim[-1]])
    assert np.array_equal(rv["xy"], g[name + "_xy"][:rv["chunk_pt_off"][-1]])
    # resuming from the last flagged packet with skip 1 continues the stream
    rest = ox.capture(pk[q + rv["resume"]:], drop=1)
    full = ox.capture(pk[q:], drop=r)
    n_done = rv["chunk_pt_off"][-1]
    assert np.array_equal(rest["xy"], full["xy"][n_done:])
