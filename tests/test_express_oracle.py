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
