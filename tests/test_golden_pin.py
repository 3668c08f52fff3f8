"""The golden generators pin the OpenBLAS dispatch, and every reference fixture records it.

The reference's float outputs depend on which OpenBLAS kernels numpy dispatches to
(``dgemv_t``/``ddot``/``dgesdd`` behind ``/root/reference/ransac_functions.py:23``, skimage
``fit.py:89,94,130-131``).  ``tests/golden/blaspin.py`` forces ``OPENBLAS_CORETYPE=SkylakeX``
before numpy loads and writes the selected core into each ``.npz``; ``census_dispatch.py``
regenerates the fixtures under other cores and counts the integer decisions that move.
"""
import ast
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, ROOT

REFERENCE_FIXTURES = ("assoc", "batch", "batch256", "big", "edge", "edge_chain", "express", "known", "live",
                      "mt_choice")
GENERATORS = ("tests/golden/make_golden.py", "tests/golden/make_golden_express.py",
              "tests/golden/make_ukf_exact.py", "tools/calibrate_twin.py")


@pytest.mark.parametrize("name", REFERENCE_FIXTURES)
def test_fixture_records_pinned_dispatch(name):
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        assert str(z["meta_blas_core"]) == "SkylakeX"
        assert "SkylakeX" in str(z["meta_blas_config"])
        assert str(z["meta_numpy"]) == "1.26.4"
        assert str(z["meta_skimage"]) == "0.18.3"
        assert str(z["meta_cpu_model"])


def _module_order(path):
    """Top-level imports in order: blaspin must come before numpy."""
    tree = ast.parse(open(os.path.join(ROOT, path)).read())
    names = []
    for node in tree.body:
        if isinstance(node, ast.Import):
            names += [a.name for a in node.names]
        elif isinstance(node, ast.ImportFrom):
            names.append(node.module)
    return names


@pytest.mark.parametrize("path", GENERATORS)
def test_generator_pins_blas_before_numpy(path):
    names = _module_order(path)
    assert "blaspin" in names and "numpy" in names
    assert names.index("blaspin") < names.index("numpy")
    src = open(os.path.join(ROOT, path)).read()
    assert "np.savez" not in src, "fixtures must go through blaspin.save_npz (metadata + reproducible bytes)"


def test_blaspin_pins_skylakex():
    tree = ast.parse(open(os.path.join(GOLDEN, "blaspin.py")).read())
    consts = {t.id: n.value.value for n in tree.body if isinstance(n, ast.Assign)
              for t in n.targets if isinstance(t, ast.Name) and isinstance(n.value, ast.Constant)}
    assert consts["PINNED_CORE"] == "SkylakeX"
    src = open(os.path.join(GOLDEN, "blaspin.py")).read()
    assert 'os.environ["OPENBLAS_CORETYPE"]' in src


def test_dispatch_census_recorded():
    """census_dispatch.py's result: the integer decisions under other kernel sets."""
    with open(os.path.join(GOLDEN, "dispatch_census.json")) as f:
        rep = json.load(f)
    assert rep["pinned_core"] == "SkylakeX"
    assert "Prescott" in rep["cores"]
    for core, r in rep["cores"].items():
        assert set(r["per_fixture"]) >= {"batch256", "batch", "live", "big"}
        n = sum(v for d in r["per_fixture"].values() for v in d["decisions"].values() if isinstance(v, int))
        assert n == r["integer_decisions_changed"], core
