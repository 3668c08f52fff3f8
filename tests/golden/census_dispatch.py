"""Dispatch census: regenerate the reference fixtures under other OpenBLAS kernel sets and count
the decisions that change against the committed (SkylakeX-pinned) fixtures.

    /opt/conda/bin/python3.9 tests/golden/census_dispatch.py [--cores Prescott Haswell ...]

The reference's floats pass through OpenBLAS (``fit.py:89,94,130-131`` behind
``/root/reference/ransac_functions.py:23``); ``blaspin`` pins the fixtures to the SkylakeX
kernels.  This script runs ``make_golden.py`` once per other core (``LSLAM_GOLDEN_CORETYPE``,
output to a scratch directory) and compares, per fixture:

* integer decisions: inlier masks, per-trial counts, winning trial, draws used, inlier counts,
  new-landmark (``is_equal``) flags, landmark ids/lives, MT end states;
* float fields: the largest relative difference.

It writes ``tests/golden/dispatch_census.json`` (read by ``test_golden_pin.py``), naming every
chunk whose integer decision flips.
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
FIXTURES = ("batch256", "batch", "live", "edge", "edge_chain", "big", "assoc")
DECISIONS = ("mask", "trial_cnt", "best_trial", "draws_used", "stop_trial", "n_inl", "new_landmark", "lm_id",
             "lm_life", "lm_in_id", "lm_in_life", "lm_out_id", "lm_out_life", "state_after_key", "state_after_pos",
             "state_after_hash", "err", "ndraw", "after_key", "after_pos", "q_off")


def _per_chunk(g, k, idx):
    """Map flat differing indices of field k to chunk indices where the layout allows."""
    if k == "mask" and "chunk_pt_off" in g:
        return sorted(set(int(np.searchsorted(g["chunk_pt_off"], i, side="right") - 1) for i in idx))
    if k == "mask" and "off" in g:
        return sorted(set(int(np.searchsorted(g["off"], i, side="right") - 1) for i in idx))
    return sorted(set(int(i) for i in idx))


def compare(ref, new):
    out = {"decisions": {}, "flipped_chunks": {}, "float_max_rel": {}}
    for k in ref.files:
        if k.startswith("meta_") or k not in new.files:
            continue
        a, b = ref[k], new[k]
        if a.shape != b.shape:
            out["decisions"][k] = "shape %s vs %s" % (a.shape, b.shape)
            continue
        if a.dtype.kind == "f":
            with np.errstate(invalid="ignore", divide="ignore"):
                both_nan = np.isnan(a) & np.isnan(b)
                rel = np.abs(a - b) / np.maximum(np.abs(a), 1e-300)
                rel[both_nan | (a == b)] = 0
            out["float_max_rel"][k] = float(np.nanmax(rel)) if rel.size else 0.0
        elif k in DECISIONS or a.dtype.kind in "iub":
            if k.endswith("_off") and k != "q_off":
                continue
            ne = np.flatnonzero((a != b).reshape(len(a), -1).any(-1)) if a.ndim else (
                np.array([0]) if a != b else np.array([], int))
            out["decisions"][k] = int(len(ne))
            if len(ne):
                out["flipped_chunks"][k] = _per_chunk(ref, k, ne)[:50]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cores", nargs="+", default=["Prescott", "Haswell", "Zen", "Sandybridge"])
    ap.add_argument("--out", default=os.path.join(HERE, "dispatch_census.json"))
    args = ap.parse_args()
    report = {"pinned_core": "SkylakeX", "fixtures": list(FIXTURES), "cores": {}}
    for core in args.cores:
        with tempfile.TemporaryDirectory() as tmp:
            env = dict(os.environ, LSLAM_GOLDEN_CORETYPE=core, LSLAM_GOLDEN_OUT=tmp)
            subprocess.check_call([sys.executable, os.path.join(HERE, "make_golden.py"),
                                   "batch256", "batch", "live", "edge", "assoc", "big"],
                                  env=env, stdout=subprocess.DEVNULL)
            per = {}
            for f in FIXTURES:
                with np.load(os.path.join(HERE, f + ".npz")) as ref, np.load(os.path.join(tmp, f + ".npz")) as new:
                    assert str(new["meta_blas_core"]).lower() == core.lower(), new["meta_blas_core"]
                    per[f] = compare(ref, new)
            flips = sum(v for d in per.values() for v in d["decisions"].values() if isinstance(v, int))
            report["cores"][core] = {"integer_decisions_changed": flips, "per_fixture": per}
            print(core, "integer decisions changed:", flips, flush=True)
    with open(args.out, "w") as f:
        json.dump(report, f, indent=1, sort_keys=True)
    print("wrote", args.out)


if __name__ == "__main__":
    main()
