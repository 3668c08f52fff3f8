"""The NumPy twin (cpu_baseline "port") reproduces the reference's masks and
landmark lists on the golden batch (same RNG stream, same per-trial structure)."""
import numpy as np

from oracle import numpy_twin as tw


def test_twin_matches_golden_batch(golden):
    g = golden("batch.npz")
    sco, cpo = g["scan_chunk_off"], g["chunk_pt_off"]
    for s in range(6):
        c0, c1 = sco[s], sco[s + 1]
        offs = cpo[c0:c1 + 1] - cpo[c0]
        xy = g["xy"][cpo[c0]:cpo[c1]]
        masks, lms = tw.process_scan(xy, offs, g["seeds"][s])
        assert np.array_equal(np.concatenate(masks).astype(np.uint8), g["mask"][cpo[c0]:cpo[c1]])
        l0, l1 = g["lm_off"][c1 - 1], g["lm_off"][c1]
        assert [L.id for L in lms] == list(g["lm_id"][l0:l1])
        assert [L.life for L in lms] == list(g["lm_life"][l0:l1])
