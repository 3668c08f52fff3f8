"""CPU simulation of the producer's window shape before building one.

    python tools/window_shape_sim.py [scans] > profiles/r05_window_shape_sim.json

Model: tests/test_table_parse_model.py (numpy's random_interval rejection behind choice(N, 2),
fit.py:819-826; the kernel's table-mode window solved by Jacobi iteration from a 0.72-accepts
guess).  C3's chunk shapes (K = 99 x 7, K = 19 x 1 per scan, 101 draws each) on random words.

Shapes compared, per full window (the chunk's last window excluded, as in the kernel's run loop):
  w64x1  the product: 64 lanes x 1 word.  One evaluation = v_mbcnt_lo/hi + a 64-bit shift of
         the lane's window row + a compare (4 VALU).
  w64x2  VERDICT r04's candidate: 64 lanes x 2 consecutive words (a 128-word window).  Lane l
         holds words 2l and 2l+1; a_2l = accepts of the lanes below (two ballots: 4 v_mbcnt),
         a_2l+1 = a_2l + accept(2l) (within the lane, same evaluation).  Each word's reject flag
         is a bit of a 128-bit row span (x in [sg, sg + 127]): pick the 64-bit half by a >= 64
         (compare + 2 selects), shift, compare: 5 VALU per word, + 1 add.  15 VALU per
         evaluation, i.e. 7.5 per 64 words.
Every window's fixed point is checked against the sequential parse.
Evaluations = iterations until a repeat (the repeat confirms the fixed point; the product runs
three before its first check, so max(3, n)).  The per-window fixed work that a 128-word window
pays once instead of twice (loop test, waits, accepted count, step/position bookkeeping) is
taken from the product's window (profiles/r05b_window_table.md): about 12 instructions."""
import json
import sys

import numpy as np

sys.path.insert(0, __import__("os").path.join(__import__("os").path.dirname(__file__), "..", "tests"))
from test_table_parse_model import mask_of  # noqa: E402

L64 = np.arange(64, dtype=np.int64)


def reject_table(K, width=384):
    """test_table_parse_model.reject_table over x in [0, width): bit x of row v rejects v at
    step i = K - (x mod K)."""
    x = np.arange(width, dtype=np.int64)
    i = K - (x % K)
    v = np.arange(128, dtype=np.uint64)[:, None]
    return (v & mask_of(i)[None, :]) > i[None, :].astype(np.uint64)


def sequential_accepts(v, sg, K):
    """Accept flags of the words v in order from step offset sg (x = sg + accepts so far)."""
    out, x = [], sg
    for w in v:
        i = K - (x % K)
        ok = (int(w) & int(mask_of(i))) <= i
        out.append(ok)
        x += ok
    return np.array(out)


def run_w64x1(words, K, G, tbl, mK, stats):
    g = sg = pos = 0
    guess = (L64 * 46) >> 6
    while G - g > 64:
        v = words[pos:pos + 64].astype(np.int64) & mK
        M = tbl[v][:, sg:sg + 64]
        a, acc, n = guess.copy(), None, 0
        while True:
            ok = ~M[L64, a]
            n += 1
            if acc is not None and np.array_equal(ok, acc):
                break
            acc = ok
            a = np.concatenate([[0], np.cumsum(ok)[:-1]])
        stats.append(max(3, n))
        assert np.array_equal(acc, sequential_accepts(v, sg, K))
        na = int(acc.sum())
        pos += 64
        g += na
        sg = (sg + na) % K
    return pos


def run_w64x2(words, K, G, tbl, mK, stats):
    g = sg = pos = 0
    guess = (2 * L64 * 46) >> 6  # a of word 2l
    while G - g > 128:
        v = words[pos:pos + 128].astype(np.int64) & mK
        M0 = tbl[v[0::2]][:, sg:sg + 128]
        M1 = tbl[v[1::2]][:, sg:sg + 128]
        a0, acc, n = guess.copy(), None, 0
        while True:
            ok0 = ~M0[L64, a0]
            ok1 = ~M1[L64, a0 + ok0]
            n += 1
            ok = np.stack([ok0, ok1])
            if acc is not None and np.array_equal(ok, acc):
                break
            acc = ok
            per = ok0.astype(np.int64) + ok1
            a0 = np.concatenate([[0], np.cumsum(per)[:-1]])
        stats.append(max(2, n))
        assert np.array_equal(acc.T.reshape(-1), sequential_accepts(v, sg, K))
        na = int(acc.sum())
        pos += 128
        g += na
        sg = (sg + na) % K
    return pos


def main():
    scans = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    rng = np.random.default_rng(5)
    s1, s2 = [], []
    for _ in range(scans):
        for K in [99] * 7 + [19]:
            G = 101 * K
            words = rng.integers(0, 2 ** 32, size=3 * G + 512, dtype=np.uint64)
            tbl = reject_table(K)
            mK = int(mask_of(K))
            run_w64x1(words, K, G, tbl, mK, s1)
            run_w64x2(words, K, G, tbl, mK, s2)
    e1, e2 = float(np.mean(s1)), float(np.mean(s2))
    fixed_saved = 12.0 / 2  # per 64 words, when a window holds 128 words
    out = {
        "model": "tests/test_table_parse_model.py; C3 chunk shapes, %d scans of random words" % scans,
        "w64x1": {"windows": len(s1), "evals_per_window": round(e1, 3), "eval_valu_per_64_words": round(4 * e1, 1)},
        "w64x2": {"windows": len(s2), "evals_per_window": round(e2, 3),
                  "eval_valu_per_64_words": round(7.5 * e2, 1),
                  "fixed_work_saved_per_64_words": fixed_saved},
        "verdict": ("w64x2 costs %.1f evaluation VALU per 64 words against w64x1's %.1f and saves ~%.0f "
                    "instructions of per-window bookkeeping per 64 words: %s"
                    % (7.5 * e2, 4 * e1, fixed_saved,
                       "not built" if 7.5 * e2 - 4 * e1 > fixed_saved else "worth building")),
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
