"""CPU simulation of the producer window's starting guess (the fixed point's first evaluation).

    python tools/guess_sim.py [scans] > profiles/r05_guess_sim.json

Model: tests/test_table_parse_model.py (numpy's random_interval rejection behind choice(N, 2),
fit.py:819-826; the kernel's table-mode window solved by Jacobi iteration).  C3's chunk shapes
(K = 99 x 7, K = 19 x 1 per scan, 101 draws each) on random words.

n = evaluations until one repeats the previous (the repeat confirms the fixed point).  The
product runs U unchecked evaluations, then one per checked turn until a turn repeats: it issues
max(U + 1, n) evaluations.  Guesses of lane l's accepted-words-below count a_l compared:
  const   the product: (46 l) >> 6, 0.72 accepts per word wherever the window starts
  rate    (l r(sg)) >> 8, r = 256 x the mean accept probability of the next 46 steps from the
          window's step sg (a per-K table of K bytes)
  path    the expected count itself: a_{l+1} = a_l + p(sg + a_l) from a_0 = 0, rounded
          (a per-K table of K x 64 bytes)."""
import json
import sys

import numpy as np

sys.path.insert(0, __import__("os").path.join(__import__("os").path.dirname(__file__), "..", "tests"))
from test_table_parse_model import mask_of  # noqa: E402

L64 = np.arange(64, dtype=np.int64)


def accept_prob(K, x):
    i = K - (np.asarray(x) % K)
    return (i + 1) / (mask_of(i).astype(np.float64) + 1)


def guesses(K):
    g = {"const": np.tile((L64 * 46) >> 6, (K, 1))}
    r = np.array([np.round(256 * accept_prob(K, np.arange(sg, sg + 46)).mean()) for sg in range(K)]).astype(np.int64)
    g["rate"] = (L64[None, :] * r[:, None]) >> 8
    path = np.zeros((K, 64))
    for sg in range(K):
        a = 0.0
        for l in range(64):
            path[sg, l] = a
            a += float(np.interp(sg + a, np.arange(sg, sg + 130), accept_prob(K, np.arange(sg, sg + 130))))
    g["path"] = np.rint(path).astype(np.int64)
    return g


def reject_table(K, width=384):
    x = np.arange(width, dtype=np.int64)
    i = K - (x % K)
    v = np.arange(128, dtype=np.uint64)[:, None]
    return (v & mask_of(i)[None, :]) > i[None, :].astype(np.uint64)


def run(words, K, G, tbl, mK, gs, stats):
    g = sg = pos = 0
    while G - g > 64:
        v = words[pos:pos + 64].astype(np.int64) & mK
        M = tbl[v][:, sg:sg + 64]
        fixed = None
        for name, gt in gs.items():
            a, acc, n = np.minimum(gt[sg], L64), None, 0
            while True:
                ok = ~M[L64, a]
                n += 1
                if acc is not None and np.array_equal(ok, acc):
                    break
                acc = ok
                a = np.concatenate([[0], np.cumsum(ok)[:-1]])
            stats[name].append(n)
            if fixed is None:
                fixed = acc
            assert np.array_equal(fixed, acc)
        na = int(fixed.sum())
        pos += 64
        g += na
        sg = (sg + na) % K


def main():
    scans = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    rng = np.random.default_rng(5)
    cache = {}
    stats = {"const": [], "rate": [], "path": []}
    for _ in range(scans):
        for K in [99] * 7 + [19]:
            if K not in cache:
                cache[K] = (reject_table(K), int(mask_of(K)), guesses(K))
            tbl, mK, gs = cache[K]
            words = rng.integers(0, 2 ** 32, size=3 * 101 * K + 512, dtype=np.uint64)
            run(words, K, 101 * K, tbl, mK, gs, stats)
    out = {"model": "tests/test_table_parse_model.py; C3 chunk shapes, %d scans of random words" % scans}
    for name, s in stats.items():
        s = np.array(s)
        out[name] = {"windows": int(s.size), "n_mean": round(float(s.mean()), 3),
                     "n_hist": {int(k): int((s == k).sum()) for k in range(1, int(s.max()) + 1)},
                     "issued_U3": round(float(np.maximum(4, s).mean()), 3),
                     "issued_U2": round(float(np.maximum(3, s).mean()), 3),
                     "issued_U1": round(float(np.maximum(2, s).mean()), 3)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
