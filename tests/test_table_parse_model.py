"""CPU model of the producer's table-mode window parse (lslam_rng_pipe.h parse_chunk_tbl).

numpy's legacy choice(N, 2) runs Fisher-Yates steps i = K..1 (K = N-1) with
j = random_interval(i): a word w is rejected while (w & mask(i)) > i
(fit.py:819-826 via numpy's mtrand).  The kernel solves 64 words at a time:
lane l holds word pos+l, a_l = accepted words below it, s_l = 63 - a_l; bit a
of the lane's 64-bit window M (bits x = sg + a of row v = w & mask(K) of the
reject table for K) is its reject flag at that count, i.e. bit 63 of M << s.
The fixed point is found by Jacobi iteration from a 0.72-accepts guess.

This restates that scheme in numpy over 64 emulated lanes (windows across
block ends, chunk-end windows with fewer steps than lanes, K < 64 with several
draw boundaries per window) and checks it against the plain sequential parse.
It pins the invariants the kernel relies on; the GPU parity tests check the
kernel itself against the golden vectors.
"""
import numpy as np
import pytest

LANES = np.arange(64, dtype=np.int64)


def mask_of(i):
    m = np.asarray(i, dtype=np.uint64)
    for sh in (1, 2, 4, 8, 16):
        m = m | (m >> np.uint64(sh))
    return m


def reject_table(K):
    """rt_word: bit x of row v = (v & mask(i)) > i with i = K - (x mod K); 7 dwords per row."""
    x = np.arange(7 * 32, dtype=np.int64)
    i = K - (x % K)
    v = np.arange(128, dtype=np.uint64)[:, None]
    rej = (v & mask_of(i)[None, :]) > i[None, :].astype(np.uint64)
    return rej  # [128, 224] booleans


def sequential(words, K, G):
    out, g, k = [], 0, 0
    while g < G:
        i = K - (g % K)
        j = int(words[k]) & int(mask_of(i))
        if j <= i:
            out.append(j)
            g += 1
        k += 1
    return np.array(out, dtype=np.int64), k


def window_parse(words, K, G):
    """Full windows while more than 64 steps remain; the chunk's last window masks lanes
    whose count reaches the remaining steps.  Returns the stored v per step and the words used."""
    mK = int(mask_of(K))
    tbl = reject_table(K)
    out = np.full(G, -1, dtype=np.int64)
    g = sg = pos = 0
    guess = (LANES * 46) >> 6
    while g < G:
        rem = G - g
        v = words[pos:pos + 64].astype(np.int64) & mK
        # bits x in [sg, sg + 63] of each lane's row
        M = tbl[v][:, sg:sg + 64]            # M[l, a] = reject flag of lane l at count a
        last = rem <= 64
        a = guess.copy()
        acc = None
        for _ in range(66):
            ok = ~M[LANES, a]
            if last:
                ok &= a < rem
            a_new = np.concatenate([[0], np.cumsum(ok)[:-1]])
            if acc is not None and np.array_equal(ok, acc):
                break
            acc, a = ok, a_new
        else:
            raise AssertionError("no fixed point")
        out[g + a[acc]] = v[acc]
        na = int(acc.sum())
        if last and na >= rem:
            pos += int(np.nonzero(acc)[0][-1]) + 1
        else:
            pos += 64
        g += na
        sg = (sg + na) % K
    return out, pos


@pytest.mark.parametrize("K,D", [(99, 101), (19, 101), (2, 40), (63, 30), (64, 30), (127, 12)])
def test_window_parse_equals_sequential(K, D):
    rng = np.random.default_rng(1000 + K)
    G = D * K
    words = rng.integers(0, 2 ** 32, size=3 * G + 256, dtype=np.uint64)
    ref, used = sequential(words, K, G)
    got, pos = window_parse(words, K, G)
    # the consumer applies mask(i) to the stored v: j_i = v & mask(i) (v & mask(i) = w & mask(i))
    i = K - (np.arange(G) % K)
    assert np.array_equal(got & mask_of(i).astype(np.int64), ref)
    assert pos == used


def test_reject_table_rows_match_random_interval():
    K = 99
    tbl = reject_table(K)
    for v in (0, 1, 63, 64, 99, 100, 127):
        for x in (0, 1, 35, 98, 99, 150, 190):
            i = K - x % K
            assert tbl[v, x] == ((v & int(mask_of(i))) > i)
