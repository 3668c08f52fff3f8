"""The association walk of `associate` (csrc/lidarslam.hip) as bit operations on the equal /
dies ballots, against the serial walk it replaces (ransac_functions.py:35-43: examine i; equal ->
stop; else decrease_life; a removal makes `i += 1` skip the next entry).  Host restatement of the
device formula, checked bit for bit on random lists; the GPU parity tests check the kernel."""
import random

M64 = (1 << 64) - 1
EVEN = 0x5555555555555555


def walk_serial(E, D, L):
    k, match, vis = 0, -1, []
    for blk in range((L + 63) >> 6):
        if match >= 0 or k >= L:
            break
        V, hi = 0, min(L, blk * 64 + 64)
        while k < hi:
            bit = k - blk * 64
            if (E[blk] >> bit) & 1:
                match = k
                break
            V |= 1 << bit
            k += 2 if (D[blk] >> bit) & 1 else 1
        vis.append(V)
    return match, vis


def walk_bits(E, D, L):
    """Mirror of the device code (64-bit wrap-around arithmetic)."""
    k, match, vis = 0, -1, []
    for blk in range((L + 63) >> 6):
        if match >= 0 or k >= L:
            break
        base = blk * 64
        s0, n = k - base, min(L, base + 64) - base
        valid = M64 if n >= 64 else (1 << n) - 1
        ge = (M64 << s0) & M64
        Dm = D[blk] & valid & ge
        run0 = Dm & ~(Dm << 1) & M64
        Re = Dm & ~((Dm + (run0 & EVEN)) & M64)
        EO = (Re & EVEN) | (Dm & ~Re & ~EVEN & M64)
        visited = ge & valid & ~((EO << 1) & M64)
        hits = visited & E[blk]
        if hits:
            m = (hits & -hits).bit_length() - 1
            match = base + m
            vis.append(visited & ((1 << m) - 1))
        else:
            vis.append(visited)
            k = base + 64 + (EO >> 63) if n >= 64 else base + n
    return match, vis


def test_walk_bits_matches_serial():
    rnd = random.Random(20261017)
    for _ in range(20000):
        L = rnd.randint(1, 200)
        nblk = (L + 63) >> 6
        pe, pd = rnd.choice([0.0, 0.01, 0.05, 0.3]), rnd.choice([0.0, 0.2, 0.5, 0.8, 1.0])
        E, D = [0] * nblk, [0] * nblk
        for j in range(L):
            if rnd.random() < pe:
                E[j >> 6] |= 1 << (j & 63)
            if rnd.random() < pd:
                D[j >> 6] |= 1 << (j & 63)
        assert walk_bits(E, D, L) == walk_serial(E, D, L)


def test_walk_bits_edge_cases():
    # every entry dies: visited 0, 2, 4, ... across the block boundary; a run ending at bit 63
    for L in (1, 2, 63, 64, 65, 66, 128, 129):
        nblk = (L + 63) >> 6
        D = [M64] * nblk
        E = [0] * nblk
        assert walk_bits(E, D, L) == walk_serial(E, D, L)
        E = [1 << 63] + [0] * (nblk - 1)
        assert walk_bits(E, D, L) == walk_serial(E, D, L)
