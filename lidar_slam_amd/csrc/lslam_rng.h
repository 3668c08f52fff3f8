// lslam_rng.h — hypothesis generation.
//
// Parity mode reproduces numpy's legacy RandomState stream that
// skimage.measure.ransac draws from (fit.py:791 -> _shared/utils.py:340-341,
// np.random.mtrand._rand): fit.py:819-826 calls choice(N, 2, replace=False) =
// permutation(N)[:2] once before the trial loop and once per trial, i.e. a full
// Fisher-Yates shuffle of arange(N) with j = random_interval(i) for
// i = N-1 .. 1, random_interval rejecting (u32 & mask) > i.
//
// Wave-parallel formulation (one scan = one stream = one wave):
//   * MT19937 state lives in LDS; the 624-word twist is done by 64 lanes in 3
//     dependency phases ([0,227) old words, [227,454) reads phase-1 words,
//     [454,624) reads phase-2 words and key[0]).
//   * the rejection parse is a sequential automaton over the word stream
//     (state = global step g; word k accepted iff (w_k & mask(i)) <= i with
//     i = K - g mod K, K = N-1).  A 64-word window is solved in parallel by a
//     fixed-point iteration on the accept ballot: lane l's state is
//     g + popcount(accepts below l); iterate accept = f(state) until the ballot
//     repeats.  Each iteration fixes at least the lowest wrong lane, so it
//     terminates (<= 64 iterations, ~3 in practice) at the unique fixpoint.
//   * the fixed point starts from a rate guess (~0.72 accepts per word), which
//     cuts the mean iteration count from ~6 to ~4.4 on 100-point chunks.
//   * each accepted j_i is scattered (LDS atomic min) into its draw's
//     next-writer table nxt[p] = min{i > max(p,1) : j_i == p}; once a draw's K
//     steps are in, the value at position q before step 1 is the end of the
//     pointer chase q -> nxt[q] -> ... (V(q) = V(nxt[q]) or q), and step 1
//     swaps x[0], x[1] iff j_1 == 0.  Draws are resolved 4 at a time (8 lanes
//     chase in parallel) from a ring of power-of-two slots.
#pragma once
#include "lslam_wave.h"

namespace lslam {

// One wave per workgroup: LDS operations of a wave are executed in program
// order, so ordering LDS accesses across lanes only needs a compiler barrier
// (no s_waitcnt, no s_barrier).
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
}

constexpr int MT_N = 624;
constexpr int MT_M = 397;
constexpr uint32_t MT_UP = 0x80000000u;
constexpr uint32_t MT_LO = 0x7fffffffu;
constexpr uint32_t MT_MA = 0x9908b0dfu;

__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

// one twisted word: far ^ (y >> 1) ^ (y odd ? MATRIX_A : 0), y = cur's top bit | nxt's low 31.
// Five VALU: y as one v_bitop3 (lo ? nxt : cur), the odd-mask from nxt's bit 0 (= y's) by
// v_bfe_i32, (mask & MATRIX_A) ^ far as one v_bitop3, the shift, the xor (the plain form
// compiles to seven).
__device__ __forceinline__ uint32_t mt_mix(uint32_t cur, uint32_t nxt, uint32_t far) {
    const uint32_t y = __builtin_amdgcn_bitop3_b32(cur, nxt, MT_LO, 0xD8);
    const uint32_t m = (uint32_t)__builtin_amdgcn_sbfe((int)nxt, 0, 1);
    const uint32_t t = __builtin_amdgcn_bitop3_b32(m, MT_MA, far, 0x6A);
    return t ^ (y >> 1);
}

// mt19937_gen on key[624] in LDS by one wave
__device__ __forceinline__ void mt_twist(uint32_t *key, int lane) {
    uint32_t v[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        int i = lane + 64 * k;
        if (i < MT_N - MT_M) v[k] = mt_mix(key[i], key[i + 1], key[i + MT_M]);
    }
    wave_lds_sync();
#pragma unroll
    for (int k = 0; k < 4; k++) {
        int i = lane + 64 * k;
        if (i < MT_N - MT_M) key[i] = v[k];
    }
    wave_lds_sync();
#pragma unroll
    for (int k = 0; k < 4; k++) {
        int i = (MT_N - MT_M) + lane + 64 * k;
        if (i < 2 * (MT_N - MT_M)) v[k] = mt_mix(key[i], key[i + 1], key[i - (MT_N - MT_M)]);
    }
    wave_lds_sync();
#pragma unroll
    for (int k = 0; k < 4; k++) {
        int i = (MT_N - MT_M) + lane + 64 * k;
        if (i < 2 * (MT_N - MT_M)) key[i] = v[k];
    }
    wave_lds_sync();
#pragma unroll
    for (int k = 0; k < 3; k++) {
        int i = 2 * (MT_N - MT_M) + lane + 64 * k;
        if (i < MT_N) {
            uint32_t nxt = (i == MT_N - 1) ? key[0] : key[i + 1];
            v[k] = mt_mix(key[i], nxt, key[i - (MT_N - MT_M)]);
        }
    }
    wave_lds_sync();
#pragma unroll
    for (int k = 0; k < 3; k++) {
        int i = 2 * (MT_N - MT_M) + lane + 64 * k;
        if (i < MT_N) key[i] = v[k];
    }
    wave_lds_sync();
}

// numpy mt19937_seed (init_genrand): sequential recurrence, lane 0
__device__ __forceinline__ void mt_seed(uint32_t *key, uint32_t seed, int lane) {
    if (lane == 0) {
        for (int i = 0; i < MT_N; i++) {
            key[i] = seed;
            seed = 1812433253u * (seed ^ (seed >> 30)) + (uint32_t)(i + 1);
        }
    }
    wave_lds_sync();
}

// q = floor(x / K), r = x - q*K for x < 2^22 (float reciprocal + one correction)
__device__ __forceinline__ void divmod_small(uint32_t x, uint32_t K, float invK, uint32_t &q, uint32_t &r) {
    q = (uint32_t)((float)x * invK);
    int rr = (int)x - (int)(q * K);
    if (rr < 0) { rr += (int)K; q -= 1; }
    else if (rr >= (int)K) { rr -= (int)K; q += 1; }
    r = (uint32_t)rr;
}

struct MTWave {
    uint32_t *key;   // LDS [624]
    uint32_t *nxt;   // LDS [nslot][N]: per draw, nxt[p] = min{i > max(p,1) : j_i == p} (0xffffffff = none)
    uint32_t *j1s;   // LDS [nslot]: j_1 (the last Fisher-Yates step) of each in-flight draw
    int pos;         // wave-uniform 0..624
#ifdef LSLAM_STAMPS
    uint64_t acc[8];
#endif
};

constexpr uint32_t MT_NONE = 0xffffffffu;

// Diagnostic build only (-DLSLAM_STAMPS): per-wave cycle accounting of the
// parse phases (guide §7 "In-kernel stamps"); never compiled into the product.
#ifdef LSLAM_STAMPS
__device__ __forceinline__ uint64_t lslam_stamp() {
    uint64_t t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#define LSLAM_STAMP_DECL uint64_t _st_prev = lslam_stamp();
#define LSLAM_STAMP(k)                         \
    do {                                       \
        const uint64_t _t = lslam_stamp();     \
        mt.acc[k] += _t - _st_prev;            \
        _st_prev = _t;                         \
    } while (0)
#else
#define LSLAM_STAMP_DECL
#define LSLAM_STAMP(k) \
    do {               \
    } while (0)
#endif

// Host-side sizing of the draw-resolution slots (power of two >= RB + ceil(64/K)).
__host__ __device__ inline int mt_resolve_batch(int N) { return N <= 512 ? 4 : 1; }
__host__ __device__ inline int mt_nslot(int N) {
    const int K = N > 2 ? N - 1 : 2;
    int need = mt_resolve_batch(N) + (64 + K - 1) / K;
    int s = 1;
    while (s < need) s <<= 1;
    return s;
}

// nxt entries carry the draw tag in the high half so that slots never need
// clearing within a chunk: entry = (0xfffe - d) << 16 | i (d <= 0xfffe, i.e.
// max_trials < 65535); atomic min keeps the newest draw's smallest i; the
// cleared value 0xffffffff matches no tag.
__device__ __forceinline__ uint32_t nxt_tag(uint32_t d) { return (0xfffeu - d) << 16; }

// Resolve draws [d0, d0+nb) (nb <= 32): lane 2k / 2k+1 chase the value at
// position 0 / 1 before step 1 of draw d0+k, then step 1 swaps iff j_1 == 0.
__device__ __forceinline__ void mt_resolve(const MTWave &mt, uint32_t N, uint32_t smask, uint32_t d0, uint32_t nb,
                                           int32_t *draws, int lane) {
    const uint32_t k = (uint32_t)lane >> 1;
    const uint32_t q = (uint32_t)lane & 1u;
    uint32_t p = q;
    const uint32_t d = d0 + k;
    const uint32_t slot = d & smask;
    const uint32_t tag = nxt_tag(d);
    if (k < nb) {
        const uint32_t *nx = mt.nxt + slot * N;
        for (;;) {
            const uint32_t t = nx[p];
            if ((t & 0xffff0000u) != tag) break;
            p = t & 0xffffu;
        }
    }
    const uint32_t other = (uint32_t)__shfl_xor((int)p, 1);
    if (k < nb && q == 0) {
        const uint32_t j1 = mt.j1s[slot];
        const uint32_t a0 = (j1 == 0u) ? other : p;
        const uint32_t a1 = (j1 == 0u) ? p : other;
        draws[2 * d] = (int32_t)a0;
        draws[2 * d + 1] = (int32_t)a1;
    }
    wave_lds_sync();
}

// Generate D draws of choice(N, 2, replace=False) from the stream.
// store: write draws[2d], draws[2d+1] (LDS).  Otherwise only advance the stream.
// FAST: K = N-1 >= 64, so one window never spans more than one draw boundary.
template <bool FAST>
__device__ void mt_draws_impl(MTWave &mt, uint32_t N, uint32_t D, int32_t *draws, bool store, int lane) {
    const uint32_t K = N - 1;  // Fisher-Yates steps per draw (N >= 3)
    const uint32_t G = D * K;
    const float invK = 1.0f / (float)K;
    const uint32_t smask = (uint32_t)mt_nslot((int)N) - 1u;
    const uint32_t RB = (uint32_t)mt_resolve_batch((int)N);
    uint32_t g = 0;            // steps done
    uint32_t dg = 0, sg = 0;   // g = dg*K + sg
    uint32_t dres = 0;         // draws resolved
    if (store) {
        for (uint32_t e = (uint32_t)lane; e < (smask + 1u) * N; e += 64) mt.nxt[e] = MT_NONE;
        wave_lds_sync();
    }
    // initial guess of the accepts below each lane: ~0.72 per word (mean
    // acceptance of random_interval's masked rejection)
    const uint32_t guess = ((uint32_t)lane * 46u) >> 6;
    // raw (untempered) word of the next window, prefetched a window ahead
    int pre_pos = -1;
    uint32_t pre_raw = 0;
    LSLAM_STAMP_DECL
    while (g < G) {
        if (mt.pos >= MT_N) {
            mt_twist(mt.key, lane);
            mt.pos = 0;
            pre_pos = -1;
        }
        LSLAM_STAMP(0);
        const int nw = min(64, MT_N - mt.pos);
        const bool act = lane < nw;
        uint32_t raw;
        if (pre_pos == mt.pos) raw = pre_raw;
        else raw = act ? mt.key[mt.pos + lane] : 0u;
        {   // prefetch the next window (consumed after the fixed point below)
            const int np = mt.pos + nw;
            pre_pos = np < MT_N ? np : -1;
            if (pre_pos >= 0) pre_raw = (np + lane < MT_N) ? mt.key[np + lane] : 0u;
        }
        const uint32_t w = act ? mt_temper(raw) : 0u;
        const uint32_t rem = G - g;
        const uint64_t actm = ballot(act);
        LSLAM_STAMP(1);
        uint32_t c = guess;
        uint64_t B = 0;
        // fixed point: B = {lanes accepted given c = popcount(B below lane)}
        for (int it = 0;; it++) {
            const uint32_t rr = sg + c;
            uint32_t r;
            if (FAST) {
                r = min(rr, rr - K);  // rr < 2K: unsigned wrap picks rr or rr-K
            } else {
                uint32_t qq;
                divmod_small(rr, K, invK, qq, r);
            }
            const uint32_t i = K - r;
            const uint32_t jv = w & (0xffffffffu >> __clz((int)i));
            const uint64_t Bn = actm & ballot(c < rem) & ballot(jv <= i);
            if (it > 0 && Bn == B) break;
            B = Bn;
            c = mbcnt(B);
        }
        const bool acc = (B >> lane) & 1ull;
        LSLAM_STAMP(2);
        const uint32_t na = (uint32_t)popc64(B);
        if (store && acc) {
            // draw index and step of this accepted word; scatter into the draw's next-writer table
            const uint32_t rr = sg + c;
            uint32_t dq, rs;
            if (FAST) {
                dq = rr >= K ? 1u : 0u;
                rs = rr - (dq ? K : 0u);
            } else {
                divmod_small(rr, K, invK, dq, rs);
            }
            const uint32_t d = dg + dq;
            const uint32_t slot = d & smask;
            const uint32_t i = K - rs;
            const uint32_t jv = w & (0xffffffffu >> __clz((int)i));
            if (i == 1u) mt.j1s[slot] = jv;
            else if (i > jv && i > 1u) atomicMin(mt.nxt + slot * N + jv, nxt_tag(d) | i);
        }
        if (na >= rem && na > 0) {
            mt.pos += fls64(B) + 1;
            pre_pos = -1;
        } else {
            mt.pos += nw;
        }
        g += na;
        if (FAST) {
            sg += na;
            if (sg >= K) { sg -= K; dg += 1; }
        } else {
            uint32_t q, rs;
            divmod_small(sg + na, K, invK, q, rs);
            dg += q;
            sg = rs;
        }
        LSLAM_STAMP(3);
        if (store && dg > dres) {
            const bool last = g >= G;
            while (dres < dg && (dg - dres >= RB || last)) {
                wave_lds_sync();
                const uint32_t nb = min(32u, dg - dres);
                mt_resolve(mt, N, smask, dres, nb, draws, lane);
                dres += nb;
            }
        }
        LSLAM_STAMP(4);
    }
    wave_lds_sync();
}

__device__ __forceinline__ void mt_draws(MTWave &mt, uint32_t N, uint32_t D, int32_t *draws, bool store, int lane) {
    if (N >= 65) mt_draws_impl<true>(mt, N, D, draws, store, lane);
    else mt_draws_impl<false>(mt, N, D, draws, store, lane);
}

// ---- Philox4x32-10 (throughput mode) ----
__device__ __forceinline__ void philox4x32_10(uint32_t ctr[4], uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; r++) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * ctr[0];
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * ctr[2];
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        const uint32_t n0 = hi1 ^ ctr[1] ^ k0;
        const uint32_t n2 = hi0 ^ ctr[3] ^ k1;
        ctr[0] = n0; ctr[1] = lo1; ctr[2] = n2; ctr[3] = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
}

// draw d of chunk `chunk_id`: a uniformly distributed distinct pair in [0, N)
__device__ __forceinline__ void philox_pair(uint32_t N, uint32_t d, uint32_t chunk_id, uint64_t seed, int32_t &a,
                                            int32_t &b) {
    uint32_t c[4] = {d, chunk_id, 0x4c534c4du, 0u};
    philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    const uint32_t x = (uint32_t)(((uint64_t)c[0] * N) >> 32);
    uint32_t y = (uint32_t)(((uint64_t)c[1] * (N - 1)) >> 32);
    if (y >= x) y += 1;
    a = (int32_t)x;
    b = (int32_t)y;
}

// D such pairs for chunk `chunk_id` into draws[2D]
__device__ __forceinline__ void philox_draws(uint32_t N, uint32_t D, uint32_t chunk_id, uint64_t seed,
                                             int32_t *draws, int lane) {
    for (uint32_t d0 = 0; d0 < D; d0 += 64) {
        const uint32_t d = d0 + (uint32_t)lane;
        if (d < D) philox_pair(N, d, chunk_id, seed, draws[2 * d], draws[2 * d + 1]);
    }
    __syncthreads();
}

}  // namespace lslam
