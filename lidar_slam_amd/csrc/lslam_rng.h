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
//   * accepted values j_i are kept in an LDS ring; when a draw's K steps are
//     complete its two output positions are resolved by chasing
//     "value at position q before step 1": V(q) = V(min{i > max(q,1) : j_i = q})
//     or q itself, searched 64 entries per ballot; then step 1 swaps x[0], x[1]
//     iff j_1 == 0.
#pragma once
#include "lslam_wave.h"

namespace lslam {

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

__device__ __forceinline__ uint32_t mt_mix(uint32_t cur, uint32_t nxt, uint32_t far) {
    uint32_t y = (cur & MT_UP) | (nxt & MT_LO);
    return far ^ (y >> 1) ^ ((y & 1u) ? MT_MA : 0u);
}

// mt19937_gen on key[624] in LDS by one wave
__device__ __forceinline__ void mt_twist(uint32_t *key, int lane) {
    uint32_t v[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        int i = lane + 64 * k;
        if (i < MT_N - MT_M) v[k] = mt_mix(key[i], key[i + 1], key[i + MT_M]);
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; k++) {
        int i = lane + 64 * k;
        if (i < MT_N - MT_M) key[i] = v[k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; k++) {
        int i = (MT_N - MT_M) + lane + 64 * k;
        if (i < 2 * (MT_N - MT_M)) v[k] = mt_mix(key[i], key[i + 1], key[i - (MT_N - MT_M)]);
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; k++) {
        int i = (MT_N - MT_M) + lane + 64 * k;
        if (i < 2 * (MT_N - MT_M)) key[i] = v[k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 3; k++) {
        int i = 2 * (MT_N - MT_M) + lane + 64 * k;
        if (i < MT_N) {
            uint32_t nxt = (i == MT_N - 1) ? key[0] : key[i + 1];
            v[k] = mt_mix(key[i], nxt, key[i - (MT_N - MT_M)]);
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 3; k++) {
        int i = 2 * (MT_N - MT_M) + lane + 64 * k;
        if (i < MT_N) key[i] = v[k];
    }
    __syncthreads();
}

// numpy mt19937_seed (init_genrand): sequential recurrence, lane 0
__device__ __forceinline__ void mt_seed(uint32_t *key, uint32_t seed, int lane) {
    if (lane == 0) {
        for (int i = 0; i < MT_N; i++) {
            key[i] = seed;
            seed = 1812433253u * (seed ^ (seed >> 30)) + (uint32_t)(i + 1);
        }
    }
    __syncthreads();
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
    uint16_t *ring;  // LDS J ring (draw resolution)
    uint32_t ring_mask;
    int pos;         // wave-uniform 0..624
};

// Resolve value at position q (0 or 1) just before step 1 for a draw whose
// step s (i = K - s) entry lives at ring[(base + s) & mask].
__device__ __forceinline__ uint32_t mt_chase(const MTWave &mt, uint32_t base, uint32_t K, uint32_t q, int lane) {
    uint32_t cur = q;
    uint32_t lo = 1;
    for (;;) {
        uint32_t start = (cur > lo ? cur : lo) + 1;
        bool found = false;
        for (uint32_t i0 = start; i0 <= K; i0 += 64) {
            uint32_t i = i0 + (uint32_t)lane;
            bool hit = false;
            if (i <= K) hit = (uint32_t)mt.ring[(base + K - i) & mt.ring_mask] == cur;
            uint64_t b = ballot(hit);
            if (b) {
                cur = i0 + (uint32_t)ffs64(b);
                found = true;
                break;
            }
        }
        if (!found) break;
        lo = cur;
    }
    return cur;
}

// Generate D draws of choice(N, 2, replace=False) from the stream.
// store: write draws[2d], draws[2d+1] to LDS `draws`.  Otherwise only advance.
__device__ void mt_draws(MTWave &mt, uint32_t N, uint32_t D, int32_t *draws, bool store, int lane) {
    const uint32_t K = N - 1;  // Fisher-Yates steps per draw (N >= 3)
    const uint32_t G = D * K;
    const float invK = 1.0f / (float)K;
    uint32_t g = 0;            // steps done
    uint32_t dg = 0, sg = 0;   // g = dg*K + sg
    uint32_t dres = 0;         // draws resolved
    while (g < G) {
        if (mt.pos >= MT_N) {
            mt_twist(mt.key, lane);
            mt.pos = 0;
        }
        const int nw = min(64, MT_N - mt.pos);
        const bool act = lane < nw;
        const uint32_t w = act ? mt_temper(mt.key[mt.pos + lane]) : 0u;
        uint64_t B = ballot(act);
        uint32_t jv = 0, s_l = 0;
        bool acc = false;
        for (;;) {
            const uint32_t c = mbcnt(B);
            const uint32_t gl = g + c;
            uint32_t q, r;
            divmod_small(sg + c, K, invK, q, r);
            s_l = r;
            const uint32_t i = K - r;
            const uint32_t m = 0xffffffffu >> __clz((int)i);
            jv = w & m;
            acc = act && (gl < G) && (jv <= i);
            const uint64_t Bn = ballot(acc);
            if (Bn == B) break;
            B = Bn;
        }
        const uint32_t na = (uint32_t)popc64(B);
        if (store && acc) {
            const uint32_t gl = g + mbcnt(B);
            mt.ring[gl & mt.ring_mask] = (uint16_t)jv;
        }
        (void)s_l;
        if (g + na >= G && na > 0) mt.pos += fls64(B) + 1;
        else mt.pos += nw;
        g += na;
        {
            uint32_t q, r;
            divmod_small(sg + na, K, invK, q, r);
            dg += q;
            sg = r;
        }
        if (store && dg > dres) {
            __syncthreads();
            for (uint32_t d = dres; d < dg; d++) {
                const uint32_t base = d * K;
                uint32_t a0 = mt_chase(mt, base, K, 0u, lane);
                uint32_t a1 = mt_chase(mt, base, K, 1u, lane);
                const uint32_t j1 = mt.ring[(base + K - 1) & mt.ring_mask];
                if (j1 == 0u) { uint32_t t = a0; a0 = a1; a1 = t; }
                if (lane == 0) {
                    draws[2 * d] = (int32_t)a0;
                    draws[2 * d + 1] = (int32_t)a1;
                }
            }
            dres = dg;
            __syncthreads();
        }
    }
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

// D uniformly distributed distinct pairs in [0, N) for chunk `chunk_id`
__device__ __forceinline__ void philox_draws(uint32_t N, uint32_t D, uint32_t chunk_id, uint64_t seed,
                                             int32_t *draws, int lane) {
    for (uint32_t d0 = 0; d0 < D; d0 += 64) {
        const uint32_t d = d0 + (uint32_t)lane;
        if (d < D) {
            uint32_t c[4] = {d, chunk_id, 0x4c534c4du, 0u};
            philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
            uint32_t a = (uint32_t)(((uint64_t)c[0] * N) >> 32);
            uint32_t b = (uint32_t)(((uint64_t)c[1] * (N - 1)) >> 32);
            if (b >= a) b += 1;
            draws[2 * d] = (int32_t)a;
            draws[2 * d + 1] = (int32_t)b;
        }
    }
    __syncthreads();
}

}  // namespace lslam
