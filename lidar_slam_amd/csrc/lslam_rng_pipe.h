// lslam_rng_pipe.h — the MT19937 hypothesis stream of a whole scan as a
// two-wave producer (parity mode).
//
// The parse of numpy's legacy stream is a sequential automaton, so a scan's
// draws are bounded by the latency of ONE dependency chain (a 4096-scan batch
// gives only 4 such chains per SIMD).  Everything that is not on that chain is
// moved to a helper wave of the same workgroup:
//   wave 0 (parser):  words -> fixed point on the accept ballot (lslam_rng.h)
//                     -> accepted j values into an LDS ring `jr`, indexed by
//                     the scan-global Fisher-Yates step counter.
//   wave 1 (helper):  (a) twists block b+1 of the MT state out of place while
//                     the parser reads block b (two 624-word slots);
//                     (b) resolves completed draws from `jr`, one lane per
//                     draw: forward scan over i = 2..K keeping the values that
//                     started at positions 0 and 1 (p <- i whenever j_i == p),
//                     then step 1 swaps them iff j_1 == 0;  (c) stores them.
// Hand-off through LDS flags.  A wave's LDS instructions are performed in
// program order, so a flag store issued after data stores publishes them, and
// a flag store issued after data loads releases their slots.
// The producer assumes no early stop (a trial with sum of squared residuals
// exactly 0); the consensus kernel flags one and the fix-up pass replays it.
#pragma once
#include "lslam_rng.h"

namespace lslam {

enum { F_BLK = 0, F_BLKUSE = 1, F_GPAR = 2, F_DRES = 3, F_NFLAGS = 8 };

// flags are LDS words: keep the address space explicit, or a volatile access
// through a generic pointer becomes a system-coherent FLAT load/store
typedef __attribute__((address_space(3))) volatile int lds_flag_t;

__device__ __forceinline__ int lds_flag_get(lds_flag_t *f) { return __builtin_amdgcn_readfirstlane(*f); }
__device__ __forceinline__ void lds_flag_put(lds_flag_t *f, int v, int lane) {
    asm volatile("" ::: "memory");
    if (lane == 0) *f = v;
    asm volatile("" ::: "memory");
}

// tempering is a bijection; the final state of the parse is written back raw
__device__ __forceinline__ uint32_t mt_untemper(uint32_t y) {
    y ^= y >> 18;
    y ^= (y << 15) & 0xefc60000u;
    uint32_t x = y;
#pragma unroll
    for (int k = 0; k < 4; k++) x = y ^ ((x << 7) & 0x9d2c5680u);
    y = x;
#pragma unroll
    for (int k = 0; k < 2; k++) x = y ^ (x >> 11);
    return x;
}

// The helper sleeps (s_sleep 127) until the parser has work for it and
// wakes it with s_wakeup: a polling helper costs the SIMD as many VALU issue
// slots as the parser's own chain.  A wakeup that arrives while the helper is
// still awake is lost; its sleep then simply runs out.
__device__ __forceinline__ void wake_helper() { asm volatile("s_wakeup" ::: "memory"); }

struct RngPipe {
    uint32_t *raw;     // LDS [624] raw MT state of the newest block (helper only)
    uint32_t *tw;      // LDS [2][624] tempered words, block b in slot b & 1
    uint16_t *jr;      // LDS [rjmask+1] accepted j by scan-global step (+64 dummy slots)
    uint32_t *nxt;     // LDS [max N] helper's next-writer table
    lds_flag_t *fl;    // LDS [F_NFLAGS]
    uint32_t rjmask;
    uint32_t ndrawn;       // parser: draws completed over the scan (wakeup cadence)
#ifdef LSLAM_STAMPS
    uint64_t acc[8];
#endif
};

// Diagnostic build only: parser cycle accounting (0 block waits, 1 ring waits,
// 2 fixed point, 3 rest of the window, 5 windows, 6 fixed-point iterations)
#ifdef LSLAM_STAMPS
#define RP_STAMP_DECL uint64_t _rp_prev = lslam_stamp();
#define RP_STAMP(k)                         \
    do {                                    \
        const uint64_t _t = lslam_stamp();  \
        rp.acc[k] += _t - _rp_prev;         \
        _rp_prev = _t;                      \
    } while (0)
#define RP_COUNT(k, n) (rp.acc[k] += (n))
#else
#define RP_STAMP_DECL
#define RP_STAMP(k) do {} while (0)
#define RP_COUNT(k, n) do {} while (0)
#endif

__device__ __forceinline__ uint32_t mbcnt_from(uint64_t m, uint32_t base) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, base));
}

// ---------------- parser wave: one chunk's D*K steps ----------------
// Full windows (64 words, chunk not ending in the window, K >= 64) are the
// common case.  They iterate on the REJECT ballot R: a lane's distance to the
// next draw boundary is d = (K-1 - sg - lane) + #rejected below the lane,
// which v_mbcnt produces directly from R, and its Fisher-Yates index is
// i = min(d, d+K) + 1 (unsigned; the window wraps past at most one boundary).
// The iteration is unrolled twice so the ballots alternate registers.
__device__ __forceinline__ uint32_t fy_index(uint32_t d, uint32_t K) { return min(d, d + K) + 1u; }
__device__ __forceinline__ uint32_t fy_j(uint32_t w, uint32_t i) { return w & (0xffffffffu >> __clz((int)i)); }

template <bool FAST>
__device__ __forceinline__ void parse_chunk(RngPipe &rp, int &blkno, int &pos, uint32_t &gs, int &dres_seen,
                                            uint32_t N, uint32_t D, int lane) {
    const uint32_t K = N - 1;
    const uint32_t G = D * K;
    const float invK = 1.0f / (float)K;
    const uint32_t guess = ((uint32_t)lane * 46u) >> 6;  // ~0.72 accepts per word
    const int rsz = (int)rp.rjmask + 1;
    uint16_t *const jdummy = rp.jr + rsz + lane;  // rejected lanes store here
    uint32_t g = 0, sg = 0;
    int pre_pos = -1;
    uint32_t pre_w = 0;
    RP_STAMP_DECL
    while (g < G) {
        RP_STAMP(3);
        if (pos >= MT_N) {
            blkno += 1;
            while (lds_flag_get(rp.fl + F_BLK) < blkno) __builtin_amdgcn_s_sleep(1);
            asm volatile("" ::: "memory");
            pos = 0;
            pre_pos = -1;
            lds_flag_put(rp.fl + F_BLKUSE, blkno, lane);
            wake_helper();
            RP_STAMP(0);
        }
        const uint32_t *tb = rp.tw + (blkno & 1) * MT_N;
        const uint32_t rem = G - g;
        const uint32_t w = (pre_pos == pos) ? pre_w : tb[min(pos + lane, MT_N - 1)];
        // next window's words (clamped inside the block; used only if the next window starts there)
        pre_pos = pos + 64;
        pre_w = tb[min(pos + 64 + lane, MT_N - 1)];
        // room in the ring for this window's (at most 64) steps
        if ((int)(gs + g + 64u) - dres_seen > rsz) {
            wake_helper();
            for (;;) {
                dres_seen = lds_flag_get(rp.fl + F_DRES);
                if ((int)(gs + g + 64u) - dres_seen <= rsz) break;
                __builtin_amdgcn_s_sleep(1);
            }
            asm volatile("" ::: "memory");
            RP_STAMP(1);
        }
        RP_STAMP(3);
        if (FAST && pos + 64 <= MT_N && rem > 64u) {
            const uint32_t b1 = K - 1u - sg;
            const uint32_t base0 = b1 - (uint32_t)lane;
            uint32_t d = b1 - guess;
            uint32_t i = fy_index(d, K);
            uint32_t jv = fy_j(w, i);
            uint64_t R0 = ballot(jv > i), R1;
            int it = 1;
            (void)it;
            for (;;) {
                d = mbcnt_from(R0, base0);
                i = fy_index(d, K);
                jv = fy_j(w, i);
                R1 = ballot(jv > i);
                if (R1 == R0) break;
                d = mbcnt_from(R1, base0);
                i = fy_index(d, K);
                jv = fy_j(w, i);
                R0 = ballot(jv > i);
                it += 2;
                if (R0 == R1) break;
            }
            RP_STAMP(2);
            RP_COUNT(5, 1);
            RP_COUNT(6, it + 1);
            // R0 == R1 == the fixed point; d, i, jv belong to it
            const bool acc = jv <= i;
            const uint32_t c = b1 - d;
            uint16_t *dst = acc ? rp.jr + ((gs + g + c) & rp.rjmask) : jdummy;
            *dst = (uint16_t)jv;
            const uint32_t na = 64u - (uint32_t)popc64(R0);
            pos += 64;
            g += na;
            sg += na;
            if (sg >= K) {
                sg -= K;
                lds_flag_put(rp.fl + F_GPAR, (int)(gs + g), lane);  // the helper only needs completed draws
                if ((++rp.ndrawn & 3u) == 0u) wake_helper();
            }
            continue;
        }
        // ---- partial window: block end, chunk end, or K < 64
        const int nw = min(64, MT_N - pos);
        const uint64_t actm = ballot(lane < nw);
        uint32_t c = guess, jv = 0;
        uint64_t B = 0;
        for (int it = 0;; it++) {
            const uint32_t rr = sg + c;
            uint32_t r;
            if (FAST) {
                r = min(rr, rr - K);
            } else {
                uint32_t qq;
                divmod_small(rr, K, invK, qq, r);
            }
            const uint32_t i = K - r;
            jv = fy_j(w, i);
            const uint64_t Bn = actm & ballot(c < rem) & ballot(jv <= i);
            if (it > 0 && Bn == B) break;
            B = Bn;
            c = mbcnt(B);
        }
        RP_STAMP(2);
        RP_COUNT(5, 1);
        const uint32_t na = (uint32_t)popc64(B);
        if ((B >> lane) & 1ull) rp.jr[(gs + g + c) & rp.rjmask] = (uint16_t)jv;
        if (na >= rem && na > 0) {
            pos += fls64(B) + 1;
            pre_pos = -1;
        } else {
            pos += nw;
        }
        g += na;
        uint32_t q, rs;
        if (FAST) {
            rs = sg + na;
            q = rs >= K ? 1u : 0u;
            if (q) rs -= K;
        } else {
            divmod_small(sg + na, K, invK, q, rs);
        }
        sg = rs;
        if (q > 0) {
            lds_flag_put(rp.fl + F_GPAR, (int)(gs + g), lane);
            rp.ndrawn += q;
            wake_helper();
        }
    }
    gs += G;
}

// ---------------- helper wave: resolution of one completed draw ----------------
// Steps s = 0..K-1 of the draw sit at ring index s0 + s (Fisher-Yates
// i = K - s, j_i <= i).  Lanes scatter the steps into the next-writer table
// nxt[p] = min{i > max(p,1) : j_i == p} (LDS atomic min; entries carry the
// draw's tag (nxt_tag, lslam_rng.h) in the high half, so the table is cleared
// once per chunk), then
// lanes 0/1 chase the values that start at positions 0/1 (p -> nxt[p] -> ...;
// the chain is ~ln K long), and step 1 swaps them iff j_1 == 0.
__device__ __forceinline__ void resolve_draw(const RngPipe &rp, uint32_t s0, uint32_t K, uint32_t d, int32_t *out,
                                             int lane) {
    const uint32_t tag = nxt_tag(d);
    for (uint32_t sb = 0; sb < K; sb += 64) {
        const uint32_t st = sb + (uint32_t)lane;
        if (st < K) {
            const uint32_t i = K - st;
            const uint32_t j = rp.jr[(s0 + st) & rp.rjmask];
            if (i > 1u && j < i) atomicMin(rp.nxt + j, tag | i);
        }
    }
    wave_lds_sync();
    const uint32_t j1 = rp.jr[(s0 + K - 1u) & rp.rjmask];
    uint32_t p = (uint32_t)lane & 1u;
    if (lane < 2) {
        for (;;) {
            const uint32_t t = rp.nxt[p];
            if ((t & 0xffff0000u) != tag) break;
            p = t & 0xffffu;
        }
    }
    const uint32_t p0 = (uint32_t)__builtin_amdgcn_readlane((int)p, 0);
    const uint32_t p1 = (uint32_t)__builtin_amdgcn_readlane((int)p, 1);
    if (lane == 0) {
        out[2 * d] = (int32_t)((j1 == 0u) ? p1 : p0);
        out[2 * d + 1] = (int32_t)((j1 == 0u) ? p0 : p1);
    }
}

}  // namespace lslam
