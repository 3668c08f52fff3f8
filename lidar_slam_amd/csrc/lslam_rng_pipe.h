// lslam_rng_pipe.h — the MT19937 hypothesis stream of a whole scan as a
// two-wave producer (parity mode).
//
// The parse of numpy's legacy stream is a sequential automaton, so a scan's
// draws are bounded by ONE dependency chain, and a 4096-scan batch gives only
// 4 such chains per SIMD.  What is not on the chain runs in a helper wave of
// the same workgroup:
//   wave 0 (parser):  tempers the words of a 64-word window, solves the accept
//                     ballot by fixed-point iteration, and stores each accepted
//                     j into an LDS ring `jr` indexed by the scan-global
//                     Fisher-Yates step counter.
//   wave 1 (helper):  (a) twists block b+1 of the MT state out of place while
//                     the parser reads block b (two 624-word slots of raw
//                     state); (b) resolves completed draws, up to RES_NB at a
//                     time: lanes scatter the steps into per-draw next-writer
//                     tables, then two lanes per draw chase positions 0 and 1;
//                     (c) stores the draws to HBM.
// The helper sleeps until the parser wakes it (s_wakeup): a polling helper
// would cost the SIMD as many VALU issue slots as the parser's own chain.
// Hand-off through LDS flags.  A wave's LDS instructions are performed in
// program order, so a flag store issued after data stores publishes them, and
// a flag store issued after data loads releases their slots.
// The producer assumes no early stop (a trial with sum of squared residuals
// exactly 0); the consensus kernel flags one and the fix-up pass replays it.
#pragma once
#include "../../include/lidarslam.h"
#include "lslam_rng.h"

namespace lslam {

enum { F_BLK = 0, F_BLKUSE = 1, F_GPAR = 2, F_DRES = 3, F_NFLAGS = 8 };
constexpr int RES_NB = 4;  // draws resolved per helper batch (next-writer tables)

// flags are LDS words: keep the address space explicit, or a volatile access
// through a generic pointer becomes a system-coherent FLAT load/store
typedef __attribute__((address_space(3))) volatile int lds_flag_t;

__device__ __forceinline__ int lds_flag_get(lds_flag_t *f) { return __builtin_amdgcn_readfirstlane(*f); }
// v is wave-uniform: every lane stores the same word (no exec-mask juggling)
__device__ __forceinline__ void lds_flag_put(lds_flag_t *f, int v, int lane) {
    (void)lane;
    asm volatile("" ::: "memory");
    *f = v;
    asm volatile("" ::: "memory");
}

// A wakeup that arrives while the helper is still awake is lost; its sleep
// then simply runs out (s_sleep 127 ~ 8k cycles).
__device__ __forceinline__ void wake_helper() { asm volatile("s_wakeup" ::: "memory"); }

// Waves of a SIMD issue by priority, then age.  With equal priorities the
// oldest parser of a SIMD races ahead and the youngest finishes last (~1.6x
// the oldest's time at 4 parsers per SIMD).  Parsers lower their priority as
// they progress (2 in the first third of the scan's steps ... 0 in the last)
// so the SIMD's parsers advance together; the helper sits above them.
__device__ __forceinline__ void set_prio_level(int lvl) {
    switch (lvl) {
        case 3: __builtin_amdgcn_s_setprio(3); break;
        case 2: __builtin_amdgcn_s_setprio(2); break;
        case 1: __builtin_amdgcn_s_setprio(1); break;
        default: __builtin_amdgcn_s_setprio(0); break;
    }
}

// out-of-place mt19937_gen: dst = twist(src) by one wave, three dependency phases
__device__ __forceinline__ void mt_twist_oop(const uint32_t *src, uint32_t *dst, int lane) {
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int i = lane + 64 * k;
        if (i < MT_N - MT_M) dst[i] = mt_mix(src[i], src[i + 1], src[i + MT_M]);
    }
    wave_lds_sync();
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int i = (MT_N - MT_M) + lane + 64 * k;
        if (i < 2 * (MT_N - MT_M)) dst[i] = mt_mix(src[i], src[i + 1], dst[i - (MT_N - MT_M)]);
    }
    wave_lds_sync();
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const int i = 2 * (MT_N - MT_M) + lane + 64 * k;
        if (i < MT_N) {
            const uint32_t nx = (i == MT_N - 1) ? dst[0] : src[i + 1];
            dst[i] = mt_mix(src[i], nx, dst[i - (MT_N - MT_M)]);
        }
    }
    wave_lds_sync();
}

// JT: uint8_t when every chunk has <= 256 points (j < N), else uint16_t
template <typename JT>
struct RngPipe {
    uint32_t *blk;     // LDS [2][624] raw MT state, block b in slot b & 1
    JT *jr;            // LDS [rjmask+1] accepted j by scan-global step, then 64 dummy slots
    uint32_t *nxt;     // LDS [RES_NB][nstride] helper's next-writer tables
    lds_flag_t *fl;    // LDS [F_NFLAGS]
    uint32_t rjmask;
    uint32_t nstride;
    uint32_t ndrawn;       // parser: draws completed over the scan (wakeup cadence)
    uint32_t total_steps;  // parser: steps of the whole scan (priority schedule)
    int prio;              // parser: current priority level
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
__device__ __forceinline__ uint32_t fy_index(uint32_t d, uint32_t K) { return min(d, d + K) + 1u; }
__device__ __forceinline__ uint32_t fy_j(uint32_t w, uint32_t i) { return w & (0xffffffffu >> __clz((int)i)); }

template <bool FAST, typename JT>
__device__ __forceinline__ void parse_chunk(RngPipe<JT> &rp, int &blkno, int &pos, uint32_t &gs, int &dres_seen,
                                            uint32_t N, uint32_t D, int lane) {
    const uint32_t K = N - 1;
    const uint32_t G = D * K;
    const float invK = 1.0f / (float)K;
    const uint32_t guess = ((uint32_t)lane * 46u) >> 6;  // ~0.72 accepts per word
    const int rsz = (int)rp.rjmask + 1;
    JT *const jdummy = rp.jr + rsz + lane;  // rejected lanes store here
    uint32_t g = 0, sg = 0;
    int pre_pos = -1;
    uint32_t pre_raw = 0;
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
            const int lvl = 2 - (int)(((uint64_t)(gs + g) * 3u) / (rp.total_steps + 1u));
            if (lvl != rp.prio) {
                rp.prio = lvl;
                set_prio_level(lvl);
            }
            RP_STAMP(0);
        }
        const uint32_t *kb = rp.blk + (blkno & 1) * MT_N;
        const uint32_t rem = G - g;
        const uint32_t raw = (pre_pos == pos) ? pre_raw : kb[min(pos + lane, MT_N - 1)];
        // next window's words (clamped inside the block; used only if the next window starts there)
        pre_pos = pos + 64;
        pre_raw = kb[min(pos + 64 + lane, MT_N - 1)];
        const uint32_t w = mt_temper(raw);
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
            uint64_t R = ballot(jv > i), Rp;
            int it = 1;
            do {
                Rp = R;
                d = mbcnt_from(Rp, base0);
                i = fy_index(d, K);
                jv = fy_j(w, i);
                R = ballot(jv > i);
                it++;
            } while (R != Rp);
            (void)it;
            RP_STAMP(2);
            RP_COUNT(5, 1);
            RP_COUNT(6, it);
            // R is the fixed point; d, i, jv belong to it.  The lane's reject
            // bit is read back from R: a boolean carried out of the loop would
            // be merged with exec on every iteration.
            const uint32_t rej = (uint32_t)(R >> lane) & 1u;
            const uint32_t c = b1 - d;
            JT *dst = rej ? jdummy : rp.jr + ((gs + g + c) & rp.rjmask);
            *dst = (JT)jv;
            const uint32_t na = 64u - (uint32_t)popc64(R);
            pos += 64;
            g += na;
            sg += na;
            if (sg >= K) {
                sg -= K;
                lds_flag_put(rp.fl + F_GPAR, (int)(gs + g), lane);  // the helper only needs completed draws
                rp.ndrawn = uniu(rp.ndrawn + 1u);
                if ((rp.ndrawn & 3u) == 0u) wake_helper();
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
        if ((B >> lane) & 1ull) rp.jr[(gs + g + c) & rp.rjmask] = (JT)jv;
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

// ---------------- helper wave: resolution of up to RES_NB completed draws ----------------
// Step s of draw d0+q sits at ring index s0 + q*K + s (Fisher-Yates i = K - s,
// j_i <= i).  Lanes scatter the steps into the draw's next-writer table
// nxt[p] = min{i > max(p,1) : j_i == p} (LDS atomic min; entries carry the
// draw's tag nxt_tag(d) in the high half, so tables are cleared once per
// chunk).  Lanes 2q / 2q+1 then chase the values that start at positions 0 / 1
// (p -> nxt[p] -> ..., ~ln K hops) and step 1 swaps them iff j_1 == 0.
template <typename JT>
__device__ __forceinline__ void resolve_batch(const RngPipe<JT> &rp, uint32_t s0, uint32_t K, uint32_t d0,
                                              uint32_t nb, int32_t *out, int lane) {
    wave_lds_sync();
    const uint32_t total = nb * K;
    for (uint32_t t0 = 0; t0 < total; t0 += 64) {
        const uint32_t t = t0 + (uint32_t)lane;
        if (t < total) {
            const uint32_t dq = (uint32_t)(t >= K) + (uint32_t)(t >= 2u * K) + (uint32_t)(t >= 3u * K);
            const uint32_t i = K - (t - dq * K);
            const uint32_t j = rp.jr[(s0 + t) & rp.rjmask];
            const uint32_t d = d0 + dq;
            if (i > 1u && j < i) atomicMin(rp.nxt + (d & (RES_NB - 1)) * rp.nstride + j, nxt_tag(d) | i);
        }
    }
    wave_lds_sync();
    const uint32_t q = (uint32_t)lane >> 1;
    uint32_t p = (uint32_t)lane & 1u;
    if (q < nb) {
        const uint32_t d = d0 + q;
        const uint32_t tag = nxt_tag(d);
        const uint32_t *tab = rp.nxt + (d & (RES_NB - 1)) * rp.nstride;
        for (;;) {
            const uint32_t t = tab[p];
            if ((t & 0xffff0000u) != tag) break;
            p = t & 0xffffu;
        }
    }
    const uint32_t other = (uint32_t)__shfl_xor((int)p, 1);
    if (q < nb && (lane & 1) == 0) {
        const uint32_t d = d0 + q;
        const uint32_t j1 = rp.jr[(s0 + q * K + K - 1u) & rp.rjmask];
        out[2 * d] = (int32_t)((j1 == 0u) ? other : p);
        out[2 * d + 1] = (int32_t)((j1 == 0u) ? p : other);
    }
}

template <typename JT>
__device__ void rng_helper(RngPipe<JT> &rp, const lslam_scan_batch &B, int c0, int c1, uint32_t D, int32_t *dst,
                           int lane) {
    auto chunk_n = [&](int c) { return B.chunk_pt_off[c + 1] - B.chunk_pt_off[c]; };
    auto clear_tables = [&]() {
        for (uint32_t e = (uint32_t)lane; e < RES_NB * rp.nstride; e += 64) rp.nxt[e] = MT_NONE;
        wave_lds_sync();
    };
    int produced = 0;
    int cc = c0;
    while (cc < c1 && chunk_n(cc) < 3) cc++;
    uint32_t K = 2u;
    if (cc < c1) {
        K = (uint32_t)chunk_n(cc) - 1u;
        clear_tables();
    }
    uint32_t base = 0, dnext = 0;
    while (cc < c1) {
        if (lds_flag_get(rp.fl + F_BLKUSE) == produced) {
            mt_twist_oop(rp.blk + (produced & 1) * MT_N, rp.blk + ((produced + 1) & 1) * MT_N, lane);
            produced += 1;
            lds_flag_put(rp.fl + F_BLK, produced, lane);
            continue;
        }
        const uint32_t gpar = (uint32_t)lds_flag_get(rp.fl + F_GPAR);
        if (gpar < base + (dnext + 1u) * K) {
            __builtin_amdgcn_s_sleep(127);  // until the parser's s_wakeup
            continue;
        }
        uint32_t nb = 1;
        while (nb < (uint32_t)RES_NB && dnext + nb < D && base + (dnext + nb + 1u) * K <= gpar) nb++;
        resolve_batch(rp, base + dnext * K, K, dnext, nb, dst + (size_t)cc * 2 * D, lane);
        dnext += nb;
        if (dnext == D) {
            base += D * K;
            dnext = 0;
            cc++;
            while (cc < c1 && chunk_n(cc) < 3) cc++;
            if (cc < c1) {
                K = (uint32_t)chunk_n(cc) - 1u;
                clear_tables();
            }
        }
        lds_flag_put(rp.fl + F_DRES, (int)(base + dnext * K), lane);
    }
}

}  // namespace lslam
