// lslam_rng_pipe.h — the MT19937 hypothesis stream of a whole scan as a
// two-wave producer (parity mode), and the resolution of the
// Fisher-Yates steps into draws (done by the consensus kernel).
//
// The parse of numpy's legacy stream is a sequential automaton, so a scan's
// draws are bounded by ONE dependency chain, and a 4096-scan batch gives only
// 4 such chains per SIMD.  The producer keeps only that chain on its critical
// wave:
//   wave 0 (parser):  tempers the words of a 64-word window, solves the accept
//                     ballot by fixed-point iteration and stores each accepted
//                     j (the step's random_interval result) to HBM:
//                     J[c][d][s] = j of step s (i = K - s) of draw d of chunk c,
//                     at D * chunk_pt_off[c] + d*K + s (u8 if every chunk has
//                     <= 256 points, else u16).
//   blocks:           block b+1 of the MT state is twisted out of place into the
//                     other of two 624-word slots of raw state (then a 64-word
//                     pad holding slot 0's head, so a window may run across the
//                     block boundary) by the parser itself, when it first needs
//                     it (rp_need_block).
// Turning the steps into the two drawn indices is bulk, data-parallel work
// (resolve_chunk below); it runs in the consensus kernel, one wave per chunk,
// where all of a chunk's draws are resolved together.
// The producer assumes no early stop (a trial with sum of squared residuals
// exactly 0); the consensus kernel flags one and the fix-up pass replays it.
#pragma once
#include "../../include/lidarslam.h"
#include "lslam_rng.h"

namespace lslam {

// Waves of a SIMD issue by priority, then age.  With equal priorities the
// oldest parser of a SIMD races ahead and the youngest finishes last.
// Parsers lower their priority as they progress (RP_PRIO_TOP in the first
// third of the scan's steps ... RP_PRIO_TOP - 2 in the last, checked at each
// chunk's start) so the SIMD's parsers advance together.  The bottom level stays above 0, the priority of
// the consumer kernels (resolve / consensus / post of the previous call) that
// share the SIMDs: they take the issue slots the parsers' chains leave idle.
#ifndef RP_PRIO_TOP
#define RP_PRIO_TOP 3
#endif
__device__ __forceinline__ void set_prio_level(int lvl) {
    switch (lvl) {
        case 3: __builtin_amdgcn_s_setprio(3); break;
        case 2: __builtin_amdgcn_s_setprio(2); break;
        case 1: __builtin_amdgcn_s_setprio(1); break;
        default: __builtin_amdgcn_s_setprio(0); break;
    }
}

// out-of-place mt19937_gen (numpy's, randomkit): dst = twist(src) by one wave in ten 64-word
// chunks, i = 64 k + lane.  dst[i] = mix(src[i], src[i + 1], far) with far = src[i + 397] for
// i < 227 and the NEW dst[i - 227] above, so chunk k reads dst only from chunks <= k - 3: four
// groups of independent chunks ({0,1,2}, {3,4,5}, {6,7,8}, {9}), each group's loads issued
// together after the previous group's stores.  The last word's "next" is the new dst[0] and is
// read as src[624]: the word after the source slot, which is dst[0] itself when dst is the slot
// after src (slot 0 -> 1), and the head pad after slot 1 when dst is slot 0 -- chunk 0 writes its
// words there too (pad != null), which is also the pad refresh of an even block.  Every chunk
// then runs the same code (one LDS address select in chunk 3, exec narrowed only in chunk 9);
// the three-phase form spent 68 VALU, 30 LDS, 14 SALU and 5 branches per block and lane, most
// of the surplus on its guarded partial iterations (SQ counters r05f).
template <int LO, int HI>
__device__ __forceinline__ void mt_twist_group(const uint32_t *src, uint32_t *dst, uint32_t *pad, int lane) {
    uint32_t a[HI - LO], b[HI - LO], c[HI - LO];
#pragma unroll
    for (int k = LO; k < HI; k++) {
        const int i = 64 * k + lane;
        if (k < 9 || i < MT_N) {
            a[k - LO] = src[i];
            b[k - LO] = src[i + 1];
            const uint32_t *f = (i < MT_N - MT_M) ? src + i + MT_M : dst + i - (MT_N - MT_M);
            c[k - LO] = *f;
        }
    }
#pragma unroll
    for (int k = LO; k < HI; k++) {
        const int i = 64 * k + lane;
        if (k < 9 || i < MT_N) {
            const uint32_t v = mt_mix(a[k - LO], b[k - LO], c[k - LO]);
            dst[i] = v;
            if (k == 0 && pad) pad[lane] = v;
        }
    }
    wave_lds_sync();
}
__device__ __forceinline__ void mt_twist_oop(const uint32_t *src, uint32_t *dst, uint32_t *pad, int lane) {
    mt_twist_group<0, 3>(src, dst, pad, lane);
    mt_twist_group<3, 6>(src, dst, pad, lane);
    mt_twist_group<6, 9>(src, dst, pad, lane);
    mt_twist_group<9, 10>(src, dst, pad, lane);
}

// ---------------- reject tables (chunks of at most 128 points) ----------------
// For K = N-1 <= 127 a word's fate depends on w only through v = w & mask(K)
// (<= 127), and on its step only through x = (step of the window's first
// word within its draw) + (words accepted before it in the window).  Row v of
// the table for K holds, bit x, whether random_interval rejects v at
// i = K - (x mod K): (v & mask(i)) > i.  A window of 64 words then needs, per
// lane, the 64 bits x in [sg, sg+63] of its row (3 dwords + 2 funnel shifts),
// and one fixed-point iteration is v_mbcnt x2, a 64-bit shift and a compare
// (the reject bit of the lane's current count), not the 9-op mask evaluation.
// x runs over at most K-1 + 63 + 32 < 224 bits: 7 dwords per row (odd, so the
// lanes' random rows spread over the LDS banks).
constexpr uint32_t RT_KMAX = 127;
constexpr int RT_ROWS = 128;
constexpr int RT_ST = 7;
constexpr int RT_DWORDS = RT_ROWS * RT_ST;  // one K's table: 3.5 KiB
__host__ __device__ inline uint32_t rt_word(uint32_t K, uint32_t v, uint32_t q) {
    uint32_t word = 0;
    for (uint32_t b = 0; b < 32; b++) {
        const uint32_t x = q * 32u + b;
        const uint32_t i = K - x % K;
        uint32_t m = i;
        m |= m >> 1; m |= m >> 2; m |= m >> 4; m |= m >> 8; m |= m >> 16;
        if ((v & m) > i) word |= 1u << b;
    }
    return word;
}

struct RngPipe;
__device__ __forceinline__ int rp_level(const RngPipe &rp, uint32_t done);

struct RngPipe {
    uint32_t *blk;         // LDS [2][624] raw MT state, block b in slot b & 1
    int have;              // the newest block in the pipe (wave-uniform: only its parser twists)
    uint32_t *tbl;         // LDS [RT_ROWS][RT_ST]: reject table of the current K
    uint32_t tblK;         // K of the table in tbl (0 = none)
    uint32_t total_steps;  // parser: steps of the whole scan (priority schedule)
    uint32_t lvl_t1, lvl_t2;  // parser: done steps at which the level drops (rp_set_schedule)
    uint32_t done_steps;   // parser: steps of the finished chunks
    int prio;              // parser: current priority level
#ifdef LSLAM_STAMPS
    uint64_t acc[8];
#endif
#ifdef LSLAM_WSTAMPS
    uint64_t wacc[8];
#endif
};

// Level RP_PRIO_TOP - floor(3 done / (total + 1)): two compares against thresholds set
// once per scan instead of a 64-bit division at every block switch.
__device__ __forceinline__ void rp_set_schedule(RngPipe &rp) {
    rp.lvl_t1 = (rp.total_steps + 1u + 2u) / 3u;        // ceil((total + 1) / 3)
    rp.lvl_t2 = (2u * (rp.total_steps + 1u) + 2u) / 3u;  // ceil(2 (total + 1) / 3)
}
__device__ __forceinline__ int rp_level(const RngPipe &rp, uint32_t done) {
    return RP_PRIO_TOP - (done >= rp.lvl_t1 ? 1 : 0) - (done >= rp.lvl_t2 ? 1 : 0);
}

// Block `need` of the pipe, before the parser reads it: twisted by the parser itself (block
// need - 1 -> slot need & 1, which held block need - 2, already parsed; an even block also
// refreshes the pad after slot 1).  rp.have = the newest block in the pipe, an SGPR: the
// parser is the pipe's only writer (an LDS flag read back at every call cost an LDS round
// trip and a readfirstlane per block).  (A helper wave per workgroup that twisted ahead was
// measured and dropped at r03: the parsers' chains got ~3 % shorter, but the producer then
// held 5 instead of 4 waves per SIMD, one consumer wave fewer.)
__device__ __forceinline__ void rp_need_block(RngPipe &rp, int need, int lane) {
    if (rp.have < need) {
        // an even block goes to slot 0: its head is copied to the pad after slot 1 by the twist
        mt_twist_oop(rp.blk + ((need - 1) & 1) * MT_N, rp.blk + (need & 1) * MT_N,
                     (need & 1) == 0 ? rp.blk + 2 * MT_N : nullptr, lane);
        rp.have = need;
    }
}

// Diagnostic build only: parser cycle accounting (0 block waits, 2 fixed point,
// 3 rest of the window, 5 windows, 6 fixed-point evaluations).  With LSLAM_WSTAMPS
// as well, those are off and the table-mode windows inside a run (tbl_window<false>)
// are cut into segments instead (rp.wacc, tools/wstamps.py): 0 next window's word
// load + temper, 1 reject-table read + funnel shifts, 2 the unchecked evaluations,
// 3 the checked loop (convergence tests, branches, further evaluations), 4 store and
// window bookkeeping; 5 windows, 6 checked iterations, 7 an empty segment (the
// stamp's own cost, to subtract from each segment).
#if defined(LSLAM_STAMPS) && !defined(LSLAM_WSTAMPS)
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
// random_interval's mask for step index i >= 1 (wave-uniform i: scalar ops)
__device__ __forceinline__ uint32_t step_mask(uint32_t i) { return 0xffffffffu >> __clz((int)i); }

// tempered word & mask(K): the two xor-with-masked-shift steps as v_bitop3 ((a & b) ^ c)
__device__ __forceinline__ uint32_t rt_temper_mask(uint32_t y, uint32_t mK) {
    y ^= (y >> 11);
    y = __builtin_amdgcn_bitop3_b32(y << 7, 0x9d2c5680u, y, 0x6a);
    y = __builtin_amdgcn_bitop3_b32(y << 15, 0xefc60000u, y, 0x6a);
    return (y ^ (y >> 18)) & mK;
}

__device__ __forceinline__ uint32_t fy_index(uint32_t d, uint32_t K) { return min(d, d + K) + 1u; }
__device__ __forceinline__ uint32_t fy_j(uint32_t w, uint32_t i) { return w & (0xffffffffu >> __clz((int)i)); }

// Store j of the accepted lanes (R = the reject ballot) without a branch: exec is
// narrowed to ~R around one store (the compiler's form re-derives the lane's bit
// from R with three VALU and a saveexec branch).  Full exec on entry.
__device__ __forceinline__ void store_accepted(uint8_t *J, uint32_t idx, uint32_t v, uint64_t R) {
    uint64_t saved;
    asm volatile(
        "s_andn1_saveexec_b64 %0, %1\n\t"  // saved = exec; exec = ~R & exec
        "global_store_byte %2, %3, %4\n\t"
        "s_mov_b64 exec, %0"
        : "=&s"(saved)
        : "s"(R), "v"(idx), "v"(v), "s"(J)
        : "memory", "scc");
}
__device__ __forceinline__ void store_accepted(uint16_t *J, uint32_t idx, uint32_t v, uint64_t R) {
    uint64_t saved;
    asm volatile(
        "s_andn1_saveexec_b64 %0, %1\n\t"
        "global_store_short %2, %3, %4\n\t"
        "s_mov_b64 exec, %0"
        : "=&s"(saved)
        : "s"(R), "v"(idx * 2u), "v"(v), "s"(J)
        : "memory", "scc");
}

// Accepted lanes of a full window = zero bits of the reject ballot.
__device__ __forceinline__ uint32_t accepted_count(uint64_t R) {
    uint32_t n;
    asm("s_bcnt0_i32_b64 %0, %1" : "=s"(n) : "s"(R) : "scc");
    return n;
}

template <bool FAST, typename JT>
__device__ __forceinline__ void parse_chunk(RngPipe &rp, int &blkno, int &pos, JT *__restrict__ J, uint32_t N,
                                            uint32_t D, int lane) {
    const uint32_t K = N - 1;
    const uint32_t G = D * K;
    const float invK = 1.0f / (float)K;
    const uint32_t guess = ((uint32_t)lane * 46u) >> 6;  // ~0.72 accepts per word
    uint32_t g = 0, sg = 0;
    int pre_pos = -1;
    uint32_t pre_raw = 0;
    RP_STAMP_DECL
    while (g < G) {
        RP_STAMP(3);
        if (pos >= MT_N) {
            blkno += 1;
            rp_need_block(rp, blkno, lane);
            asm volatile("" ::: "memory");
            pos -= MT_N;  // > 0 after a window that ran across the block boundary (table mode)
            pre_pos = -1;
            // the priority schedule at block switches too: a one-chunk scan (C5) has no other
            // chunk start, and without it a SIMD's oldest parser finishes first and its youngest
            // runs on alone (stamps r06: 23 vs 41 us by age rank in one epoch launch)
            const int lvl = rp_level(rp, rp.done_steps + g);
            if (lvl != rp.prio) {
                rp.prio = lvl;
                set_prio_level(lvl);
            }
            RP_STAMP(0);
        }
        const uint32_t *kb = rp.blk + (blkno & 1) * MT_N;
        const uint32_t rem = G - g;
        // a run of full windows short of the chunk's end (window r of the run still has > 64 steps
        // left: r < (rem - 1) / 64), up to and including the window across the block's end: as in
        // table mode, the next block is twisted first and its words follow the block's in the LDS
        // ([slot 0][slot 1][pad]), so a block's last words need no partial window (C5: one in
        // eleven of its windows was the partial form, ~10 % of the producer)
        // The next block is twisted when the parser enters a block (not when a run first crosses:
        // a run cut short by the chunk's end prefetches the next run's first words, which may lie
        // past the block's end, so those must already be the next block's).
        if (FAST) {
            rp_need_block(rp, blkno + 1, lane);
            asm volatile("" ::: "memory");
        }
        const int nrun = FAST ? min((MT_N - pos + 63) >> 6, (int)((rem - 1u) >> 6)) : 0;
        if (nrun > 0) {
            uint32_t raw = (pre_pos == pos) ? pre_raw : kb[pos + lane];
            // software-pipelined temper: window r+1's words are tempered beside window r's fixed
            // point (this path is latency-bound: C5's one-chunk scans give 4 parsers per SIMD and
            // little else to issue, ~680 cycles per window alone, stamps r06)
            uint32_t w = rt_temper_mask(raw, 0xffffffffu);
            for (int r = 0; r < nrun; r++) {
                // next window's words: past the block's end this reads the rest of the pipe's LDS
                // (the other block, the flags, the next pipe) or out-of-range zeros; never used
                const uint32_t nraw = kb[pos + 64 + lane];
                RP_STAMP(3);
                const uint32_t b1 = K - 1u - sg;
                const uint32_t base0 = b1 - (uint32_t)lane;
                uint32_t d = b1 - guess;
                uint32_t i = fy_index(d, K);
                uint32_t jv = fy_j(w, i);
                uint64_t R = ballot(jv > i), Rp;
                const uint32_t wn = rt_temper_mask(nraw, 0xffffffffu);
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
                // R is the fixed point; d, jv belong to it: the accepted lanes
                // (exec & ~R) store their j
                store_accepted(J, g + (b1 - d), jv, R);
                const uint32_t na = accepted_count(R);
                pos += 64;
                g += na;
                sg += na;
                if (sg >= K) sg -= K;
                raw = nraw;
                w = wn;
            }
            pre_pos = pos;
            pre_raw = raw;
            continue;
        }
        const uint32_t raw = (pre_pos == pos) ? pre_raw : kb[min(pos + lane, MT_N - 1)];
        pre_pos = -1;
        const uint32_t w = mt_temper(raw);
        RP_STAMP(3);
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
        if ((B >> lane) & 1ull) J[g + c] = (JT)jv;
        if (na >= rem && na > 0) {
            pos += fls64(B) + 1;
            pre_pos = -1;
        } else {
            pos += nw;
        }
        g += na;
        if (FAST) {
            sg += na;
            if (sg >= K) sg -= K;
        } else {
            uint32_t q, rs;
            divmod_small(sg + na, K, invK, q, rs);
            sg = rs;
        }
    }
    rp.done_steps += G;
}

// ---------------- parser wave, table mode (K <= 127) ----------------
// Lane l of a window holds word pos+l; a_l = accepted words below it, and
// s_l = 63 - a_l = v_mbcnt(reject ballot, 63 - l).  Bit a of the lane's 64-bit
// window M (x = sg + a) is its reject flag at that count, i.e. bit 63 of
// M << s.  Accepted lanes store v at step g + a_l; the consumer applies
// mask(i) itself (v & mask(i) = the step's j), so no per-lane i is formed here.

// The sign test reads the shifted window's high dword only (an empty asm keeps the compiler
// from folding it back into a 64-bit compare of the whole shift).  A/B at r04: C3 0.785 vs
// 0.804 ms per step, producer 0.737 vs 0.749 ms (2 x 2 runs, one box).
__device__ __forceinline__ bool rt_rej(uint64_t M, uint32_t s) {
    uint32_t hi = (uint32_t)((M << s) >> 32);
    asm("" : "+v"(hi));
    return (int32_t)hi < 0;
}

// (sg + na) mod K for sg < K, na <= 64: one conditional subtraction when K >= 64
// (KGE64, known at compile time: no per-window test of K)
template <bool KGE64>
__device__ __forceinline__ uint32_t rt_wrap(uint32_t x, uint32_t K) {
    x = min(x, x - K);  // unsigned: x - K wraps high when x < K
    if (!KGE64)
        while (x >= K) x -= K;
    return x;
}

typedef __attribute__((address_space(3))) const uint32_t lds_u32_t;
__device__ __forceinline__ uint64_t rt_window(const uint32_t *tbl, uint32_t v, uint32_t sg) {
    // 32-bit LDS byte address: v * 28 (v <= 127) as one u24 multiply-add onto the scalar
    // part (table base + dword sg / 32), not a 64-bit generic-pointer multiply-add.  The scalar
    // part is s_lshr + s_lshl2_add (the compiler's shift, mask and add is one SALU more per window)
    uint32_t q, base;
    asm("s_lshr_b32 %0, %1, 5" : "=s"(q) : "s"(sg) : "scc");
    asm("s_lshl2_add_u32 %0, %1, %2" : "=s"(base) : "s"(q), "s"((uint32_t)(uintptr_t)(lds_u32_t *)tbl) : "scc");
    lds_u32_t *row = (lds_u32_t *)(uintptr_t)(__umul24(v, RT_ST * 4u) + base);
    const uint32_t d0 = row[0], d1 = row[1], d2 = row[2];
    const uint32_t r = sg & 31u;
    const uint32_t lo = __builtin_amdgcn_alignbit(d1, d0, r);
    const uint32_t hi = __builtin_amdgcn_alignbit(d2, d1, r);
    return ((uint64_t)hi << 32) | lo;
}

// One full table-mode window (64 words, short of the chunk's end).  The last window of a run may
// run across the block's end: the next block is in the pipe already (parse_chunk_tbl twists it
// when the parser enters a block), so no window tests for the crossing.
// gq = g + 63 (steps of the chunk before this window, + 63): lane l's step is gq - s_l.
//
// The fixed point: three evaluations (the first at the 0.72-accepts guess s0) without a
// convergence check (a further evaluation of the fixed point leaves it unchanged; ~4.5 reach
// it on average), then one per checked turn.  Two unchecked after the first measured fastest
// at r04 (C3 step 0.777 vs 0.793 ms with three; one: 0.765-0.773 vs 0.761-0.769): the
// producer's instruction count, not its checks' latency, is what the consumers beside it feel.
// Measured and dropped: a count-based convergence test (6 VALU per checked turn), reading each
// test one turn late (one evaluation more per window: 0.81 vs 0.77 ms).
//
// The product form is one asm block: the evaluations, the checked turns and the store.  The
// checked turns keep the ballot in VCC and in s[40:41] in turn, so no turn copies the ballot
// it compares against (the compiler's loop spends an s_mov_b64 per turn).  Both exits leave
// the fixed point in VCC (equal to s[40:41]) and its counts in S; v[28:29] is the shift's
// scratch pair.  Wait states (gfx950, tests/test_isa_hazards.py checks them in the built code
// object): one between v_lshlrev_b64 and the v_cmp that reads its high dword (the compiler
// puts the same s_nop 0 there: tools/hazard_probe.hip), two between a v_cmp writing VCC or an
// SGPR pair and the v_mbcnt reading it as a lane mask (VALU SGPR write -> VALU read of that
// SGPR as a constant: an s_nop 1, or the s_cmp + s_cbranch of a checked turn).  Nothing after
// the exec restore reads EXEC as DPP data, so the block ends without a wait state (A/B at r04:
// 0.765 vs 0.768 ms with a trailing s_nop).  The diagnostic stamp build (LSLAM_STAMPS) keeps
// the compiler's form of the same iteration, cut into stamped segments.
template <bool KGE64, typename JT>
__device__ __forceinline__ void tbl_window(RngPipe &rp, const uint32_t *kb, int &pos, uint32_t &raw, uint32_t &gq,
                                           uint32_t &sg, JT *__restrict__ J, uint32_t K, uint32_t mK, uint32_t sbase,
                                           uint32_t s0, int lane) {
#ifdef LSLAM_WSTAMPS
    const bool wst = true;
    uint64_t _w = wst ? lslam_stamp() : 0;
#define WSTAMP(k)                                  \
    do {                                           \
        if (wst) {                                 \
            const uint64_t _t = lslam_stamp();     \
            rp.wacc[k] += _t - _w;                 \
            _w = _t;                               \
        }                                          \
    } while (0)
    if (wst) {
        WSTAMP(7);
        rp.wacc[5] += 1;
    }
#else
#define WSTAMP(k) do {} while (0)
#endif
    // next window's words (after a window across the block's end: discarded by the block switch)
    const uint32_t nraw = kb[pos + 64 + lane];
    const uint32_t v = rt_temper_mask(raw, mK);
    WSTAMP(0);
    const uint64_t M = rt_window(rp.tbl, v, sg);
#ifdef LSLAM_WSTAMPS
    if (wst) asm volatile("" ::"v"((uint32_t)M), "v"((uint32_t)(M >> 32)));
#endif
    WSTAMP(1);
#ifndef LSLAM_STAMPS
    uint32_t na, tS, tI;
    uint64_t tE;
#define TBL_EVAL_VCC                                \
    "v_mbcnt_lo_u32_b32 %[S], vcc_lo, %[sb]\n\t"  \
    "v_mbcnt_hi_u32_b32 %[S], vcc_hi, %[S]\n\t"   \
    "v_lshlrev_b64 v[28:29], %[S], %[M]\n\t"      \
    "s_nop 0\n\t"                                 \
    "v_cmp_gt_i32_e32 vcc, 0, v29\n\t"            \
    "s_nop 1\n\t"
#define TBL_TURNS                                                   \
    "v_lshlrev_b64 v[28:29], %[s0], %[M]\n\t"                     \
    "s_nop 0\n\t"                                                 \
    "v_cmp_gt_i32_e32 vcc, 0, v29\n\t"                            \
    "s_nop 1\n\t" TBL_EVAL_VCC TBL_EVAL_VCC                        \
    "TBLA_%=:\n\t"                                            \
    "v_mbcnt_lo_u32_b32 %[S], vcc_lo, %[sb]\n\t"                  \
    "v_mbcnt_hi_u32_b32 %[S], vcc_hi, %[S]\n\t"                   \
    "v_lshlrev_b64 v[28:29], %[S], %[M]\n\t"                      \
    "s_nop 0\n\t"                                                 \
    "v_cmp_gt_i32_e64 s[40:41], 0, v29\n\t"                       \
    "s_cmp_eq_u64 s[40:41], vcc\n\t"                              \
    "s_cbranch_scc1 TBLX_%=\n\t"                              \
    "v_mbcnt_lo_u32_b32 %[S], s40, %[sb]\n\t"                     \
    "v_mbcnt_hi_u32_b32 %[S], s41, %[S]\n\t"                      \
    "v_lshlrev_b64 v[28:29], %[S], %[M]\n\t"                      \
    "s_nop 0\n\t"                                                 \
    "v_cmp_gt_i32_e32 vcc, 0, v29\n\t"                            \
    "s_cmp_eq_u64 vcc, s[40:41]\n\t"                              \
    "s_cbranch_scc0 TBLA_%=\n"                                 \
    "TBLX_%=:\n\t"                                            \
    "v_sub_u32 %[I], %[gq], %[S]\n\t"
    if constexpr (sizeof(JT) == 1) {
        asm volatile(TBL_TURNS
                     "s_andn1_saveexec_b64 %[E], vcc\n\t"
                     "global_store_byte %[I], %[v], %[J]\n\t"
                     "s_mov_b64 exec, %[E]\n\t"
                     "s_bcnt0_i32_b64 %[na], vcc"
                     : [na] "=s"(na), [S] "=&v"(tS), [I] "=&v"(tI), [E] "=&s"(tE)
                     : [M] "v"(M), [s0] "v"(s0), [sb] "v"(sbase), [v] "v"(v), [gq] "s"(gq), [J] "s"(J)
                     : "vcc", "scc", "v28", "v29", "s40", "s41", "memory");
    } else {
        asm volatile(TBL_TURNS
                     "v_lshlrev_b32 %[I], 1, %[I]\n\t"
                     "s_andn1_saveexec_b64 %[E], vcc\n\t"
                     "global_store_short %[I], %[v], %[J]\n\t"
                     "s_mov_b64 exec, %[E]\n\t"
                     "s_bcnt0_i32_b64 %[na], vcc"
                     : [na] "=s"(na), [S] "=&v"(tS), [I] "=&v"(tI), [E] "=&s"(tE)
                     : [M] "v"(M), [s0] "v"(s0), [sb] "v"(sbase), [v] "v"(v), [gq] "s"(gq), [J] "s"(J)
                     : "vcc", "scc", "v28", "v29", "s40", "s41", "memory");
    }
#undef TBL_TURNS
#undef TBL_EVAL_VCC
#else
    uint64_t R = ballot(rt_rej(M, s0));
#pragma unroll
    for (int e = 0; e < 2; e++) R = ballot(rt_rej(M, mbcnt_from(R, sbase)));
#ifdef LSLAM_WSTAMPS
    if (wst) asm volatile("" ::"s"(R));
#endif
    WSTAMP(2);
    uint32_t s;
    RP_COUNT(6, 3);
    for (;;) {
        s = mbcnt_from(R, sbase);
        const uint64_t Rn = ballot(rt_rej(M, s));
        RP_COUNT(6, 1);
#ifdef LSLAM_WSTAMPS
        if (wst) rp.wacc[6] += 1;
#endif
        if (Rn == R) break;
        R = Rn;
    }
    RP_COUNT(5, 1);
    WSTAMP(3);
    store_accepted(J, gq - s, v, R);
    const uint32_t na = accepted_count(R);
#endif
    pos += 64;
    gq += na;
    sg = rt_wrap<KGE64>(sg + na, K);
    raw = nraw;
#ifdef LSLAM_WSTAMPS
    if (wst) asm volatile("" ::"s"(sg), "s"(gq));
#endif
    WSTAMP(4);
#undef WSTAMP
}

template <bool KGE64, typename JT>
__device__ __forceinline__ void parse_chunk_tbl(RngPipe &rp, int &blkno, int &pos, JT *__restrict__ J, uint32_t N,
                                                uint32_t D, int lane) {
    const uint32_t K = N - 1;
    const uint32_t G = D * K;
    const uint32_t mK = 0xffffffffu >> __clz((int)K);
    const uint32_t sbase = 63u - (uint32_t)lane;
    const uint32_t s0 = 63u - (((uint32_t)lane * 46u) >> 6);  // ~0.72 accepts per word below the lane
    uint32_t g = 0, sg = 0;
    int pre_pos = -1;
    uint32_t pre_raw = 0;
    RP_STAMP_DECL
    while (g < G) {
        RP_STAMP(3);
        if (pos >= MT_N) {
            blkno += 1;
            rp_need_block(rp, blkno, lane);
            asm volatile("" ::: "memory");
            pos -= MT_N;  // > 0 after a window that ran across the block boundary (table mode)
            pre_pos = -1;
            RP_STAMP(0);
        }
        // the next block is twisted as soon as the parser enters a block (its slot held the block
        // before this one, already parsed), so a run's last window may run across the boundary
        // without a check: the LDS holds [block slot 0][slot 1][pad = head of slot 0], and the
        // words after the boundary follow contiguously.  (One block per scan is twisted and never
        // read: the one after the scan's last.)
        rp_need_block(rp, blkno + 1, lane);
        asm volatile("" ::: "memory");
        const uint32_t *kb = rp.blk + (blkno & 1) * MT_N;
        const uint32_t rem = G - g;
        // A run of full windows short of the chunk's end, up to the block's end
        const int nrun = min((MT_N - pos + 63) >> 6, (int)((rem - 1u) >> 6));
        if (nrun > 0) {
            uint32_t raw = (pre_pos == pos) ? pre_raw : kb[pos + lane];
            uint32_t gq = g + 63u;
            const int pos_end = pos + 64 * nrun;
            // two windows per loop turn (one loop test and one address step per pair: the second
            // window's loads take the first's address plus an immediate)
            if (nrun & 1) tbl_window<KGE64>(rp, kb, pos, raw, gq, sg, J, K, mK, sbase, s0, lane);
            while (pos != pos_end) {
                tbl_window<KGE64>(rp, kb, pos, raw, gq, sg, J, K, mK, sbase, s0, lane);
                tbl_window<KGE64>(rp, kb, pos, raw, gq, sg, J, K, mK, sbase, s0, lane);
            }
            g = gq - 63u;
            RP_STAMP(2);
            pre_pos = pos;
            pre_raw = raw;
            continue;
        }
        // ---- the chunk's last window (rem <= 64), possibly across the block boundary.
        // A = accept ballot (lanes whose count is below rem); ~A counts the others as rejected.
        if (pos + 64 > MT_N) {
            rp_need_block(rp, blkno + 1, lane);
            asm volatile("" ::: "memory");
            pre_pos = -1;
        }
        const uint32_t raw = (pre_pos == pos) ? pre_raw : kb[pos + lane];
        pre_pos = -1;
        const uint32_t v = rt_temper_mask(raw, mK);
        const uint64_t M = rt_window(rp.tbl, v, sg);
        RP_STAMP(3);
        const int nw = 64;
        const uint64_t actm = ~0ull;
        const int thr = 63 - (int)min(rem, 64u);  // a < rem  <=>  s > thr
        uint64_t A = actm & ballot(!rt_rej(M, s0) && (int)s0 > thr);
        uint32_t s;
        for (;;) {
            s = mbcnt_from(~A, sbase);
            const uint64_t An = actm & ballot(!rt_rej(M, s) && (int)s > thr);
            if (An == A) break;
            A = An;
        }
        RP_STAMP(2);
        RP_COUNT(5, 1);
        if ((A >> lane) & 1ull) J[(g + 63u) - s] = (JT)v;
        const uint32_t na = (uint32_t)popc64(A);
        if (na >= rem && na > 0) pos += fls64(A) + 1;
        else pos += nw;
        g += na;
        sg = rt_wrap<KGE64>(sg + na, K);
    }
    rp.done_steps += G;
}

// ---------------- resolution: steps -> draws, one wave per chunk ----------------
// Lanes are draws.  For draw d, step s has i = K - s and j_i = J[d*K + s] &
// mask(i) (j_i <= i; the table-mode parser stores w & mask(K), the other the
// masked j itself, and masking again leaves it unchanged).  Fisher-Yates swaps x[i] and x[j_i] for i = K..1, so a forward
// scan over i = 2..K recovers where the values that START at positions 0 and 1
// of the last step's input come from: p <- i whenever j_i == p (the value at p
// was swapped there by step i, and no later, smaller-i step writes position
// i > p).  Step 1 then swaps them iff j_1 == 0.  numpy's permutation(N)[:2] =
// (x[0], x[1]) after all steps.  The chunk's steps are staged in LDS when they
// fit (16-byte loads, one HBM latency); otherwise lanes stream them from HBM.
template <typename JT>
__device__ __forceinline__ void resolve_draws_fwd(const JT *__restrict__ Js, uint32_t K, uint32_t d0, uint32_t D,
                                                  int32_t *__restrict__ draws, int lane) {
    const uint32_t d = d0 + (uint32_t)lane;
    const bool live = d < D;
    const JT *Jd = Js + (size_t)(live ? d : d0) * K;
    uint32_t c0 = 0, c1 = 1;
    // i = 2..K in runs of one mask class [2^b, 2^(b+1)): the mask is loop-invariant
    for (uint32_t lo = 2; lo <= K;) {
        const uint32_t m = step_mask(lo);
        const uint32_t hi = min(K, m);
        uint32_t i = lo;
        for (; i + 8 <= hi + 1; i += 8) {
            uint32_t jj[8];
#pragma unroll
            for (int u = 0; u < 8; u++) jj[u] = Jd[K - i - u] & m;
#pragma unroll
            for (int u = 0; u < 8; u++) {
                c0 = (jj[u] == c0) ? i + u : c0;
                c1 = (jj[u] == c1) ? i + u : c1;
            }
        }
        for (; i <= hi; i++) {
            const uint32_t j = Jd[K - i] & m;
            c0 = (j == c0) ? i : c0;
            c1 = (j == c1) ? i : c1;
        }
        lo = hi + 1;
    }
    if (live) {
        const uint32_t j1 = Jd[K - 1] & 1u;
        draws[2 * d] = (int32_t)((j1 == 0u) ? c1 : c0);
        draws[2 * d + 1] = (int32_t)((j1 == 0u) ? c0 : c1);
    }
}

template <typename JT>
__device__ __forceinline__ void resolve_chunk(const JT *__restrict__ J, uint32_t K, uint32_t D, uint32_t stage_cap,
                                              unsigned char *stage, int32_t *__restrict__ draws, int lane) {
    const uint32_t bytes = D * K * (uint32_t)sizeof(JT);
    const uintptr_t gs = (uintptr_t)J;
    const uintptr_t a0 = gs & ~(uintptr_t)15;
    const uint32_t skew = (uint32_t)(gs - a0);
    const uint32_t n16 = (skew + bytes + 15u) >> 4;
    if (n16 * 16u <= stage_cap) {
        for (uint32_t e = (uint32_t)lane; e < n16; e += 64) ((uint4 *)stage)[e] = ((const uint4 *)a0)[e];
        __syncthreads();
        const JT *Js = (const JT *)(stage + skew);
        for (uint32_t d0 = 0; d0 < D; d0 += 64) resolve_draws_fwd(Js, K, d0, D, draws, lane);
    } else {
        for (uint32_t d0 = 0; d0 < D; d0 += 64) resolve_draws_fwd(J, K, d0, D, draws, lane);
    }
}

}  // namespace lslam
