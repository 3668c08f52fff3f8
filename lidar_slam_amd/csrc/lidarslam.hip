// lidarslam.hip — MI355X (gfx950) kernels + C ABI for the per-scan hot path of
// Farofeiro231/LiDAR_SLAM.  See include/lidarslam.h for the reference entry
// points each function replaces and DESIGN.md for the layout/roofline notes.
//
// Execution model (lslam_scan_pipeline, parity mode):
//   rng_kernel     (producer stream) one parser wave per scan, 4 parsers per
//                  workgroup, each twisting its own MT blocks: the scan's chained legacy
//                  MT19937 stream (ransac_functions.py:73 + fit.py:791) -> the
//                  j of every Fisher-Yates step, assuming no early stop
//                  (lslam_rng_pipe.h)
//   resolve_reg8_kernel one wave per (chunk, 64 draws) (resolve_kernel / _walk /
//                  _big for other sizes and epochs): steps -> the T+1 draws
//   chunk_kernel   one wave per chunk: A4/A5 counts (lane = hypothesis), A6 tie
//                  sums + selection, mask + A7 refit, A8 line parameters
//                  (chunks of > 128 points: model / count / select kernels)
//   scan_kernel    (fix-up) one wave per scan; exits at once unless one of its
//                  chunks stopped early, then replays the scan sequentially
//   ukf_group_kernel U1-U8 on lane groups (16 lanes per scan at L = 20), 4-wave
//                  workgroups, between the fix-up and the post pass
//   scan_kernel    (post) one wave per scan: A9/A10 association walk over the
//                  chunks in order (list in registers up to 64 landmarks), y_proj
//                  (LSLAM_UKF_MAP: predict, world-frame association, update)
// Philox / explicit hypotheses skip the producer and the fix-up.  A chunk's
// points, draws and scratch live in LDS; HBM sees the points once per pass.
//
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fPIC -shared.
// -ffp-contract=off is REQUIRED: hipcc contracts a*b+c into v_fma_f64 by
// default, which would change the reference's rounding.
#include <hip/hip_runtime.h>
#include <math.h>
#include "lslam_host_math.h"
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <atomic>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "../../include/lidarslam.h"
#include "lslam_express.h"
#include "lslam_rng.h"
#include "lslam_rng_pipe.h"
#include "lslam_ransac.h"
#include "lslam_ukf.h"
#include "lslam_wave.h"

using namespace lslam;

static_assert(sizeof(lslam_chunk_model) == 112, "chunk model ABI");

// functions.py:59-60 for one measure; polar_kernel and every fused point load
// use this one definition, so both give the same bits.  Out of line: inlined
// sin/cos in every point-staging loop slowed the xy path of C3 by 2.5 %.
__device__ __attribute__((noinline)) double2 polar_xy(double th, double d) {
    const double ang = -th * (LS_PI / 180.0) + LS_PI / 2.0;
    return make_double2(d * cos(ang), d * sin(ang));
}

// A batch's points: Cartesian xy, or raw (theta, d) measures converted on load
// (A1 fused, lslam_scan_batch.theta_deg / dist_mm).  The choice is uniform.
struct PtSrc {
    const double2 *xy;
    const double *th, *dd;
    __device__ __forceinline__ double2 operator[](int64_t i) const { return xy ? xy[i] : polar_xy(th[i], dd[i]); }
    __device__ __forceinline__ PtSrc operator+(int64_t o) const {
        PtSrc r = *this;
        if (xy) r.xy += o;
        else { r.th += o; r.dd += o; }
        return r;
    }
};
__device__ __forceinline__ PtSrc batch_points(const lslam_scan_batch &B) {
    return PtSrc{(const double2 *)B.xy, B.theta_deg, B.dist_mm};
}
// a chunk's points -> LDS, the xy loop kept free of the polar path
__device__ __forceinline__ void stage_points(const lslam_scan_batch &B, int p0, int N, double2 *P, int lane) {
    if (B.xy) {
        const double2 *src = (const double2 *)B.xy + p0;
        for (int p = lane; p < N; p += 64) P[p] = src[p];
    } else {
        for (int p = lane; p < N; p += 64) P[p] = polar_xy(B.theta_deg[p0 + p], B.dist_mm[p0 + p]);
    }
}
static_assert(sizeof(lslam_landmark) == 56, "landmark ABI");

// owning scan of chunk c: the last s with scan_chunk_off[s] <= c.  Batches of
// equal scans (C3: 8 chunks each) hit the proportional guess with one load
// pair; otherwise a binary search (a chain of dependent loads).
__device__ __forceinline__ int owning_scan(const lslam_scan_batch &B, int c) {
    const int g = (int)(((int64_t)c * B.n_scans) / (B.n_chunks > 0 ? B.n_chunks : 1));
    if (g < B.n_scans && B.scan_chunk_off[g] <= c && c < B.scan_chunk_off[g + 1]) return uni(g);
    int lo = 0, hi = B.n_scans;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (B.scan_chunk_off[mid] <= c) lo = mid;
        else hi = mid;
    }
    return uni(lo);
}

enum { MODE_RANSAC = 1, MODE_ASSOC = 2, MODE_UKF = 4, MODE_HYP_ONLY = 8, MODE_POST = 16 };

// A chunk's bounding-box terms and residual cutoffs (chunk_consensus, cut_finish).
typedef float cut_t;  // the count loops' cutoffs: FP32 on the residual's high dword (count_one)
struct ChunkCut {
    double tq;      // tie brackets: an upper bound of E2 + R (sqrt(E2) + 1) (tie_bound_q)
    double margin;  // the exact-test band around ecut
    cut_t c_lo, c_hi;
    int finite;     // every point finite and the box bounds finite
    int scan;       // cut_lane_kernel: the chunk's owning scan (owning_scan), for chunk_kernel
};

// ------------------------------------------------------------------------
// kernel arguments (passed by value)
// ------------------------------------------------------------------------
struct KArgs {
    lslam_scan_batch b;
    double ecut;
    double ecut_q;  // sqrt(ecut) * 1.01 + 1 (host)
    double thr;
    double tol_a, tol_b, tol_dist;
    double tol_dist_sq;  // largest v with RN(sqrt(v)) <= tol_dist (host: sqrt_le_bound)
    uint64_t philox_seed;
    int T;
    int hyp_source;
    int life;
    // LDS layout (byte offsets into dynamic shared memory)
    int off_pts, off_key, off_ring, off_draws, off_cnt, off_tied, off_tsum;
    int off_vstack, off_nstack, off_snap, off_lmk, off_vis, off_mask, off_corg, off_zobs;
    int corg_cap;
    int off_recs;       // post pass: the scan's chunk records + chunk offsets (-1: per-chunk loop)
    int off_ukf;
    int off_j1;
    int pts_cap;
    int lmk_cap;
    int hist_cap;
    UkfConst ukf;
    // split pipeline
    void *jbuf;         // producer -> consensus: Fisher-Yates j per step, [D * n_points] (u8 or u16)
    int j8;             // jbuf holds u8
    int res_g;          // resolve_kernel: LDS staging capacity (bytes)
    int32_t *draws_scr; // resolve_kernel -> chunk_kernel: [n_chunks][T+1][2] (= draws_out when given)
    uint32_t *state_scr;  // producer's end-of-scan MT state [n_scans][625]; the fix-up copies it out
    int off_blk, off_nxt, off_vtmp, off_stage;
    int rng_pipe_bytes;  // rng_kernel: LDS bytes per parser pipe
    int off_stbl;        // rng_kernel: [2] K claims then 2 shared reject tables, after the pipes
    const uint32_t *rt_all;  // rng_kernel: reject tables for K = 2..127
    const uint32_t *seed_state;  // rng_kernel: seed_kernel's initial states [n_scans][624] (null: none)
    // producer epochs (one-chunk scans whose steps exceed the slot budget): this launch
    // covers draws [ep_d0, ep_d0 + ep_nd) of every chunk; ep_nd = 0: all T + 1 draws
    int ep_d0, ep_nd;
    int ep_count;        // host: producer launches of the call
    size_t slot_jbytes;  // host: steps bytes of a slot (its MT state area follows)
    int fixup;          // scan_kernel: only scans with an early-stopped chunk run
    const uint8_t *spec_dirty_in;  // fix-up: scans whose speculative producer input was stale (replay)
    uint8_t *spec_dirty_out;       // fix-up: scans replayed by this call (the next call's dirty_in)
    int write_yproj;    // chunk_kernel: y_proj with the chunk's own line (no association pass)
    int lmk_reg;        // post pass (association only, lmk_cap <= 64): landmark list in registers
    // large chunks (N > 128): count_kernel -> select_kernel
    int32_t *cnt_scr;   // [n_chunks][T] inlier counts (= trial_cnt_out when given)
    double *models;     // [n_chunks][T][4] 2-point models (origin, direction)
    int cnt_blocks;     // count_kernel workgroups per chunk
    const ChunkCut *cuts;  // chunk_kernel: [n_chunks] box terms and cutoffs from cut_lane_kernel (null: in-kernel)
    unsigned long long *dbg;  // diagnostic build only: [n_scans][8] cycle accumulators
    unsigned long long *wcen;  // diagnostic build only: wave census records [256][cap / 256][3] (WaveCensus)
    unsigned int *wcen_n;      // [256] records claimed so far per bucket
    unsigned int wcen_cap;
    unsigned int call_seq;     // host's pipeline-call counter (census tag)
};

// Diagnostic build only (-DLSLAM_STAMPS): one record per wave of a consumer or producer
// kernel, {kernel id | call << 8 | HW_ID << 24 | XCC_ID << 56, s_memrealtime at entry,
// at exit} (100 MHz chip clock), for tools/census.py: when each wave of each dispatch
// became resident, how long it lived, and on which SIMD.  The product build has none.
enum { WC_RNG_PARSER = 1, WC_RNG_HELPER, WC_RESOLVE, WC_CHUNK, WC_FIXUP, WC_POST, WC_UKF };
#if defined(LSLAM_STAMPS) || defined(LSLAM_CENSUS)
struct WaveCensus {
    const KArgs &a;
    uint32_t kid;
    uint64_t t0;
    __device__ WaveCensus(const KArgs &a_, uint32_t kid_) : a(a_), kid(kid_), t0(__builtin_amdgcn_s_memrealtime()) {}
    __device__ ~WaveCensus() {
        if (!a.wcen || (threadIdx.x & 63) != 0) return;
        const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
        const uint32_t hw = (uint32_t)__builtin_amdgcn_s_getreg(4 | (0 << 6) | (31 << 11));
        const uint32_t xcc = (uint32_t)__builtin_amdgcn_s_getreg(20 | (0 << 6) | (3 << 11));
        // 256 buckets of wcen_cap / 256 records, one counter each: one counter for every
        // wave of a launch was a hot spot that slowed the consumers' last instructions
        const unsigned int bk = (blockIdx.x * 7u + (threadIdx.x >> 6)) & 255u, per = a.wcen_cap >> 8;
        const unsigned int i = atomicAdd(a.wcen_n + bk, 1u);
        if (i >= per) return;
        unsigned long long *r = a.wcen + 3 * ((size_t)bk * per + i);
        r[0] = (uint64_t)kid | ((uint64_t)(a.call_seq & 0xffffu) << 8) | ((uint64_t)hw << 24) | ((uint64_t)xcc << 56);
        r[1] = t0;
        r[2] = t1;
    }
};
#define WAVE_CENSUS(a, kid) WaveCensus _wave_census((a), (kid))
#else
#define WAVE_CENSUS(a, kid) \
    do {                    \
    } while (0)
#endif

// ------------------------------------------------------------------------
// per-chunk RANSAC on one wave
// ------------------------------------------------------------------------
struct ChunkOut {
    Model m;          // final model (valid if flags & VALID)
    int n_inl;
    int last_inl;
    int best;
    int n_draws;
    int flags;
    int stop;         // trial at which the stop criterion fired, -1 if none
};

// counts for T trials over N points; returns M = max count
__device__ __forceinline__ int count_pass(const double2 *P, int N, const int32_t *draws, int32_t *cnt, int T,
                                          double ecut, int lane) {
    int M = 0;
    for (int tb = 0; tb < T; tb += 64) {
        const int t = tb + lane;
        const int tt = t < T ? t : 0;
        const Model m = model2(P[draws[2 * tt]], P[draws[2 * tt + 1]]);
        int c0 = 0, c1 = 0, c2 = 0, c3 = 0;
        int p = 0;
        for (; p + 4 <= N; p += 4) {
            const double2 q0 = P[p], q1 = P[p + 1], q2 = P[p + 2], q3 = P[p + 3];
            c0 += resid2(q0, m) < ecut;
            c1 += resid2(q1, m) < ecut;
            c2 += resid2(q2, m) < ecut;
            c3 += resid2(q3, m) < ecut;
        }
        for (; p < N; p++) c0 += resid2(P[p], m) < ecut;
        const int c = (c0 + c1) + (c2 + c3);
        if (t < T) cnt[t] = c;
        M = max(M, wave_max(t < T ? c : 0));
    }
    __syncthreads();
    return M;
}

__device__ ChunkOut chunk_finish_fit(const KArgs &a, double2 *P, int N, const int32_t *draws, uint8_t *mk,
                                     int best, ChunkOut o, int lane);

// The whole ransac() call for one chunk whose draws are in LDS `draws`.
__device__ ChunkOut chunk_ransac(const KArgs &a, double2 *P, int N, const int32_t *draws, int32_t *cnt,
                                 int32_t *tied, double *tsum, uint8_t *mk, double *vstack, int *nstack,
                                 int32_t *cnt_out, int lane) {
    ChunkOut o;
    o.flags = 0;
    o.best = -1;
    o.stop = -1;
    o.n_inl = 0;
    o.last_inl = -1;
    o.n_draws = a.T + 1;
    const int T = a.T;
    const double ecut = a.ecut;
    const int M = uni(count_pass(P, N, draws, cnt, T, ecut, lane));
    if (cnt_out)
        for (int t = lane; t < T; t += 64) cnt_out[t] = cnt[t];
    // compact the max-count trials in trial order
    int ntied = 0;
    for (int tb = 0; tb < T; tb += 64) {
        const int t = tb + lane;
        const bool h = t < T && cnt[t] == M;
        const uint64_t bm = ballot(h);
        if (h) tied[ntied + (int)mbcnt(bm)] = t;
        ntied += popc64(bm);
    }
    __syncthreads();
    // tie sums: only needed if they can change the outcome or trigger the stop
    const bool need_sums = ntied > 1 || M == N || !(ecut > 0.0);
    if (need_sums) {
        for (int kb = 0; kb < ntied; kb += 64) {
            const int k = kb + lane;
            const int t = tied[k < ntied ? k : 0];
            const Model m = model2(P[draws[2 * t]], P[draws[2 * t + 1]]);
            const double s = pw_sum(P, N, m, vstack, nstack, lane);
            if (k < ntied) tsum[k] = s;
        }
        __syncthreads();
    }
    // sequential selection over the tied trials (fit.py:850-869)
    int bcnt = 0, best = -1;
    double bsum = __builtin_inf();
    if (T > 0) {
        if (!need_sums) {
            best = tied[0];
            bcnt = M;
        } else {
            for (int k = 0; k < ntied; k++) {
                const int t = uni(tied[k]);
                const double s = unid(tsum[k]);
                if (M > bcnt || (M == bcnt && s < bsum)) {
                    best = t;
                    bcnt = M;
                    bsum = s;
                    if (bsum <= 0.0) {
                        o.stop = t;
                        break;
                    }
                }
            }
        }
    }
    return chunk_finish_fit(a, P, N, draws, mk, uni(best), o, lane);
}

// after selection: stop bookkeeping, inlier mask of the winner, refit.  The mask pass writes the
// LDS mask mk[0..N) and compacts the inlier points in place to P[0..nin) in data order (inlier
// k of pass j lands at nin_j + rank <= its own index, after the pass has read its points), so the
// refit reads them contiguously: no index list, no gathers.  P's original order is gone
// afterwards: callers take the projections through the mask's ranks (chunk_yproj).
__device__ ChunkOut chunk_finish_fit(const KArgs &a, double2 *P, int N, const int32_t *draws, uint8_t *mk,
                                     int best, ChunkOut o, int lane) {
    const double ecut = a.ecut;
    o.best = best;
    __syncthreads();  // tsum (read above) is dead from here
    if (o.stop >= 0) {
        o.n_draws = o.stop + 2;
        o.flags |= LSLAM_EARLY_STOP;
    }
    if (best < 0) {
        o.flags |= LSLAM_NO_INLIERS;
        return o;
    }
    // inlier mask of the winner; inlier points compacted to P[0..nin)
    const Model mw = model2(P[draws[2 * best]], P[draws[2 * best + 1]]);
    int nin = 0;
    for (int pb = 0; pb < N; pb += 64) {
        const int p = pb + lane;
        const double2 q = P[p < N ? p : 0];
        const bool h = p < N && resid2(q, mw) < ecut;
        const uint64_t bm = ballot(h);
        if (p < N) mk[p] = h ? 1 : 0;
        if (h) P[nin + (int)mbcnt(bm)] = q;
        nin += popc64(bm);
    }
    __syncthreads();
    o.n_inl = nin;
    o.last_inl = nin - 1;
    if (nin == 0) {
        o.flags |= LSLAM_NO_INLIERS;
        return o;
    }
    if (nin == 1) {
        o.flags |= LSLAM_EST_FAIL;
        return o;
    }
    const Model f = (nin == 2) ? model2(P[0], P[1]) : refit_line(P, nin, lane);
    o.m = f;
    o.flags |= LSLAM_VALID;
    if (f.ux == 0.0) o.flags |= LSLAM_VERTICAL;
    return o;
}

// ------------------------------------------------------------------------
// A4-A6 for chunk_kernel (N <= 128): cheap residual test, exact fall-backs
// ------------------------------------------------------------------------
// For a unit direction u the residual is the cross product: r^2 = (e x u)^2.
// With |u|^2 = 1 + d, |d| <= 2^-46 (checked per hypothesis), the reference's
// r^2 (fit.py:129-132 rounding) and c2 = fl(fl(ex*uy - ey*ux)^2) differ by
// < 160 u |e|^2 (u = 2^-53), and the tie-break terms RN(sqrt(r^2))^2 by
// < 165 u |e|^2, where |e|^2 <= E2 = squared bounding-box diagonal.  Hence
//   count: c2 further than 2^-42 (E2 + ecut) from ecut decides r^2 < ecut;
//          closer than that, the exact residual is computed;
//   ties:  S~ = sum of c2 brackets the exact pairwise sum within
//          B(S~) = 2^-42 (N E2 + (N + 32) S~); only tied trials whose lower
//          bound reaches the least upper bound get exact sums (usually one),
//          visited in trial order, so best and the stop trial are unchanged.
// A hypothesis whose direction is not unit (duplicate points: u = d) and
// non-finite coordinates take the exact paths.
__device__ __forceinline__ double tie_bound(double S, int N, double E2) {
    return ((double)N * E2 + (double)(N + 32) * S) * 0x1p-42;
}

// the same for sums of the reassociated cross product (chunk_consensus): each
// term may further differ by ~8 u R |r| <= 8 u R sqrt(E2)
__device__ __forceinline__ double tie_bound_r(double S, int N, double E2, double R) {
    return ((double)N * (E2 + R * (sqrt(E2) + 1.0)) + (double)(N + 32) * S) * 0x1p-42;
}
// the same with tq >= E2 + R (sqrt(E2) + 1) made once per chunk (ChunkCut)
__device__ __forceinline__ double tie_bound_q(double S, int N, double tq) {
    return ((double)N * tq + (double)(N + 32) * S) * 0x1p-42;
}

// The count pass reads the chunk's points with scalar loads (through the
// scalar cache, into SGPRs) when the batch holds Cartesian xy: every lane (a
// hypothesis) uses the same point, which then is an FP64 SGPR operand of its
// FMAs.  The LDS-broadcast form of the same loop is bound by the LDS return
// path (1 KiB per point and wave) and by its load latency.  Scalar loads can
// return out of order, so their wait is lgkmcnt(0): the loop issues the next
// group's load right AFTER waiting for the current one, and the current
// group's arithmetic covers the latency.  The loads are inline asm (the
// compiler would wait for the prefetch before the current group); the waits
// are asm statements that the loaded values pass through.
typedef unsigned u32x16 __attribute__((ext_vector_type(16)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

template <int OFF = 0>  // byte offset, the instruction's immediate
__device__ __forceinline__ u32x16 sload_4pts(const double2 *p) {
    u32x16 v;
    asm volatile("s_load_dwordx16 %0, %1, %2" : "=s"(v) : "s"(p), "i"(OFF) : "memory");
    return v;
}
__device__ __forceinline__ u32x4 sload_pt(const double2 *p) {
    u32x4 v;
    asm volatile("s_load_dwordx4 %0, %1, 0x0" : "=s"(v) : "s"(p) : "memory");
    return v;
}
__device__ __forceinline__ void swait(u32x16 &v) { asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(v)::"memory"); }
__device__ __forceinline__ void swait(u32x4 &v) { asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(v)::"memory"); }
__device__ __forceinline__ double sd(unsigned lo, unsigned hi) {
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// one point against the lane's hypothesis: r = fl(x uy - fl(y ux + k)),
// S += r^2, lo += |r| <= r_lo, hi += |r| < r_hi
// The two cutoffs are tested on r's HIGH dword read as a float (sign, exponent and the top 20
// mantissa bits of the double; for non-negative values its order is the double's): the sure
// inliers are |hi(r)| < hi(r_lo) (so |r| < r_lo), the possible ones |hi(r)| <= hi(r_hi) (every
// |r| < r_hi).  A point between them (|r| within 2^-20 relative of the threshold, ~15 nm at
// 20 mm) makes lo != hi, and the lane recounts exactly, as for the band.  Two FP32 compares
// with the free |.| modifier instead of two FP64 compares (half rate on CDNA4).
__device__ __forceinline__ cut_t count_cut(double c) { return __uint_as_float((uint32_t)(__double_as_longlong(c) >> 32)); }
__device__ __forceinline__ bool sure_in(double r, cut_t c) { return __builtin_fabsf(count_cut(r)) < c; }
__device__ __forceinline__ bool maybe_in(double r, cut_t c) { return __builtin_fabsf(count_cut(r)) <= c; }
__device__ __forceinline__ void count_one(double x, double y, double ux, double uy, double k, cut_t c_lo,
                                          cut_t c_hi, int &lo, int &hi, double &S) {
    // r = fma(x, uy, -fma(y, ux, k)) as two three-address FMAs (left to itself the compiler
    // turns some into v_fmac + a 64-bit copy of k)
    double t, r;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(t) : "s"(y), "v"(ux), "v"(k));
    asm("v_fma_f64 %0, %1, %2, -%3" : "=v"(r) : "s"(x), "v"(uy), "v"(t));
    S = __builtin_fma(r, r, S);
    lo += sure_in(r, c_lo) ? 1 : 0;
    hi += maybe_in(r, c_hi) ? 1 : 0;
    asm volatile("" : "+v"(lo), "+v"(hi));  // keep one compare + add-with-carry per count
}

// Four points against the lane's hypothesis: count_one x 4 in point order (the same S chain,
// the same counts) as one asm block.  gfx950 needs two wait states between a v_cmp writing an
// SGPR pair and the v_addc reading it as the carry-in, and none between a v_fma_f64 and a VALU
// reading its result (tools/hazard_probe.hip; tests/test_isa_hazards.py checks the first in the
// code object); the compiler pads around inline asm it cannot see into, which cost the
// point-by-point form three s_nops per point.  Here every mask is read four or more
// instructions after its compare.  r_i lives in v[40:47] (its high dword is the FP32 key the
// cutoffs test), the compare masks in s[80:87]; each add-with-carry writes its (unused)
// carry-out over the mask it has just read.
__device__ __forceinline__ void count_four(const u32x16 &A, double ux, double uy, double k, cut_t c_lo, cut_t c_hi,
                                           int &lo, int &hi, double &S) {
    asm volatile(
        "v_fma_f64 v[40:41], %[y0], %[ux], %[k]\n\t"
        "v_fma_f64 v[42:43], %[y1], %[ux], %[k]\n\t"
        "v_fma_f64 v[44:45], %[y2], %[ux], %[k]\n\t"
        "v_fma_f64 v[46:47], %[y3], %[ux], %[k]\n\t"
        "v_fma_f64 v[40:41], %[x0], %[uy], -v[40:41]\n\t"
        "v_fma_f64 v[42:43], %[x1], %[uy], -v[42:43]\n\t"
        "v_fma_f64 v[44:45], %[x2], %[uy], -v[44:45]\n\t"
        "v_fma_f64 v[46:47], %[x3], %[uy], -v[46:47]\n\t"
        "v_cmp_lt_f32_e64 s[80:81], |v41|, %[cl]\n\t"
        "v_cmp_le_f32_e64 s[82:83], |v41|, %[ch]\n\t"
        "v_cmp_lt_f32_e64 s[84:85], |v43|, %[cl]\n\t"
        "v_cmp_le_f32_e64 s[86:87], |v43|, %[ch]\n\t"
        "v_fma_f64 %[S], v[40:41], v[40:41], %[S]\n\t"
        "v_addc_co_u32_e64 %[lo], s[80:81], %[lo], 0, s[80:81]\n\t"
        "v_addc_co_u32_e64 %[hi], s[82:83], %[hi], 0, s[82:83]\n\t"
        "v_fma_f64 %[S], v[42:43], v[42:43], %[S]\n\t"
        "v_cmp_lt_f32_e64 s[80:81], |v45|, %[cl]\n\t"
        "v_cmp_le_f32_e64 s[82:83], |v45|, %[ch]\n\t"
        "v_addc_co_u32_e64 %[lo], s[84:85], %[lo], 0, s[84:85]\n\t"
        "v_addc_co_u32_e64 %[hi], s[86:87], %[hi], 0, s[86:87]\n\t"
        "v_fma_f64 %[S], v[44:45], v[44:45], %[S]\n\t"
        "v_cmp_lt_f32_e64 s[84:85], |v47|, %[cl]\n\t"
        "v_cmp_le_f32_e64 s[86:87], |v47|, %[ch]\n\t"
        "v_addc_co_u32_e64 %[lo], s[80:81], %[lo], 0, s[80:81]\n\t"
        "v_addc_co_u32_e64 %[hi], s[82:83], %[hi], 0, s[82:83]\n\t"
        "v_fma_f64 %[S], v[46:47], v[46:47], %[S]\n\t"
        "v_addc_co_u32_e64 %[lo], s[84:85], %[lo], 0, s[84:85]\n\t"
        "v_addc_co_u32_e64 %[hi], s[86:87], %[hi], 0, s[86:87]"
        : [lo] "+v"(lo), [hi] "+v"(hi), [S] "+v"(S)
        : [x0] "s"(sd(A[0], A[1])), [y0] "s"(sd(A[2], A[3])), [x1] "s"(sd(A[4], A[5])), [y1] "s"(sd(A[6], A[7])),
          [x2] "s"(sd(A[8], A[9])), [y2] "s"(sd(A[10], A[11])), [x3] "s"(sd(A[12], A[13])),
          [y3] "s"(sd(A[14], A[15])), [ux] "v"(ux), [uy] "v"(uy), [k] "v"(k), [cl] "v"(c_lo), [ch] "v"(c_hi)
        : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "s80", "s81", "s82", "s83", "s84", "s85", "s86",
          "s87");
}

// one hypothesis per lane against all N points (gP: global, wave-uniform).  Groups of 4 points
// through two SGPR buffers in turn; the loop walks a pointer (one 64-bit add per 8 points, the
// loads' offsets are immediates) and tests it once per 8 points (the index form spent ~15 SALU per 4 points on 64-bit address
// arithmetic and two bounds tests).
__device__ __forceinline__ void count_points_sgpr(const double2 *gP, int N, double ux, double uy, double k,
                                                  cut_t r_lo, cut_t r_hi, int &lo, int &hi, double &S) {
    const double2 *q = gP;
    if (N >= 8) {
        // each buffer is waited on before the other one's load issues (scalar loads return out of
        // order, so lgkmcnt(0) is the only wait); the last group of 8 is peeled so that the loop
        // has one exit test at its bottom
        const double2 *const qlast = gP + ((N >> 3) - 1) * 8;
        u32x16 A = sload_4pts(q), B;
        swait(A);
        while (q != qlast) {
            B = sload_4pts<64>(q);
            count_four(A, ux, uy, k, r_lo, r_hi, lo, hi, S);
            swait(B);
            A = sload_4pts<128>(q);
            count_four(B, ux, uy, k, r_lo, r_hi, lo, hi, S);
            q += 8;
            swait(A);
        }
        B = sload_4pts<64>(q);
        count_four(A, ux, uy, k, r_lo, r_hi, lo, hi, S);
        swait(B);
        count_four(B, ux, uy, k, r_lo, r_hi, lo, hi, S);
        q += 8;
    }
    if (N & 4) {
        u32x16 A = sload_4pts(q);
        swait(A);
        count_four(A, ux, uy, k, r_lo, r_hi, lo, hi, S);
        q += 4;
    }
    for (int r = N & 3; r > 0; r--, q++) {
        u32x4 v = sload_pt(q);
        swait(v);
        count_one(sd(v[0], v[1]), sd(v[2], v[3]), ux, uy, k, r_lo, r_hi, lo, hi, S);
    }
}

// the same from the LDS copy (polar batches: points converted on load)
__device__ __forceinline__ void count_points_lds(const double2 *P, int N, double ux, double uy, double k, cut_t r_lo,
                                                 cut_t r_hi, int &lo, int &hi, double &S) {
    int p = 0;
    for (; p + 2 <= N; p += 2) {
        const double2 q0 = P[p], q1 = P[p + 1];
        count_one(q0.x, q0.y, ux, uy, k, r_lo, r_hi, lo, hi, S);
        count_one(q1.x, q1.y, ux, uy, k, r_lo, r_hi, lo, hi, S);
    }
    if (p < N) count_one(P[p].x, P[p].y, ux, uy, k, r_lo, r_hi, lo, hi, S);
}

// diagnostic build only: chunk_kernel phase cycles into dbg[c][k] (k < 8)
#ifdef LSLAM_STAMPS
#define CH_STAMP(k)                                                            \
    do {                                                                       \
        const uint64_t _t = lslam_stamp();                                     \
        if (chdbg && lane == 0) chdbg[(k)] += _t - _ch_prev;                   \
        _ch_prev = _t;                                                         \
    } while (0)
#define CH_STAMP_DECL uint64_t _ch_prev = lslam_stamp();
#define CH_STAMP_DECL_RESET _ch_prev = lslam_stamp();
#elif defined(LSLAM_CHUNK_EXIT)
// diagnostic build only (tools/chunkphase.sh): the wave ends after phase LSLAM_CHUNK_EXIT, so the
// SQ instruction counters of the launch hold the phases up to it
#define CH_STAMP_DECL_RESET
#define CH_STAMP(k)                                           \
    do {                                                      \
        if ((k) == LSLAM_CHUNK_EXIT) asm volatile("s_endpgm"); \
    } while (0)
#define CH_STAMP_DECL
#else
#define CH_STAMP_DECL_RESET
#define CH_STAMP(k) do {} while (0)
#define CH_STAMP_DECL
#endif

// The chunk's box as upper bounds, not the box itself: the high dword of each coordinate as a
// signed-order key (key(-x) = ~key(x)), so max x, -min x, max y, -min y are four integer maxima
// (per lane, then over the wave by DPP), and a key decodes to the largest double with that high
// dword.  A looser E2 or R only widens the cutoffs' band and the tie brackets, both decided
// exactly beyond them: the counts, winners and sums are the same bits.
__device__ __forceinline__ int hkey(double d) {
    const int h = (int)(__double_as_longlong(d) >> 32);
    return h ^ ((h >> 31) & 0x7fffffff);
}
__device__ __forceinline__ double key_up(int k) {  // >= every double whose key is k
    const int h = k ^ ((k >> 31) & 0x7fffffff);
    return __longlong_as_double((long long)(((unsigned long long)(uint32_t)h << 32) | (h >= 0 ? 0xffffffffull : 0ull)));
}
__device__ __forceinline__ bool key_finite(int k) {
    const int h = k ^ ((k >> 31) & 0x7fffffff);
    return (h & 0x7ff00000) != 0x7ff00000;
}
struct BoxAcc {
    int xh = INT_MIN, xl = INT_MAX, yh = INT_MIN, yl = INT_MAX;  // max / min key of x and y
    __device__ __forceinline__ void add(double2 q) {
        const int kx = hkey(q.x), ky = hkey(q.y);
        xh = max(xh, kx);
        xl = min(xl, kx);
        yh = max(yh, ky);
        yl = min(yl, ky);
    }
};
__device__ __forceinline__ ChunkCut cut_finish(BoxAcc b, double ecut, double ecut_q);
template <typename PP>
__device__ __forceinline__ ChunkCut chunk_cut(PP P, int N, double ecut, double ecut_q, int lane) {
    BoxAcc b;
    for (int p = lane; p < N; p += 64) b.add(P[p]);
    return cut_finish(b, ecut, ecut_q);
}

// max over the wave (every lane active), uniform: DPP within rows of 16, the row broadcasts to
// lane 63, one readlane -- no LDS round trips (beside the producer, whose parsers keep the LDS
// busy, six ds_bpermute levels per value were most of the box's cost)
template <int CTRL, int ROWS>
__device__ __forceinline__ int dpp_max_step(int v) {
    return max(v, __builtin_amdgcn_update_dpp(INT_MIN, v, CTRL, ROWS, 0xf, false));  // INT_MIN where no source
}
__device__ __forceinline__ int wave_max_dpp(int v) {
    v = dpp_max_step<0xB1, 0xf>(v);   // quad_perm [1,0,3,2]
    v = dpp_max_step<0x4E, 0xf>(v);   // quad_perm [2,3,0,1]
    v = dpp_max_step<0x124, 0xf>(v);  // row_ror:4
    v = dpp_max_step<0x128, 0xf>(v);  // row_ror:8
    v = dpp_max_step<0x142, 0xa>(v);  // row_bcast:15 -> rows 1, 3
    v = dpp_max_step<0x143, 0xc>(v);  // row_bcast:31 -> rows 2, 3
    return __builtin_amdgcn_readlane(v, 63);
}

// High-dword cutoffs (count_one) without the exact square-root search: c_lo <= hi(sq_floor_lt(e)),
// c_hi >= hi(sq_ceil_gt(e)).  v_sqrt_f32 of (float)e is within 2^-22 relative of the root, a
// quarter of a high-dword unit; two units of slack leave the band only wider.  Outside float's
// comfortable range, the exact search.
__device__ __forceinline__ float hi_units(double s, int d) {
    return __uint_as_float((uint32_t)(__double_as_longlong(s) >> 32) + (uint32_t)d);
}
__device__ __forceinline__ cut_t cut_lo_of(double e) {
    if (!(e > 0.0)) return -1.0f;
    if (e >= 0x1p-100 && e <= 0x1p100) return hi_units((double)__builtin_amdgcn_sqrtf((float)e), -2);
    return count_cut(sq_floor_lt(e));
}
__device__ __forceinline__ cut_t cut_hi_of(double e) {
    if (e >= 0x1p-100 && e <= 0x1p100) return hi_units((double)__builtin_amdgcn_sqrtf((float)e), 2);
    return count_cut(sq_ceil_gt(e));
}

// from the four key maxima (x max, -x min, y max, -y min) of the chunk's points
__device__ __forceinline__ ChunkCut cut_from_keys(int kxh, int kxl, int kyh, int kyl, double ecut, double ecut_q) {
    ChunkCut cc;
    cc.finite = key_finite(kxh) && key_finite(kxl) && key_finite(kyh) && key_finite(kyl);
    const double hx = key_up(kxh), lx = key_up(kxl), hy = key_up(kyh), ly = key_up(kyl);
    const double bx = hx + lx, by = hy + ly;  // >= max x - min x, max y - min y
    const double E2 = (bx * bx + by * by) * (1.0 + 0x1p-20);
    const double Rb = (fmax(hx, lx) + fmax(hy, ly)) * (1.0 + 0x1p-40);  // >= max|x| + max|y|
    cc.finite = cc.finite && E2 < __builtin_inf();
    cc.scan = 0;
    cc.tq = 0.0;
    cc.margin = 0.0;
    cc.c_lo = count_cut(-1.0);
    cc.c_hi = count_cut(0.0);
    if (cc.finite && ecut < __builtin_inf()) {
        // Reassociated cross product r = fl(x uy - fl(y ux + k)) (two fmas), k = ox uy - oy ux per
        // hypothesis, with the band widened by the R sqrt(ecut) term (see count_kernel;
        // ecut_q = sqrt(ecut) * 1.01 + 1 from the host) and tested as two cutoffs on |r|
        cc.margin = (E2 + ecut + Rb * ecut_q) * 0x1p-42;
        cc.c_lo = cut_lo_of(ecut - cc.margin);
        cc.c_hi = cut_hi_of(ecut + cc.margin);
        const double sE = (double)__builtin_amdgcn_sqrtf((float)E2) * (1.0 + 0x1p-20);  // >= sqrt(E2)
        cc.tq = E2 + Rb * (sE + 1.0);
    }
    return cc;
}
__device__ __forceinline__ ChunkCut cut_finish(BoxAcc b, double ecut, double ecut_q) {
    return cut_from_keys(wave_max_dpp(b.xh), wave_max_dpp(~b.xl), wave_max_dpp(b.yh), wave_max_dpp(~b.yl), ecut,
                         ecut_q);
}

// pcut: the chunk's box terms and cutoffs computed ahead (cut_lane_kernel), or null
__device__ ChunkOut chunk_consensus(const KArgs &a, double2 *P, const double2 *gP, int N, const int32_t *draws,
                                    int32_t *cnt, int32_t *tied, double *tsum, uint8_t *mk, double *vtmp,
                                    double *vstack, int *nstack, int32_t *cnt_out, int lane, const ChunkCut *pcut,
                                    unsigned long long *chdbg = nullptr) {
    CH_STAMP_DECL
    const int T = a.T;
    const double ecut = a.ecut;
    const ChunkCut cc = pcut ? *pcut : chunk_cut(P, N, ecut, a.ecut_q, lane);
    if (N > 128 || !cc.finite || !(ecut < __builtin_inf()))
        return chunk_ransac(a, P, N, draws, cnt, tied, tsum, mk, vstack, nstack, cnt_out, lane);

    ChunkOut o;
    o.flags = 0;
    o.best = -1;
    o.stop = -1;
    o.n_inl = 0;
    o.last_inl = -1;
    o.n_draws = T + 1;
    // 2 FP64 ops + S + two counts per evaluation.  A lane whose counts differ (a point in the band)
    // or whose direction is not unit recounts exactly.
    const double margin = cc.margin;
    const cut_t c_lo = cc.c_lo, c_hi = cc.c_hi;
    int M = 0;
    CH_STAMP(1);
    for (int tb = 0; tb < T; tb += 64) {
        const int t = tb + lane;
        const int tt = t < T ? t : 0;
        const Model m = model2(P[draws[2 * tt]], P[draws[2 * tt + 1]]);
        const double un = m.ux * m.ux + m.uy * m.uy;
        const bool exact_all = !(fabs(un - 1.0) <= 0x1p-46);
        const double k = __builtin_fma(m.ox, m.uy, -(m.oy * m.ux));
        int lo = 0, hi = 0;
        double S = 0.0;
        if (gP) count_points_sgpr(gP, N, m.ux, m.uy, k, c_lo, c_hi, lo, hi, S);
        else count_points_lds(P, N, m.ux, m.uy, k, c_lo, c_hi, lo, hi, S);
        int c = lo;
        if (exact_all || lo != hi) {  // rare: lane-divergent exact recount
            c = 0;
            for (int q = 0; q < N; q++) {
                const double r = __builtin_fma(P[q].x, m.uy, -__builtin_fma(P[q].y, m.ux, k));
                const double v = r * r;
                bool in = v < ecut;
                if (exact_all || fabs(v - ecut) <= margin) in = resid2(P[q], m) < ecut;
                c += (int)in;
            }
        }
        if (t < T) {
            cnt[t] = c;
            tsum[t] = exact_all ? -1.0 : S;  // negative: no bracket, always a candidate
            if (cnt_out) cnt_out[t] = c;
        }
        M = max(M, wave_max_dpp(t < T ? c : 0));
    }
    M = uni(M);
    CH_STAMP(2);
    __syncthreads();
    // compact the max-count trials in trial order
    int ntied = 0;
    for (int tb = 0; tb < T; tb += 64) {
        const int t = tb + lane;
        const bool h = t < T && cnt[t] == M;
        const uint64_t bm = ballot(h);
        if (h) tied[ntied + (int)mbcnt(bm)] = t;
        ntied += popc64(bm);
    }
    __syncthreads();
    int best = -1;
    if (T > 0) {
        const bool need_sums = ntied > 1 || M == N || !(ecut > 0.0);
        if (!need_sums) {
            best = tied[0];
        } else {
            double U = __builtin_inf();
            for (int k = lane; k < ntied; k += 64) {
                const double S = tsum[tied[k]];
                if (S >= 0.0) U = fmin(U, S + tie_bound_q(S, N, cc.tq));
            }
            U = wave_min_d(U);
            // a single candidate wins without its exact sum unless the stop test
            // (sum == 0, only possible with M == N) could fire
            int ncand = 0, cand1 = -1;
            for (int kb = 0; kb < ntied; kb += 64) {
                const int k = kb + lane;
                bool cand = false;
                if (k < ntied) {
                    const double S = tsum[tied[k]];
                    cand = S < 0.0 || S - tie_bound_q(S, N, cc.tq) <= U;
                }
                const uint64_t cm = ballot(cand);
                if (cm && cand1 < 0) cand1 = kb + ffs64(cm);
                ncand += popc64(cm);
            }
            const bool lone = ncand == 1 && M < N && ecut > 0.0;
            if (lone) best = uni(tied[cand1]);
            int bcnt = 0;
            double bsum = __builtin_inf();
            for (int kb = 0; !lone && kb < ntied && o.stop < 0; kb += 64) {
                const int k = kb + lane;
                bool cand = false;
                if (k < ntied) {
                    const double S = tsum[tied[k]];
                    cand = S < 0.0 || S - tie_bound_q(S, N, cc.tq) <= U;
                }
                uint64_t cm = ballot(cand);
                while (cm) {
                    const int bit = ffs64(cm);
                    cm &= cm - 1ull;
                    const int t = uni(tied[kb + bit]);
                    const Model m = model2(P[draws[2 * t]], P[draws[2 * t + 1]]);
                    const double s = pw_sum_regs(P, N, m, lane);
                    if (M > bcnt || (M == bcnt && s < bsum)) {
                        best = t;
                        bcnt = M;
                        bsum = s;
                        if (bsum <= 0.0) {
                            o.stop = t;
                            break;
                        }
                    }
                }
            }
        }
    }
    CH_STAMP(3);
    const ChunkOut of = chunk_finish_fit(a, P, N, draws, mk, uni(best), o, lane);
    CH_STAMP(4);
    return of;
}

// mask (LDS copy + global) and A8 line parameters (ransac_functions.py:25-31).  A valid fit's
// mask was written by chunk_finish_fit's pass; any other outcome has no inliers.  P holds the
// inliers compacted (the tip is the last of them).
__device__ bool finish_chunk(const KArgs &a, const ChunkOut &o, const double2 *P, uint8_t *mk, int p0, int N,
                             lslam_chunk_model &rec, int lane) {
    const lslam_scan_batch &B = a.b;
    const bool valid = (o.flags & LSLAM_VALID) != 0;
    if (!valid)
        for (int p = lane; p < N; p += 64) mk[p] = 0;
    __syncthreads();
    if (B.inlier_mask)
        for (int p = lane; p < N; p += 64) B.inlier_mask[p0 + p] = mk[p];
    rec.n_inliers = valid ? o.n_inl : 0;
    rec.best_trial = o.best;
    rec.n_draws = o.n_draws;
    rec.flags = o.flags;
    if (valid) {
        const Model fm = o.m;
        const double av = fm.uy / fm.ux;
        const double bv = fm.oy - av * fm.ox;
        const double tx = P[o.last_inl].x;
        const double ty = tx * av + bv;
        rec.ox = fm.ox; rec.oy = fm.oy; rec.ux = fm.ux; rec.uy = fm.uy;
        rec.a = av; rec.b = bv; rec.tip_x = tx; rec.tip_y = ty;
        rec.proj_a = av; rec.proj_b = bv;
    }
    return valid;
}

// projected points y = pa x + pb of the inliers, 0 elsewhere (ransac_functions.py:46,49,53,55),
// with P holding the inliers compacted (chunk_finish_fit): point p's x is P[rank of p].x
__device__ __forceinline__ void chunk_yproj(double *y, const double2 *P, const uint8_t *mk, int N, bool have_model,
                                            double pa, double pb, int lane) {
    int base = 0;
    for (int pb0 = 0; pb0 < N; pb0 += 64) {
        const int p = pb0 + lane;
        const bool h = have_model && p < N && mk[p];
        const uint64_t bm = ballot(h);
        if (p < N) y[p] = h ? (pa * P[base + (int)mbcnt(bm)].x + pb) : 0.0;
        base += popc64(bm);
    }
}

// ------------------------------------------------------------------------
// landmark association (ransac_functions.py:34-54, landmarking.py:48-77)
// list in LDS: lmk[0..L)
// ------------------------------------------------------------------------
__device__ __forceinline__ bool is_equal(const lslam_landmark &Lk, double a, double b, double px, double py,
                                         double ex, double ey, const KArgs &ka) {
    const double distA = fabs(Lk.a - a);
    const double distB = fabs(Lk.b - b);
    const double vx = Lk.end_x - px, vy = Lk.end_y - py;
    const double eEO = __builtin_fma(vy, vy, vx * vx);
    const double wx = Lk.pos_x - ex, wy = Lk.pos_y - ey;
    const double eOE = __builtin_fma(wy, wy, wx * wx);
    // landmarking.py:57-72 compare the distances sqrt(e); sqrt is correctly rounded and monotone,
    // so RN(sqrt(e)) <= tol_dist  <=>  e <= tol_dist_sq (NaN: false either way)
    if (distA <= ka.tol_a && distB <= ka.tol_b) return (eEO <= ka.tol_dist_sq || eOE <= ka.tol_dist_sq);
    return false;
}

// returns match index (pre-call) or -1; updates list + count; proj line out
__device__ int associate(const KArgs &ka, lslam_landmark *lmk, uint64_t *vis, int &L, double a, double b,
                         double px, double py, double ex, double ey, int id, double &pa, double &pb,
                         bool &overflow, int32_t *walk_out, int lane, double2 *mpos = nullptr,
                         unsigned long long *st = nullptr) {
#ifdef LSLAM_STAMPS
    uint64_t _as_prev = lslam_stamp();
#define AS_STAMP(k)                                                    \
    do {                                                               \
        const uint64_t _t = lslam_stamp();                             \
        if (st && lane == 0) st[(k)] += _t - _as_prev;                 \
        _as_prev = _t;                                                 \
    } while (0)
#else
#define AS_STAMP(k) do {} while (0)
#endif
    const int nblk = (L + 63) >> 6;
    for (int i = lane; i < nblk; i += 64) vis[i] = 0ull;
    __syncthreads();
    int match = -1;
    int k = 0;
    // walk (ransac_functions.py:35-43) over pre-call indices: examine k; equal ->
    // stop; else decrease_life; if it died it is removed and `i += 1` then skips
    // the element that slid into its slot, i.e. pre-call index k+1.
    for (int blk = 0; blk < nblk && match < 0 && k < L; blk++) {
        if (k >= blk * 64 + 64) continue;
        const int j = blk * 64 + lane;
        bool eq = false, dies = false;
        if (j < L) {
            eq = is_equal(lmk[j], a, b, px, py, ex, ey, ka);
            dies = lmk[j].life <= 1;
        }
        const uint64_t E = ballot(eq);
        const uint64_t D = ballot(dies);
        AS_STAMP(12);
        // The walk as bit operations on the two ballots (a serial loop here was SALU and
        // branch bound: ~half the post pass beside the producer, whose parsers keep the CU's
        // scalar unit busy).  Position p is visited unless p-1 was visited and died (its
        // removal makes `i += 1` skip p): in a run of dying entries [r, e] that starts at a
        // visited position, r, r+2, r+4, ... are visited and r+1, r+3, ... (up to e+1) skipped.
        // Adding a run's start bit carries through the run, so Dm & ~(Dm + starts) selects the
        // runs by the parity of their start.  tests/test_assoc_walk_bits.py checks this form
        // against the serial walk on random lists of 1..200 entries.
        const int base = blk * 64;
        const int s0 = k - base;                   // 0, or 1 after a skip across the block end
        const int n = min(L, base + 64) - base;    // list positions in this block
        const uint64_t valid = n >= 64 ? ~0ull : ((1ull << n) - 1ull);
        const uint64_t ge = ~0ull << s0;
        const uint64_t Dm = D & valid & ge;
        const uint64_t run0 = Dm & ~(Dm << 1);     // first entry of each run of dying entries
        const uint64_t EVEN = 0x5555555555555555ull;
        const uint64_t Re = Dm & ~(Dm + (run0 & EVEN));        // runs starting at an even position
        const uint64_t EO = (Re & EVEN) | (Dm & ~Re & ~EVEN);  // even offset within their run
        const uint64_t visited = ge & valid & ~(EO << 1);
        const uint64_t hits = visited & E;
        uint64_t V;
        if (hits) {
            const int m = ffs64(hits);
            match = base + m;
            V = visited & ((1ull << m) - 1ull);
        } else {
            V = visited;
            k = n >= 64 ? base + 64 + (int)(EO >> 63) : base + n;
        }
        if (lane == 0) vis[blk] = V;
        __syncthreads();
    }
    AS_STAMP(9);
    pa = a;
    pb = b;
    if (match >= 0) {
        pa = unid(lmk[match].a);
        pb = unid(lmk[match].b);
        if (mpos) *mpos = make_double2(unid(lmk[match].pos_x), unid(lmk[match].pos_y));
    }
    // apply decrease_life / removal / reset_life, then compact in list order
    int w = 0;
    for (int blk = 0; blk < nblk; blk++) {
        const int j = blk * 64 + lane;
        const uint64_t V = vis[blk];
        lslam_landmark e;
        bool keep = false;
        if (j < L) {
            e = lmk[j];
            if ((V >> lane) & 1ull) {
                if (e.life > 0) e.life -= 1;
                keep = e.life != 0;
            } else {
                keep = true;
            }
            if (j == match) e.life = ka.life;
            if (walk_out) walk_out[j] = e.life;
        }
        const uint64_t km = ballot(keep);
        __syncthreads();
        if (keep) lmk[w + (int)mbcnt(km)] = e;
        w += popc64(km);
        __syncthreads();
    }
    L = w;
    AS_STAMP(10);
    overflow = false;
    if (match < 0) {
        if (L < ka.lmk_cap) {
            if (lane == 0) {
                lslam_landmark F;
                F.a = a; F.b = b; F.pos_x = px; F.pos_y = py; F.end_x = ex; F.end_y = ey;
                F.id = id; F.life = ka.life;
                lmk[L] = F;
            }
            L += 1;
        } else {
            overflow = true;
        }
    }
    __syncthreads();
    AS_STAMP(11);
    return match;
}

// ------------------------------------------------------------------------
// landmark map (LSLAM_UKF_MAP): a fitted chunk line (robot frame,
// ransac_functions.py:25-31) moved into the world frame of pose (tx, ty, th):
// p_w = R(th) p + t for the origin and the tip, the direction rotated, then
// a, b exactly as ransac_functions.py:26-27 form them.  At th = 0, t = 0 every
// value is unchanged bit for bit (c = 1, s = 0).
// ------------------------------------------------------------------------
struct MapLine {
    double a, b, px, py, ex, ey;
};
__device__ __forceinline__ MapLine to_world(const lslam_chunk_model &r, double c, double s, double tx, double ty) {
    MapLine w;
    w.px = (c * r.ox - s * r.oy) + tx;
    w.py = (s * r.ox + c * r.oy) + ty;
    w.ex = (c * r.tip_x - s * r.tip_y) + tx;
    w.ey = (s * r.tip_x + c * r.tip_y) + ty;
    const double ux = c * r.ux - s * r.uy;
    const double uy = s * r.ux + c * r.uy;
    w.a = uy / ux;
    w.b = w.py - w.a * w.px;
    return w;
}

// The measurement a chunk that matched map landmark j contributes (robot frame):
// is_equal (landmarking.py:66-77) matches any segment continuing the same wall,
// so the chunk's own origin may lie a segment length away from pos_j.  The
// measured point is instead the foot of pos_j (moved into the robot frame by the
// predicted pose) on the observed line o + t u; z = [|f|, atan2(f_y, f_x)] is
// compared with hx(x, pos_j) (UKFMethods.py:26-34).  Same wall => consistent.
__device__ __forceinline__ double2 observe_point(const lslam_chunk_model &r, double2 pw, double c, double s, double tx,
                                                 double ty) {
    const double dx = pw.x - tx, dy = pw.y - ty;
    const double qx = c * dx + s * dy;
    const double qy = c * dy - s * dx;
    const double t = (qx - r.ox) * r.ux + (qy - r.oy) * r.uy;
    const double fx = r.ox + t * r.ux;
    const double fy = r.oy + t * r.uy;
    return make_double2(cr_sqrt(fx * fx + fy * fy), atan2(fy, fx));
}

// ------------------------------------------------------------------------
// A9/A10 post pass over fitted models (ransac_functions.py:34-55, landmarking.py:48-77),
// not MAP mode.  The per-chunk loop of scan_body makes ~3 dependent HBM round trips per
// chunk (its record, its mask, its x); a post wave is one scan's serial chain, and beside
// the next call's producer (5 of a SIMD's 8 wave slots) a 4096-scan batch needs two rounds
// of post waves, so those round trips set the kernel's time.  Here the scan's records and
// chunk offsets come in with one 16-byte load per lane, the walk runs on LDS only, and the
// records and y_proj go out in flat passes (4 points per lane in flight).  Same values,
// same order of list updates as the loop.
// ------------------------------------------------------------------------
// diagnostic build only: post-pass phase cycles into dbg[(n_chunks + s) * 16 + k]
#ifdef LSLAM_STAMPS
#define PS_STAMP(k)                                                                               \
    do {                                                                                          \
        const uint64_t _t = lslam_stamp();                                                        \
        if (a.dbg && lane == 0) a.dbg[((size_t)a.b.n_chunks + s) * 16 + (k)] += _t - _ps_prev;  \
        _ps_prev = _t;                                                                            \
    } while (0)
#define PS_STAMP_DECL uint64_t _ps_prev = lslam_stamp();
#else
#define PS_STAMP(k) do {} while (0)
#define PS_STAMP_DECL
#endif
__device__ void post_assoc_fast(const KArgs &a, int s, int c0, int nchunks, int id0, lslam_landmark *lmk,
                                uint64_t *vis, int &L, double2 *corg, unsigned char *rbuf, int lane) {
    static_assert(sizeof(lslam_chunk_model) == 112, "a chunk record is 7 x 16 bytes");
    PS_STAMP_DECL
    const lslam_scan_batch &B = a.b;
    lslam_chunk_model *recs = (lslam_chunk_model *)rbuf;
    int32_t *off = (int32_t *)(rbuf + (((int)sizeof(lslam_chunk_model) * a.hist_cap + 15) & ~15));  // hist_cap = max_scan_chunks
    {
        const uint4 *src = (const uint4 *)(B.models + c0);
        uint4 *dst = (uint4 *)rbuf;
        for (int e = lane; e < nchunks * 7; e += 64) dst[e] = src[e];
        for (int e = lane; e <= nchunks; e += 64) off[e] = B.chunk_pt_off[c0 + e];
    }
    __syncthreads();
    PS_STAMP(1);
    int32_t *walk = B.lmk_walk ? B.lmk_walk + (size_t)s * a.lmk_cap : nullptr;
    for (int ci = 0; ci < nchunks; ci++) {
        lslam_chunk_model rec = recs[ci];
        rec.landmark_id = id0 + ci;
        const bool have_model = (rec.flags & LSLAM_VALID) != 0;
        if (ci < a.corg_cap && lane == 0)
            corg[ci] = have_model ? make_double2(rec.ox, rec.oy) : make_double2(__builtin_nan(""), __builtin_nan(""));
        if (have_model) {
            double pa, pb;
            bool overflow = false;
#ifdef LSLAM_STAMPS
            unsigned long long *st = a.dbg ? a.dbg + ((size_t)a.b.n_chunks + s) * 16 : nullptr;
#else
            unsigned long long *st = nullptr;
#endif
            const int m = associate(a, lmk, vis, L, rec.a, rec.b, rec.ox, rec.oy, rec.tip_x, rec.tip_y,
                                    rec.landmark_id, pa, pb, overflow, walk, lane, nullptr, st);
            rec.match_index = m;
            rec.proj_a = pa;
            rec.proj_b = pb;
            rec.flags |= (m >= 0) ? LSLAM_MATCHED : LSLAM_NEW_LANDMARK;
            if (overflow) rec.flags |= LSLAM_CAPACITY;
        }
        __syncthreads();  // every lane has its copy of recs[ci]
        if (lane == 0) recs[ci] = rec;
    }
    __syncthreads();
    PS_STAMP(2);
    {
        const uint4 *src = (const uint4 *)rbuf;
        uint4 *dst = (uint4 *)(B.models + c0);
        for (int e = lane; e < nchunks * 7; e += 64) dst[e] = src[e];
    }
    PS_STAMP(3);
    if (!B.y_proj) return;
    // y_proj: point q of chunk ci (off[ci] <= q < off[ci + 1]); a lane's points ascend, so
    // its chunk index only moves forward
    const int q0 = off[0], q1 = off[nchunks];
    int ci = 0;
    for (int qb = q0; qb < q1; qb += 4 * 64) {
        uint8_t mk[4];
        double xs[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int q = qb + u * 64 + lane;
            mk[u] = 0;
            xs[u] = 0.0;
            if (q < q1) {
                mk[u] = B.inlier_mask[q];
                xs[u] = B.xy ? B.xy[2 * (size_t)q] : polar_xy(B.theta_deg[q], B.dist_mm[q]).x;
            }
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int q = qb + u * 64 + lane;
            if (q < q1) {
                while (ci + 1 < nchunks && off[ci + 1] <= q) ci++;
                const lslam_chunk_model &r = recs[ci];
                const bool have_model = (r.flags & LSLAM_VALID) != 0;
                B.y_proj[q] = (have_model && mk[u]) ? (r.proj_a * xs[u] + r.proj_b) : 0.0;
            }
        }
    }
    PS_STAMP(4);
}

// ------------------------------------------------------------------------
// The same post pass with the scan's landmark list in registers (lmk_cap <= 64: entry i in
// lane i).  Beside the next call's producer the post pass was bound by its LDS (4.8 KiB per
// wave, 3.6 of them the list: ~9 waves per CU); here it holds 1.2 KiB.  The walk is the same
// bit operations on the same ballots (associate), removal is a compaction by ds_permute (kept
// entries to their rank, removed ones above the new length), the matched entry's line is read
// with a lane shuffle before the list changes.  Same values, same list order.
// ------------------------------------------------------------------------
struct LmkReg {
    double a, b, px, py, ex, ey;
    int id, life;
};

__device__ __forceinline__ bool is_equal_reg(const LmkReg &Lk, double a, double b, double px, double py, double ex,
                                             double ey, const KArgs &ka) {
    const double distA = fabs(Lk.a - a);
    const double distB = fabs(Lk.b - b);
    const double vx = Lk.ex - px, vy = Lk.ey - py;
    const double eEO = __builtin_fma(vy, vy, vx * vx);
    const double wx = Lk.px - ex, wy = Lk.py - ey;
    const double eOE = __builtin_fma(wy, wy, wx * wx);
    if (distA <= ka.tol_a && distB <= ka.tol_b) return (eEO <= ka.tol_dist_sq || eOE <= ka.tol_dist_sq);
    return false;
}

__device__ __forceinline__ double permute_d(int addr, double v) {
    const long long u = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_ds_permute(addr, (int)(unsigned)u);
    const int hi = __builtin_amdgcn_ds_permute(addr, (int)(unsigned)(u >> 32));
    return __longlong_as_double(((long long)(unsigned)hi << 32) | (unsigned)lo);
}

__device__ int associate_reg(const KArgs &ka, LmkReg &e, int &L, double a, double b, double px, double py, double ex,
                             double ey, int id, double &pa, double &pb, bool &overflow, int32_t *walk_out, int lane) {
    const bool have = lane < L;
    bool eq = false, dies = false;
    if (have) {
        eq = is_equal_reg(e, a, b, px, py, ex, ey, ka);
        dies = e.life <= 1;
    }
    const uint64_t E = ballot(eq);
    const uint64_t D = ballot(dies);
    // the walk of associate() for one block starting at position 0 (see the comment there)
    int match = -1;
    uint64_t V = 0ull;
    if (L > 0) {
        const uint64_t valid = L >= 64 ? ~0ull : ((1ull << L) - 1ull);
        const uint64_t Dm = D & valid;
        const uint64_t run0 = Dm & ~(Dm << 1);
        const uint64_t EVEN = 0x5555555555555555ull;
        const uint64_t Re = Dm & ~(Dm + (run0 & EVEN));
        const uint64_t EO = (Re & EVEN) | (Dm & ~Re & ~EVEN);
        const uint64_t visited = valid & ~(EO << 1);
        const uint64_t hits = visited & E;
        V = visited;
        if (hits) {
            const int m = ffs64(hits);
            match = m;
            V = visited & ((1ull << m) - 1ull);
        }
    }
    pa = a;
    pb = b;
    if (match >= 0) {
        pa = unid(__shfl(e.a, match));
        pb = unid(__shfl(e.b, match));
    }
    // decrease_life / removal / reset_life, then compaction in list order
    bool keep = false;
    if (have) {
        if ((V >> lane) & 1ull) {
            if (e.life > 0) e.life -= 1;
            keep = e.life != 0;
        } else {
            keep = true;
        }
        if (lane == match) e.life = ka.life;
        if (walk_out) walk_out[lane] = e.life;
    }
    const uint64_t km = ballot(keep);
    const int nL = popc64(km);
    if (nL != L) {  // something was removed: kept entries to their rank, the others above nL
        const int dst = keep ? (int)mbcnt(km) : nL + (int)mbcnt(~km);
        const int ad = dst << 2;
        e.a = permute_d(ad, e.a);
        e.b = permute_d(ad, e.b);
        e.px = permute_d(ad, e.px);
        e.py = permute_d(ad, e.py);
        e.ex = permute_d(ad, e.ex);
        e.ey = permute_d(ad, e.ey);
        e.id = __builtin_amdgcn_ds_permute(ad, e.id);
        e.life = __builtin_amdgcn_ds_permute(ad, e.life);
    }
    L = nL;
    overflow = false;
    if (match < 0) {
        if (L < ka.lmk_cap) {
            if (lane == L) {
                e.a = a; e.b = b; e.px = px; e.py = py; e.ex = ex; e.ey = ey;
                e.id = id; e.life = ka.life;
            }
            L += 1;
        } else {
            overflow = true;
        }
    }
    return match;
}

// staged: the scan's chunk records and offsets are copied into rbuf (LDS, max_scan_chunks =
// hist_cap records) and back; a scan with more chunks than the batch declared walks its records
// in place (HBM) and writes y_proj chunk by chunk: the same results, one extra load per record.
// STAGED (the scan's records fit the LDS area): the records are read through an LDS pointer (ds
// loads, lgkmcnt) instead of a generic one (FLAT loads that wait on every outstanding vector memory
// access, the y_proj prefetch included)
template <bool staged>
__device__ void post_assoc_reg_t(const KArgs &a, int s, unsigned char *rbuf, int lane) {
    PS_STAMP_DECL
    const lslam_scan_batch &B = a.b;
    const int c0 = B.scan_chunk_off[s], nchunks = B.scan_chunk_off[s + 1] - c0;
    const int id0 = B.id_base ? B.id_base[s] : 0;
    lslam_chunk_model *recs = staged ? (lslam_chunk_model *)rbuf : B.models + c0;
    int32_t *off = (int32_t *)(rbuf + (((int)sizeof(lslam_chunk_model) * a.hist_cap + 15) & ~15));
    if (staged) {
        const uint4 *src = (const uint4 *)(B.models + c0);
        uint4 *dst = (uint4 *)rbuf;
        for (int e = lane; e < nchunks * 7; e += 64) dst[e] = src[e];
        for (int e = lane; e <= nchunks; e += 64) off[e] = B.chunk_pt_off[c0 + e];
    }
    int L = min(uni(B.lmk_count[s]), a.lmk_cap);
    lslam_landmark *lst = B.landmarks + (size_t)s * a.lmk_cap;
    LmkReg e;
    if (lane < L) {
        const lslam_landmark g = lst[lane];
        e.a = g.a; e.b = g.b; e.px = g.pos_x; e.py = g.pos_y; e.ex = g.end_x; e.ey = g.end_y;
        e.id = g.id; e.life = g.life;
    } else {
        e.a = e.b = e.px = e.py = e.ex = e.ey = 0.0;
        e.id = 0;
        e.life = 0;
    }
    // y_proj's inputs (inlier flags and x of up to 768 points) are loaded now, after the list, so
    // that their latency runs under the association walk (loads complete in issue order: the
    // walk's wait for the list does not wait for them)
    constexpr int YPF = 12;
    const int yq0 = B.chunk_pt_off[c0], yq1 = B.chunk_pt_off[c0 + nchunks];
    const bool ypf = staged && B.y_proj && B.xy && yq1 - yq0 <= YPF * 64;
    double yx[YPF];
    asm volatile("" ::: "memory");
    if (ypf) {
        // unconditional loads (an index past the scan reads its first point, dropped at the use):
        // a conditional one ends in a merge that waits for the load right there.  The inlier
        // flags are loaded late, all at once (a byte load is widened, and so waited for, at once)
#pragma unroll
        for (int u = 0; u < YPF; u++) {
            const int q0u = yq0 + u * 64 + lane;
            yx[u] = B.xy[2 * (size_t)(q0u < yq1 ? q0u : yq0)];
        }
    }
    __syncthreads();
    PS_STAMP(1);
    int32_t *walk = B.lmk_walk ? B.lmk_walk + (size_t)s * a.lmk_cap : nullptr;
    for (int ci = 0; ci < nchunks; ci++) {
        // the record's fields read and written one by one (a copy of the whole record lived in
        // scratch memory): landmark_id always, the association's fields for a valid line
        lslam_chunk_model &R = recs[ci];
        const int flags = R.flags;
        const bool valid = (flags & LSLAM_VALID) != 0;
        const int lid = id0 + ci;
        int m = -1, nflags = flags;
        double pa = 0.0, pb = 0.0;
        if (valid) {
            bool overflow = false;
            m = associate_reg(a, e, L, R.a, R.b, R.ox, R.oy, R.tip_x, R.tip_y, lid, pa, pb, overflow, walk, lane);
            nflags |= (m >= 0) ? LSLAM_MATCHED : LSLAM_NEW_LANDMARK;
            if (overflow) nflags |= LSLAM_CAPACITY;
        }
        __syncthreads();  // every lane has read recs[ci]
        if (lane == 0) {
            R.landmark_id = lid;
            if (valid) {
                R.match_index = m;
                R.proj_a = pa;
                R.proj_b = pb;
                R.flags = nflags;
            }
        }
        if (!staged && B.y_proj) {
            const int q0 = B.chunk_pt_off[c0 + ci], q1 = B.chunk_pt_off[c0 + ci + 1];
            for (int q = q0 + lane; q < q1; q += 64) {
                const double x = B.xy ? B.xy[2 * (size_t)q] : polar_xy(B.theta_deg[q], B.dist_mm[q]).x;
                B.y_proj[q] = (valid && B.inlier_mask[q]) ? (pa * x + pb) : 0.0;
            }
        }
    }
    PS_STAMP(2);
    if (lane < L) {
        lslam_landmark g;
        g.a = e.a; g.b = e.b; g.pos_x = e.px; g.pos_y = e.py; g.end_x = e.ex; g.end_y = e.ey;
        g.id = e.id; g.life = e.life;
        lst[lane] = g;
    }
    if (lane == 0) B.lmk_count[s] = L;
    if (!staged) return;
    __syncthreads();
    {
        const uint4 *src = (const uint4 *)rbuf;
        uint4 *dst = (uint4 *)(B.models + c0);
        for (int k = lane; k < nchunks * 7; k += 64) dst[k] = src[k];
    }
    PS_STAMP(3);
    if (!B.y_proj) return;
    if (ypf) {
        uint32_t ym[YPF];
#pragma unroll
        for (int u = 0; u < YPF; u++) {
            const int q0u = yq0 + u * 64 + lane;
            ym[u] = B.inlier_mask[q0u < yq1 ? q0u : yq0];
        }
        int ci = 0;
#pragma unroll
        for (int u = 0; u < YPF; u++) {
            const int q = yq0 + u * 64 + lane;
            if (q < yq1) {
                while (ci + 1 < nchunks && off[ci + 1] <= q) ci++;
                const lslam_chunk_model &r = recs[ci];
                const bool have_model = (r.flags & LSLAM_VALID) != 0;
                B.y_proj[q] = (have_model && ym[u]) ? (r.proj_a * yx[u] + r.proj_b) : 0.0;
            }
        }
        PS_STAMP(4);
        return;
    }
    const int q0 = off[0], q1 = off[nchunks];
    int ci = 0;
    for (int qb = q0; qb < q1; qb += 4 * 64) {
        uint8_t mk[4];
        double xs[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int q = qb + u * 64 + lane;
            mk[u] = 0;
            xs[u] = 0.0;
            if (q < q1) {
                mk[u] = B.inlier_mask[q];
                xs[u] = B.xy ? B.xy[2 * (size_t)q] : polar_xy(B.theta_deg[q], B.dist_mm[q]).x;
            }
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int q = qb + u * 64 + lane;
            if (q < q1) {
                while (ci + 1 < nchunks && off[ci + 1] <= q) ci++;
                const lslam_chunk_model &r = recs[ci];
                const bool have_model = (r.flags & LSLAM_VALID) != 0;
                B.y_proj[q] = (have_model && mk[u]) ? (r.proj_a * xs[u] + r.proj_b) : 0.0;
            }
        }
    }
    PS_STAMP(4);
}
__device__ void post_assoc_reg(const KArgs &a, int s, unsigned char *rbuf, bool staged, int lane) {
    if (staged) post_assoc_reg_t<true>(a, s, rbuf, lane);
    else post_assoc_reg_t<false>(a, s, rbuf, lane);
}

// ------------------------------------------------------------------------
// the scan kernel
// ------------------------------------------------------------------------
template <int HYP, int MODE>
__device__ __forceinline__ void scan_body(const KArgs &a, const int s, unsigned char *smem) {
    const int lane = (int)threadIdx.x;
    const lslam_scan_batch &B = a.b;

    double2 *P = (double2 *)(smem + a.off_pts);
    uint32_t *key = (uint32_t *)(smem + a.off_key);
    int32_t *draws = (int32_t *)(smem + a.off_draws);
    int32_t *cnt = (int32_t *)(smem + a.off_cnt);
    int32_t *tied = (int32_t *)(smem + a.off_tied);
    double *tsum = (double *)(smem + a.off_tsum);
    uint8_t *mk = (uint8_t *)(smem + a.off_mask);
    double *vstack = (double *)(smem + a.off_vstack);
    int *nstack = (int *)(smem + a.off_nstack);
    uint32_t *snap = (uint32_t *)(smem + a.off_snap);  // MT state at the current chunk's start (rewind)
    double2 *corg = (double2 *)(smem + a.off_corg);
    double2 *zobs = (double2 *)(smem + a.off_zobs);
    lslam_landmark *lmk = (lslam_landmark *)(smem + a.off_lmk);
    uint64_t *vis = (uint64_t *)(smem + a.off_vis);

    const int c0 = B.scan_chunk_off[s], c1 = B.scan_chunk_off[s + 1];
    const int nchunks = c1 - c0;
    const int T = a.T;

    constexpr bool kRansac = (MODE & (MODE_RANSAC | MODE_HYP_ONLY)) != 0;
    constexpr bool use_mt = kRansac && HYP == LSLAM_HYP_MT19937;
    constexpr bool kPost = !kRansac && (MODE & (MODE_ASSOC | MODE_POST)) != 0;
    if (kRansac && a.fixup) {
        // fix-up pass after rng_kernel + chunk_kernel: only a scan with an
        // early-stopped chunk consumed a different stream; replay it whole
        bool any = false;
        for (int c = c0 + lane; c < c1; c += 64) any |= (B.models[c].flags & LSLAM_EARLY_STOP) != 0;
        // a speculative producer (map mode) parsed this scan from the previous call's end state
        // before that call's fix-up: if the fix-up replayed the scan, its draws are stale too
        if (a.spec_dirty_in && lane == 0) any |= a.spec_dirty_in[s] != 0;
        const bool replay = ballot(any) != 0ull;
        if (a.spec_dirty_out && lane == 0) a.spec_dirty_out[s] = replay ? 1 : 0;
        if (!replay) {
            // the producer's end state is the scan's
            if (B.mt_state_out && a.state_scr)
                for (int i = lane; i < 625; i += 64)
                    B.mt_state_out[(size_t)s * 625 + i] = a.state_scr[(size_t)s * 625 + i];
            return;
        }
    }

    MTWave mt;
    mt.key = key;
    mt.nxt = (uint32_t *)(smem + a.off_ring);
    mt.j1s = (uint32_t *)(smem + a.off_j1);
    mt.pos = MT_N;
#ifdef LSLAM_STAMPS
    for (int k = 0; k < 8; k++) mt.acc[k] = 0;
#endif

    auto mt_init = [&]() {
        if (B.mt_state_in) {
            const uint32_t *src = B.mt_state_in + (size_t)s * 625;
            for (int i = lane; i < MT_N; i += 64) key[i] = src[i];
            mt.pos = uni((int)src[624]);
            __syncthreads();
        } else {
            mt_seed(key, B.seeds ? B.seeds[s] : 0u, lane);
            mt.pos = MT_N;
        }
    };

    if (use_mt) mt_init();

    // the staged post passes hold the scan's chunk records in an LDS area of max_scan_chunks
    // (hist_cap) records: a scan with more chunks than the batch declared walks them in place
    // (post_assoc_reg) or takes the per-chunk loop below, with the same results
    // (test_gpu_bounds.py); only map mode's measurement slots end there (LSLAM_CHUNK_BOUND)
    const bool recs_fit = nchunks <= a.hist_cap;
    if constexpr (kPost && (MODE & MODE_ASSOC) != 0 && (MODE & MODE_UKF) == 0) {
        if (a.lmk_reg) {  // the list in registers (association-only post pass, lmk_cap <= 64)
            post_assoc_reg(a, s, smem + a.off_recs, recs_fit, lane);
            return;
        }
    }
    // landmark list of this scan -> LDS
    int L = 0;
    if (MODE & MODE_ASSOC) {
        if (B.landmarks) {
            L = uni(B.lmk_count[s]);
            if (L > a.lmk_cap) L = a.lmk_cap;
            const lslam_landmark *src = B.landmarks + (size_t)s * a.lmk_cap;
            for (int i = lane; i < L; i += 64) lmk[i] = src[i];
        }
        __syncthreads();
    }
    const int id0 = B.id_base ? B.id_base[s] : 0;

    // landmark MAP mode (LSLAM_UKF_MAP): predict first; the chunks' lines are
    // associated in the world frame of the predicted pose; matches feed the update
    constexpr bool kMapable = kPost && (MODE & MODE_ASSOC) && (MODE & MODE_UKF);
    const bool map_mode = kMapable && (a.ukf.flags & LSLAM_UKF_MAP);
    double mx[3], mP[9], mu[2];
    double cth = 1.0, sth = 0.0;
    int n_meas = 0;
    if (kMapable && map_mode) {
        for (int i = 0; i < 3; i++) mx[i] = B.ukf_x[3 * (size_t)s + i];
        for (int i = 0; i < 9; i++) mP[i] = B.ukf_P[9 * (size_t)s + i];
        mu[0] = B.ukf_u[2 * (size_t)s];
        mu[1] = B.ukf_u[2 * (size_t)s + 1];
        if (a.ukf.flags & LSLAM_UKF_PREDICT) {
            UkfLds us;
            us.carve((double *)(smem + a.off_ukf), a.ukf.L);
            ukf_step(mx, mP, mu[0], mu[1], nullptr, B.ukf_R_diag,
                     [](int, double &, double &) { return false; }, a.ukf, LSLAM_UKF_PREDICT, us, lane);
        }
        cth = cos(mx[2]);
        sth = sin(mx[2]);
    }

    bool chunks_done = false;
    if constexpr (kPost && (MODE & MODE_ASSOC) != 0) {
        if (!map_mode && a.off_recs >= 0 && recs_fit) {
            post_assoc_fast(a, s, c0, nchunks, id0, lmk, vis, L, corg, smem + a.off_recs, lane);
            chunks_done = true;
        }
    }
    for (int ci = 0; ci < nchunks && (kRansac || kPost) && !chunks_done; ci++) {
        const int c = c0 + ci;
        const int p0 = B.chunk_pt_off[c];
        const int N = B.chunk_pt_off[c + 1] - p0;
        lslam_chunk_model rec;
        memset(&rec, 0, sizeof(rec));
        rec.best_trial = -1;
        rec.match_index = -1;
        rec.landmark_id = id0 + ci;
        rec.n_points = N;
        bool have_model = false;
        if (kRansac) {
            if (ci < a.corg_cap && lane == 0) corg[ci] = make_double2(__builtin_nan(""), __builtin_nan(""));
            if (N < 3) {
                // fit.py:798-799: ValueError before any draw; nothing consumed
                rec.flags = LSLAM_N_TOO_SMALL;
                if (lane == 0 && B.models) B.models[c] = rec;
                for (int p = lane; p < N; p += 64) {
                    if (B.inlier_mask) B.inlier_mask[p0 + p] = 0;
                    if (B.y_proj) B.y_proj[p0 + p] = 0.0;
                }
                if (B.trial_cnt_out)  // no trials: a zero row (lidarslam.h)
                    for (int t = lane; t < a.T; t += 64) B.trial_cnt_out[(size_t)c * a.T + t] = 0;
                __syncthreads();
                continue;
            }
            // ---- A3: draws
            const int D = T + 1;
            int snap_pos = 0;
            if (use_mt && !(MODE & MODE_HYP_ONLY)) {  // the stream at the chunk's start, for an early stop
                for (int i = lane; i < MT_N; i += 64) snap[i] = key[i];
                snap_pos = mt.pos;
                __syncthreads();
            }
            if (HYP == LSLAM_HYP_MT19937) {
                mt_draws(mt, (uint32_t)N, (uint32_t)D, draws, true, lane);
            } else if (HYP == LSLAM_HYP_PHILOX) {
                philox_draws((uint32_t)N, (uint32_t)D, (uint32_t)c, a.philox_seed, draws, lane);
            } else {
                const int32_t *h = B.hyp + (size_t)c * 2 * D;
                for (int i = lane; i < 2 * D; i += 64) draws[i] = h[i];
                __syncthreads();
            }
            if (B.draws_out) {
                int32_t *dst = B.draws_out + (size_t)c * 2 * D;
                for (int i = lane; i < 2 * D; i += 64) dst[i] = draws[i];
            }
            if (MODE & MODE_HYP_ONLY) {
                __syncthreads();
                continue;
            }
            // ---- stage the chunk's points in LDS (16 B per lane, coalesced)
            stage_points(B, p0, N, P, lane);
            __syncthreads();
            // ---- A4-A7
            const ChunkOut o = chunk_ransac(a, P, N, draws, cnt, tied, tsum, mk, vstack, nstack,
                                            B.trial_cnt_out ? B.trial_cnt_out + (size_t)c * T : nullptr, lane);
            if (use_mt && o.n_draws < D) {
                // early stop: rewind the stream to the chunk's start, then exactly o.n_draws draws
                // (the snapshot holds any number of chunks: max_scan_chunks does not bound it)
                __syncthreads();
                for (int i = lane; i < MT_N; i += 64) key[i] = snap[i];
                mt.pos = snap_pos;
                __syncthreads();
                mt_draws(mt, (uint32_t)N, (uint32_t)o.n_draws, nullptr, false, lane);
            }
            have_model = finish_chunk(a, o, P, mk, p0, N, rec, lane);
            if (have_model && ci < a.corg_cap && lane == 0) corg[ci] = make_double2(rec.ox, rec.oy);
        } else {
            // post pass: models and masks come from a previous ransac launch
            rec = B.models[c];
            rec.landmark_id = id0 + ci;  // id_base as this pass reads it (MAP mode advances it)
            have_model = (rec.flags & LSLAM_VALID) != 0;
            if (ci < a.corg_cap && lane == 0)
                corg[ci] = have_model ? make_double2(rec.ox, rec.oy) : make_double2(__builtin_nan(""), __builtin_nan(""));
            if (MODE & MODE_ASSOC)
                for (int p = lane; p < N; p += 64) mk[p] = B.inlier_mask[p0 + p];
            __syncthreads();
        }

        // ---- A9/A10 association + projection
        if (MODE & MODE_ASSOC) {
            if (kMapable && map_mode) {
                if (ci < a.corg_cap && lane == 0) corg[ci] = make_double2(__builtin_nan(""), __builtin_nan(""));
            }
            if (kMapable && map_mode && have_model) {
                // the chunk's line in the world frame of the predicted pose
                const MapLine w = to_world(rec, cth, sth, mx[0], mx[1]);
                double pa, pb;
                bool overflow = false;
                double2 mp = make_double2(0.0, 0.0);
                const int m = associate(a, lmk, vis, L, w.a, w.b, w.px, w.py, w.ex, w.ey, rec.landmark_id, pa, pb,
                                        overflow, B.lmk_walk ? B.lmk_walk + (size_t)s * a.lmk_cap : nullptr, lane,
                                        &mp);
                rec.match_index = m;
                rec.flags |= (m >= 0) ? LSLAM_MATCHED : LSLAM_NEW_LANDMARK;
                if (overflow) rec.flags |= LSLAM_CAPACITY;
                if (m >= 0 && ci >= a.corg_cap) rec.flags |= LSLAM_CHUNK_BOUND;  // no measurement slot
                if (m >= 0 && ci < a.corg_cap) {
                    // measurement of map landmark m (hx = range/bearing of its pos): the point of the
                    // observed line nearest to that pos seen from the predicted pose (observe_point)
                    if (lane == 0) {
                        corg[ci] = mp;
                        zobs[ci] = observe_point(rec, mp, cth, sth, mx[0], mx[1]);
                    }
                    n_meas++;
                }
            } else if (have_model) {
                double pa, pb;
                bool overflow = false;
                const int m = associate(a, lmk, vis, L, rec.a, rec.b, rec.ox, rec.oy, rec.tip_x, rec.tip_y,
                                        rec.landmark_id, pa, pb, overflow,
                                        B.lmk_walk ? B.lmk_walk + (size_t)s * a.lmk_cap : nullptr, lane);
                rec.match_index = m;
                rec.proj_a = pa;
                rec.proj_b = pb;
                rec.flags |= (m >= 0) ? LSLAM_MATCHED : LSLAM_NEW_LANDMARK;
                if (overflow) rec.flags |= LSLAM_CAPACITY;
            }
        }
        if (B.y_proj && (kRansac || (MODE & MODE_ASSOC))) {
            const double pa = rec.proj_a, pb = rec.proj_b;
            if (B.xy) {
                for (int p = lane; p < N; p += 64) {
                    const double x = B.xy[2 * (size_t)(p0 + p)];
                    B.y_proj[p0 + p] = (have_model && mk[p]) ? (pa * x + pb) : 0.0;
                }
            } else {
                for (int p = lane; p < N; p += 64) {
                    const double x = polar_xy(B.theta_deg[p0 + p], B.dist_mm[p0 + p]).x;
                    B.y_proj[p0 + p] = (have_model && mk[p]) ? (pa * x + pb) : 0.0;
                }
            }
        }
        if (lane == 0 && B.models && (kRansac || (MODE & MODE_ASSOC))) B.models[c] = rec;
        __syncthreads();
    }

#ifdef LSLAM_STAMPS
    if (a.dbg && lane == 0)
        for (int k = 0; k < 8; k++) a.dbg[(size_t)s * 8 + k] = mt.acc[k];
#endif
    if (use_mt && B.mt_state_out) {
        uint32_t *dst = B.mt_state_out + (size_t)s * 625;
        for (int i = lane; i < MT_N; i += 64) dst[i] = key[i];
        if (lane == 0) dst[624] = (uint32_t)mt.pos;
    }
    if ((MODE & MODE_ASSOC) && B.landmarks) {
        lslam_landmark *dst = B.landmarks + (size_t)s * a.lmk_cap;
        for (int i = lane; i < L; i += 64) dst[i] = lmk[i];
        if (lane == 0) B.lmk_count[s] = L;
    }

    // ---- UKF update of MAP mode: the matched chunks are the measurements
    if (kMapable && map_mode) {
        __syncthreads();
        if ((a.ukf.flags & LSLAM_UKF_UPDATE) && n_meas > 0) {
            const int nslot = min(nchunks, a.corg_cap);
            auto slot_fn = [&](int j, double &px, double &py) {
                if (j >= nslot) return false;
                const double2 q = corg[j];
                px = q.x;
                py = q.y;
                return q.x == q.x;
            };
            UkfLds us;
            us.carve((double *)(smem + a.off_ukf), a.ukf.L);
            ukf_step(mx, mP, mu[0], mu[1], (const double *)zobs, B.ukf_R_diag, slot_fn, a.ukf, LSLAM_UKF_UPDATE, us,
                     lane);
        }
        if (lane == 0) {
            for (int i = 0; i < 3; i++) B.ukf_x[3 * (size_t)s + i] = mx[i];
            for (int i = 0; i < 9; i++) B.ukf_P[9 * (size_t)s + i] = mP[i];
            // landmarkNumber += 1 per chunk (ransac_functions.py:77): the map's id source is in/out
            if (B.id_base) const_cast<int32_t *>(B.id_base)[s] = id0 + nchunks;
        }
    }
    // ---- UKF step (U1-U8)
    if ((MODE & MODE_UKF) && !map_mode) {
        __syncthreads();
        double x[3], Pm[9], u[2];
        for (int i = 0; i < 3; i++) x[i] = B.ukf_x[3 * (size_t)s + i];
        for (int i = 0; i < 9; i++) Pm[i] = B.ukf_P[9 * (size_t)s + i];
        u[0] = B.ukf_u[2 * (size_t)s];
        u[1] = B.ukf_u[2 * (size_t)s + 1];
        const int Lu = a.ukf.L;
        const double *lm = B.ukf_lmk + (size_t)s * 2 * Lu;
        // no LMK_FROM_RANSAC here: this one-wave step runs stand-alone (lslam_ukf_step with
        // LSLAM_UKF_MAP; no RANSAC in the call), and the fused pipeline never gives its post pass
        // a non-map UKF (lslam_scan_pipeline sends it to ukf_group_kernel, whose origins are not
        // capped by the LDS staging; checked on the host)
        auto lmk_fn = [&](int j, double &px, double &py) {
            px = lm[2 * j];
            py = lm[2 * j + 1];
            return true;
        };
        UkfLds us;
        us.carve((double *)(smem + a.off_ukf), Lu);
        ukf_step(x, Pm, u[0], u[1], B.ukf_z + (size_t)s * 2 * Lu, B.ukf_R_diag, lmk_fn, a.ukf, a.ukf.flags, us, lane);
        if (lane == 0) {
            for (int i = 0; i < 3; i++) B.ukf_x[3 * (size_t)s + i] = x[i];
            for (int i = 0; i < 9; i++) B.ukf_P[9 * (size_t)s + i] = Pm[i];
        }
    }
}
// Consumer kernels loop over their items with a grid capped at a few waves per
// CU (launch_cap): they then fill the issue slots the producer's chains leave
// idle instead of competing with them for residency (which made the producer's
// placement, and so the step time, vary from run to run).
// Two register budgets for the same body.  Left alone the compiler spends all
// 512 registers of a lone wave on the UKF (occupancy 1): right beside the MT
// producer (parity mode) that is what runs best, one post wave per SIMD taking
// few issue slots from the parsers.  Without the producer (Philox / explicit
// hypotheses, the stand-alone entry points) the waves_per_eu(4) build keeps a
// batch's 4 waves per SIMD resident: fused post pass 181 -> 88 us on C3.
template <int HYP, int MODE>
__global__ __launch_bounds__(64) void scan_kernel(const KArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    WAVE_CENSUS(a, a.fixup ? WC_FIXUP : WC_POST);
    for (int s = blockIdx.x; s < a.b.n_scans; s += gridDim.x) {
#ifdef LSLAM_STAMPS
        const uint64_t t0 = lslam_stamp();
#endif
        scan_body<HYP, MODE>(a, s, smem);
        __syncthreads();
#ifdef LSLAM_STAMPS
        if (!a.fixup && a.dbg && threadIdx.x == 0) {
            a.dbg[((size_t)a.b.n_chunks + s) * 16 + 7] += lslam_stamp() - t0;
            a.dbg[((size_t)a.b.n_chunks + s) * 16 + 8] = t0;
        }
#endif
    }
}
// The association-only post pass with the list in registers (lmk_cap <= 64) as its own kernel:
// inside scan_kernel it took the general scan body's register count (112 VGPRs), so only three
// of its waves fit per SIMD beside the producer's four; alone it needs what the walk needs.
__global__ __launch_bounds__(64) void post_reg_kernel(const KArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    WAVE_CENSUS(a, WC_POST);
    for (int s = blockIdx.x; s < a.b.n_scans; s += gridDim.x) {
#ifdef LSLAM_STAMPS
        const uint64_t t0 = lslam_stamp();
#endif
        const int nchunks = a.b.scan_chunk_off[s + 1] - a.b.scan_chunk_off[s];
        post_assoc_reg(a, s, smem + a.off_recs, nchunks <= a.hist_cap, (int)threadIdx.x);
        __syncthreads();
#ifdef LSLAM_STAMPS
        if (a.dbg && threadIdx.x == 0) {
            a.dbg[((size_t)a.b.n_chunks + s) * 16 + 7] += lslam_stamp() - t0;
            a.dbg[((size_t)a.b.n_chunks + s) * 16 + 8] = t0;
        }
#endif
    }
}
template <int HYP, int MODE>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4))) void scan_kernel_w4(const KArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    for (int s = blockIdx.x; s < a.b.n_scans; s += gridDim.x) {
        scan_body<HYP, MODE>(a, s, smem);
        __syncthreads();
    }
}

// UKF step of the fused pipeline on groups of Pg lanes per scan (lslam_ukf.h: ukf_step_group),
// after the association pass; the landmark slots [0, nchunks) take the scan's fitted chunk
// origins (LMK_FROM_RANSAC) exactly as the post pass's corg does (models with LSLAM_VALID)
// VAR != 0 (lslam_ukf_step's sigma cache / lslam_ukf_trace, lslam_ukf.h UKF_VAR_*) instantiates the same
// step with those extra loads and stores; the pipeline's launches are VAR = 0.
template <int VAR>
__global__ __launch_bounds__(256) void ukf_group_kernel(const KArgs a, int Pg, int fuse, double *trace) {
    const lslam_scan_batch &B = a.b;
    const int lane = (int)threadIdx.x & 63;
    const int g = lane & (Pg - 1);
    const int wave = (int)blockIdx.x * (int)(blockDim.x >> 6) + ((int)threadIdx.x >> 6);
    const int s = wave * (64 / Pg) + lane / Pg;
    WAVE_CENSUS(a, WC_UKF);
    if (s >= B.n_scans) return;  // whole groups only: the butterfly stays inside a group
    double x[3], Pm[9];
    for (int i = 0; i < 3; i++) x[i] = B.ukf_x[3 * (size_t)s + i];
    for (int i = 0; i < 9; i++) Pm[i] = B.ukf_P[9 * (size_t)s + i];
    const double u0 = B.ukf_u[2 * (size_t)s], u1 = B.ukf_u[2 * (size_t)s + 1];
    const int Lu = a.ukf.L;
    const double *lm = B.ukf_lmk + (size_t)s * 2 * Lu;
    const int c0 = B.scan_chunk_off[s];
    // fuse: a pipeline call's post pass, whose chunk models exist (the stand-alone step has none)
    const int nfuse = (fuse && (a.ukf.flags & LSLAM_UKF_LMK_FROM_RANSAC)) ? B.scan_chunk_off[s + 1] - c0 : 0;
    auto lmk_fn = [&](int j, double &px, double &py) {
        px = lm[2 * j];
        py = lm[2 * j + 1];
        if (j < nfuse) {
            const lslam_chunk_model &m = B.models[c0 + j];
            if (m.flags & LSLAM_VALID) {
                px = m.ox;
                py = m.oy;
            }
        }
        return true;
    };
    double *sio = (VAR & UKF_VAR_SIGMAS) ? B.ukf_sigmas + (size_t)s * 21 : nullptr;
    double *tr = (VAR & UKF_VAR_TRACE) ? trace + (size_t)s * ukf_tr_doubles(Lu) : nullptr;
    ukf_step_group<VAR>(x, Pm, u0, u1, B.ukf_z + (size_t)s * 2 * Lu, B.ukf_R_diag, lmk_fn, a.ukf, a.ukf.flags, g, Pg,
                        sio, tr);
    if (g == 0) {
        for (int i = 0; i < 3; i++) B.ukf_x[3 * (size_t)s + i] = x[i];
        for (int i = 0; i < 9; i++) B.ukf_P[9 * (size_t)s + i] = Pm[i];
    }
}

// lanes per scan: about two landmarks per lane, up to a wave (C3: 16 lanes, 4 scans per wave,
// one round of waves beside the producer; one landmark per lane: +1 % per C3 step, five: +2 %)
static void launch_ukf_group(const KArgs &k, int n_landmarks, hipStream_t stream, bool fuse, double *trace = nullptr) {
    int Pg = 1;
    while (Pg < (n_landmarks + 1) / 2 && Pg < 64) Pg <<= 1;
    const int per = 64 / Pg;
    // waves per workgroup: a workgroup's waves go to different SIMDs of one CU, so 4-wave groups
    // keep the 253-VGPR waves at one per SIMD, where single-wave groups stack two on some SIMDs
    // (full register file) and hold the next producer off that CU
    constexpr int wpg = 4;
    const int nwaves = (k.b.n_scans + per - 1) / per;
    const dim3 grid((unsigned)((nwaves + wpg - 1) / wpg)), block(64 * wpg);
    const int var = (trace ? UKF_VAR_TRACE : 0) | (k.b.ukf_sigmas ? UKF_VAR_SIGMAS : 0);
    switch (fuse ? 0 : var) {
        case 0: hipLaunchKernelGGL(ukf_group_kernel<0>, grid, block, 0, stream, k, Pg, fuse ? 1 : 0, nullptr); break;
        case 1: hipLaunchKernelGGL(ukf_group_kernel<1>, grid, block, 0, stream, k, Pg, 0, trace); break;
        case 2: hipLaunchKernelGGL(ukf_group_kernel<2>, grid, block, 0, stream, k, Pg, 0, nullptr); break;
        default: hipLaunchKernelGGL(ukf_group_kernel<3>, grid, block, 0, stream, k, Pg, 0, trace); break;
    }
}

// ------------------------------------------------------------------------
// rng_kernel: the chained parity stream of one scan -> every chunk's draws
// (lslam_rng_pipe.h)
// ------------------------------------------------------------------------
// RNG_PPW parser waves (one scan each) per workgroup, each twisting its own MT blocks: a
// 4096-scan batch holds 4 waves per SIMD, and the previous call's consumers run beside it in
// the other wave slots.
// numpy's init_genrand (mt19937_seed, the np.random.seed(s) of every scan's stream), one lane
// per scan.  The recurrence is sequential within a scan; the parser waves used to run it on one
// lane each before their first twist (scalar chain + one LDS write per word: ~4.1k counted
// instructions per scan of the producer's ~122k, SQ counters r05f).  Here 64 scans share a wave
// (3 VALU per word for all 64).  No LDS: it runs beside the previous call's producer and
// consumers (launch_seed), where a resident seed wave holding LDS could keep a producer
// workgroup off its CU; each lane stores its own scan's row of out[S][624] (10 MB per C3 call,
// merged in L2), and the producer's parsers read their rows coalesced.  Wave priority 2: above
// the consumers, below the parsers, so it is done long before the next producer launches.
__global__ __launch_bounds__(64) void seed_kernel(const uint32_t *__restrict__ seeds, int S, uint32_t *__restrict__ out) {
    __builtin_amdgcn_s_setprio(2);
    const int s = (int)blockIdx.x * 64 + (int)threadIdx.x;
    if (s >= S) return;
    uint32_t x = seeds ? seeds[s] : 0u;
    uint32_t *row = out + (size_t)s * MT_N;
#pragma unroll 8
    for (int i = 0; i < MT_N; i++) {
        row[i] = x;
        x = 1812433253u * (x ^ (x >> 30)) + (uint32_t)(i + 1);
    }
}

// The chunks' box terms and cutoffs (chunk_cut) one lane per chunk, launched with seed_kernel on
// the seeding stream beside the previous call (launch_seed), so the consensus on the context
// stream -- the longer of the pipeline's two loops at r06 -- reads 32 bytes per
// chunk instead of reducing its box over the wave (~220 of its ~3.3k instructions per chunk).
// The same key maxima as cut_finish's DPP reduction, so the same ChunkCut.
__global__ __launch_bounds__(64) void cut_lane_kernel(const KArgs a, ChunkCut *__restrict__ out) {
    __builtin_amdgcn_s_setprio(2);
    const lslam_scan_batch &B = a.b;
    const int c = (int)blockIdx.x * 64 + (int)threadIdx.x;
    if (c >= B.n_chunks) return;
    const int p0 = B.chunk_pt_off[c];
    const int N = B.chunk_pt_off[c + 1] - p0;
    BoxAcc b;
    if (B.xy) {
        const double2 *src = (const double2 *)B.xy + p0;
#pragma unroll 4
        for (int p = 0; p < N; p++) b.add(src[p]);
    } else {
        for (int p = 0; p < N; p++) b.add(polar_xy(B.theta_deg[p0 + p], B.dist_mm[p0 + p]));
    }
    ChunkCut cc = cut_from_keys(b.xh, ~b.xl, b.yh, ~b.yl, a.ecut, a.ecut_q);
    // owning scan (owning_scan's guess and search, per lane): the consensus wave then skips its
    // 64-bit division and dependent loads
    int g = (int)(((int64_t)c * B.n_scans) / (B.n_chunks > 0 ? B.n_chunks : 1));
    if (!(g < B.n_scans && B.scan_chunk_off[g] <= c && c < B.scan_chunk_off[g + 1])) {
        int lo = 0, hi = B.n_scans;
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (B.scan_chunk_off[mid] <= c) lo = mid;
            else hi = mid;
        }
        g = lo;
    }
    cc.scan = g;
    out[c] = cc;
}

constexpr int RNG_PPW = 4;
template <typename JT>
__global__ __launch_bounds__(64 * RNG_PPW) void rng_kernel(const KArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = (int)threadIdx.x & 63;
    const int wave = uni((int)threadIdx.x >> 6);
    const lslam_scan_batch &B = a.b;
    const uint32_t D = a.ep_nd > 0 ? (uint32_t)a.ep_nd : (uint32_t)a.T + 1u;  // draws of this launch
    WAVE_CENSUS(a, WC_RNG_PARSER);
    RngPipe rp;
    {
        unsigned char *base = smem + (size_t)wave * a.rng_pipe_bytes;
        rp.blk = (uint32_t *)(base + a.off_blk);
        rp.have = 0;  // block 0 = the initial state
        rp.tbl = nullptr;
        rp.tblK = 0;
    }
    // Shared reject tables: the workgroup's parsers claim up to two table Ks (K = N-1 <= RT_KMAX
    // of their chunks) and the workgroup loads those two tables once; a chunk whose K got no slot
    // is parsed in mask mode (same steps).  Per-parser tables held 4 x 3.5 KiB of each
    // workgroup's LDS: ~142 of a CU's 160 KiB with 4 workgroups, which left the consumers beside
    // the producer ~4 consensus waves per CU (wave census).
    int *kslot = (int *)(smem + a.off_stbl);
    uint32_t *stbl = (uint32_t *)(smem + a.off_stbl + 16);
    if (threadIdx.x < 2) kslot[threadIdx.x] = 0;
    const int s = (int)blockIdx.x * RNG_PPW + wave;
    // block 0 = the initial state (raw); flags
    if (s < B.n_scans) {
        if (B.mt_state_in) {
            const uint32_t *src = B.mt_state_in + (size_t)s * 625;
            for (int i = lane; i < MT_N; i += 64) rp.blk[i] = src[i];
        } else if (a.seed_state) {  // seeded by seed_kernel (a fresh state: pos = MT_N below)
            const uint32_t *src = a.seed_state + (size_t)s * MT_N;
            for (int i = lane; i < MT_N; i += 64) rp.blk[i] = src[i];
        } else {
            mt_seed(rp.blk, B.seeds ? B.seeds[s] : 0u, lane);
        }
    }
    __syncthreads();
    if (s < B.n_scans && lane == 0) {
        for (int c = B.scan_chunk_off[s]; c < B.scan_chunk_off[s + 1]; c++) {
            const int K = B.chunk_pt_off[c + 1] - B.chunk_pt_off[c] - 1;
            if (K < 2 || K > (int)RT_KMAX) continue;
            const int o = atomicCAS(kslot, 0, K);
            if (o == 0 || o == K) continue;
            (void)atomicCAS(kslot + 1, 0, K);  // taken by another K: no table, mask mode
        }
    }
    __syncthreads();
    // the claimed Ks, wave-uniform (SGPRs): the parser's table base then stays scalar, and a row's
    // LDS address costs one VALU (rt_window)
    const int kt0 = uni(kslot[0]), kt1 = uni(kslot[1]);
    for (int t = 0; t < 2; t++) {
        const int K = t ? kt1 : kt0;
        if (K == 0) continue;
        const uint32_t mK = 0xffffffffu >> __clz(K);
        const uint4 *src = (const uint4 *)(a.rt_all + (size_t)(K - 2) * RT_DWORDS);
        uint4 *dst = (uint4 *)(stbl + t * RT_DWORDS);
        const uint32_t n4 = (mK + 1u) * RT_ST / 4u;  // rows 0..mK (mK + 1 >= 4, a power of two)
        for (uint32_t e = threadIdx.x; e < n4; e += blockDim.x) dst[e] = src[e];
    }
    __syncthreads();
#ifdef LSLAM_WSTAMPS
    for (int k = 0; k < 8; k++) rp.wacc[k] = 0;
#endif
#ifdef LSLAM_STAMPS
    for (int k = 0; k < 8; k++) rp.acc[k] = 0;
    const uint64_t t_start = lslam_stamp();
    const uint64_t rt_start = __builtin_amdgcn_s_memrealtime();
#endif
    if (s >= B.n_scans) return;
    // ---- parser: its chain is the kernel's critical path
    const int c0 = B.scan_chunk_off[s], c1 = B.scan_chunk_off[s + 1];
    rp.total_steps = 0;
    rp.done_steps = 0;
    for (int c = c0; c < c1; c++) {
        const int N = B.chunk_pt_off[c + 1] - B.chunk_pt_off[c];
        if (N >= 3) rp.total_steps += D * (uint32_t)(N - 1);
    }
    rp_set_schedule(rp);
    rp.prio = RP_PRIO_TOP;
    set_prio_level(RP_PRIO_TOP);
    int blkno = 0;
    int pos = B.mt_state_in ? uni((int)B.mt_state_in[(size_t)s * 625 + 624]) : MT_N;
    JT *J = (JT *)a.jbuf;
    for (int c = c0; c < c1; c++) {
        const int p0 = B.chunk_pt_off[c];
        const int N = B.chunk_pt_off[c + 1] - p0;
        if (N < 3) continue;
        JT *Jc = J + (size_t)D * (size_t)p0;
        const int K = N - 1;
        // the priority schedule moves at chunk starts (a block switch is ~20 times as frequent)
        const int lvl = rp_level(rp, rp.done_steps);
        if (lvl != rp.prio) {
            rp.prio = lvl;
            set_prio_level(lvl);
        }
        const bool tbl = K <= (int)RT_KMAX && (kt0 == K || kt1 == K);
        if (tbl) {
            rp.tbl = stbl + (kt0 == K ? 0 : RT_DWORDS);
            rp.tblK = (uint32_t)K;
        }
        if (tbl && K >= 64) parse_chunk_tbl<true>(rp, blkno, pos, Jc, (uint32_t)N, D, lane);
        else if (tbl) parse_chunk_tbl<false>(rp, blkno, pos, Jc, (uint32_t)N, D, lane);
        else if (N >= 65) parse_chunk<true>(rp, blkno, pos, Jc, (uint32_t)N, D, lane);
        else parse_chunk<false>(rp, blkno, pos, Jc, (uint32_t)N, D, lane);
    }
    if (pos > MT_N) {  // the last window ran across the block end: its block is in (numpy twisted too)
        blkno += 1;
        pos -= MT_N;
    }
    if (B.mt_state_out) {
        uint32_t *o = B.mt_state_out + (size_t)s * 625;
        const uint32_t *kb = rp.blk + (blkno & 1) * MT_N;
        for (int i = lane; i < MT_N; i += 64) o[i] = kb[i];
        if (lane == 0) o[624] = (uint32_t)pos;
    }
#ifdef LSLAM_STAMPS
    rp.acc[7] = lslam_stamp() - t_start;
    rp.acc[4] = rt_start;  // residency census (100 MHz chip-wide clock)
    rp.acc[3] = __builtin_amdgcn_s_memrealtime();
#ifdef LSLAM_WSTAMPS
    if (a.dbg && lane == 0) {
        for (int k = 0; k < 8; k++) a.dbg[(size_t)s * 16 + k] = rp.acc[k];
        for (int k = 0; k < 8; k++) a.dbg[(size_t)s * 16 + 8 + k] = rp.wacc[k];
    }
#else
    if (a.dbg && lane == 0) {
        for (int k = 0; k < 8; k++) a.dbg[(size_t)s * 16 + k] = rp.acc[k];
        // placement census: HW_ID simd / cu / se of the parser, xcc
        a.dbg[(size_t)s * 16 + 8] = (uint32_t)__builtin_amdgcn_s_getreg(4 | (4 << 6) | (1 << 11));
        a.dbg[(size_t)s * 16 + 9] = (uint32_t)__builtin_amdgcn_s_getreg(4 | (8 << 6) | (3 << 11));
        a.dbg[(size_t)s * 16 + 10] = (uint32_t)__builtin_amdgcn_s_getreg(4 | (13 << 6) | (2 << 11));
        a.dbg[(size_t)s * 16 + 11] = (uint32_t)__builtin_amdgcn_s_getreg(20 | (0 << 6) | (3 << 11));
        a.dbg[(size_t)s * 16 + 13] = (uint32_t)__builtin_amdgcn_s_getreg(4 | (12 << 6) | (0 << 11));
    }
#endif
#endif
}

// ------------------------------------------------------------------------
// resolve_kernel: one wave per chunk, the producer's Fisher-Yates steps ->
// the chunk's T+1 draws (lslam_rng_pipe.h: resolve_chunk)
// ------------------------------------------------------------------------
template <typename JT>
__global__ __launch_bounds__(64) void resolve_kernel(const KArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = (int)threadIdx.x;
    const lslam_scan_batch &B = a.b;
    const uint32_t Dall = (uint32_t)a.T + 1u;
    const uint32_t D = a.ep_nd > 0 ? (uint32_t)a.ep_nd : Dall;  // draws of this launch (from ep_d0)
    for (int c = blockIdx.x; c < B.n_chunks; c += gridDim.x) {
        const int p0 = B.chunk_pt_off[c];
        const int N = B.chunk_pt_off[c + 1] - p0;
        if (N >= 3)
            resolve_chunk((const JT *)a.jbuf + (size_t)D * (size_t)p0, (uint32_t)N - 1u, D, (uint32_t)a.res_g, smem,
                          a.draws_scr + (size_t)c * 2 * Dall + 2 * (size_t)a.ep_d0, lane);
        __syncthreads();
    }
}

// The staged walk without LDS (u8 steps, C3): lanes = draws, each lane loads its own row 16
// steps at a time (one unaligned 16-byte load; the 64 rows of a group lie in ~50 cache lines
// that stay in the vector L1) and walks the bytes from registers.  Beside the producer, whose
// workgroups hold most of each CU's LDS, the staged resolve fits only ~2 waves per CU.
__device__ __forceinline__ uint4 load16_unaligned(const uint8_t *p) {
    uint4 v;
    __builtin_memcpy(&v, p, 16);
    return v;
}
__global__ __launch_bounds__(64) void resolve_reg_kernel(const KArgs a) {
    const int lane = (int)threadIdx.x;
    const lslam_scan_batch &B = a.b;
    const uint32_t Dall = (uint32_t)a.T + 1u;
    const uint32_t D = a.ep_nd > 0 ? (uint32_t)a.ep_nd : Dall;
    for (int c = blockIdx.x; c < B.n_chunks; c += gridDim.x) {
        const int p0 = B.chunk_pt_off[c];
        const int N = B.chunk_pt_off[c + 1] - p0;
        if (N < 3) continue;
        const uint32_t K = (uint32_t)N - 1u;
        const uint8_t *J = (const uint8_t *)a.jbuf + (size_t)D * (size_t)p0;
        int32_t *draws = a.draws_scr + (size_t)c * 2 * Dall + 2 * (size_t)a.ep_d0;
        for (uint32_t d0 = 0; d0 < D; d0 += 64) {
            const uint32_t d = d0 + (uint32_t)lane;
            const bool live = d < D;
            const uint8_t *row = J + (size_t)(live ? d : d0) * K;  // step i at row[K - i]
            uint32_t c0 = 0, c1 = 1;
            uint32_t i0 = 2;
            // 16 steps i0 .. i0 + 15 = bytes K - i0 - 15 .. K - i0, walked from the top byte down
            for (; i0 + 15u <= K; i0 += 16u) {
                const uint4 v = load16_unaligned(row + (K - i0 - 15u));
                const uint32_t w[4] = {v.w, v.z, v.y, v.x};
#pragma unroll
                for (int u = 0; u < 16; u++) {
                    const uint32_t i = i0 + (uint32_t)u;
                    const uint32_t j = ((w[u >> 2] >> (8 * (3 - (u & 3)))) & 0xffu) & step_mask(i);
                    c0 = (j == c0) ? i : c0;
                    c1 = (j == c1) ? i : c1;
                }
            }
            for (; i0 <= K; i0++) {
                const uint32_t j = (uint32_t)row[K - i0] & step_mask(i0);
                c0 = (j == c0) ? i0 : c0;
                c1 = (j == c1) ? i0 : c1;
            }
            if (live) {
                const uint32_t j1 = (uint32_t)row[K - 1u] & 1u;
                draws[2 * d] = (int32_t)((j1 == 0u) ? c1 : c0);
                draws[2 * d + 1] = (int32_t)((j1 == 0u) ? c0 : c1);
            }
        }
    }
}

// The register walk for K <= 127 and at most 128 draws (C3), with the whole row in
// registers before the walk starts.  resolve_reg_kernel loads 16 steps, walks them,
// then loads the next 16: between a wave's loads the other waves of its XCD stream
// their own rows (and the producer its steps) through the L2, so a cache line of
// the 64 rows was fetched from HBM ~4x per launch (PMC 1.21 GB read vs 0.29 GB of
// steps, profiles/r03a_rocprof.md).  Here a wave (one chunk, 64 draws) issues all
// of its rows' loads (up to 8 x 16 bytes per lane) back to back, so every line of
// its 64 rows is requested once, while it is in flight.
// Group t of a row is bytes [K - 16(t+1), K - 16t) = steps i = 16t+1 .. 16t+16 (step
// i at byte K - i); the lowest group may start up to 15 bytes before the row (the
// previous row, or the slot's front pad JBUF_FRONT) and walks only i <= K.
constexpr int RR_GROUPS = 8;  // K <= 127
constexpr size_t JBUF_FRONT = 128;  // bytes of a producer slot before its steps (resolve_reg8_kernel's loads)
// One step of both trackers, c = (j == c) ? i : c.  The two trackers are independent
// chains, so both compares are issued (masks in two SGPR pairs) before both selects; the
// v_mov of i between them gives each select the two VALU wait states gfx950 requires
// between a VALU write of a mask SGPR and v_cndmask reading it (the compiler's order --
// compare, select, compare, select through VCC -- padded every step with s_nops: ~475 per
// wave).  Only VALU instructions inside.
template <uint32_t I>
__device__ __forceinline__ void rr_step(uint32_t j, uint32_t &c0, uint32_t &c1) {
    uint64_t m0, m1;
    uint32_t iv;
    asm volatile(
        "v_cmp_eq_u32_e64 %[m0], %[j], %[c0]\n\t"
        "v_cmp_eq_u32_e64 %[m1], %[j], %[c1]\n\t"
        "v_mov_b32 %[iv], %[i]\n\t"
        "v_cndmask_b32_e64 %[c0], %[c0], %[iv], %[m0]\n\t"
        "v_cndmask_b32_e64 %[c1], %[c1], %[iv], %[m1]"
        : [c0] "+v"(c0), [c1] "+v"(c1), [m0] "=&s"(m0), [m1] "=&s"(m1), [iv] "=&v"(iv)
        : [j] "v"(j), [i] "i"(I));
}

// steps i = 16T+1+U .. 16T+16 of a row's group T (byte 15 - U), all indices compile-time
template <bool CHECK, uint32_t T, int U>
__device__ __forceinline__ void rr_walk_from(const uint32_t (&w)[4], uint32_t K, uint32_t &c0, uint32_t &c1) {
    if constexpr (U < 16) {
        constexpr uint32_t i = 16u * T + 1u + (uint32_t)U;
        if constexpr (i >= 2u) {  // step 1 (i = 1): j_1 decides the final swap, not a tracker step
            if (CHECK && i > K) return;
            constexpr int off = 15 - U;
            constexpr uint32_t nb = 32u - (uint32_t)__builtin_clz(i);  // mask(i) = 2^nb - 1
            const uint32_t j = __builtin_amdgcn_ubfe(w[off >> 2], (uint32_t)(8 * (off & 3)), nb);
            rr_step<i>(j, c0, c1);
        }
        rr_walk_from<CHECK, T, U + 1>(w, K, c0, c1);
    }
}

// Steps i <= 64: i is an inline constant of the selects, so no v_mov is needed; the next
// step's byte extract (independent of the trackers) stands between the compares and the
// selects as the second wait state: 5 VALU per step instead of 6.
template <uint32_t I>
__device__ __forceinline__ void rr_step_nx(uint32_t j, uint32_t &c0, uint32_t &c1, uint32_t &jn, uint32_t wn) {
    static_assert(I >= 2 && I < 64, "inline-constant step");
    constexpr int offn = 15 - (int)((I % 16u));        // byte of step I + 1 within its group
    constexpr uint32_t nbn = 32u - (uint32_t)__builtin_clz(I + 1u);
    uint64_t m0, m1;
    asm volatile(
        "v_cmp_eq_u32_e64 %[m0], %[j], %[c0]\n\t"
        "v_cmp_eq_u32_e64 %[m1], %[j], %[c1]\n\t"
        "v_bfe_u32 %[jn], %[wn], %[off], %[nb]\n\t"
        "v_cndmask_b32_e64 %[c0], %[c0], %[i], %[m0]\n\t"
        "v_cndmask_b32_e64 %[c1], %[c1], %[i], %[m1]"
        : [c0] "+v"(c0), [c1] "+v"(c1), [m0] "=&s"(m0), [m1] "=&s"(m1), [jn] "=&v"(jn)
        : [j] "v"(j), [wn] "v"(wn), [off] "i"(8 * (offn & 3)), [nb] "i"(nbn), [i] "i"(I));
}

// group T <= 3 (steps 16T+1 .. 16T+16 <= 64), j of the current step given
template <bool CHECK, uint32_t T, int U>
__device__ __forceinline__ void rr_walk_fast(const uint32_t (&w)[4], uint32_t K, uint32_t &c0, uint32_t &c1, uint32_t j) {
    if constexpr (U < 16) {
        constexpr uint32_t i = 16u * T + 1u + (uint32_t)U;
        if (CHECK && i > K) return;
        if constexpr (U < 15) {
            constexpr int offn = 15 - (U + 1);
            uint32_t jn;
            if constexpr (i >= 2u) {
                rr_step_nx<i>(j, c0, c1, jn, w[offn >> 2]);
            } else {  // step 1 decides the final swap, not a tracker step
                jn = __builtin_amdgcn_ubfe(w[offn >> 2], (uint32_t)(8 * (offn & 3)), 32u - (uint32_t)__builtin_clz(i + 1u));
            }
            rr_walk_fast<CHECK, T, U + 1>(w, K, c0, c1, jn);
        } else {
            rr_step<i>(j, c0, c1);
        }
    }
}

template <bool CHECK, uint32_t T>
__device__ __forceinline__ void rr_walk_group(const uint32_t (&ws)[4], uint32_t K, uint32_t &c0, uint32_t &c1) {
    if constexpr (T <= 3u) {  // 5-VALU steps for i <= 64 (rr_step_nx)
        constexpr uint32_t i0 = 16u * T + 1u;
        const uint32_t j0 = __builtin_amdgcn_ubfe(ws[3], 24u, 32u - (uint32_t)__builtin_clz(i0));  // byte 15
        rr_walk_fast<CHECK, T, 0>(ws, K, c0, c1, j0);
    } else {
        rr_walk_from<CHECK, T, 0>(ws, K, c0, c1);
    }
}

// A full group (all 16 steps <= the wave's longest K) as SDWA byte compares: 4 VALU per step
// instead of rr_step_nx's 5 (the byte extract goes) or rr_step's 6 (i > 64: no inline constant
// for the select, so a v_mov of i).  Per dword of 4 steps one pre-op: steps i <= 64 mask their
// bytes with mask(i) (one v_and with the 4 masks as a literal); steps i >= 65 all have mask 127
// = the stored byte's own bound, and run in the XOR-64 domain: the bytes and the trackers are
// XORed with 64 (a bijection on 0..127), so the select writes i ^ 64 = i - 64, an inline
// constant 1..63.  The trackers enter that domain at group 4 and leave it after the last full
// group (rr_walk_row).
// Wait states (gfx950; checked on the built code object by tests/test_isa_hazards.py): two
// between a v_cmp writing a mask SGPR pair and the v_cndmask reading it (the compiler's own
// requirement, tools/hazard_probe.hip), and -- conservatively -- one between a v_cndmask and
// the next SDWA compare, and between any VALU write of a VGPR and an SDWA read of it (the
// compiler's SDWA compare/select chains put an s_nop 0 there in most but not all places).
// Per step: cmp c0, cmp c1, F, select c0, select c1, G -- each compare two slots ahead of its
// select, each select at least one slot ahead of the next SDWA compare.  F and G are the next
// dwords' pre-ops where one is due, else s_nop 0 (waits inside dependency chains: ~free in
// issue, profiles/r05_ubench_issue.json).
#define RZ_CMP2(t, sel)                                                                  \
    "v_cmp_eq_u32_sdwa %[mA], %[" t "], %[c0] src0_sel:BYTE_" sel " src1_sel:DWORD\n\t" \
    "v_cmp_eq_u32_sdwa %[mB], %[" t "], %[c1] src0_sel:BYTE_" sel " src1_sel:DWORD\n\t"
#define RZ_SEL2(k)                                               \
    "v_cndmask_b32_e64 %[c0], %[c0], %[ib]+" k ", %[mA]\n\t" \
    "v_cndmask_b32_e64 %[c1], %[c1], %[ib]+" k ", %[mB]\n\t"
#define RZ_STEP(t, sel, k, F) RZ_CMP2(t, sel) F RZ_SEL2(k) RZ_NOP
#define RZ_NOP "s_nop 0\n\t"
#define RZ_AND(t, k) "v_and_b32_e32 %[" t "], %[M" k "], %[w" k "]\n\t"
#define RZ_XOR(t, k) "v_xor_b32_e32 %[" t "], 0x40404040, %[w" k "]\n\t"
// steps U = 1..15 of a group (byte 15 - U: dword 3 - U/4, byte 3 - U%4); step U = 0 is FIRST
#define RZ_GROUP(P, FIRST)                                                                        \
    P("tA", "3") P("tB", "2") FIRST RZ_STEP("tA", "2", "1", RZ_NOP) RZ_STEP("tA", "1", "2", RZ_NOP)  \
    RZ_STEP("tA", "0", "3", RZ_NOP) RZ_STEP("tB", "3", "4", P("tA", "1"))                            \
    RZ_STEP("tB", "2", "5", RZ_NOP) RZ_STEP("tB", "1", "6", RZ_NOP) RZ_STEP("tB", "0", "7", RZ_NOP)  \
    RZ_STEP("tA", "3", "8", P("tB", "0")) RZ_STEP("tA", "2", "9", RZ_NOP)                            \
    RZ_STEP("tA", "1", "10", RZ_NOP) RZ_STEP("tA", "0", "11", RZ_NOP) RZ_STEP("tB", "3", "12", RZ_NOP) \
    RZ_STEP("tB", "2", "13", RZ_NOP) RZ_STEP("tB", "1", "14", RZ_NOP) RZ_STEP("tB", "0", "15", RZ_NOP)
#define RZ_ENTER_X "v_xor_b32_e32 %[c0], 64, %[c0]\n\tv_xor_b32_e32 %[c1], 64, %[c1]\n\t"

// the 4 masks mask(i) of dword k's bytes (byte b <-> step i = 16T + 16 - 4k - b)
__host__ __device__ constexpr uint32_t rz_dword_masks(uint32_t T, uint32_t k) {
    uint32_t m = 0;
    for (uint32_t b = 0; b < 4; b++) {
        const uint32_t i = 16u * T + 16u - 4u * k - b;
        uint32_t mk = i;
        for (uint32_t sh = 1; sh < 32; sh <<= 1) mk |= mk >> sh;
        m |= (mk & 0xffu) << (8u * b);
    }
    return m;
}

template <uint32_t T>
__device__ __forceinline__ void rr_group_sdwa(const uint4 &w, uint32_t &c0, uint32_t &c1) {
    static_assert(T < (uint32_t)RR_GROUPS, "K <= 127");
    uint64_t mA, mB;
    uint32_t tA, tB;
    constexpr int ib = T >= 4u ? (int)(16u * T + 1u) - 64 : (int)(16u * T + 1u);
#define RZ_OPS                                                                                           \
    : [c0] "+v"(c0), [c1] "+v"(c1), [mA] "=&s"(mA), [mB] "=&s"(mB), [tA] "=&v"(tA), [tB] "=&v"(tB)    \
    : [w0] "v"(w.x), [w1] "v"(w.y), [w2] "v"(w.z), [w3] "v"(w.w), [ib] "i"(ib),                        \
      [M0] "i"(rz_dword_masks(T, 0)), [M1] "i"(rz_dword_masks(T, 1)), [M2] "i"(rz_dword_masks(T, 2)),  \
      [M3] "i"(rz_dword_masks(T, 3))
    if constexpr (T == 0u) {  // step 1 decides the final swap, not a tracker step
        asm volatile(RZ_GROUP(RZ_AND, "") RZ_OPS);
    } else if constexpr (T < 4u) {
        asm volatile(RZ_GROUP(RZ_AND, RZ_STEP("tA", "3", "0", RZ_NOP)) RZ_OPS);
    } else if constexpr (T == 4u) {
        asm volatile(RZ_ENTER_X RZ_GROUP(RZ_XOR, RZ_STEP("tA", "3", "0", RZ_NOP)) RZ_OPS);
    } else {
        asm volatile(RZ_GROUP(RZ_XOR, RZ_STEP("tA", "3", "0", RZ_NOP)) RZ_OPS);
    }
#undef RZ_OPS
}
#undef RZ_CMP2
#undef RZ_SEL2
#undef RZ_STEP
#undef RZ_NOP
#undef RZ_AND
#undef RZ_XOR
#undef RZ_GROUP
#undef RZ_ENTER_X

template <uint32_t T>
__device__ __forceinline__ void rr_full_groups(const uint4 (&w)[RR_GROUPS], uint32_t nfull, uint32_t &c0, uint32_t &c1) {
    if constexpr (T < (uint32_t)RR_GROUPS) {
        if (T < nfull) {
            rr_group_sdwa<T>(w[T], c0, c1);
            rr_full_groups<T + 1>(w, nfull, c0, c1);
        }
    }
}

template <uint32_t T>
__device__ __forceinline__ void rr_partial_group(const uint4 (&w)[RR_GROUPS], uint32_t K, uint32_t nfull, uint32_t &c0,
                                                 uint32_t &c1) {
    if constexpr (T < (uint32_t)RR_GROUPS) {
        if (T == nfull) {
            const uint32_t ws[4] = {w[T].x, w[T].y, w[T].z, w[T].w};
            rr_walk_group<true, T>(ws, K, c0, c1);
        } else {
            rr_partial_group<T + 1>(w, K, nfull, c0, c1);
        }
    }
}

// K: the wave's longest row (uniform).  K >> 4 full groups as SDWA compares, then the group
// holding step K (if any) step by step with its bound checked.
__device__ __forceinline__ void rr_walk_row(const uint4 (&w)[RR_GROUPS], uint32_t K, uint32_t &c0, uint32_t &c1) {
    const uint32_t nfull = K >> 4;
    rr_full_groups<0>(w, nfull, c0, c1);
    if (nfull > 4u) {  // leave the XOR-64 domain of groups 4..
        c0 ^= 64u;
        c1 ^= 64u;
    }
    rr_partial_group<0>(w, K, nfull, c0, c1);
}

// Invalid steps of a lane whose chunk is shorter than the wave's longest (packed waves, below):
// group t holds steps 16t+1 .. 16t+16 at bytes 15 .. 0, so steps past the lane's K are the group's
// low 16 - clamp(K - 16t, 0, 16) bytes; they get all their low 7 bits set, so the step's
// extraction yields mask(i) >= i > either tracker: never a match.
__device__ __forceinline__ void rr_poison(uint4 &w, uint32_t K, uint32_t t) {
    const int cnt = min(max((int)K - 16 * (int)t, 0), 16);  // valid steps of the group
    const int nbad = 16 - cnt;                                // its low nbad bytes
    uint32_t *d = (uint32_t *)&w;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int nb = min(max(nbad - 4 * k, 0), 4);  // invalid bytes of dword k (from its low end)
        d[k] |= (uint32_t)(0x7f7f7f7full & ((1ull << (8 * nb)) - 1ull));
    }
}

// Lanes are (chunk, draw) items of the whole launch in chunk-major order, 64 consecutive items
// per wave: a chunk's 101 draws no longer leave the second of its two waves 37 of 64 lanes,
// and a draw the consensus never reads (draw T: skimage draws it after its last trial,
// fit.py:826) is not resolved unless the caller asked for draws_out.  C3: 12.5 instead of 16
// waves per scan.  A wave whose lanes' chunks differ in size walks the longest chunk's steps,
// the shorter rows poisoned past their K (rr_poison).
__global__ __launch_bounds__(64) void resolve_reg8_kernel(const KArgs a, int Dres) {
    const int lane = (int)threadIdx.x;
    const lslam_scan_batch &B = a.b;
    const uint32_t Dall = (uint32_t)a.T + 1u;
    const uint32_t D = a.ep_nd > 0 ? (uint32_t)a.ep_nd : Dall;  // draws in the slot per chunk
    WAVE_CENSUS(a, WC_RESOLVE);
    const uint32_t total = (uint32_t)B.n_chunks * (uint32_t)Dres;  // < 2^31 (host)
    for (uint32_t wb = blockIdx.x * 64u; wb < total; wb += gridDim.x * 64u) {
        const uint32_t g = wb + (uint32_t)lane;
        const bool live = g < total;
        const int c = live ? (int)(g / (uint32_t)Dres) : 0;
        const uint32_t d = live ? g - (uint32_t)c * (uint32_t)Dres : 0u;
        const int p0 = B.chunk_pt_off[c];
        const int N = B.chunk_pt_off[c + 1] - p0;
        const bool act = live && N >= 3;
        const uint32_t K = act ? (uint32_t)N - 1u : 0u;  // <= 127 (host)
        const uint32_t kmax = (uint32_t)wave_max_dpp(act ? (int)K : 0);
        const uint32_t kmin = (uint32_t)-wave_max_dpp(act ? -(int)K : INT_MIN + 1);
        if (kmax < 2u) continue;
        const uint8_t *row = (const uint8_t *)a.jbuf + (size_t)D * (size_t)p0 + (size_t)d * K;
        uint4 w[RR_GROUPS];
#pragma unroll
        for (int t = 0; t < RR_GROUPS; t++)
            if ((uint32_t)(16 * t) < kmax) w[t] = load16_unaligned(row + (int)K - 16 * (t + 1));
        if (kmin != kmax) {
#pragma unroll
            for (int t = 0; t < RR_GROUPS; t++)
                if ((uint32_t)(16 * t) < kmax && (uint32_t)(16 * t + 16) > kmin) rr_poison(w[t], K, (uint32_t)t);
        }
        uint32_t c0 = 0, c1 = 1;
        rr_walk_row(w, kmax, c0, c1);
        if (act) {
            const uint32_t j1 = (w[0].w >> 24) & 1u;  // byte K - 1: step 1
            int32_t *draws = a.draws_scr + (size_t)c * 2 * Dall + 2 * (size_t)(a.ep_d0 + d);
            draws[0] = (int32_t)((j1 == 0u) ? c1 : c0);
            draws[1] = (int32_t)((j1 == 0u) ? c0 : c1);
        }
    }
}

// Chunks whose steps do not fit the 16 KiB stage (C5: 2049 draws x 4095 steps x 2 B = 16.8 MB
// per chunk), without LDS: one wave per (chunk, draw), lanes = 64 consecutive
// steps i of the draw, so each load is one coalesced 128-byte (u16) read
// straight from HBM and a wave keeps RW windows of loads in flight.  The
// trackers c0, c1 are wave-uniform: a window's matches j_i == c come out of one
// compare as a lane mask; the lowest matching lane l moves c to i0 + l, after
// which only lanes above l can match the new c (j_i <= i) - a hop is rare
// (probability 1/(i+1) per step).  Per window: one load, the mask, two compares.
template <typename JT, int RW>  // RW: windows of 64 steps in flight per wave
__global__ __launch_bounds__(64) void resolve_walk_kernel(const KArgs a) {
    const int lane = (int)threadIdx.x;
    const lslam_scan_batch &B = a.b;
    const uint32_t Dall = (uint32_t)a.T + 1u;
    const uint32_t D = a.ep_nd > 0 ? (uint32_t)a.ep_nd : Dall;  // draws of this launch (from ep_d0)
    const int64_t total = (int64_t)B.n_chunks * D;
    for (int64_t e = blockIdx.x; e < total; e += gridDim.x) {
        const int c = (int)(e / D);
        const uint32_t d = (uint32_t)(e - (int64_t)c * D);
        const int p0 = B.chunk_pt_off[c];
        const int N = B.chunk_pt_off[c + 1] - p0;
        if (N < 3) continue;
        const uint32_t K = (uint32_t)N - 1u;
        const JT *Jd = (const JT *)a.jbuf + (size_t)D * (size_t)p0 + (size_t)d * K;  // step i at K - i
        uint32_t c0 = 0, c1 = 1;
        auto track = [&](uint32_t jv, uint32_t i0) {
            uint64_t m0 = ballot(jv == c0), m1 = ballot(jv == c1);
            while (m0) {
                const int l = ffs64(m0);
                c0 = i0 + (uint32_t)l;
                m0 = ballot(jv == c0) & ((~0ull << l) << 1);
            }
            while (m1) {
                const int l = ffs64(m1);
                c1 = i0 + (uint32_t)l;
                m1 = ballot(jv == c1) & ((~0ull << l) << 1);
            }
        };
        // Groups of RW windows, their loads issued together; in the last group the lanes past K
        // read step K (in range) and never match.  Double-buffered: group g + 1's loads are in
        // flight while group g is walked (beside the next epoch's parsers a wave otherwise
        // waited out each group's load latency with nothing to issue).
        auto load_group = [&](uint32_t ib, uint32_t (&raw)[RW]) {
            if (ib + 64u * RW - 1u <= K) {
                const JT *q = Jd + (K - ib - (uint32_t)lane);
#pragma unroll
                for (int u = 0; u < RW; u++) raw[u] = (uint32_t)q[-64 * u];
            } else {
#pragma unroll
                for (int u = 0; u < RW; u++) {
                    const uint32_t i = ib + 64u * (uint32_t)u + (uint32_t)lane;
                    raw[u] = (uint32_t)Jd[K - (i <= K ? i : K)];
                }
            }
        };
        auto walk_group = [&](uint32_t ib, const uint32_t (&raw)[RW]) {
            if (ib + 64u * RW - 1u <= K) {
#pragma unroll
                for (int u = 0; u < RW; u++) {
                    const uint32_t i = ib + 64u * (uint32_t)u + (uint32_t)lane;
                    track(raw[u] & step_mask(i), ib + 64u * (uint32_t)u);
                }
            } else {
#pragma unroll
                for (int u = 0; u < RW; u++) {
                    const uint32_t i0 = ib + 64u * (uint32_t)u, i = i0 + (uint32_t)lane;
                    if (i0 > K) break;
                    track(i <= K ? (raw[u] & step_mask(i)) : 0xffffffffu, i0);
                }
            }
        };
        uint32_t rawA[RW], rawB[RW];
        if (2u <= K) load_group(2u, rawA);
        for (uint32_t ib = 2; ib <= K; ib += 128u * RW) {
            const uint32_t ib2 = ib + 64u * RW;
            if (ib2 <= K) load_group(ib2, rawB);
            walk_group(ib, rawA);
            if (ib2 > K) break;
            if (ib2 + 64u * RW <= K) load_group(ib2 + 64u * RW, rawA);
            walk_group(ib2, rawB);
        }
        if (lane == 0) {
            const uint32_t j1 = (uint32_t)Jd[K - 1u] & 1u;
            int32_t *draws = a.draws_scr + (size_t)c * 2 * Dall + 2 * (size_t)a.ep_d0;
            draws[2 * d] = (int32_t)((j1 == 0u) ? c1 : c0);
            draws[2 * d + 1] = (int32_t)((j1 == 0u) ? c0 : c1);
        }
    }
}

// ------------------------------------------------------------------------
// chunk_kernel: one wave per chunk, A4-A8 with the draws given
// ------------------------------------------------------------------------
template <int HYP>
__device__ __forceinline__ void chunk_body(const KArgs &a, const int c, unsigned char *smem) {
    const int lane = (int)threadIdx.x;
    const lslam_scan_batch &B = a.b;
    double2 *P = (double2 *)(smem + a.off_pts);
    int32_t *draws = (int32_t *)(smem + a.off_draws);
    int32_t *cnt = (int32_t *)(smem + a.off_cnt);
    int32_t *tied = (int32_t *)(smem + a.off_tied);
    double *tsum = (double *)(smem + a.off_tsum);
    uint8_t *mk = (uint8_t *)(smem + a.off_mask);
    double *vstack = (double *)(smem + a.off_vstack);
    int *nstack = (int *)(smem + a.off_nstack);
    double *vtmp = (double *)(smem + a.off_vtmp);

    const int s = a.cuts ? uni(a.cuts[c].scan) : owning_scan(B, c);
    const int p0 = B.chunk_pt_off[c];
    const int N = B.chunk_pt_off[c + 1] - p0;
    const int T = a.T;
#ifdef LSLAM_STAMPS
    unsigned long long *chdbg = a.dbg ? a.dbg + (size_t)c * 16 : nullptr;
#else
    unsigned long long *chdbg = nullptr;
#endif
    CH_STAMP_DECL
    lslam_chunk_model rec;
    memset(&rec, 0, sizeof(rec));
    rec.best_trial = -1;
    rec.match_index = -1;
    rec.landmark_id = (B.id_base ? B.id_base[s] : 0) + (c - B.scan_chunk_off[s]);
    rec.n_points = N;
    if (N < 3) {
        rec.flags = LSLAM_N_TOO_SMALL;
        if (lane == 0 && B.models) B.models[c] = rec;
        for (int p = lane; p < N; p += 64) {
            if (B.inlier_mask) B.inlier_mask[p0 + p] = 0;
            if (B.y_proj && a.write_yproj) B.y_proj[p0 + p] = 0.0;
        }
        if (B.trial_cnt_out)  // no trials: a zero row (lidarslam.h)
            for (int t = lane; t < a.T; t += 64) B.trial_cnt_out[(size_t)c * a.T + t] = 0;
        return;
    }
    const int D = T + 1;
    // explicit draws, or the parity stream's draws resolved by the resolve kernel, are read where
    // they lie (no LDS copy: beside the producer, whose workgroups hold most of each CU's LDS,
    // every KiB of ours is residency); Philox draws are generated into LDS
    const int32_t *dr = draws;
    if (HYP == LSLAM_HYP_PHILOX) {
        philox_draws((uint32_t)N, (uint32_t)D, (uint32_t)c, a.philox_seed, draws, lane);
        if (B.draws_out)
            for (int i = lane; i < 2 * D; i += 64) B.draws_out[(size_t)c * 2 * D + i] = draws[i];
    } else {
        const int32_t *h = (HYP == LSLAM_HYP_EXPLICIT ? B.hyp : a.draws_scr) + (size_t)c * 2 * D;
        dr = h;
        if (N <= 128 && B.xy) {
            double2 pv[2];
            const double2 *src = (const double2 *)B.xy + p0;
#pragma unroll
            for (int k = 0; k < 2; k++) pv[k] = (lane + 64 * k < N) ? src[lane + 64 * k] : make_double2(0.0, 0.0);
#pragma unroll
            for (int k = 0; k < 2; k++)
                if (lane + 64 * k < N) P[lane + 64 * k] = pv[k];
        } else {
            stage_points(B, p0, N, P, lane);
        }
        if (HYP == LSLAM_HYP_EXPLICIT && B.draws_out)
            for (int i = lane; i < 2 * D; i += 64) B.draws_out[(size_t)c * 2 * D + i] = h[i];
    }
    CH_STAMP(0);
    if (HYP == LSLAM_HYP_PHILOX) stage_points(B, p0, N, P, lane);
    __syncthreads();
    CH_STAMP(6);
    const double2 *gP = B.xy ? (const double2 *)B.xy + p0 : nullptr;
    const ChunkOut o = chunk_consensus(a, P, gP, N, dr, cnt, tied, tsum, mk, vtmp, vstack, nstack,
                                       B.trial_cnt_out ? B.trial_cnt_out + (size_t)c * T : nullptr, lane,
                                       a.cuts ? a.cuts + c : nullptr, chdbg);
    CH_STAMP_DECL_RESET
    const bool have_model = finish_chunk(a, o, P, mk, p0, N, rec, lane);
    if (B.y_proj && a.write_yproj) chunk_yproj(B.y_proj + p0, P, mk, N, have_model, rec.proj_a, rec.proj_b, lane);
    if (lane == 0 && B.models) B.models[c] = rec;
    CH_STAMP(5);
}

// At most 128 VGPRs (four waves per SIMD by registers): three consensus waves per SIMD then fit
// beside the producer's four parsers.  An unbounded build drifted to 132 after an unrelated edit
// and left two: consensus 0.382 vs 0.359 ms, step +3.4 % (r06g A/B).
template <int HYP>
__global__ __launch_bounds__(64, 4) void chunk_kernel(const KArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    WAVE_CENSUS(a, WC_CHUNK);
    for (int c = blockIdx.x; c < a.b.n_chunks; c += gridDim.x) {
        chunk_body<HYP>(a, c, smem);
        __syncthreads();
    }
}

// ------------------------------------------------------------------------
// Large chunks (N > 128, e.g. C5: 4096 points x 2048 hypotheses): the
// count pass is split from the selection so that it can use many waves per
// chunk:
//   model_kernel   one lane per trial: the 2-point model (A4) -> HBM
//   count_kernel   workgroup = one chunk x up to 1024 hypotheses; lanes hold
//                  points in registers, the hypothesis is wave-uniform (scalar
//                  loads, SGPR operands), so one test costs 4 FP64 ops + 2
//                  compares and the per-hypothesis count is a scalar popcount
//                  of the compare mask.  The cheap cross-product test of
//                  chunk_consensus is applied as two cutoffs on |r| (no
//                  squaring); a hypothesis with a point between them, a
//                  non-unit direction or non-finite data is recounted exactly.
//   select_kernel  one wave per chunk: max count, tied trials, tie brackets,
//                  exact pairwise sums of the candidates (lanes over points),
//                  then the same finish as chunk_kernel.
// ------------------------------------------------------------------------
constexpr int CNT_TPB = 256;          // 4 waves
constexpr int CNT_HYP_BLOCK = 1024;   // hypotheses per count workgroup

typedef const __attribute__((address_space(4))) double cdouble_t;  // scalar-load path

// bounding-box E2 and finiteness of P[0..N) (every lane gets the same values)
struct ChunkBox {
    double E2;
    bool finite;
};

template <typename Src>
__device__ __forceinline__ void box_partial(const Src src, int N, int tid, int nthr, double2 *P, double &xmn,
                                            double &xmx, double &ymn, double &ymx, bool &fin) {
    xmn = __builtin_inf(); xmx = -__builtin_inf(); ymn = __builtin_inf(); ymx = -__builtin_inf();
    fin = true;
    auto take = [&](int p, double2 q) {
        if (P) P[p] = q;
        xmn = fmin(xmn, q.x); xmx = fmax(xmx, q.x);
        ymn = fmin(ymn, q.y); ymx = fmax(ymx, q.y);
        fin = fin && (q.x - q.x == 0.0) && (q.y - q.y == 0.0);
    };
    int p = tid;
    // 8 independent loads in flight per lane
    for (; p + 7 * nthr < N; p += 8 * nthr) {
        double2 q[8];
#pragma unroll
        for (int j = 0; j < 8; j++) q[j] = src[p + j * nthr];
#pragma unroll
        for (int j = 0; j < 8; j++) take(p + j * nthr, q[j]);
    }
    for (; p < N; p += nthr) take(p, src[p]);
    xmn = wave_min_d(xmn); xmx = wave_max_d(xmx);
    ymn = wave_min_d(ymn); ymx = wave_max_d(ymx);
}

__device__ __forceinline__ ChunkBox box_finish(double xmn, double xmx, double ymn, double ymx, bool fin) {
    const double bx = xmx - xmn, by = ymx - ymn;
    ChunkBox b;
    b.E2 = (bx * bx + by * by) * (1.0 + 0x1p-20);
    b.finite = fin && b.E2 < __builtin_inf();
    return b;
}

// the hypothesis pair of trial t (draw t) of chunk c
template <int HYP>
__device__ __forceinline__ void trial_pair(const KArgs &a, int c, int N, int D, int t, int32_t &i0, int32_t &i1) {
    if (HYP == LSLAM_HYP_PHILOX) {
        philox_pair((uint32_t)N, (uint32_t)t, (uint32_t)c, a.philox_seed, i0, i1);
    } else {
        const int32_t *h = (HYP == LSLAM_HYP_EXPLICIT ? a.b.hyp : a.draws_scr) + ((size_t)c * D + t) * 2;
        i0 = h[0];
        i1 = h[1];
    }
}

// A4 for every trial of every large chunk (and the Philox draws they use)
template <int HYP>
__global__ __launch_bounds__(256) void model_kernel(const KArgs a) {
    const lslam_scan_batch &B = a.b;
    const int T = a.T, D = T + 1;
    const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (idx >= (int64_t)B.n_chunks * D) return;
    const int c = (int)(idx / D), t = (int)(idx % D);
    const int p0 = B.chunk_pt_off[c];
    const int N = B.chunk_pt_off[c + 1] - p0;
    if (N < 3) return;
    int32_t i0, i1;
    trial_pair<HYP>(a, c, N, D, t, i0, i1);
    if (HYP == LSLAM_HYP_PHILOX) {  // the draws select_kernel (and draws_out) read
        a.draws_scr[((size_t)c * D + t) * 2] = i0;
        a.draws_scr[((size_t)c * D + t) * 2 + 1] = i1;
    }
    if (t >= T) return;
    const PtSrc xy = batch_points(B) + p0;
    const Model m = model2(xy[i0], xy[i1]);
    double *o = a.models + ((size_t)c * T + t) * 4;
    *(double4 *)o = make_double4(m.ox, m.oy, m.ux, m.uy);
}

// PPL points per lane (a tile of 256 * PPL points per pass)
template <int PPL>
__global__ __launch_bounds__(CNT_TPB) void count_kernel(const KArgs a) {
    __shared__ int s_lo[CNT_HYP_BLOCK], s_hi[CNT_HYP_BLOCK];
    __shared__ uint8_t s_ex[CNT_HYP_BLOCK];
    __shared__ double s_box[4][4];
    __shared__ int s_fin[4];
    const lslam_scan_batch &B = a.b;
    const int c = (int)blockIdx.x / a.cnt_blocks;
    const int t0 = ((int)blockIdx.x % a.cnt_blocks) * CNT_HYP_BLOCK;
    const int tid = (int)threadIdx.x, w = tid >> 6, lane = tid & 63;
    const int p0 = B.chunk_pt_off[c];
    const int N = B.chunk_pt_off[c + 1] - p0;
    const int T = a.T;
    if (t0 >= T) return;
    const int nt = min(CNT_HYP_BLOCK, T - t0);
    if (N < 3) {  // no trials: a zero row (lidarslam.h)
        for (int h = (int)threadIdx.x; h < nt; h += CNT_TPB) a.cnt_scr[(size_t)c * T + t0 + h] = 0;
        return;
    }
    for (int h = tid; h < nt; h += CNT_TPB) {
        s_lo[h] = 0;
        s_hi[h] = 0;
        s_ex[h] = 0;
    }
    const PtSrc xy = batch_points(B) + p0;
    double xmn, xmx, ymn, ymx;
    bool fin;
    box_partial(xy, N, tid, CNT_TPB, nullptr, xmn, xmx, ymn, ymx, fin);
    const bool wfin = ballot(!fin) == 0ull;
    if (lane == 0) {
        s_box[w][0] = xmn; s_box[w][1] = xmx; s_box[w][2] = ymn; s_box[w][3] = ymx;
        s_fin[w] = wfin;
    }
    __syncthreads();
    xmn = fmin(fmin(s_box[0][0], s_box[1][0]), fmin(s_box[2][0], s_box[3][0]));
    xmx = fmax(fmax(s_box[0][1], s_box[1][1]), fmax(s_box[2][1], s_box[3][1]));
    ymn = fmin(fmin(s_box[0][2], s_box[1][2]), fmin(s_box[2][2], s_box[3][2]));
    ymx = fmax(fmax(s_box[0][3], s_box[1][3]), fmax(s_box[2][3], s_box[3][3]));
    const ChunkBox bx = box_finish(xmn, xmx, ymn, ymx, s_fin[0] && s_fin[1] && s_fin[2] && s_fin[3]);
    const double ecut = a.ecut;
    const bool cheap = bx.finite && ecut < __builtin_inf();
    // The main loop evaluates the cross product as r = fl(x uy - fl(y ux + k))
    // (two fmas), k = fl(ox uy - oy ux) per hypothesis: 2 FP64 ops instead of 4.
    // |y ux + k| <= 2R, so the inner rounding is <= 2uR, the outer <= u|r| and
    // k's own <= 2uR: against the direct fl(ex uy - ey ux) this adds at most
    // ~8 u R |r| to r^2 (R = max|x| + max|y| over the chunk box, which holds
    // o), so the band gets an R sqrt(ecut) term; 2^-42 leaves a factor 2^8 of
    // slack on it as on the E2 term.  Outside the band the cheap test decides
    // as before.
    const double Rb = fmax(fabs(xmn), fabs(xmx)) + fmax(fabs(ymn), fabs(ymx));
    const double margin = (bx.E2 + ecut + Rb * a.ecut_q) * 0x1p-42;
    // c2 < ecut - margin  <=  |r| below c_lo;   c2 > ecut + margin  <=  |r| above c_hi (cut_lo_of);
    // only for a cheap chunk (the exact square-root search would not end for ecut = inf)
    const cut_t c_lo = cheap ? cut_lo_of(ecut - margin) : count_cut(-1.0);
    const cut_t c_hi = cheap ? cut_hi_of(ecut + margin) : count_cut(0.0);
    cdouble_t *mp = (cdouble_t *)(a.models + ((size_t)c * T + t0) * 4);
    const double nan = __builtin_nan("");
    if (cheap) {
        for (int tile = 0; tile < N; tile += CNT_TPB * PPL) {
            double qx[PPL], qy[PPL];
#pragma unroll
            for (int j = 0; j < PPL; j++) {
                const int p = tile + (w * PPL + j) * 64 + lane;
                const double2 q = p < N ? xy[p] : make_double2(nan, nan);  // NaN: neither cutoff holds
                qx[j] = q.x;
                qy[j] = q.y;
            }
            int acc_lo = 0, acc_hi = 0;  // lane k: counts of hypothesis (t & ~63) + k
            double nox = mp[0], noy = mp[1], nux = mp[2], nuy = mp[3];
            for (int t = 0; t < nt; t++) {
                const double ox = nox, oy = noy, ux = nux, uy = nuy;
                if (t + 1 < nt) {  // next hypothesis' scalar loads in flight during this one
                    nox = mp[4 * t + 4]; noy = mp[4 * t + 5]; nux = mp[4 * t + 6]; nuy = mp[4 * t + 7];
                }
                const double k = __builtin_fma(ox, uy, -(oy * ux));
                uint32_t nlo = 0, nhi = 0;
#pragma unroll
                for (int j = 0; j < PPL; j++) {
                    const double r = __builtin_fma(qx[j], uy, -__builtin_fma(qy[j], ux, k));
                    nlo += (uint32_t)popc64(ballot(sure_in(r, c_lo)));
                    nhi += (uint32_t)popc64(ballot(maybe_in(r, c_hi)));
                }
                const bool mine = lane == (t & 63);
                acc_lo = mine ? (int)nlo : acc_lo;
                acc_hi = mine ? (int)nhi : acc_hi;
                if ((t & 63) == 63 || t == nt - 1) {
                    const int h = (t & ~63) + lane;
                    if (h <= t) {
                        atomicAdd(&s_lo[h], acc_lo);
                        atomicAdd(&s_hi[h], acc_hi);
                    }
                    acc_lo = 0;
                    acc_hi = 0;
                }
            }
        }
    }
    __syncthreads();
    // hypotheses the cutoffs cannot decide: non-unit direction (duplicate points),
    // a point between the cutoffs, or a chunk that is not finite
    for (int h = tid; h < nt; h += CNT_TPB) {
        const double ux = mp[4 * h + 2], uy = mp[4 * h + 3];
        const double un = ux * ux + uy * uy;
        s_ex[h] = (!cheap || !(fabs(un - 1.0) <= 0x1p-46) || s_lo[h] != s_hi[h]) ? 1 : 0;
    }
    __syncthreads();
    for (int hb = 0; hb < nt; hb += 64) {
      // the flagged hypotheses of this group of 64, one ballot instead of 64 LDS round trips
      uint64_t fm = ballot(hb + lane < nt && s_ex[hb + lane] != 0);
      while (fm) {
        const int h = hb + ffs64(fm);
        fm &= fm - 1ull;
        Model m;
        m.ox = mp[4 * h]; m.oy = mp[4 * h + 1]; m.ux = mp[4 * h + 2]; m.uy = mp[4 * h + 3];
        const double un = m.ux * m.ux + m.uy * m.uy;
        const bool exact_all = !cheap || !(fabs(un - 1.0) <= 0x1p-46);
        int cnt = 0;
        for (int p = tid; p < N; p += CNT_TPB) {
            const double2 q = xy[p];
            const double r = __builtin_fma(q.x - m.ox, m.uy, -((q.y - m.oy) * m.ux));
            const double v = r * r;
            bool in = v < ecut;
            if (exact_all || fabs(v - ecut) <= margin) in = resid2(q, m) < ecut;
            cnt += (int)in;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
        __syncthreads();
        if (tid == 0) s_lo[h] = 0;
        __syncthreads();
        if (lane == 0) atomicAdd(&s_lo[h], cnt);
        __syncthreads();
      }
    }
    for (int h = tid; h < nt; h += CNT_TPB) a.cnt_scr[(size_t)c * T + t0 + h] = s_lo[h];
}

// diagnostic build only: select_kernel phase cycles into dbg[c][8 + k]
#ifdef LSLAM_STAMPS
#define SEL_STAMP(k)                                                         \
    do {                                                                     \
        const uint64_t _t = lslam_stamp();                                   \
        if (a.dbg && lane == 0) a.dbg[(size_t)c * 16 + 8 + (k)] += _t - _sel_prev; \
        _sel_prev = _t;                                                      \
    } while (0)
#else
#define SEL_STAMP(k) do {} while (0)
#endif

template <int HYP>
__global__ __launch_bounds__(64) void select_kernel(const KArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int c = blockIdx.x;
    const int lane = (int)threadIdx.x;
    const lslam_scan_batch &B = a.b;
    double2 *P = (double2 *)(smem + a.off_pts);
    int32_t *tied = (int32_t *)(smem + a.off_tied);
    double *tsum = (double *)(smem + a.off_tsum);
    uint8_t *mk = (uint8_t *)(smem + a.off_mask);
    double *vst = (double *)(smem + a.off_vstack);
    int *nstack = (int *)(smem + a.off_nstack);
    double *vtmp = (double *)(smem + a.off_vtmp);
    const int s = owning_scan(B, c);
    const int p0 = B.chunk_pt_off[c];
    const int N = B.chunk_pt_off[c + 1] - p0;
    const int T = a.T, D = T + 1;
    lslam_chunk_model rec;
    memset(&rec, 0, sizeof(rec));
    rec.best_trial = -1;
    rec.match_index = -1;
    rec.landmark_id = (B.id_base ? B.id_base[s] : 0) + (c - B.scan_chunk_off[s]);
    rec.n_points = N;
    if (N < 3) {
        rec.flags = LSLAM_N_TOO_SMALL;
        if (lane == 0 && B.models) B.models[c] = rec;
        for (int p = lane; p < N; p += 64) {
            if (B.inlier_mask) B.inlier_mask[p0 + p] = 0;
            if (B.y_proj && a.write_yproj) B.y_proj[p0 + p] = 0.0;
        }
        if (B.trial_cnt_out)  // no trials: a zero row (lidarslam.h)
            for (int t = lane; t < a.T; t += 64) B.trial_cnt_out[(size_t)c * a.T + t] = 0;
        return;
    }
#ifdef LSLAM_STAMPS
    uint64_t _sel_prev = lslam_stamp();
#endif
    const int32_t *draws = (HYP == LSLAM_HYP_EXPLICIT ? B.hyp : a.draws_scr) + (size_t)c * 2 * D;
    if (HYP == LSLAM_HYP_EXPLICIT && B.draws_out)
        for (int i = lane; i < 2 * D; i += 64) B.draws_out[(size_t)c * 2 * D + i] = draws[i];
    double xmn, xmx, ymn, ymx;
    bool fin;
    box_partial(batch_points(B) + p0, N, lane, 64, P, xmn, xmx, ymn, ymx, fin);
    SEL_STAMP(0);
    const ChunkBox bx = box_finish(unid(xmn), unid(xmx), unid(ymn), unid(ymx), ballot(!fin) == 0ull);
    __syncthreads();
    const double ecut = a.ecut;
    const bool cheap = bx.finite && ecut < __builtin_inf();
    // the chunk's per-trial counts -> LDS (many loads in flight), then the max
    int32_t *cnt = (int32_t *)(smem + a.off_cnt);
    {
        const int32_t *g = a.cnt_scr + (size_t)c * T;
        int t = lane;
        for (; t + 7 * 64 < T; t += 8 * 64) {
            int32_t v[8];
#pragma unroll
            for (int j = 0; j < 8; j++) v[j] = g[t + j * 64];
#pragma unroll
            for (int j = 0; j < 8; j++) cnt[t + j * 64] = v[j];
        }
        for (; t < T; t += 64) cnt[t] = g[t];
    }
    __syncthreads();
    int M = 0;
    for (int t = lane; t < T; t += 64) M = max(M, cnt[t]);
    M = uni(wave_max(M));
    int ntied = 0;
    for (int tb = 0; tb < T; tb += 64) {
        const int t = tb + lane;
        const bool h = t < T && cnt[t] == M;
        const uint64_t bm = ballot(h);
        if (h) tied[ntied + (int)mbcnt(bm)] = t;
        ntied += popc64(bm);
    }
    __syncthreads();
    SEL_STAMP(1);
    ChunkOut o;
    o.flags = 0;
    o.best = -1;
    o.stop = -1;
    o.n_inl = 0;
    o.last_inl = -1;
    o.n_draws = D;
    int best = -1;
    if (T > 0) {
        const bool need_sums = ntied > 1 || M == N || !(ecut > 0.0);
        if (!need_sums) {
            best = tied[0];
        } else {
            // brackets of the tied trials' sums (-1: always a candidate): one tied
            // trial at a time, lanes over points (any summation order is covered
            // by tie_bound)
            for (int k = 0; k < ntied; k++) {
                const int t = uni(tied[k]);
                const Model m = model2(P[draws[2 * t]], P[draws[2 * t + 1]]);
                const double un = m.ux * m.ux + m.uy * m.uy;
                double S = -1.0;
                if (cheap && fabs(un - 1.0) <= 0x1p-46) {
                    double s0 = 0.0, s1 = 0.0;
                    int p = lane;
                    for (; p + 64 < N; p += 128) {
                        const double2 q0 = P[p], q1 = P[p + 64];
                        const double r0 = __builtin_fma(q0.x - m.ox, m.uy, -((q0.y - m.oy) * m.ux));
                        const double r1 = __builtin_fma(q1.x - m.ox, m.uy, -((q1.y - m.oy) * m.ux));
                        s0 += r0 * r0;
                        s1 += r1 * r1;
                    }
                    if (p < N) {
                        const double r = __builtin_fma(P[p].x - m.ox, m.uy, -((P[p].y - m.oy) * m.ux));
                        s0 += r * r;
                    }
                    S = unid(wave_sum(s0 + s1));
                }
                if (lane == 0) tsum[k] = S;
            }
            __syncthreads();
            SEL_STAMP(2);
            double U = __builtin_inf();
            for (int k = lane; k < ntied; k += 64) {
                const double S = tsum[k];
                if (S >= 0.0) U = fmin(U, S + tie_bound(S, N, bx.E2));
            }
            U = wave_min_d(U);
            // a single candidate wins without its exact sum unless the stop test
            // (sum == 0, only possible with M == N) could fire
            int ncand = 0, cand1 = -1;
            for (int kb = 0; kb < ntied; kb += 64) {
                const int k = kb + lane;
                bool cand = false;
                if (k < ntied) {
                    const double S = tsum[k];
                    cand = S < 0.0 || S - tie_bound(S, N, bx.E2) <= U;
                }
                const uint64_t cm = ballot(cand);
                if (cm && cand1 < 0) cand1 = kb + ffs64(cm);
                ncand += popc64(cm);
            }
            const bool lone = ncand == 1 && M < N && ecut > 0.0;
            if (lone) best = uni(tied[cand1]);
            int bcnt = 0;
            double bsum = __builtin_inf();
            for (int kb = 0; !lone && kb < ntied && o.stop < 0; kb += 64) {
                const int k = kb + lane;
                bool cand = false;
                if (k < ntied) {
                    const double S = tsum[k];
                    cand = S < 0.0 || S - tie_bound(S, N, bx.E2) <= U;
                }
                uint64_t cm = ballot(cand);
                while (cm) {
                    const int bit = ffs64(cm);
                    cm &= cm - 1ull;
                    const int t = uni(tied[kb + bit]);
                    const Model m = model2(P[draws[2 * t]], P[draws[2 * t + 1]]);
                    const double sum = pw_sum_lanes_any(P, N, m, vtmp, vst, nstack, lane);
                    if (M > bcnt || (M == bcnt && sum < bsum)) {
                        best = t;
                        bcnt = M;
                        bsum = sum;
                        if (bsum <= 0.0) {
                            o.stop = t;
                            break;
                        }
                    }
                }
            }
        }
    }
    SEL_STAMP(3);
    o = chunk_finish_fit(a, P, N, draws, mk, uni(best), o, lane);
    SEL_STAMP(4);
    const bool have_model = finish_chunk(a, o, P, mk, p0, N, rec, lane);
    if (B.y_proj && a.write_yproj) chunk_yproj(B.y_proj + p0, P, mk, N, have_model, rec.proj_a, rec.proj_b, lane);
    if (lane == 0 && B.models) B.models[c] = rec;
    SEL_STAMP(5);
#ifdef LSLAM_STAMPS
    if (a.dbg && lane == 0) {
        a.dbg[(size_t)c * 16 + 14] += (uint64_t)ntied;
        a.dbg[(size_t)c * 16 + 15] += (uint64_t)o.n_inl;
    }
#endif
}

// A1: polar -> Cartesian (functions.py:59-60)
__global__ __launch_bounds__(256) void polar_kernel(const double *__restrict__ th, const double *__restrict__ d,
                                                    double2 *__restrict__ xy, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        xy[i] = polar_xy(th[i], d[i]);
    }
}

// ------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------
constexpr int LSLAM_EV_RING = 64;
constexpr int LSLAM_MAX_OUTS = 48;

constexpr int NSLOTS = 2;  // producer slots in the ring
struct lslam_ctx {
    int device;
    hipStream_t stream;
    bool timing;
    // per kernel id: a ring of (start, stop) event pairs harvested lazily, so
    // timing never blocks the host between back-to-back launches
    hipEvent_t ev0[LSLAM_K_COUNT][LSLAM_EV_RING], ev1[LSLAM_K_COUNT][LSLAM_EV_RING];
    int head[LSLAM_K_COUNT], npend[LSLAM_K_COUNT];
    double total_ms[LSLAM_K_COUNT];
    int64_t launches[LSLAM_K_COUNT];
    // main-stream scratch: resolved draws (when the caller gives no draws_out)
    void *scr;
    size_t scr_bytes;
    // express-scan revolution builder scratch (per-packet flags/ranks, per-revolution info)
    void *escr;
    size_t escr_bytes;
    // large-chunk consensus scratch: per-trial counts (+ Philox draws)
    void *cscr;
    size_t cscr_bytes;
    // grid cap of the one-wave consumer kernels (resolve, chunk, fix-up, post)
    int resolve_beside;  // this call's resolves will likely run beside the next call's producer
    int n_cus;         // compute units of the device
    uint32_t timing_mask;  // kernel ids timed when timing is on (lslam_set_timing_mask)
    // reject tables of the table-mode parser, K = 2..127 (lslam_rng_pipe.h)
    uint32_t *rt_all;
    // seed_kernel -> rng_kernel: initial MT states [n_scans][624].  [0], [1]: the pipeline's, by
    // call parity, seeded on sstream ahead of their producers (launch_seed); [2]: producers on the
    // ctx stream (lslam_hyp_mt19937), seeded in stream order
    uint32_t *seedst[3];
    size_t seedst_bytes[3];
    hipStream_t sstream;
    hipEvent_t ev_seeded[2];     // on sstream, after seed_kernel into seedst[i]
    hipEvent_t ev_seed_read[2];  // on pstream, after the producer that read seedst[i]
    int seed_next;               // the pipeline's next seed buffer
    // cut_lane_kernel -> chunk_kernel: [n_chunks] ChunkCut, a ring of four by seeded call: the
    // buffer of call n is written after the producer of seeded call n - 2 (ev_seed_read), which
    // waited for its slot, released by the fix-up of the mt call two before it -- after the
    // consensus of seeded call n - 4, the buffer's previous reader
    ChunkCut *cutb[4];
    size_t cutb_bytes[4];
    int cut_next;
    size_t steps_budget;  // producer slot budget (prepare_steps)
    // The MT producer of call k+1 runs on its own stream while call k's
    // consumers finish on `stream`: two producer slots (Fisher-Yates steps +
    // end-of-scan MT state), each released by an event once its consumers ran.
    // (Measured and dropped at r04: a third slot, 0.79-0.86 vs 0.76 ms per C3 step; the resolve
    // on a stream of its own after its producer, 0.871 vs 0.763 ms.)
    hipStream_t pstream;
    void *pslot[NSLOTS];
    size_t pslot_bytes;
    int next_slot;
    hipEvent_t ev_slot_free[NSLOTS];  // on stream, after the slot's resolve + fix-up
    hipEvent_t ev_produced;      // on pstream, after rng_kernel
    hipEvent_t ev_copy;          // on stream, after the latest lslam_h2d / lslam_memset
    // destinations written by copies since the producer last waited for ev_copy: the producer
    // waits only if one of them is its input (seeds, CSR, MT state), so an xy upload per call
    // overlaps the stream parse
    struct { const void *p; size_t n; } copy_rng[32];
    int n_copy_rng;
    int copy_unknown;
    hipEvent_t ev_call;          // on stream, at the end of the latest pipeline call
    // A UKF step that does not read the call's RANSAC results runs on its own
    // stream beside the RANSAC chain; the main stream joins it before ev_call.
    hipStream_t ustream;
    hipEvent_t ev_ukf;           // on ustream, after the side UKF
    // Every buffer written by a call since the producer last waited for ev_call: the union
    // over calls, not only the latest (the producer of call k may start once call k-2's
    // fix-up has run).  A producer input that overlaps one of them makes it wait.
    const void *out_ptr[LSLAM_MAX_OUTS];
    size_t out_len[LSLAM_MAX_OUTS];
    int n_out;
    int out_unknown;             // the union overflowed: the producer waits for ev_call
    // the latest call's mt_state_out, complete once ev_slot_free[prev_slot] (after its fix-up) fired
    const void *prev_state_out;
    int prev_slot;
    int prev_fixed;
    // speculative producer (map mode): a call whose only producer hazard is the previous call's
    // mt_state_out parses from the previous producer's end state (its slot's state area) without
    // waiting for that call's fix-up; the fix-up replays the scans it replayed (spec_dirty)
    int speculate;            // env LSLAM_MT_SPECULATE=0: wait for the fix-up (test_gpu_speculate.py)
    int spec_ok;              // the previous call was a one-epoch pipeline call with dirty flags
    int spec_run;             // consecutive speculative calls (bounded by SPEC_RESYNC)
    const uint32_t *prev_state_scr;
    int prev_spec_scans;
    uint8_t *spec_dirty[2];   // [n_scans] replayed-by-fix-up flags, by call parity
    int spec_dirty_n;
    int spec_cur;             // the buffer the latest fix-up wrote
};

static thread_local std::string g_err;

static size_t default_steps_budget() { return (size_t)2 << 30; }  // lslam_set_steps_budget

// rows v = 0..127 of every K = 2..127, built once per process (rt_word, lslam_rng_pipe.h)
static const std::vector<uint32_t> &reject_tables() {
    static const std::vector<uint32_t> t = [] {
        std::vector<uint32_t> v((size_t)(RT_KMAX - 1) * RT_DWORDS);
        for (uint32_t K = 2; K <= RT_KMAX; K++)
            for (uint32_t r = 0; r < (uint32_t)RT_ROWS; r++)
                for (uint32_t q = 0; q < (uint32_t)RT_ST; q++)
                    v[(size_t)(K - 2) * RT_DWORDS + r * RT_ST + q] = rt_word(K, r, q);
        return v;
    }();
    return t;
}

static int set_err(int code, const char *msg) {
    g_err = msg;
    return code;
}

#define HIPCHK(expr)                                                                  \
    do {                                                                              \
        hipError_t _e = (expr);                                                       \
        if (_e != hipSuccess) {                                                       \
            g_err = std::string(#expr) + ": " + hipGetErrorString(_e);                \
            return LSLAM_ERR_HIP;                                                     \
        }                                                                             \
    } while (0)

extern "C" {

#define LSLAM_STR_(x) #x
#define LSLAM_STR(x) LSLAM_STR_(x)
#ifndef LSLAM_SRC_HASH
#define LSLAM_SRC_HASH "0000000000000000"  // lidar_slam_amd/build.py passes the sources' sha256 prefix
#endif
const char *lslam_version(void) {
    return "lidarslam-mi355x 0.3.0 (abi " LSLAM_STR(LSLAM_ABI_VERSION) ", src " LSLAM_SRC_HASH ", gfx950)";
}

const char *lslam_status_string(int st) {
    switch (st) {
        case LSLAM_OK: return "ok";
        case LSLAM_ERR_ARG: return "invalid argument";
        case LSLAM_ERR_HIP: return "HIP runtime error";
        case LSLAM_ERR_NOMEM: return "out of memory";
        case LSLAM_ERR_CAPACITY: return "capacity exceeded";
        case LSLAM_ERR_UNSUPPORTED: return "unsupported";
        default: return "unknown status";
    }
}

const char *lslam_last_error(void) { return g_err.c_str(); }

int lslam_device_count(int *n) {
    if (!n) return LSLAM_ERR_ARG;
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    if (e != hipSuccess) c = 0;
    *n = c;
    return LSLAM_OK;
}

int lslam_ctx_create(int device, lslam_ctx **out) {
    if (!out) return LSLAM_ERR_ARG;
    *out = nullptr;
    int n = 0;
    HIPCHK(hipGetDeviceCount(&n));
    if (device < 0 || device >= n) return set_err(LSLAM_ERR_ARG, "device index out of range");
    HIPCHK(hipSetDevice(device));
    lslam_ctx *c = new (std::nothrow) lslam_ctx();
    if (!c) return LSLAM_ERR_NOMEM;
    c->device = device;
    c->n_cus = 0;
    HIPCHK(hipDeviceGetAttribute(&c->n_cus, hipDeviceAttributeMultiprocessorCount, device));
    if (c->n_cus < 1) c->n_cus = 1;
    c->timing = false;
    c->scr = nullptr;
    c->scr_bytes = 0;
    for (int i = 0; i < 3; i++) {
        c->seedst[i] = nullptr;
        c->seedst_bytes[i] = 0;
    }
    c->sstream = nullptr;
    c->seed_next = 0;
    for (int i = 0; i < 4; i++) {
        c->cutb[i] = nullptr;
        c->cutb_bytes[i] = 0;
    }
    c->cut_next = 0;
    c->escr = nullptr;
    c->escr_bytes = 0;
    c->cscr = nullptr;
    c->cscr_bytes = 0;
    c->resolve_beside = 0;
    c->timing_mask = 0xffffffffu;
    c->rt_all = nullptr;
    c->steps_budget = default_steps_budget();
    c->pstream = nullptr;
    c->ustream = nullptr;
    for (int i = 0; i < NSLOTS; i++) c->pslot[i] = nullptr;
    c->pslot_bytes = 0;
    c->next_slot = 0;
    c->speculate = 1;
    if (const char *e = getenv("LSLAM_MT_SPECULATE")) c->speculate = atoi(e) != 0;
    c->spec_ok = 0;
    c->spec_run = 0;
    c->prev_state_scr = nullptr;
    c->prev_spec_scans = 0;
    c->spec_dirty[0] = c->spec_dirty[1] = nullptr;
    c->spec_dirty_n = 0;
    c->spec_cur = 0;
    c->n_out = 0;
    for (int k = 0; k < LSLAM_K_COUNT; k++) {
        c->total_ms[k] = 0;
        c->launches[k] = 0;
        c->head[k] = 0;
        c->npend[k] = 0;
        for (int r = 0; r < LSLAM_EV_RING; r++) c->ev0[k][r] = c->ev1[k][r] = nullptr;
    }
    hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete c;
        return set_err(LSLAM_ERR_HIP, hipGetErrorString(e));
    }
    for (int k = 0; k < LSLAM_K_COUNT; k++)
        for (int r = 0; r < LSLAM_EV_RING; r++) {
            HIPCHK(hipEventCreate(&c->ev0[k][r]));
            HIPCHK(hipEventCreate(&c->ev1[k][r]));
        }
    // the producer's chains are the critical path: its stream gets the highest
    // priority so that its workgroups are dispatched ahead of the previous call's
    // consumers (resolve / consensus / post) that run beside it
    {
        int lo_pri = 0, hi_pri = 0;
        if (hipDeviceGetStreamPriorityRange(&lo_pri, &hi_pri) != hipSuccess) hi_pri = 0;
        HIPCHK(hipStreamCreateWithPriority(&c->pstream, hipStreamNonBlocking, hi_pri));
    }
    HIPCHK(hipStreamCreateWithFlags(&c->sstream, hipStreamNonBlocking));
    for (int i = 0; i < 2; i++) {
        HIPCHK(hipEventCreateWithFlags(&c->ev_seeded[i], hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&c->ev_seed_read[i], hipEventDisableTiming));
        HIPCHK(hipEventRecord(c->ev_seed_read[i], c->stream));
    }
    for (int i = 0; i < NSLOTS; i++) HIPCHK(hipEventCreateWithFlags(&c->ev_slot_free[i], hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&c->ev_produced, hipEventDisableTiming));
    HIPCHK(hipStreamCreateWithFlags(&c->ustream, hipStreamNonBlocking));
    HIPCHK(hipEventCreateWithFlags(&c->ev_ukf, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&c->ev_copy, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&c->ev_call, hipEventDisableTiming));
    for (int i = 0; i < NSLOTS; i++) HIPCHK(hipEventRecord(c->ev_slot_free[i], c->stream));
    HIPCHK(hipEventRecord(c->ev_copy, c->stream));
    HIPCHK(hipEventRecord(c->ev_call, c->stream));
    {
        const std::vector<uint32_t> &t = reject_tables();
        HIPCHK(hipMalloc(&c->rt_all, t.size() * 4));
        HIPCHK(hipMemcpy(c->rt_all, t.data(), t.size() * 4, hipMemcpyHostToDevice));
    }
    *out = c;
    return LSLAM_OK;
}

int lslam_ctx_destroy(lslam_ctx *c) {
    if (!c) return LSLAM_OK;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    for (int k = 0; k < LSLAM_K_COUNT; k++)
        for (int r = 0; r < LSLAM_EV_RING; r++) {
            if (c->ev0[k][r]) (void)hipEventDestroy(c->ev0[k][r]);
            if (c->ev1[k][r]) (void)hipEventDestroy(c->ev1[k][r]);
        }
    if (c->pstream) (void)hipStreamSynchronize(c->pstream);
    if (c->ustream) (void)hipStreamSynchronize(c->ustream);
    if (c->sstream) (void)hipStreamSynchronize(c->sstream);
    if (c->scr) (void)hipFree(c->scr);
    for (int i = 0; i < 3; i++)
        if (c->seedst[i]) (void)hipFree(c->seedst[i]);
    for (int i = 0; i < 4; i++)
        if (c->cutb[i]) (void)hipFree(c->cutb[i]);
    for (int i = 0; i < 2; i++) {
        if (c->ev_seeded[i]) (void)hipEventDestroy(c->ev_seeded[i]);
        if (c->ev_seed_read[i]) (void)hipEventDestroy(c->ev_seed_read[i]);
    }
    if (c->escr) (void)hipFree(c->escr);
    if (c->cscr) (void)hipFree(c->cscr);
    for (int i = 0; i < NSLOTS; i++)
        if (c->pslot[i]) (void)hipFree(c->pslot[i]);
    if (c->rt_all) (void)hipFree(c->rt_all);
    for (int i = 0; i < 2; i++)
        if (c->spec_dirty[i]) (void)hipFree(c->spec_dirty[i]);
    hipEvent_t evs[6] = {c->ev_slot_free[0], c->ev_slot_free[1], c->ev_produced, c->ev_copy, c->ev_call, c->ev_ukf};
    for (hipEvent_t e : evs)
        if (e) (void)hipEventDestroy(e);
    if (c->pstream) (void)hipStreamDestroy(c->pstream);
    if (c->ustream) (void)hipStreamDestroy(c->ustream);
    if (c->sstream) (void)hipStreamDestroy(c->sstream);
    (void)hipStreamDestroy(c->stream);
    delete c;
    return LSLAM_OK;
}

int lslam_sync(lslam_ctx *c) {
    if (!c) return LSLAM_ERR_ARG;
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(c->pstream));
    HIPCHK(hipStreamSynchronize(c->ustream));
    HIPCHK(hipStreamSynchronize(c->sstream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return LSLAM_OK;
}

int lslam_malloc(lslam_ctx *c, size_t bytes, void **p) {
    if (!c || !p) return LSLAM_ERR_ARG;
    HIPCHK(hipSetDevice(c->device));
    *p = nullptr;
    if (bytes == 0) bytes = 16;
    hipError_t e = hipMalloc(p, bytes);
    if (e == hipErrorOutOfMemory) return set_err(LSLAM_ERR_NOMEM, "hipMalloc: out of memory");
    HIPCHK(e);
    return LSLAM_OK;
}

int lslam_free(lslam_ctx *c, void *p) {
    if (!c) return LSLAM_ERR_ARG;
    if (!p) return LSLAM_OK;
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipFree(p));
    return LSLAM_OK;
}

int lslam_host_alloc(size_t bytes, void **p) {
    if (!p) return LSLAM_ERR_ARG;
    HIPCHK(hipHostMalloc(p, bytes ? bytes : 16, hipHostMallocDefault));
    return LSLAM_OK;
}

int lslam_host_free(void *p) {
    if (p) HIPCHK(hipHostFree(p));
    return LSLAM_OK;
}

static void note_copy(lslam_ctx *c, const void *p, size_t n) {
    if (!p || !n) return;
    for (int i = 0; i < c->n_copy_rng; i++)
        if (c->copy_rng[i].p == p && c->copy_rng[i].n == n) return;
    if (c->n_copy_rng == 32) {
        c->copy_unknown = 1;
        return;
    }
    c->copy_rng[c->n_copy_rng].p = p;
    c->copy_rng[c->n_copy_rng].n = n;
    c->n_copy_rng++;
}

int lslam_h2d(lslam_ctx *c, void *dst, const void *src, size_t n) {
    if (!c || (!dst && n) || (!src && n)) return LSLAM_ERR_ARG;
    if (!n) return LSLAM_OK;
    HIPCHK(hipSetDevice(c->device));
    // (the previous calls, which may still read dst, are ahead of this on the ctx stream)
    HIPCHK(hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipEventRecord(c->ev_copy, c->stream));
    note_copy(c, dst, n);
    return LSLAM_OK;
}

int lslam_d2h(lslam_ctx *c, void *dst, const void *src, size_t n) {
    if (!c || (!dst && n) || (!src && n)) return LSLAM_ERR_ARG;
    if (!n) return LSLAM_OK;
    HIPCHK(hipSetDevice(c->device));
    // (the previous calls, which may still read dst, are ahead of this on the ctx stream)
    HIPCHK(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, c->stream));
    return LSLAM_OK;
}

int lslam_d2d(lslam_ctx *c, void *dst, const void *src, size_t n) {
    if (!c || (!dst && n) || (!src && n)) return LSLAM_ERR_ARG;
    if (!n) return LSLAM_OK;
    HIPCHK(hipSetDevice(c->device));
    // (the previous calls, which may still read dst, are ahead of this on the ctx stream)
    HIPCHK(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(hipEventRecord(c->ev_copy, c->stream));
    note_copy(c, dst, n);
    return LSLAM_OK;
}

int lslam_host_register(void *p, size_t n) {
    if (!p || !n) return LSLAM_ERR_ARG;
    const hipError_t e = hipHostRegister(p, n, hipHostRegisterDefault);
    if (e != hipSuccess) {
        (void)hipGetLastError();  // not sticky: the caller falls back to pageable copies
        return set_err(LSLAM_ERR_HIP, hipGetErrorString(e));
    }
    return LSLAM_OK;
}

int lslam_host_unregister(void *p) {
    if (!p) return LSLAM_ERR_ARG;
    HIPCHK(hipHostUnregister(p));
    return LSLAM_OK;
}

int lslam_ctx_stream(lslam_ctx *c, void **stream) {
    if (!c || !stream) return LSLAM_ERR_ARG;
    *stream = (void *)c->stream;
    return LSLAM_OK;
}

int lslam_abi_sizes(int64_t *sizes, int n) {
    const int64_t s[7] = {(int64_t)sizeof(lslam_chunk_model), (int64_t)sizeof(lslam_landmark),
                          (int64_t)sizeof(lslam_ransac_params), (int64_t)sizeof(lslam_ukf_params),
                          (int64_t)sizeof(lslam_scan_batch), (int64_t)sizeof(lslam_express_measures),
                          (int64_t)sizeof(lslam_express_revs)};
    for (int i = 0; i < n && i < 7 && sizes; i++) sizes[i] = s[i];
    return 7;
}

int lslam_memset(lslam_ctx *c, void *dst, int v, size_t n) {
    if (!c || (!dst && n)) return LSLAM_ERR_ARG;
    if (!n) return LSLAM_OK;
    HIPCHK(hipSetDevice(c->device));
    // (the previous calls, which may still read dst, are ahead of this on the ctx stream)
    HIPCHK(hipMemsetAsync(dst, v, n, c->stream));
    HIPCHK(hipEventRecord(c->ev_copy, c->stream));
    note_copy(c, dst, n);
    return LSLAM_OK;
}

// fold the oldest `keep_free` pending event pairs (all of them if < 0) into the totals
static int harvest(lslam_ctx *c, int k, int upto_free = -1) {
    while (c->npend[k] > 0 && (upto_free < 0 || LSLAM_EV_RING - c->npend[k] < upto_free)) {
        const int r = (c->head[k] - c->npend[k] + LSLAM_EV_RING) % LSLAM_EV_RING;
        HIPCHK(hipEventSynchronize(c->ev1[k][r]));
        float ms = 0.f;
        HIPCHK(hipEventElapsedTime(&ms, c->ev0[k][r], c->ev1[k][r]));
        c->total_ms[k] += ms;
        c->launches[k] += 1;
        c->npend[k] -= 1;
    }
    return LSLAM_OK;
}

static int timer_begin(lslam_ctx *c, int k, hipStream_t st_ = nullptr) {
    if (!c->timing || !((c->timing_mask >> k) & 1u)) return LSLAM_OK;
    int st = harvest(c, k, 1);
    if (st) return st;
    HIPCHK(hipEventRecord(c->ev0[k][c->head[k]], st_ ? st_ : c->stream));
    return LSLAM_OK;
}

static int timer_end(lslam_ctx *c, int k, hipStream_t st_ = nullptr) {
    if (!c->timing || !((c->timing_mask >> k) & 1u)) return LSLAM_OK;
    HIPCHK(hipEventRecord(c->ev1[k][c->head[k]], st_ ? st_ : c->stream));
    c->head[k] = (c->head[k] + 1) % LSLAM_EV_RING;
    c->npend[k] += 1;
    return LSLAM_OK;
}

int lslam_set_timing(lslam_ctx *c, int en) {
    if (!c) return LSLAM_ERR_ARG;
    c->timing = en != 0;
    return LSLAM_OK;
}

int lslam_set_timing_mask(lslam_ctx *c, uint32_t mask) {
    if (!c) return LSLAM_ERR_ARG;
    c->timing_mask = mask;
    return LSLAM_OK;
}

int lslam_timing(lslam_ctx *c, int k, double *ms, int64_t *n) {
    if (!c || k < 0 || k >= LSLAM_K_COUNT) return LSLAM_ERR_ARG;
    HIPCHK(hipSetDevice(c->device));
    int st = harvest(c, k);
    if (st) return st;
    if (ms) *ms = c->total_ms[k];
    if (n) *n = c->launches[k];
    return LSLAM_OK;
}

int lslam_timing_reset(lslam_ctx *c) {
    if (!c) return LSLAM_ERR_ARG;
    for (int k = 0; k < LSLAM_K_COUNT; k++) {
        int st = harvest(c, k);
        if (st) return st;
        c->total_ms[k] = 0;
        c->launches[k] = 0;
    }
    return LSLAM_OK;
}

int lslam_ransac_params_default(lslam_ransac_params *p) {
    if (!p) return LSLAM_ERR_ARG;
    memset(p, 0, sizeof(*p));
    p->residual_threshold = 20.0;  // ransac_functions.py:9
    p->max_trials = 100;           // :10
    p->min_samples = 2;            // :11
    p->hyp_source = LSLAM_HYP_MT19937;
    p->life = 40;                  // landmarking.py:3
    p->tol_a = 0.1;                // :4
    p->tol_b = 10.0;               // :5
    p->tol_dist = 100.0;           // :6
    p->philox_seed = 0x5eed5eedull;
    return LSLAM_OK;
}

int lslam_ukf_params_default(lslam_ukf_params *p, int32_t L) {
    if (!p || L < 0) return LSLAM_ERR_ARG;
    memset(p, 0, sizeof(*p));
    p->n_landmarks = L;
    p->flags = LSLAM_UKF_PREDICT | LSLAM_UKF_UPDATE;
    p->dt = 0.005;          // systemClass.py:10
    p->wheel_radius = 50;   // UKFMethods.py:6
    p->wheel_base = 200;    // UKFMethods.py:7
    p->alpha = 1e-4;        // systemClass.py:20
    p->beta = 2.0;
    p->kappa = 0.0;
    for (int i = 0; i < 9; i++) p->Q[i] = (i % 4 == 0) ? 0.001 : 0.0;  // systemClass.py:29
    return LSLAM_OK;
}

double lslam_inlier_cutoff(double thr) {
    if (isnan(thr)) return NAN;
    if (!(thr > 0)) return 0.0;
    if (isinf(thr)) return INFINITY;
    double e = thr * thr;
    while (e > 0 && sqrt(e) >= thr) e = nextafter(e, 0.0);
    while (sqrt(e) < thr) e = nextafter(e, INFINITY);
    return e;
}

int lslam_ukf_weights(const lslam_ukf_params *p, double *Wm, double *Wc, double *lpn) {
    if (!p || !Wm || !Wc) return LSLAM_ERR_ARG;
    // filterpy MerweScaledSigmaPoints._compute_weights, n = 3
    const double n = 3.0;
    const double lambda_ = p->alpha * p->alpha * (n + p->kappa) - n;
    const double c = .5 / (n + lambda_);
    for (int i = 0; i < 7; i++) Wm[i] = Wc[i] = c;
    Wc[0] = lambda_ / (n + lambda_) + (1 - p->alpha * p->alpha + p->beta);
    Wm[0] = lambda_ / (n + lambda_);
    if (lpn) *lpn = lambda_ + n;
    return LSLAM_OK;
}

int lslam_mt_seed_state(uint32_t seed, uint32_t *st) {
    if (!st) return LSLAM_ERR_ARG;
    for (int i = 0; i < 624; i++) {
        st[i] = seed;
        seed = 1812433253u * (seed ^ (seed >> 30)) + (uint32_t)(i + 1);
    }
    st[624] = 624;
    return LSLAM_OK;
}

}  // extern "C"

// ---- launch plumbing ----
static inline int align16(int x) { return (x + 15) & ~15; }

static int validate_batch(const lslam_scan_batch *b, bool need_points) {
    if (!b) return set_err(LSLAM_ERR_ARG, "batch is NULL");
    if (b->n_scans < 0 || b->n_chunks < 0 || b->n_points < 0) return set_err(LSLAM_ERR_ARG, "negative sizes");
    if (b->n_scans == 0) return LSLAM_OK;
    if (!b->scan_chunk_off || !b->chunk_pt_off) return set_err(LSLAM_ERR_ARG, "missing CSR offsets");
    if (need_points && !b->xy && (!b->theta_deg || !b->dist_mm) && b->n_points > 0)
        return set_err(LSLAM_ERR_ARG, "missing points (xy, or theta_deg + dist_mm)");
    if (b->max_chunk_points < 0 || b->max_scan_chunks < 0) return set_err(LSLAM_ERR_ARG, "bad maxima");
    return LSLAM_OK;
}

#if defined(LSLAM_STAMPS) || defined(LSLAM_CENSUS)
static unsigned long long *g_wcen = nullptr;  // wave census (diagnostic builds)
static unsigned int *g_wcen_n = nullptr;
static unsigned int g_wcen_cap = 0;
static unsigned int g_call_seq = 0;
extern "C" int lslam_debug_set_census(unsigned long long *dev_buf, unsigned int *dev_count, unsigned int cap) {
    g_wcen = dev_buf;
    g_wcen_n = dev_count;
    g_wcen_cap = cap;
    return LSLAM_OK;
}
#endif
#ifdef LSLAM_STAMPS
static unsigned long long *g_dbg = nullptr;
extern "C" int lslam_debug_set_stamps(unsigned long long *dev_buf) {
    g_dbg = dev_buf;
    return LSLAM_OK;
}
#endif

static int build_args(KArgs &k, const lslam_scan_batch *b, const lslam_ransac_params *p, const lslam_ukf_params *u,
                      int mode, int &lds) {
    memset(&k, 0, sizeof(k));
#ifdef LSLAM_STAMPS
    k.dbg = g_dbg;
#endif
#if defined(LSLAM_STAMPS) || defined(LSLAM_CENSUS)
    k.wcen = g_wcen;
    k.wcen_n = g_wcen_n;
    k.wcen_cap = g_wcen_cap;
    k.call_seq = g_call_seq;
#endif
    k.b = *b;
    if (p) {
        if (p->min_samples != 2) return set_err(LSLAM_ERR_UNSUPPORTED, "only min_samples == 2 (ransac_functions.py:11)");
        if (p->residual_threshold < 0) return set_err(LSLAM_ERR_ARG, "`residual_threshold` must be greater than zero");
        if (p->max_trials < 0) return set_err(LSLAM_ERR_ARG, "`max_trials` must be greater than zero");
        if (p->max_trials > 65533) return set_err(LSLAM_ERR_UNSUPPORTED, "max_trials > 65533");
        if (p->hyp_source < 0 || p->hyp_source > 2) return set_err(LSLAM_ERR_ARG, "bad hyp_source");
        if (p->hyp_source == LSLAM_HYP_EXPLICIT && !b->hyp) return set_err(LSLAM_ERR_ARG, "explicit hyp without hyp");
        k.thr = p->residual_threshold;
        k.ecut = lslam_inlier_cutoff(p->residual_threshold);
        k.ecut_q = std::sqrt(k.ecut) * 1.01 + 1.0;
        k.tol_a = p->tol_a;
        k.tol_b = p->tol_b;
        k.tol_dist = p->tol_dist;
        k.tol_dist_sq = sqrt_le_bound(p->tol_dist);
        k.philox_seed = p->philox_seed;
        k.T = p->max_trials;
        k.hyp_source = p->hyp_source;
        k.life = p->life;
    }
    if ((mode & MODE_ASSOC) && b->landmarks && !b->lmk_count) return set_err(LSLAM_ERR_ARG, "landmarks without lmk_count");
    const int N = b->max_chunk_points > 0 ? b->max_chunk_points : 1;
    const int T = k.T;
    int off = 0;
    if (mode & (MODE_RANSAC | MODE_HYP_ONLY)) {
        k.off_pts = off; off += align16(16 * N);
        k.off_key = off; off += align16(4 * 624);
        // phase-exclusive scratch shares one region: the draw-resolution tables
        // (draw generation), then the tie sums (selection)
        const int nxt_bytes = 4 * mt_nslot(N) * N;
        const int uni_bytes = max(nxt_bytes, 8 * (T > 0 ? T : 1));
        k.off_ring = off;
        k.off_tsum = off;
        off += align16(uni_bytes);
        k.off_j1 = off;
        off += align16(4 * mt_nslot(N));
        k.off_draws = off; off += align16(8 * (T + 1));
        k.off_cnt = off; off += align16(4 * (T > 0 ? T : 1));
        k.off_tied = off; off += align16(4 * (T > 0 ? T : 1));
        k.off_mask = off; off += align16(N);
        k.off_vstack = off; off += (N > 128) ? align16(8 * 64 * 24) : 0;
        k.off_nstack = off; off += (N > 128) ? align16(4 * 72) : 0;
        k.off_recs = -1;
    } else {
        // post pass (association / UKF over fitted models): only the chunk's mask
        k.off_mask = off; off += align16(N);
        // and the scan's chunk records + offsets, staged up front (post_assoc_fast)
        const int msc = b->max_scan_chunks > 0 ? b->max_scan_chunks : 1;
        if (msc <= 256) {
            k.off_recs = off;
            off += align16((int)sizeof(lslam_chunk_model) * msc) + align16(4 * (msc + 1));
        } else {
            k.off_recs = -1;
        }
    }
    // the UKF runs after the last chunk: its scratch aliases the RANSAC scratch
    // above (offset 0); only the persistent region below (chunk history, chunk
    // origins, landmark list) is live across both
    if (u && u->n_landmarks > 0) {
        k.off_ukf = 0;
        off = max(off, align16(8 * UkfLds::doubles(u->n_landmarks)));
    }
    k.hist_cap = b->max_scan_chunks > 0 ? b->max_scan_chunks : 1;
    k.off_snap = off; off += (mode & MODE_RANSAC) ? align16(4 * MT_N) : 0;
    k.corg_cap = k.hist_cap;
    k.off_corg = off; off += align16(16 * k.corg_cap);
    k.off_zobs = off; off += (u && (u->flags & LSLAM_UKF_MAP)) ? align16(16 * k.corg_cap) : 0;
    k.lmk_cap = (mode & MODE_ASSOC) ? b->lmk_capacity : 0;
    if ((mode & MODE_ASSOC) && k.lmk_cap <= 0) return set_err(LSLAM_ERR_ARG, "lmk_capacity must be > 0");
    // the association-only post pass keeps a list of at most 64 entries in registers
    k.lmk_reg = (mode == MODE_ASSOC && k.lmk_cap > 0 && k.lmk_cap <= 64 && k.off_recs >= 0 &&
                 !(u && (u->flags & LSLAM_UKF_MAP)) && b->landmarks) ? 1 : 0;
    k.off_lmk = off; off += k.lmk_reg ? 0 : align16((int)sizeof(lslam_landmark) * (k.lmk_cap > 0 ? k.lmk_cap : 1));
    k.off_vis = off; off += k.lmk_reg ? 0 : align16(8 * ((k.lmk_cap + 63) / 64 + 1));
    k.pts_cap = N;
    if (u) {
        if (u->n_landmarks <= 0) return set_err(LSLAM_ERR_ARG, "n_landmarks must be > 0");
        const bool map = (u->flags & LSLAM_UKF_MAP) != 0;
        if (!b->ukf_x || !b->ukf_P || !b->ukf_u || !b->ukf_R_diag || (!map && (!b->ukf_z || !b->ukf_lmk)))
            return set_err(LSLAM_ERR_ARG, "UKF buffers missing");
        if (map && (!(mode & MODE_ASSOC) || !b->landmarks))
            return set_err(LSLAM_ERR_ARG, "LSLAM_UKF_MAP needs the landmark lists (the map) in lslam_scan_pipeline");
        if (map && u->n_landmarks < b->max_scan_chunks)
            return set_err(LSLAM_ERR_CAPACITY, "LSLAM_UKF_MAP: n_landmarks (measurement slots) < max_scan_chunks");
        double lpn = 0;
        lslam_ukf_weights(u, k.ukf.Wm, k.ukf.Wc, &lpn);
        for (int i = 0; i < 7; i++)
            if (k.ukf.Wc[i] == 0.0) return set_err(LSLAM_ERR_UNSUPPORTED, "zero covariance weight");
        k.ukf.cfac = lpn;
        k.ukf.dt = u->dt;
        k.ukf.wr = u->wheel_radius;
        k.ukf.wb = u->wheel_base;
        for (int i = 0; i < 9; i++) k.ukf.Q[i] = u->Q[i];
        k.ukf.L = u->n_landmarks;
        k.ukf.flags = u->flags;
    }
    lds = off;
    if (lds > 160 * 1024) return set_err(LSLAM_ERR_CAPACITY, "chunk/trial/landmark sizes exceed the 160 KiB LDS");
    return LSLAM_OK;
}

template <int MODE>
static hipError_t launch_mode(const KArgs &k, int lds, hipStream_t st) {
    const dim3 grid((unsigned)k.b.n_scans), block(64);
    switch (k.hyp_source) {
        case LSLAM_HYP_PHILOX:
            hipLaunchKernelGGL((scan_kernel<LSLAM_HYP_PHILOX, MODE>), grid, block, lds, st, k);
            break;
        case LSLAM_HYP_EXPLICIT:
            hipLaunchKernelGGL((scan_kernel<LSLAM_HYP_EXPLICIT, MODE>), grid, block, lds, st, k);
            break;
        default:
            hipLaunchKernelGGL((scan_kernel<LSLAM_HYP_MT19937, MODE>), grid, block, lds, st, k);
            break;
    }
    return hipGetLastError();
}

template <int MODE>
static int run_scan_kernel(lslam_ctx *c, const KArgs &k, int lds, int timer) {
    HIPCHK(hipSetDevice(c->device));
    if (k.b.n_scans == 0) return LSLAM_OK;
    static std::once_flag once;
    std::call_once(once, [] {
        const int mx = 160 * 1024;
        (void)hipFuncSetAttribute((const void *)scan_kernel<0, MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, mx);
        (void)hipFuncSetAttribute((const void *)scan_kernel<1, MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, mx);
        (void)hipFuncSetAttribute((const void *)scan_kernel<2, MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, mx);
        set_max_lds(scan_kernel_w4<LSLAM_HYP_EXPLICIT, MODE>);
    });
    int st = timer_begin(c, timer);
    if (st) return st;
    if (MODE == MODE_UKF && !(k.ukf.flags & LSLAM_UKF_MAP)) {  // stand-alone UKF: lane groups
        launch_ukf_group(k, k.ukf.L, c->stream, false);
        HIPCHK(hipGetLastError());
    } else if (MODE == MODE_ASSOC || MODE == MODE_UKF) {  // stand-alone association / UKF: no producer beside them
        hipLaunchKernelGGL((scan_kernel_w4<LSLAM_HYP_EXPLICIT, MODE>), dim3((unsigned)k.b.n_scans), dim3(64), lds,
                           c->stream, k);
        HIPCHK(hipGetLastError());
    } else {
        HIPCHK(launch_mode<MODE>(k, lds, c->stream));
    }
    st = timer_end(c, timer);
    if (st) return st;
    return LSLAM_OK;
}


// chunk_kernel LDS: one chunk's points, draws and consensus scratch
static int layout_chunk(KArgs &k, const lslam_scan_batch *b, int &lds) {
    const int N = b->max_chunk_points > 0 ? b->max_chunk_points : 1;
    const int T = k.T;
    int off = 0;
    k.off_pts = off; off += align16(16 * N);
    k.off_draws = off; off += (k.hyp_source == LSLAM_HYP_PHILOX) ? align16(8 * (T + 1)) : 0;  // else read in place
    k.off_cnt = off; off += align16(4 * (T > 0 ? T : 1));
    k.off_tied = off; off += align16(4 * (T > 0 ? T : 1));
    k.off_tsum = off; off += align16(8 * (T > 0 ? T : 1));  // tie sums
    k.off_mask = off; off += align16(N);
    k.off_vstack = off; off += (N > 128) ? align16(8 * 64 * 24) : 0;
    k.off_nstack = off; off += (N > 128) ? align16(4 * 72) : 0;
    k.off_vtmp = off;  // (pairwise sums from registers: pw_sum_regs)
    lds = off;
    if (lds > 160 * 1024) return set_err(LSLAM_ERR_CAPACITY, "chunk/trial sizes exceed the 160 KiB LDS");
    return LSLAM_OK;
}

// rng_kernel LDS: two raw MT blocks + flags
static int layout_rng(KArgs &k, const lslam_scan_batch *b, int &lds) {
    const int N = b->max_chunk_points > 3 ? b->max_chunk_points : 3;
    if (N > 65536) return set_err(LSLAM_ERR_UNSUPPORTED, "chunks of more than 65536 points");
    int off = 0;
    k.off_blk = off; off += align16(4 * (2 * 624 + 64));  // two block slots + the head pad
    k.rng_pipe_bytes = off;
    lds = off * RNG_PPW;
    // two K claims (16 B) + two reject tables shared by the workgroup's parsers, after the
    // pipes: table mode is chosen per chunk (N - 1 <= RT_KMAX), so a batch whose largest chunk
    // is bigger may still parse its small chunks with them
    k.off_stbl = lds;
    lds += 16 + 2 * 4 * RT_DWORDS;
    return LSLAM_OK;
}

// consumer grids: one workgroup per item, at most 2^30 (kernels loop over their items)
static inline unsigned launch_cap(const lslam_ctx *c, int64_t n) {
    (void)c;
    return (unsigned)(n < (1 << 30) ? (n > 0 ? n : 1) : (1 << 30));
}

static int ensure_scratch(lslam_ctx *c, size_t bytes) {
    if (c->scr_bytes >= bytes) return LSLAM_OK;
    HIPCHK(hipStreamSynchronize(c->stream));
    HIPCHK(hipStreamSynchronize(c->pstream));
    if (c->scr) HIPCHK(hipFree(c->scr));
    c->scr = nullptr;
    c->scr_bytes = 0;
    hipError_t e = hipMalloc(&c->scr, bytes);
    if (e == hipErrorOutOfMemory) return set_err(LSLAM_ERR_NOMEM, "hipMalloc: out of memory (step scratch)");
    HIPCHK(e);
    c->scr_bytes = bytes;
    return LSLAM_OK;
}

// allow up to 160 KiB of LDS per workgroup (static + dynamic); a failure here must
// not linger as the runtime's last error for the next launch check
template <typename F>
static void set_max_lds(F *fn) {
    hipFuncAttributes at;
    size_t stat = 0;
    if (hipFuncGetAttributes(&at, (const void *)fn) == hipSuccess) stat = at.sharedSizeBytes;
    (void)hipFuncSetAttribute((const void *)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)(160 * 1024 - stat));
    (void)hipGetLastError();
}

// Producer slot: one j per Fisher-Yates step (D * n_points entries; chunk c at
// D * chunk_pt_off[c]; + slack for 16-byte staging loads) and the end-of-scan
// MT state.  The resolved draws live in the main-stream scratch unless the
// caller asked for draws_out.
// Epochs: when every scan is one chunk (C5) and the steps of all T + 1 draws
// exceed the slot budget (lslam_set_steps_budget, default 2 GiB), the producer
// runs in launches of ep_nd draws, each resolved before its slot is reused; the
// MT state chains through the slots' state areas.  k.ep_count launches.
static int prepare_steps(lslam_ctx *c, KArgs &k, int slot) {
    const int N = k.b.max_chunk_points;
    k.j8 = N <= 256 ? 1 : 0;
    const size_t per_draw = (size_t)(k.b.n_points > 0 ? k.b.n_points : 1) * (k.j8 ? 1 : 2);
    const size_t budget = c->steps_budget;
    const int D = k.T + 1;
    int De = D;
    if (k.b.max_scan_chunks == 1 && (size_t)D * per_draw > budget) {
        const size_t fit = budget / per_draw;
        De = fit < 1 ? 1 : (fit < (size_t)D ? (int)fit : D);
    }
    k.ep_nd = De < D ? De : 0;
    k.ep_d0 = 0;
    k.ep_count = (D + De - 1) / De;
    const size_t jbytes = ((size_t)De * per_draw + JBUF_FRONT + 64 + 255) & ~(size_t)255;
    const size_t sbytes = ((size_t)(k.b.n_scans > 0 ? k.b.n_scans : 1) * 625 * 4 + 255) & ~(size_t)255;
    if (c->pslot_bytes < jbytes + sbytes) {
        HIPCHK(hipStreamSynchronize(c->stream));
        HIPCHK(hipStreamSynchronize(c->pstream));
        for (int i = 0; i < NSLOTS; i++) {
            if (c->pslot[i]) HIPCHK(hipFree(c->pslot[i]));
            c->pslot[i] = nullptr;
        }
        c->pslot_bytes = 0;
        for (int i = 0; i < NSLOTS; i++) {
            hipError_t e = hipMalloc(&c->pslot[i], jbytes + sbytes);
            if (e == hipErrorOutOfMemory) return set_err(LSLAM_ERR_NOMEM, "hipMalloc: out of memory (producer slot)");
            HIPCHK(e);
        }
        c->pslot_bytes = jbytes + sbytes;
        c->spec_ok = 0;  // the previous producer's end state went with the old slots
    }
    k.jbuf = (unsigned char *)c->pslot[slot] + JBUF_FRONT;
    k.state_scr = (uint32_t *)((unsigned char *)c->pslot[slot] + jbytes);
    k.slot_jbytes = jbytes;
    if (k.b.draws_out) {
        k.draws_scr = k.b.draws_out;
    } else {
        int st = ensure_scratch(c, (size_t)(k.b.n_chunks > 0 ? k.b.n_chunks : 1) * 2 * (k.T + 1) * 4);
        if (st) return st;
        k.draws_scr = (int32_t *)c->scr;
    }
    return LSLAM_OK;
}

// resolve_kernel LDS: the chunk's staged steps (if they fit)
static int launch_resolve(lslam_ctx *c, const KArgs &base, hipStream_t rs) {
    if (base.b.n_chunks == 0) return LSLAM_OK;
    KArgs k = base;
    const int N = k.b.max_chunk_points > 3 ? k.b.max_chunk_points : 3;
    const int esz = k.j8 ? 1 : 2;
    // stage a chunk's steps in LDS when they fit 16 KiB (C3: 101 x 99 B), else stream them from HBM
    const int De = k.ep_nd > 0 ? k.ep_nd : k.T + 1;  // draws of this launch
    const int64_t need = ((int64_t)De * (N - 1) * esz + 46) & ~(int64_t)15;  // + alignment skew
    const int lds = need <= 16 * 1024 ? (int)need : 0;
    k.res_g = lds;  // staging capacity in bytes
    if (lds == 0) {  // steps streamed from HBM, waves over (chunk, draw)
        const int64_t items = (int64_t)k.b.n_chunks * De;
        // beside the next epoch's producer (produce_draws): four waves per SIMD beside its four
        // parsers.  The epoch loop is max(producer, resolve beside it): with the double-buffered
        // walk, three waves per SIMD measured 65.7-66.1 vs 68.9-69.3 ms per C5 call at two (r06d,
        // four: 66.0-66.3); once mask-mode runs crossed block ends (r06f: a 9 % faster producer)
        // the resolve was the longer again, and four gave 61.4-61.6 vs 63.5-63.6 ms at three.
        // (At r02, with five producer waves per SIMD, three displaced parser workgroups: 107 vs
        // 78 ms.  Measured and dropped: LDS tiles of [64 draws][128 steps], 1.0 vs 0.43 ms per
        // epoch.)
        const int64_t cap = k.ep_count > 1 ? 16 * (int64_t)c->n_cus : (1 << 20);
        const dim3 grid(launch_cap(c, items > cap ? cap : items)), block(64);
        if (k.j8) hipLaunchKernelGGL((resolve_walk_kernel<uint8_t, 16>), grid, block, 0, rs, k);
        else hipLaunchKernelGGL((resolve_walk_kernel<uint16_t, 16>), grid, block, 0, rs, k);
        HIPCHK(hipGetLastError());
        return LSLAM_OK;
    }
    if (k.j8 && c->resolve_beside) {  // no LDS: the producer's workgroups hold most of it
        if (N - 1 <= 16 * RR_GROUPS - 1) {
            // draws of this launch to resolve per chunk: all but draw T (never read by the
            // consensus) unless the caller wants the draws
            const bool has_last = k.ep_d0 + De == k.T + 1;
            const int Dres = (has_last && !k.b.draws_out && De > 1) ? De - 1 : De;
            if ((int64_t)k.b.n_chunks * Dres >= ((int64_t)1 << 31) - 64)
                return set_err(LSLAM_ERR_UNSUPPORTED, "more than 2^31 chunk draws in one call");
            const dim3 grid(launch_cap(c, ((int64_t)k.b.n_chunks * Dres + 63) / 64)), block(64);
            hipLaunchKernelGGL(resolve_reg8_kernel, grid, block, 0, rs, k, Dres);
        } else {
            const dim3 grid(launch_cap(c, k.b.n_chunks)), block(64);
            hipLaunchKernelGGL(resolve_reg_kernel, grid, block, 0, rs, k);
        }
        HIPCHK(hipGetLastError());
        return LSLAM_OK;
    }
    static std::once_flag once;
    std::call_once(once, [] {
        set_max_lds(resolve_kernel<uint8_t>);
        set_max_lds(resolve_kernel<uint16_t>);
    });
    const dim3 grid(launch_cap(c, k.b.n_chunks)), block(64);
    if (k.j8) hipLaunchKernelGGL(resolve_kernel<uint8_t>, grid, block, lds, rs, k);
    else hipLaunchKernelGGL(resolve_kernel<uint16_t>, grid, block, lds, rs, k);
    HIPCHK(hipGetLastError());
    return LSLAM_OK;
}

// Fresh streams (np.random.seed per scan, no mt_state_in): seed_kernel fills a seed buffer and
// k.seed_state points the producer at it.  In the pipeline (on_side) it runs on its own stream
// as soon as the call is enqueued -- after the input waits the producer would make (copies into
// the seeds, a previous call writing them) and after the producer that last read its buffer
// (two buffers by call parity) -- so it overlaps the previous call's producer, and the producer
// only waits for its event.  Measured and dropped: seed_kernel in the producer's stream order,
// right before rng_kernel (every producer launch 40 us later, moved onto the next resolve's
// launch: 0.917 vs 0.715 ms per C3 step) or before its slot wait (0.786 vs 0.716 ms: the
// producers no longer run back to back).  Returns the buffer index used (-1: none).
static int launch_seed(lslam_ctx *c, KArgs &k, hipStream_t stream, bool on_side, bool wait_copy, bool wait_call,
                       int &buf) {
    k.seed_state = nullptr;
    buf = -1;
    if (k.b.mt_state_in || k.b.n_scans <= 0) return LSLAM_OK;
    const int i = on_side ? c->seed_next : 2;
    const size_t need = (size_t)k.b.n_scans * MT_N * 4;
    if (c->seedst_bytes[i] < need) {
        HIPCHK(hipStreamSynchronize(c->stream));
        HIPCHK(hipStreamSynchronize(c->pstream));
        HIPCHK(hipStreamSynchronize(c->sstream));
        if (c->seedst[i]) HIPCHK(hipFree(c->seedst[i]));
        c->seedst[i] = nullptr;
        c->seedst_bytes[i] = 0;
        hipError_t e = hipMalloc(&c->seedst[i], need);
        if (e == hipErrorOutOfMemory) return set_err(LSLAM_ERR_NOMEM, "hipMalloc: out of memory (seed states)");
        HIPCHK(e);
        c->seedst_bytes[i] = need;
    }
    hipStream_t ss = stream;
    if (on_side) {
        ss = c->sstream;
        HIPCHK(hipStreamWaitEvent(ss, c->ev_seed_read[i], 0));
        if (wait_copy) HIPCHK(hipStreamWaitEvent(ss, c->ev_copy, 0));
        if (wait_call) HIPCHK(hipStreamWaitEvent(ss, c->ev_call, 0));
    }
    hipLaunchKernelGGL(seed_kernel, dim3((unsigned)((k.b.n_scans + 63) / 64)), dim3(64), 0, ss, k.b.seeds,
                       (int)k.b.n_scans, c->seedst[i]);
    HIPCHK(hipGetLastError());
    k.cuts = nullptr;
    if (on_side && k.b.n_chunks > 0 && k.b.max_chunk_points <= 128) {  // chunk_kernel's chunks
        const int j = c->cut_next;
        const size_t cneed = (size_t)k.b.n_chunks * sizeof(ChunkCut);
        if (c->cutb_bytes[j] < cneed) {
            HIPCHK(hipStreamSynchronize(c->stream));
            HIPCHK(hipStreamSynchronize(c->pstream));
            HIPCHK(hipStreamSynchronize(c->sstream));
            if (c->cutb[j]) HIPCHK(hipFree(c->cutb[j]));
            c->cutb[j] = nullptr;
            c->cutb_bytes[j] = 0;
            hipError_t e = hipMalloc(&c->cutb[j], cneed);
            if (e == hipErrorOutOfMemory) return set_err(LSLAM_ERR_NOMEM, "hipMalloc: out of memory (chunk cutoffs)");
            HIPCHK(e);
            c->cutb_bytes[j] = cneed;
        }
        hipLaunchKernelGGL(cut_lane_kernel, dim3((unsigned)((k.b.n_chunks + 63) / 64)), dim3(64), 0, ss, k, c->cutb[j]);
        HIPCHK(hipGetLastError());
        k.cuts = c->cutb[j];
        c->cut_next = (j + 1) & 3;
    }
    if (on_side) {
        HIPCHK(hipEventRecord(c->ev_seeded[i], ss));
        HIPCHK(hipStreamWaitEvent(stream, c->ev_seeded[i], 0));
        c->seed_next ^= 1;
    }
    k.seed_state = c->seedst[i];
    buf = on_side ? i : -1;
    return LSLAM_OK;
}

static int launch_rng(lslam_ctx *c, const KArgs &base, hipStream_t stream) {
    KArgs k = base;
    k.rt_all = c->rt_all;
    if (k.b.mt_state_in || k.ep_d0 != 0) k.seed_state = nullptr;  // a chained state, or a later epoch
    int lds = 0;
    int st = layout_rng(k, &k.b, lds);
    if (st) return st;
    static std::once_flag once;
    std::call_once(once, [] {
        set_max_lds(rng_kernel<uint8_t>);
        set_max_lds(rng_kernel<uint16_t>);
    });
    st = timer_begin(c, LSLAM_K_RNG, stream);
    if (st) return st;
    const dim3 grid((unsigned)((k.b.n_scans + RNG_PPW - 1) / RNG_PPW)), block(64 * RNG_PPW);
    if (k.j8) hipLaunchKernelGGL((rng_kernel<uint8_t>), grid, block, lds, stream, k);
    else hipLaunchKernelGGL((rng_kernel<uint16_t>), grid, block, lds, stream, k);
    HIPCHK(hipGetLastError());
    return timer_end(c, LSLAM_K_RNG, stream);
}

// Producer + resolve of a call: one launch, or k.ep_count epochs in alternating
// slots (prepare_steps).  rng_kernel runs on `ps` (after the previous epoch's
// resolve released its slot), the resolve on the ctx stream.  final_out: where
// the last launch writes the end state (null: the slot's state area).  On return
// k.state_scr is the end state's area and last_slot the slot the caller releases.
static int produce_draws(lslam_ctx *c, KArgs &k, int slot, hipStream_t ps, uint32_t *final_out, int &last_slot) {
    const int D = k.T + 1;
    // An epoch's resolve (the lane walk on a grid of two waves per SIMD) runs on the ctx
    // stream beside the next epoch's producer on ps, the slots alternating (C5: 78 vs 89 ms
    // per call with the epochs one after the other).
    const uint32_t *prev_state = nullptr;
    int sl = slot;
    for (int e = 0; e < k.ep_count; e++) {
        KArgs ke = k;
        if (k.ep_count > 1) {
            ke.ep_d0 = e * k.ep_nd;
            ke.ep_nd = std::min(k.ep_nd, D - ke.ep_d0);
            ke.jbuf = (unsigned char *)c->pslot[sl] + JBUF_FRONT;
            ke.state_scr = (uint32_t *)((unsigned char *)c->pslot[sl] + k.slot_jbytes);
            if (e > 0) {
                if (ps != c->stream) HIPCHK(hipStreamWaitEvent(ps, c->ev_slot_free[sl], 0));
                ke.b.mt_state_in = prev_state;  // the previous epoch's end state (same parser, draw boundary)
            }
        }
        const bool last = e == k.ep_count - 1;
        ke.b.mt_state_out = (last && final_out) ? final_out : ke.state_scr;
        int st = launch_rng(c, ke, ps);
        if (st) return st;
        if (ps != c->stream) {
            HIPCHK(hipEventRecord(c->ev_produced, ps));
            HIPCHK(hipStreamWaitEvent(c->stream, c->ev_produced, 0));
        }
        st = launch_resolve(c, ke, c->stream);
        if (st) return st;
        if (!last) HIPCHK(hipEventRecord(c->ev_slot_free[sl], c->stream));
        prev_state = ke.state_scr;
        last_slot = sl;
        sl = (sl + 1) % NSLOTS;
    }
    k.state_scr = const_cast<uint32_t *>(prev_state);
    c->next_slot = sl;
    return LSLAM_OK;
}

static bool ranges_overlap(const void *a, size_t na, const void *b, size_t nb) {
    if (!a || !b || !na || !nb) return false;
    const uintptr_t x = (uintptr_t)a, y = (uintptr_t)b;
    return x < y + nb && y < x + na;
}

// did a copy since the producer last synchronised with ev_copy write [p, p + n)?
static bool copy_unknown_or_hits(const lslam_ctx *c, const void *p, size_t n) {
    if (c->copy_unknown) return true;
    for (int j = 0; j < c->n_copy_rng; j++)
        if (ranges_overlap(p, n, c->copy_rng[j].p, c->copy_rng[j].n)) return true;
    return false;
}

// did a copy since the producer last synchronised with ev_copy write one of its inputs?
static bool copy_hazard(const lslam_ctx *c, const lslam_scan_batch *b) {
    if (c->copy_unknown) return true;
    const void *in[4] = {b->seeds, b->scan_chunk_off, b->chunk_pt_off, b->mt_state_in};
    const size_t len[4] = {(size_t)b->n_scans * 4, (size_t)(b->n_scans + 1) * 4, (size_t)(b->n_chunks + 1) * 4,
                           (size_t)b->n_scans * 625 * 4};
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < c->n_copy_rng; j++)
            if (ranges_overlap(in[i], len[i], c->copy_rng[j].p, c->copy_rng[j].n)) return true;
    return false;
}

// does the producer of this call read anything the previous pipeline call wrote?
// 0: no; 1: only the previous call's mt_state_out (final once that call's fix-up ran:
// a chained stream, e.g. LandmarkMap steps); 2: something else (wait for the whole call)
static int producer_hazard(const lslam_ctx *c, const lslam_scan_batch *b) {
    if (c->out_unknown) return 2;
    const void *in[4] = {b->seeds, b->scan_chunk_off, b->chunk_pt_off, b->mt_state_in};
    const size_t len[4] = {(size_t)b->n_scans * 4, (size_t)(b->n_scans + 1) * 4, (size_t)(b->n_chunks + 1) * 4,
                           (size_t)b->n_scans * 625 * 4};
    int level = 0;
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < c->n_out; j++)
            if (ranges_overlap(in[i], len[i], c->out_ptr[j], c->out_len[j]))
                level = max(level, (i == 3 && c->out_ptr[j] == c->prev_state_out && c->prev_fixed) ? 1 : 2);
    return level;
}

// add [p, p + n) to the union of buffers written since the producer last waited for ev_call
static void note_out(lslam_ctx *c, const void *p, size_t n) {
    if (!p || !n) return;
    for (int i = 0; i < c->n_out; i++)
        if (c->out_ptr[i] == p && c->out_len[i] == n) return;
    if (c->n_out == LSLAM_MAX_OUTS) {
        c->out_unknown = 1;
        return;
    }
    c->out_ptr[c->n_out] = p;
    c->out_len[c->n_out] = n;
    c->n_out++;
}

static void remember_outputs(lslam_ctx *c, const lslam_scan_batch *b, int T, int L) {
    const size_t S = (size_t)b->n_scans, C = (size_t)b->n_chunks, P = (size_t)b->n_points;
    const void *p[11] = {b->inlier_mask, b->models, b->y_proj, b->draws_out, b->trial_cnt_out, b->mt_state_out,
                         b->landmarks, b->lmk_count, b->lmk_walk, b->ukf_x, b->ukf_P};
    const size_t n[11] = {P, C * sizeof(lslam_chunk_model), P * 8, C * 2 * (T + 1) * 4, C * T * 4, S * 625 * 4,
                          S * b->lmk_capacity * sizeof(lslam_landmark), S * 4, S * b->lmk_capacity * 4,
                          L ? S * 24 : 0, L ? S * 72 : 0};
    for (int i = 0; i < 11; i++) note_out(c, p[i], n[i]);
}

// Every entry point that enqueues device work ends here.  Each call's work on the producer
// and side streams joins the ctx stream before the call returns, so "every call so far" is the
// ctx stream's tail: copies on the ctx stream follow it by stream order, and another stream
// that must wait for it records ev_call at that moment (mark_calls) and waits on that.  An
// event recorded at every call's end would be a marker packet inside the pipelined ctx chain
// (~7 us between two kernels on the MI355X).
static int end_call(lslam_ctx *c) {
    (void)c;
    return LSLAM_OK;
}
static int mark_calls(lslam_ctx *c) {
    HIPCHK(hipEventRecord(c->ev_call, c->stream));
    return LSLAM_OK;
}

// select_kernel LDS: the chunk's points, tied trials, tie sums, mask, sum scratch
static int layout_select(KArgs &k, const lslam_scan_batch *b, int &lds) {
    const int N = b->max_chunk_points > 0 ? b->max_chunk_points : 1;
    const int T = k.T > 0 ? k.T : 1;
    int off = 0;
    k.off_pts = off; off += align16(16 * N);
    k.off_tied = off; off += align16(4 * T);
    k.off_cnt = off; off += align16(4 * T);
    k.off_tsum = off; off += align16(8 * T);
    k.off_mask = off; off += align16(N);
    k.off_vstack = off; off += align16(8 * 24);
    k.off_nstack = off; off += align16(4 * 72);
    k.off_vtmp = off; off += align16(8 * 128);
    lds = off;
    if (lds > 160 * 1024) return set_err(LSLAM_ERR_CAPACITY, "chunk/trial sizes exceed the 160 KiB LDS");
    return LSLAM_OK;
}

static int ensure_cscr(lslam_ctx *c, size_t bytes) {
    if (c->cscr_bytes >= bytes) return LSLAM_OK;
    HIPCHK(hipStreamSynchronize(c->stream));
    if (c->cscr) HIPCHK(hipFree(c->cscr));
    c->cscr = nullptr;
    c->cscr_bytes = 0;
    hipError_t e = hipMalloc(&c->cscr, bytes);
    if (e == hipErrorOutOfMemory) return set_err(LSLAM_ERR_NOMEM, "hipMalloc: out of memory (consensus scratch)");
    HIPCHK(e);
    c->cscr_bytes = bytes;
    return LSLAM_OK;
}

// chunks of more than 128 points: count_kernel (many waves per chunk) + select_kernel
static int launch_chunks_large(lslam_ctx *c, KArgs &k) {
    const int T = k.T;
    const size_t nc = (size_t)k.b.n_chunks;
    const size_t cnt_bytes = (k.b.trial_cnt_out || T == 0) ? 0 : ((nc * T * 4 + 255) & ~(size_t)255);
    const bool philox = k.hyp_source == LSLAM_HYP_PHILOX;
    const size_t drw_bytes = (philox && !k.b.draws_out) ? ((nc * 2 * (size_t)(T + 1) * 4 + 255) & ~(size_t)255) : 0;
    const size_t mdl_bytes = nc * (size_t)(T > 0 ? T : 1) * 32;
    int st = ensure_cscr(c, cnt_bytes + drw_bytes + mdl_bytes);
    if (st) return st;
    unsigned char *base = (unsigned char *)c->cscr;
    k.cnt_scr = k.b.trial_cnt_out ? k.b.trial_cnt_out : (int32_t *)base;
    if (philox) k.draws_scr = k.b.draws_out ? k.b.draws_out : (int32_t *)(base + cnt_bytes);
    k.models = (double *)(base + cnt_bytes + drw_bytes);
    const int N = k.b.max_chunk_points;
    int lds_sel = 0;
    st = layout_select(k, &k.b, lds_sel);
    if (st) return st;
    k.cnt_blocks = T > 0 ? (T + CNT_HYP_BLOCK - 1) / CNT_HYP_BLOCK : 0;
    static std::once_flag once;
    std::call_once(once, [] {
        set_max_lds(select_kernel<LSLAM_HYP_MT19937>);
        set_max_lds(select_kernel<LSLAM_HYP_PHILOX>);
        set_max_lds(select_kernel<LSLAM_HYP_EXPLICIT>);
    });
    const size_t nmod = nc * (size_t)(T + 1);
    const dim3 mgrid((unsigned)((nmod + 255) / 256)), block(256);
    switch (k.hyp_source) {
        case LSLAM_HYP_PHILOX: hipLaunchKernelGGL(model_kernel<LSLAM_HYP_PHILOX>, mgrid, block, 0, c->stream, k); break;
        case LSLAM_HYP_EXPLICIT: hipLaunchKernelGGL(model_kernel<LSLAM_HYP_EXPLICIT>, mgrid, block, 0, c->stream, k); break;
        default: hipLaunchKernelGGL(model_kernel<LSLAM_HYP_MT19937>, mgrid, block, 0, c->stream, k); break;
    }
    HIPCHK(hipGetLastError());
    if (k.cnt_blocks > 0) {
        const dim3 grid((unsigned)(nc * k.cnt_blocks)), cblock(CNT_TPB);
        // points per lane: the smallest power of two covering the chunk, at most 16 (then tiles)
        if (N <= 256) hipLaunchKernelGGL(count_kernel<1>, grid, cblock, 0, c->stream, k);
        else if (N <= 512) hipLaunchKernelGGL(count_kernel<2>, grid, cblock, 0, c->stream, k);
        else if (N <= 1024) hipLaunchKernelGGL(count_kernel<4>, grid, cblock, 0, c->stream, k);
        else if (N <= 2048) hipLaunchKernelGGL(count_kernel<8>, grid, cblock, 0, c->stream, k);
        else hipLaunchKernelGGL(count_kernel<16>, grid, cblock, 0, c->stream, k);
        HIPCHK(hipGetLastError());
    }
    const dim3 grid((unsigned)nc), sblock(64);
    switch (k.hyp_source) {
        case LSLAM_HYP_PHILOX: hipLaunchKernelGGL(select_kernel<LSLAM_HYP_PHILOX>, grid, sblock, lds_sel, c->stream, k); break;
        case LSLAM_HYP_EXPLICIT: hipLaunchKernelGGL(select_kernel<LSLAM_HYP_EXPLICIT>, grid, sblock, lds_sel, c->stream, k); break;
        default: hipLaunchKernelGGL(select_kernel<LSLAM_HYP_MT19937>, grid, sblock, lds_sel, c->stream, k); break;
    }
    HIPCHK(hipGetLastError());
    return LSLAM_OK;
}

static int launch_chunks(lslam_ctx *c, const KArgs &base, bool write_yproj) {
    if (base.b.n_chunks == 0) return LSLAM_OK;
    KArgs k = base;
    k.write_yproj = write_yproj ? 1 : 0;
    int st = timer_begin(c, LSLAM_K_CONSENSUS);
    if (st) return st;
    if (k.b.max_chunk_points > 128) {
        st = launch_chunks_large(c, k);
        if (st) return st;
        return timer_end(c, LSLAM_K_CONSENSUS);
    }
    int lds = 0;
    st = layout_chunk(k, &k.b, lds);
    if (st) return st;
    static std::once_flag once;
    std::call_once(once, [] {
        set_max_lds(chunk_kernel<LSLAM_HYP_MT19937>);
        set_max_lds(chunk_kernel<LSLAM_HYP_PHILOX>);
        set_max_lds(chunk_kernel<LSLAM_HYP_EXPLICIT>);
    });
    const dim3 grid(launch_cap(c, k.b.n_chunks)), block(64);
    switch (k.hyp_source) {
        case LSLAM_HYP_PHILOX: hipLaunchKernelGGL(chunk_kernel<LSLAM_HYP_PHILOX>, grid, block, lds, c->stream, k); break;
        case LSLAM_HYP_EXPLICIT: hipLaunchKernelGGL(chunk_kernel<LSLAM_HYP_EXPLICIT>, grid, block, lds, c->stream, k); break;
        default: hipLaunchKernelGGL(chunk_kernel<LSLAM_HYP_MT19937>, grid, block, lds, c->stream, k); break;
    }
    HIPCHK(hipGetLastError());
    return timer_end(c, LSLAM_K_CONSENSUS);
}

template <int MODE>
static int launch_post(lslam_ctx *c, const KArgs &k, int lds) {
    static std::once_flag once;
    std::call_once(once, [] {
        set_max_lds(scan_kernel<LSLAM_HYP_EXPLICIT, MODE>);
        set_max_lds(scan_kernel_w4<LSLAM_HYP_EXPLICIT, MODE>);
    });
    const dim3 grid(launch_cap(c, k.b.n_scans));
    if (MODE == MODE_ASSOC && k.lmk_reg) {
        static std::once_flag once_reg;
        std::call_once(once_reg, [] { set_max_lds(post_reg_kernel); });
        hipLaunchKernelGGL(post_reg_kernel, grid, dim3(64), lds, c->stream, k);
    } else if (k.hyp_source == LSLAM_HYP_MT19937)  // beside the next call's producer
        hipLaunchKernelGGL((scan_kernel<LSLAM_HYP_EXPLICIT, MODE>), grid, dim3(64), lds, c->stream, k);
    else
        hipLaunchKernelGGL((scan_kernel_w4<LSLAM_HYP_EXPLICIT, MODE>), grid, dim3(64), lds, c->stream, k);
    HIPCHK(hipGetLastError());
    return LSLAM_OK;
}

// rng_kernel -> chunk_kernel -> fix-up -> association/UKF post pass, all on the ctx stream
static int run_split(lslam_ctx *c, const lslam_scan_batch *b, const lslam_ransac_params *p,
                     const lslam_ukf_params *u) {
    HIPCHK(hipSetDevice(c->device));
    if (b->n_scans == 0) return LSLAM_OK;
#if defined(LSLAM_STAMPS) || defined(LSLAM_CENSUS)
    g_call_seq += 1;
#endif
    const bool assoc = b->landmarks != nullptr;
    KArgs k;
    int lds_fix = 0;
    int st = build_args(k, b, p, nullptr, MODE_RANSAC, lds_fix);
    if (st) return st;
    const bool mt = k.hyp_source == LSLAM_HYP_MT19937;
    bool spec = false;
    int seed_buf = -1;  // the seed buffer this call's producer reads (launch_seed)
    int slot = c->next_slot;
    if (mt) {
        st = prepare_steps(c, k, slot);
        if (st) return st;
        c->next_slot = (c->next_slot + 1) % NSLOTS;
    }
    KArgs kp;
    int lds_post = 0;
    // a UKF step that reads nothing of this call's RANSAC (no LMK_FROM_RANSAC / MAP) runs
    // on the side stream, off the resolve -> consensus -> association chain
    // (Philox / explicit hypotheses only: beside the MT producer a third stream of UKF waves
    // slows the resolve -> consensus chain more than it saves, 1.23 -> 1.27-1.32 ms on C3, and
    // made the step bimodal)
    const bool ukf_side = p->hyp_source != LSLAM_HYP_MT19937 && u &&
                          !(u->flags & (LSLAM_UKF_LMK_FROM_RANSAC | LSLAM_UKF_MAP));
    // the UKF of the fused call on lane groups after the association pass (not in MAP mode,
    // whose measurements come out of the association walk itself)
    const bool ukf_lane = u && !ukf_side && !(u->flags & LSLAM_UKF_MAP);
    const int pmode = (assoc ? MODE_ASSOC : MODE_POST) | (u && !ukf_side && !ukf_lane ? MODE_UKF : 0);
    if ((pmode & MODE_UKF) && !(u->flags & LSLAM_UKF_MAP))  // scan_body's one-wave UKF fuses no origins
        return set_err(LSLAM_ERR_UNSUPPORTED, "post pass given a non-map UKF step");
    if (assoc || (u && !ukf_side && !ukf_lane)) {
        st = build_args(kp, b, p, (ukf_side || ukf_lane) ? nullptr : u, pmode, lds_post);
        if (st) return st;
    }
    KArgs kl;
    if (ukf_lane) {
        int lds_l = 0;
        st = build_args(kl, b, p, u, MODE_UKF, lds_l);
        if (st) return st;
        if ((u->flags & LSLAM_UKF_LMK_FROM_RANSAC) && !b->models)
            return set_err(LSLAM_ERR_ARG, "LSLAM_UKF_LMK_FROM_RANSAC needs the chunk models");
    }
    KArgs ku;
    int lds_u = 0;
    if (ukf_side) {
        st = build_args(ku, b, nullptr, u, MODE_UKF, lds_u);
        if (st) return st;
    }
    st = timer_begin(c, LSLAM_K_PIPELINE);
    if (st) return st;
    if (ukf_side) {
        // after the previous call (its outputs may be this step's inputs) and the latest copies
        if ((st = mark_calls(c))) return st;
        HIPCHK(hipStreamWaitEvent(c->ustream, c->ev_call, 0));
        HIPCHK(hipStreamWaitEvent(c->ustream, c->ev_copy, 0));
        launch_ukf_group(ku, u->n_landmarks, c->ustream, false);
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(c->ev_ukf, c->ustream));
    }
    if (mt) {
        // producer on its own stream: it waits for input copies, (on a hazard) for the previous
        // call, and for its slot's previous consumers; the consumers wait for it.  A fresh
        // stream's seed_kernel goes between the input waits and the slot wait (launch_seed).
        // a copy into this call's MT state (e.g. a caller's upload into the previous call's
        // mt_state_out) invalidates speculating from the previous producer's end state
        const bool state_copied = copy_unknown_or_hits(c, b->mt_state_in, (size_t)b->n_scans * 625 * 4);
        const bool chz = copy_hazard(c, b);
        if (chz) {
            HIPCHK(hipStreamWaitEvent(c->pstream, c->ev_copy, 0));
            c->n_copy_rng = 0;
            c->copy_unknown = 0;
        }
        const int hz = producer_hazard(c, b);
        if (hz == 2) {
            // ev_call follows every call enqueued so far: the union starts afresh
            if ((st = mark_calls(c))) return st;
            HIPCHK(hipStreamWaitEvent(c->pstream, c->ev_call, 0));
            c->n_out = 0;
            c->out_unknown = 0;
        }
        if ((st = launch_seed(c, k, c->pstream, true, chz, hz == 2, seed_buf))) return st;
        HIPCHK(hipStreamWaitEvent(c->pstream, c->ev_slot_free[slot], 0));
        // speculation (a chained stream, e.g. LandmarkMap steps): parse from the previous
        // producer's end state, which precedes this producer on pstream, instead of waiting for
        // the previous fix-up; this call's fix-up replays the scans that one replayed
        spec = hz == 1 && c->speculate && c->spec_ok && k.ep_count == 1 && c->prev_state_scr &&
               c->prev_spec_scans == b->n_scans && b->mt_state_in == c->prev_state_out && !state_copied;
        // a scan replayed by a speculative call stays dirty in every later one (its producer state
        // is never repaired): every SPEC_RESYNC-th chained call waits for the
        // previous fix-up instead, which clears the flags (test_gpu_speculate.py runs past it)
        constexpr int SPEC_RESYNC = 32;
        if (spec && ++c->spec_run >= SPEC_RESYNC) spec = false;
        if (!spec) c->spec_run = 0;
        if (hz == 1 && !spec) HIPCHK(hipStreamWaitEvent(c->pstream, c->ev_slot_free[c->prev_slot], 0));
        // a producer that waited on the previous call will most likely wait on this one too, so
        // this call's resolve runs alone: the LDS-staged form is faster there (map mode 1.48 vs
        // 1.39 ms per step); otherwise the next call's producer runs beside it and holds the LDS
        // (C3 0.93 vs 1.03 ms)
        c->resolve_beside = hz == 0 || spec;
        const uint32_t *true_in = k.b.mt_state_in;
        if (spec) k.b.mt_state_in = c->prev_state_scr;
        st = produce_draws(c, k, slot, c->pstream, nullptr, slot);  // slot <- the last epoch's
        k.b.mt_state_in = true_in;  // the fix-up's replays start from the true state
        if (st) return st;
        if (seed_buf >= 0) HIPCHK(hipEventRecord(c->ev_seed_read[seed_buf], c->pstream));
    }
    // A UKF that reads nothing of this call's RANSAC runs between the fix-up and the post pass.
    // The fix-up releases this call's steps slot; the next producer starts ~40 us after that
    // event, so a UKF placed right behind the fix-up runs alone (35 us) instead of beside the
    // parsers (~180 us): C3 0.893 -> 0.858 ms per step, the producer 0.79 -> 0.71 ms in the
    // pipeline.  (Measured and dropped, DESIGN.md §8: the UKF before the fix-up, +2.7 %, or
    // before the consensus, +0.8 %; the slot released after the post pass or at the call's end.)
    const bool ukf_indep = ukf_lane && !(u->flags & (LSLAM_UKF_LMK_FROM_RANSAC | LSLAM_UKF_MAP));
    st = launch_chunks(c, k, !assoc);
    if (st) return st;
    if (mt) {
        KArgs kf = k;
        kf.fixup = 1;
        // replay flags: this call's, for the next call's speculation (one epoch only: the
        // end state is then the slot's state area)
        if (k.ep_count == 1 && b->mt_state_out) {
            if (c->spec_dirty_n < b->n_scans) {
                HIPCHK(hipStreamSynchronize(c->stream));
                for (int i = 0; i < 2; i++) {
                    if (c->spec_dirty[i]) HIPCHK(hipFree(c->spec_dirty[i]));
                    c->spec_dirty[i] = nullptr;
                }
                c->spec_dirty_n = 0;
                for (int i = 0; i < 2; i++) {
                    hipError_t e = hipMalloc(&c->spec_dirty[i], (size_t)b->n_scans);
                    if (e == hipErrorOutOfMemory) return set_err(LSLAM_ERR_NOMEM, "hipMalloc: out of memory (flags)");
                    HIPCHK(e);
                }
                c->spec_dirty_n = b->n_scans;
                if (spec) return set_err(LSLAM_ERR_HIP, "speculation without replay flags");  // unreachable
            }
            kf.spec_dirty_in = spec ? c->spec_dirty[c->spec_cur] : nullptr;
            kf.spec_dirty_out = c->spec_dirty[c->spec_cur ^ 1];
        }
        static std::once_flag once;
        std::call_once(once, [] { set_max_lds(scan_kernel<LSLAM_HYP_MT19937, MODE_RANSAC>); });
        hipLaunchKernelGGL((scan_kernel<LSLAM_HYP_MT19937, MODE_RANSAC>), dim3(launch_cap(c, b->n_scans)), dim3(64), lds_fix,
                           c->stream, kf);
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(c->ev_slot_free[slot], c->stream));
    }
    if (ukf_indep) {
        launch_ukf_group(kl, u->n_landmarks, c->stream, true);
        HIPCHK(hipGetLastError());
    }
    // (mt_state_out is final after the fix-up: the next call's producer may chain from it early)
    c->prev_state_out = mt ? b->mt_state_out : nullptr;
    c->prev_slot = slot;
    c->prev_fixed = mt ? 1 : 0;
    c->spec_ok = (mt && k.ep_count == 1 && b->mt_state_out) ? 1 : 0;
    if (c->spec_ok) {
        c->spec_cur ^= 1;  // the buffer this call's fix-up writes
        c->prev_state_scr = k.state_scr;
        c->prev_spec_scans = b->n_scans;
    }
    switch (pmode) {
        case MODE_ASSOC | MODE_UKF: st = launch_post<MODE_ASSOC | MODE_UKF>(c, kp, lds_post); break;
        case MODE_POST | MODE_UKF: st = launch_post<MODE_POST | MODE_UKF>(c, kp, lds_post); break;
        case MODE_ASSOC: st = launch_post<MODE_ASSOC>(c, kp, lds_post); break;
        default: break;
    }
    if (st) return st;
    if (ukf_lane && !ukf_indep) {  // reads this call's chunk models (LMK_FROM_RANSAC)
        launch_ukf_group(kl, u->n_landmarks, c->stream, true);
        HIPCHK(hipGetLastError());
    }
    if (ukf_side) HIPCHK(hipStreamWaitEvent(c->stream, c->ev_ukf, 0));
    remember_outputs(c, b, k.T, u ? u->n_landmarks : 0);
    if ((st = end_call(c))) return st;
    return timer_end(c, LSLAM_K_PIPELINE);
}


// ---- express-scan codec (lslam_express.h) ----

static inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

static int ensure_escr(lslam_ctx *c, size_t bytes) {
    if (c->escr_bytes >= bytes) return LSLAM_OK;
    HIPCHK(hipStreamSynchronize(c->stream));
    if (c->escr) HIPCHK(hipFree(c->escr));
    c->escr = nullptr;
    c->escr_bytes = 0;
    hipError_t e = hipMalloc(&c->escr, bytes);
    if (e == hipErrorOutOfMemory) return set_err(LSLAM_ERR_NOMEM, "hipMalloc: out of memory (express scratch)");
    HIPCHK(e);
    c->escr_bytes = bytes;
    return LSLAM_OK;
}

// packet streams are read as dwords: 4-byte alignment, and every rank fits int32
static int express_check(const uint8_t *packets, int64_t n) {
    if (n < 0 || (n > 0 && !packets)) return set_err(LSLAM_ERR_ARG, "express: bad packet stream");
    if (((uintptr_t)packets & 3) != 0) return set_err(LSLAM_ERR_ARG, "express: packet stream must be 4-byte aligned");
    if (n > ((int64_t)1 << 26)) return set_err(LSLAM_ERR_ARG, "express: more than 2^26 packets per call");
    return LSLAM_OK;
}

extern "C" {

int lslam_polar_to_xy(lslam_ctx *c, const double *th, const double *d, double *xy, int64_t n) {
    if (!c || n < 0 || (n > 0 && (!th || !d || !xy))) return LSLAM_ERR_ARG;
    if (n == 0) return LSLAM_OK;
    HIPCHK(hipSetDevice(c->device));
    int64_t blocks = (n + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    int st = timer_begin(c, LSLAM_K_POLAR);
    if (st) return st;
    hipLaunchKernelGGL(polar_kernel, dim3((unsigned)blocks), dim3(256), 0, c->stream, th, d, (double2 *)xy, n);
    HIPCHK(hipGetLastError());
    st = timer_end(c, LSLAM_K_POLAR);
    if (st) return st;
    note_out(c, xy, (size_t)n * 16);
    return end_call(c);
}

int lslam_set_steps_budget(lslam_ctx *c, int64_t bytes) {
    if (!c) return LSLAM_ERR_ARG;
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(c->pstream));
    HIPCHK(hipStreamSynchronize(c->stream));
    c->steps_budget = bytes > 0 ? (size_t)bytes : default_steps_budget();
    return LSLAM_OK;
}

int lslam_hyp_mt19937(lslam_ctx *c, const lslam_scan_batch *b, int32_t max_trials) {
    if (!c) return LSLAM_ERR_ARG;
    int st = validate_batch(b, false);
    if (st) return st;
    if (!b->draws_out) return set_err(LSLAM_ERR_ARG, "draws_out required");
    lslam_ransac_params p;
    lslam_ransac_params_default(&p);
    p.max_trials = max_trials;
    KArgs k;
    int lds = 0;
    st = build_args(k, b, &p, nullptr, MODE_HYP_ONLY, lds);
    if (st) return st;
    HIPCHK(hipSetDevice(c->device));
    if (b->n_scans == 0) return LSLAM_OK;
    k.hyp_source = LSLAM_HYP_MT19937;
    const int slot = c->next_slot;
    st = prepare_steps(c, k, slot);
    if (st) return st;
    c->next_slot = (c->next_slot + 1) % NSLOTS;
    st = timer_begin(c, LSLAM_K_HYP);
    if (st) return st;
    HIPCHK(hipStreamWaitEvent(c->stream, c->ev_slot_free[slot], 0));
    int last = slot;
    // on the main stream; the end state goes straight to mt_state_out
    c->resolve_beside = 0;  // alone on the ctx stream
    int seed_buf = -1;
    if ((st = launch_seed(c, k, c->stream, false, false, false, seed_buf))) return st;
    st = produce_draws(c, k, slot, c->stream, b->mt_state_out, last);
    if (st) return st;
    HIPCHK(hipEventRecord(c->ev_slot_free[last], c->stream));
    // the end state is written by the rng kernel itself, final at ev_slot_free[slot]: a
    // pipeline call chaining from it waits for that event, anything else for ev_call
    note_out(c, b->draws_out, (size_t)b->n_chunks * 2 * (size_t)(max_trials + 1) * 4);
    note_out(c, b->mt_state_out, (size_t)b->n_scans * 625 * 4);
    c->prev_state_out = b->mt_state_out;
    c->prev_slot = last;
    c->prev_fixed = b->mt_state_out ? 1 : 0;
    c->spec_ok = 0;
    c->spec_run = 0;
    if ((st = end_call(c))) return st;
    return timer_end(c, LSLAM_K_HYP);
}

int lslam_ransac(lslam_ctx *c, const lslam_scan_batch *b, const lslam_ransac_params *p) {
    if (!c || !p) return LSLAM_ERR_ARG;
    int st = validate_batch(b, true);
    if (st) return st;
    return run_split(c, b, p, nullptr);
}

int lslam_landmarks(lslam_ctx *c, const lslam_scan_batch *b, const lslam_ransac_params *p) {
    if (!c || !p) return LSLAM_ERR_ARG;
    int st = validate_batch(b, true);
    if (st) return st;
    if (!b->models || !b->landmarks || !b->inlier_mask) return set_err(LSLAM_ERR_ARG, "models/landmarks/mask required");
    KArgs k;
    int lds = 0;
    st = build_args(k, b, p, nullptr, MODE_ASSOC, lds);
    if (st) return st;
    if ((st = run_scan_kernel<MODE_ASSOC>(c, k, lds, LSLAM_K_LANDMARK))) return st;
    remember_outputs(c, b, k.T, 0);
    return end_call(c);
}

static int ukf_step_impl(lslam_ctx *c, const lslam_scan_batch *b, const lslam_ukf_params *u, double *trace) {
    if (!c || !u || !b) return LSLAM_ERR_ARG;
    if (b->n_scans < 0) return LSLAM_ERR_ARG;
    lslam_scan_batch bb = *b;
    // UKF-only: no chunks are touched; give the kernel an empty CSR if absent
    KArgs k;
    int lds = 0;
    if (!bb.scan_chunk_off) return set_err(LSLAM_ERR_ARG, "scan_chunk_off required (may describe 0 chunks)");
    int st = build_args(k, &bb, nullptr, u, MODE_UKF, lds);
    if (st) return st;
    const bool lanes = !(u->flags & LSLAM_UKF_MAP);  // MAP: the one-wave form (its post pass's step)
    if ((u->flags & LSLAM_UKF_SIGMAS_IN) && !b->ukf_sigmas)
        return set_err(LSLAM_ERR_ARG, "LSLAM_UKF_SIGMAS_IN without ukf_sigmas");
    if ((b->ukf_sigmas || trace) && !lanes)
        return set_err(LSLAM_ERR_UNSUPPORTED, "ukf_sigmas / trace need the lane-group UKF (not LSLAM_UKF_MAP)");
    if (trace && !(u->flags & LSLAM_UKF_UPDATE)) return set_err(LSLAM_ERR_ARG, "lslam_ukf_trace needs LSLAM_UKF_UPDATE");
    if (trace || b->ukf_sigmas) {
        HIPCHK(hipSetDevice(c->device));
        if (k.b.n_scans > 0) {
            if ((st = timer_begin(c, LSLAM_K_UKF))) return st;
            launch_ukf_group(k, k.ukf.L, c->stream, false, trace);
            HIPCHK(hipGetLastError());
            if ((st = timer_end(c, LSLAM_K_UKF))) return st;
        }
    } else if ((st = run_scan_kernel<MODE_UKF>(c, k, lds, LSLAM_K_UKF))) {
        return st;
    }
    note_out(c, b->ukf_x, (size_t)b->n_scans * 24);
    note_out(c, b->ukf_P, (size_t)b->n_scans * 72);
    if (b->ukf_sigmas) note_out(c, b->ukf_sigmas, (size_t)b->n_scans * 168);
    if (trace) note_out(c, trace, (size_t)b->n_scans * 8 * ukf_tr_doubles(u->n_landmarks));
    return end_call(c);
}

int lslam_ukf_step(lslam_ctx *c, const lslam_scan_batch *b, const lslam_ukf_params *u) {
    return ukf_step_impl(c, b, u, nullptr);
}

int lslam_ukf_trace(lslam_ctx *c, const lslam_scan_batch *b, const lslam_ukf_params *u, double *trace) {
    if (!trace) return set_err(LSLAM_ERR_ARG, "trace buffer required");
    return ukf_step_impl(c, b, u, trace);
}

int lslam_scan_pipeline(lslam_ctx *c, const lslam_scan_batch *b, const lslam_ransac_params *p,
                        const lslam_ukf_params *u) {
    if (!c || !p) return LSLAM_ERR_ARG;
    int st = validate_batch(b, true);
    if (st) return st;
    if (u && ((u->flags & LSLAM_UKF_SIGMAS_IN) || b->ukf_sigmas))
        return set_err(LSLAM_ERR_UNSUPPORTED, "ukf_sigmas / LSLAM_UKF_SIGMAS_IN are lslam_ukf_step's (filterpy's cache)");
    return run_split(c, b, p, u);
}

int lslam_express_decode(lslam_ctx *c, const uint8_t *packets, int64_t n_packets, const lslam_express_measures *out) {
    if (!c || !out) return LSLAM_ERR_ARG;
    int st = express_check(packets, n_packets);
    if (st) return st;
    if (n_packets == 0) return LSLAM_OK;
    HIPCHK(hipSetDevice(c->device));
    ExpressOut o{out->angle_deg, out->dist_mm, out->new_scan, out->valid, (double2 *)out->xy, out->pkt_valid};
    if ((st = timer_begin(c, LSLAM_K_EXPRESS))) return st;
    const int64_t blocks = (n_packets + EXP_DEC_PER_WG - 1) / EXP_DEC_PER_WG;
    hipLaunchKernelGGL(express_decode_kernel, dim3((unsigned)blocks), dim3(256), 0, c->stream, packets, n_packets, o);
    HIPCHK(hipGetLastError());
    if ((st = timer_end(c, LSLAM_K_EXPRESS))) return st;
    const size_t nm = (size_t)(n_packets > 1 ? n_packets - 1 : 0) * 32;
    note_out(c, out->angle_deg, nm * 8);
    note_out(c, out->dist_mm, nm * 8);
    note_out(c, out->new_scan, nm);
    note_out(c, out->valid, nm);
    note_out(c, out->xy, nm * 16);
    note_out(c, out->pkt_valid, (size_t)n_packets);
    return end_call(c);
}

int lslam_express_scans(lslam_ctx *c, const uint8_t *packets, int64_t n_packets, int32_t skip,
                        const lslam_express_revs *out) {
    if (!c || !out || !out->counts || !out->scan_chunk_off || !out->chunk_pt_off) return LSLAM_ERR_ARG;
    if (out->cap_scans < 0 || out->cap_chunks < 0 || out->cap_points < 0 || (out->cap_points > 0 && !out->xy))
        return set_err(LSLAM_ERR_ARG, "express: bad output capacities");
    int st = express_check(packets, n_packets);
    if (st) return st;
    if (skip < 0 || skip > 31) return set_err(LSLAM_ERR_ARG, "express: skip must be in [0, 31]");
    HIPCHK(hipSetDevice(c->device));
    const int64_t np = n_packets > 1 ? n_packets - 1 : 0;  // packets that carry measures
    const int64_t tiles = (np + EXP_TILE - 1) / EXP_TILE;
    size_t off = 0;
    const size_t o_flags = off;
    off = align256(off + (size_t)np);
    const size_t o_tile = off;
    off = align256(off + (size_t)tiles * sizeof(int2));
    const size_t o_rank = off;
    off = align256(off + (size_t)np * sizeof(int2));
    const size_t o_rend = off;
    off = align256(off + (size_t)np * sizeof(int2));
    const size_t o_rinfo = off;
    off = align256(off + (size_t)np * sizeof(int4));
    if ((st = ensure_escr(c, off > 0 ? off : 256))) return st;
    uint8_t *base = (uint8_t *)c->escr;
    ExpressScratch s{base + o_flags, (int2 *)(base + o_tile), (int2 *)(base + o_rank), (int2 *)(base + o_rend),
                     (int4 *)(base + o_rinfo), out->counts};
    ExpressScans o{(double2 *)out->xy, out->scan_chunk_off, out->chunk_pt_off, out->cap_points, out->cap_scans,
                   out->cap_chunks};
    if ((st = timer_begin(c, LSLAM_K_EXPRESS))) return st;
    if (tiles > 0) {
        hipLaunchKernelGGL(express_flags_kernel, dim3((unsigned)tiles), dim3(256), 0, c->stream, packets, n_packets,
                           (int)skip, s);
        HIPCHK(hipGetLastError());
        hipLaunchKernelGGL(express_rank_kernel, dim3((unsigned)tiles), dim3(256), 0, c->stream, n_packets, (int)skip, s);
        HIPCHK(hipGetLastError());
    }
    // revolutions <= packets with measures: one 256-revolution workgroup per packet tile
    hipLaunchKernelGGL(express_revs_kernel, dim3((unsigned)(tiles > 0 ? tiles : 1)), dim3(256), 0, c->stream,
                       (int)tiles, s, o);
    HIPCHK(hipGetLastError());
    if (np > 0) {
        if ((st = timer_begin(c, LSLAM_K_EXPRESS_SCATTER))) return st;
        const int64_t blocks = (np + EXP_DEC_PER_WG - 1) / EXP_DEC_PER_WG;
        hipLaunchKernelGGL(express_scatter_kernel, dim3((unsigned)blocks), dim3(256), 0, c->stream, packets, n_packets,
                           (int)skip, s, o);
        HIPCHK(hipGetLastError());
        if ((st = timer_end(c, LSLAM_K_EXPRESS_SCATTER))) return st;
    }
    if ((st = timer_end(c, LSLAM_K_EXPRESS))) return st;
    // the outputs may feed a pipeline call whose MT producer runs on the other stream
    HIPCHK(hipEventRecord(c->ev_copy, c->stream));
    note_copy(c, out->xy, (size_t)out->cap_points * 16);
    note_copy(c, out->scan_chunk_off, ((size_t)out->cap_scans + 1) * 4);
    note_copy(c, out->chunk_pt_off, ((size_t)out->cap_chunks + 1) * 4);
    note_copy(c, out->counts, 16);
    return end_call(c);
}

}  // extern "C"
