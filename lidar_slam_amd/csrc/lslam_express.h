// lslam_express.h — RPLidar express-scan packets -> measures -> revolutions
// of chunked Cartesian points, on the GPU (SURVEY §8f rank 2 + rows A1/A2).
//
// Reference: lidar.py:55-59 twos_comp, :59-91 ExpressPacket.decode,
// :179-187 Lidar._process_express_scan, :327-338 the measure stream of
// Lidar.scan('express') (packet p's 32 measures use packet p+1's start
// angle); functions.py:56-76 the capture loop (A1 polar -> Cartesian, A2 a
// chunk every 100 points, on the new-revolution flag the remainder if it has
// more than 2 points, then the revolution delimiter).
//
// A packet whose sync nibbles or XOR checksum are wrong raises ValueError in
// the reference (and ends its capture process); here it is flagged, the
// measures that need it (its own and its predecessor's) are invalid, and the
// revolution builder skips them.
//
// Kernels (all HBM-bound byte/integer work, a few exact FP64 ops per measure):
//   express_decode_kernel   measure-level SoA outputs (angle, dist, flags, xy)
//   express_flags_kernel    per packet: valid + new-revolution bits, per-tile sums
//   express_rank_kernel     per packet: measure rank + revolution index
//   express_revs_kernel     per revolution: kept points, chunks -> CSR offsets
//   express_scatter_kernel  decode + A1 + write each kept measure's xy in place
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lslam {

constexpr int EXP_PKT = 84;          // bytes per express packet
constexpr int EXP_ROWS = 4;          // decode/scatter: each lane handles cabin k of 4 packets
constexpr int EXP_DEC_PER_WG = 8 * EXP_ROWS;  // 256 lanes = 8 packet rows x 32 cabins, 4 times
constexpr int EXP_TILE = 256;        // flags/rank: one packet per lane
constexpr int EXP_CHUNK = 100;       // functions.py:14 MIN_NEIGHBOORS
constexpr int EXP_MIN_REM = 2;       // functions.py:70 len(distancesList) > 2

// pkt_flags bits
constexpr uint8_t EXP_OK = 1;        // packets p and p+1 decode: p's 32 measures exist
constexpr uint8_t EXP_NEW = 2;       // p's measure 0 carries the new-revolution flag

// lidar.py:55-59: only bit (bits-1) is tested, higher bits pass through
__device__ __forceinline__ int twos_comp5(int v) { return (v & 16) ? v - 32 : v; }

// Stage packets [p0, p0 + n) of the stream into LDS with 16-byte loads from the
// 16-byte aligned-down start; returns the byte offset of packet p0 in `st`.
// Requires a 4-byte aligned stream (checked by the host), so the offset is a
// multiple of 4 and packets can be read as dwords.
__device__ __forceinline__ int stage_packets(uint8_t *st, const uint8_t *pk, int64_t p0, int64_t n) {
    const uintptr_t g0 = (uintptr_t)(pk + p0 * EXP_PKT);
    const uintptr_t a0 = g0 & ~(uintptr_t)15;
    const uintptr_t gend = g0 + (uintptr_t)n * EXP_PKT;
    const int n16 = (int)((gend - a0 + 15) >> 4);
    for (int e = (int)threadIdx.x; e < n16; e += (int)blockDim.x) {
        const uintptr_t ua = a0 + (uintptr_t)e * 16;
        if (ua + 16 <= gend) {
            *(uint4 *)(st + e * 16) = *(const uint4 *)ua;
        } else {  // the tail unit stops at the stream end: dwords (gend is 4-aligned)
            for (int k = 0; k < 16 && ua + k < gend; k += 4) *(uint32_t *)(st + e * 16 + k) = *(const uint32_t *)(ua + k);
        }
    }
    return (int)(g0 - a0);
}

// sync nibbles + XOR of bytes 2..83 against the checksum nibbles (lidar.py:68-77)
__device__ __forceinline__ bool packet_ok(const uint8_t *b) {
    const uint32_t *w = (const uint32_t *)b;
    const uint32_t w0 = w[0];
    uint32_t x = w0 >> 16;
#pragma unroll
    for (int j = 1; j < EXP_PKT / 4; j++) x ^= w[j];
    x ^= x >> 16;
    x ^= x >> 8;
    x &= 0xFF;
    const uint32_t b0 = w0 & 0xFF, b1 = (w0 >> 8) & 0xFF;
    return (b0 >> 4) == 0xA && (b1 >> 4) == 0x5 && x == ((b0 & 0xF) | ((b1 & 0xF) << 4));
}

// start angle in 1/64 degree (lidar.py:79): an integer, so < compares like the floats
__device__ __forceinline__ int start_q6(const uint8_t *b) { return b[2] + ((b[3] & 0x7F) << 8); }

// cabin k of a packet (lidar.py:80-91): distance (mm) and the Q3 angle offset
__device__ __forceinline__ void cabin(const uint8_t *b, int k, int &dist, int &corr) {
    const int i = 5 * (k >> 1);
    if ((k & 1) == 0) {
        dist = (b[i + 4] >> 2) + (b[i + 5] << 6);
        corr = twos_comp5((b[i + 8] & 0xF) + ((b[i + 4] & 3) << 4));
    } else {
        dist = (b[i + 6] >> 2) + (b[i + 7] << 6);
        corr = twos_comp5(((b[i + 8] >> 4) & 0xF) + ((b[i + 6] & 3) << 4));
    }
}

// lidar.py:185 with trame = k + 1, in integer units of 2^-11 degree.  Every
// operand of the reference's float expression is a multiple of 2^-11 below
// 2^20 units, so each of its steps is exact and the result is j / 2048 for
//   j = floor_mod(32 s + floor_mod(na - s, 360*64) (k + 1) - 256 corr, 360*2048)
// (s, na in 1/64 degree): bit-identical angles from integer arithmetic.
constexpr int EXP_Q6_TURN = 360 * 64;
constexpr int EXP_Q11_TURN = 360 * 2048;

__device__ __forceinline__ int floor_mod(int x, int m) {
    const int r = x % m;
    return r < 0 ? r + m : r;
}

__device__ __forceinline__ int measure_angle_q11(int s_q6, int na_q6, int k, int corr) {
    const int x = floor_mod(na_q6 - s_q6, EXP_Q6_TURN);
    return floor_mod(32 * s_q6 + x * (k + 1) - 256 * corr, EXP_Q11_TURN);
}

// sin and cos of j * 2^-11 degrees (0 <= j < 360 * 2048): exact quadrant split
// in integers, then fdlibm's |x| <= pi/4 kernels (~1 ulp) on the remainder.
__device__ __forceinline__ void sincos_q11(int j, double &sn, double &cs) {
    constexpr int QUAD = 90 * 2048;
    const int q = (j + QUAD / 2) / QUAD;  // nearest quadrant, 0..4
    const int r = j - q * QUAD;           // [-45, 45) degrees
    const double x = (double)r * (3.14159265358979323846 / (180.0 * 2048.0));
    const double z = x * x;
    const double ps = __builtin_fma(z, __builtin_fma(z, __builtin_fma(z, __builtin_fma(z, __builtin_fma(z,
                          1.58969099521155010221e-10, -2.50507602534068634195e-08), 2.75573137070700676789e-06),
                          -1.98412698298579493134e-04), 8.33333333332248946124e-03), -1.66666666666666324348e-01);
    const double pc = __builtin_fma(z, __builtin_fma(z, __builtin_fma(z, __builtin_fma(z, __builtin_fma(z,
                          -1.13596475577881948265e-11, 2.08757232129817482790e-09), -2.75573143513906633035e-07),
                          2.48015872894767294178e-05), -1.38888888888741095749e-03), 4.16666666666666019037e-02);
    const double s0 = __builtin_fma(x * z, ps, x);
    const double c0 = 1.0 - (0.5 * z - z * z * pc);
    // quadrant q: (sin, cos) = (s0, c0), (c0, -s0), (-s0, -c0), (-c0, s0); selects
    // and sign-bit flips instead of a divergent switch
    const bool odd = q & 1;
    const uint64_t neg_s = (uint64_t)((q >> 1) & 1) << 63, neg_c = (uint64_t)(((q + 1) >> 1) & 1) << 63;
    sn = __longlong_as_double(__double_as_longlong(odd ? c0 : s0) ^ neg_s);
    cs = __longlong_as_double(__double_as_longlong(odd ? s0 : c0) ^ neg_c);
}

// functions.py:59-60 for an angle of j * 2^-11 degrees:
// d cos(-a + pi/2) = d sin(a), d sin(-a + pi/2) = d cos(a)
__device__ __forceinline__ double2 polar_xy_q11(int j, double d) {
    double sn, cs;
    sincos_q11(j, sn, cs);
    return make_double2(d * sn, d * cs);
}

// block-wide (256 lanes = 4 waves) inclusive scan of two ints; returns the block totals
__device__ __forceinline__ int2 block_scan2_256(int &a, int &b, int2 *wtot) {
    const int lane = (int)threadIdx.x & 63, w = (int)threadIdx.x >> 6;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int ta = __shfl_up(a, o), tb = __shfl_up(b, o);
        if (lane >= o) {
            a += ta;
            b += tb;
        }
    }
    if (lane == 63) wtot[w] = make_int2(a, b);
    __syncthreads();
    int2 pre = make_int2(0, 0), tot = make_int2(0, 0);
#pragma unroll
    for (int v = 0; v < 4; v++) {
        const int2 t = wtot[v];
        if (v < w) pre.x += t.x, pre.y += t.y;
        tot.x += t.x, tot.y += t.y;
    }
    a += pre.x;
    b += pre.y;
    __syncthreads();
    return tot;
}

struct ExpressOut {
    double *angle_deg;   // [(M-1)*32]
    double *dist_mm;     // [(M-1)*32]
    uint8_t *new_scan;   // [(M-1)*32]
    uint8_t *valid;      // [(M-1)*32]
    double2 *xy;         // [(M-1)*32] (A1 fused)
    uint8_t *pkt_valid;  // [M]
};

// Measure-level decode: lane (q, k) of a workgroup = cabin k of packets p0 + q + 8r, r < EXP_ROWS.
__global__ __launch_bounds__(256) void express_decode_kernel(const uint8_t *__restrict__ pk, int64_t M, ExpressOut o) {
    __shared__ __attribute__((aligned(16))) uint8_t st[(EXP_DEC_PER_WG + 1) * EXP_PKT + 32];
    __shared__ int s_start[EXP_DEC_PER_WG + 1];
    __shared__ int s_ok[EXP_DEC_PER_WG + 1];
    const int64_t p0 = (int64_t)blockIdx.x * EXP_DEC_PER_WG;
    const int tid = (int)threadIdx.x;
    const int64_t npk = min((int64_t)(EXP_DEC_PER_WG + 1), M - p0);
    const uint8_t *sp = st + stage_packets(st, pk, p0, npk);
    __syncthreads();
    if (tid < EXP_DEC_PER_WG + 1) {
        const bool in = tid < npk;
        s_ok[tid] = in && packet_ok(sp + tid * EXP_PKT);
        s_start[tid] = in ? start_q6(sp + tid * EXP_PKT) : 0;
    }
    __syncthreads();
    const int k = tid & 31;
#pragma unroll
    for (int r = 0; r < EXP_ROWS; r++) {
        const int q = (tid >> 5) + 8 * r;
        const int64_t p = p0 + q;
        if (o.pkt_valid && k == 0 && p < M) o.pkt_valid[p] = (uint8_t)s_ok[q];  // grid covers all M packets
        if (p >= M - 1) break;  // the last packet only lends its start angle
        const bool ok = s_ok[q] && s_ok[q + 1];
        int dist, corr;
        cabin(sp + q * EXP_PKT, k, dist, corr);
        const int j = ok ? measure_angle_q11(s_start[q], s_start[q + 1], k, corr) : 0;
        const double ang = (double)j * (1.0 / 2048.0);
        const double d = ok ? (double)dist : 0.0;
        const int64_t m = p * 32 + k;
        if (o.angle_deg) o.angle_deg[m] = ang;
        if (o.dist_mm) o.dist_mm[m] = d;
        if (o.new_scan) o.new_scan[m] = (uint8_t)(ok && k == 0 && s_start[q + 1] < s_start[q]);
        if (o.valid) o.valid[m] = (uint8_t)ok;
        if (o.xy) o.xy[m] = polar_xy_q11(j, d);
    }
}

// ---- revolution builder (A2 over the measure stream) ----
//
// Measures are ranked over the valid ones in stream order, after dropping the
// first `skip` measures of packet 0 (a resumed stream).  A flagged measure is
// always cabin 0 of its packet and ENDS its revolution (functions.py:61 appends
// it before :68 checks the flag).  Revolution j holds ranks
// [rev_end[j-1] + 1, rev_end[j]]; the open revolution after the last flag is
// not emitted (the caller resumes from its flagged packet with skip = 1).

struct ExpressScratch {
    uint8_t *pkt_flags;  // [M-1]
    int2 *tile_sum;      // [tiles]: (valid measures, flags)
    int2 *pkt_rank;      // [M-1]: (rank of the packet's first kept measure, flags at packets <= p)
    int2 *rev_end;       // [M-1]: (rank of the flagged measure, its packet)
    int4 *rev_info;      // [M-1]: (first rank, kept points, first output point, -)
    int32_t *counts;     // [4]: n_scans, n_chunks, n_points, resume packet (-1 if no revolution)
};

struct ExpressScans {
    double2 *xy;              // [cap_points]
    int32_t *scan_chunk_off;  // [cap_scans + 1]
    int32_t *chunk_pt_off;    // [cap_chunks + 1]
    int64_t cap_points;
    int32_t cap_scans, cap_chunks;
};

__global__ __launch_bounds__(256) void express_flags_kernel(const uint8_t *__restrict__ pk, int64_t M, int skip,
                                                            ExpressScratch s) {
    __shared__ __attribute__((aligned(16))) uint8_t st[(EXP_TILE + 1) * EXP_PKT + 32];
    __shared__ int s_start[EXP_TILE + 1];
    __shared__ int s_ok[EXP_TILE + 1];
    __shared__ int2 wtot[4];
    const int64_t p0 = (int64_t)blockIdx.x * EXP_TILE;
    const int tid = (int)threadIdx.x;
    const int64_t npk = min((int64_t)(EXP_TILE + 1), M - p0);
    const uint8_t *sp = st + stage_packets(st, pk, p0, npk);
    __syncthreads();
    for (int q = tid; q < EXP_TILE + 1; q += 256) {
        const bool in = q < npk;
        s_ok[q] = in && packet_ok(sp + q * EXP_PKT);
        s_start[q] = in ? start_q6(sp + q * EXP_PKT) : 0;
    }
    __syncthreads();
    const int64_t p = p0 + tid;
    int cnt = 0, fl = 0;
    if (p < M - 1) {
        const bool ok = s_ok[tid] && s_ok[tid + 1];
        const int sk = p == 0 ? skip : 0;
        fl = ok && sk == 0 && s_start[tid + 1] < s_start[tid];
        cnt = ok ? 32 - sk : 0;
        s.pkt_flags[p] = (uint8_t)((ok ? EXP_OK : 0) | (fl ? EXP_NEW : 0));
    }
    const int2 tot = block_scan2_256(cnt, fl, wtot);
    if (tid == 0) s.tile_sum[blockIdx.x] = tot;
}

__global__ __launch_bounds__(256) void express_rank_kernel(int64_t M, int skip, ExpressScratch s) {
    __shared__ int2 wtot[4];
    const int tid = (int)threadIdx.x;
    // exclusive prefix over the earlier tiles (a few hundred int2: cheaper than a third pass)
    int a = 0, b = 0;
    for (int h = tid; h < (int)blockIdx.x; h += 256) {
        const int2 t = s.tile_sum[h];
        a += t.x;
        b += t.y;
    }
    int2 pre = block_scan2_256(a, b, wtot);
    const int64_t p = (int64_t)blockIdx.x * EXP_TILE + tid;
    const uint8_t f = p < M - 1 ? s.pkt_flags[p] : 0;
    const int c0 = (f & EXP_OK) ? 32 - (p == 0 ? skip : 0) : 0;
    int cnt = c0, fl = (f & EXP_NEW) ? 1 : 0;
    block_scan2_256(cnt, fl, wtot);
    if (p < M - 1) {
        const int rank0 = pre.x + cnt - c0;  // exclusive
        const int rev = pre.y + fl;          // inclusive
        s.pkt_rank[p] = make_int2(rank0, rev);
        if (f & EXP_NEW) s.rev_end[rev - 1] = make_int2(rank0, (int)p);
    }
}

// revolution j: first rank, kept points (a remainder of <= 2 is dropped), chunks
__device__ __forceinline__ void rev_size(const ExpressScratch &s, int j, int &first, int &kept, int &nch) {
    first = j ? s.rev_end[j - 1].x + 1 : 0;
    const int n = s.rev_end[j].x - first + 1;
    const int rem = n % EXP_CHUNK;
    nch = n / EXP_CHUNK + (rem > EXP_MIN_REM);
    kept = n - (rem > EXP_MIN_REM ? 0 : rem);
}

// Workgroup g: revolutions [256g, 256g + 256) -> kept points and chunks -> CSR
// offsets.  Its prefix over the earlier revolutions is summed directly (a few
// thousand L2-resident int2 at most: cheaper than another pass).
__global__ __launch_bounds__(256) void express_revs_kernel(int n_tiles, ExpressScratch s, ExpressScans o) {
    __shared__ int2 wtot[4];
    const int tid = (int)threadIdx.x;
    int nr = 0, zero = 0;
    for (int h = tid; h < n_tiles; h += 256) nr += s.tile_sum[h].y;
    const int nrev = block_scan2_256(nr, zero, wtot).x;
    const int j0 = (int)blockIdx.x * 256;
    if (j0 >= nrev && blockIdx.x != 0) return;
    int pk = 0, pc = 0;
    for (int j = tid; j < j0; j += 256) {
        int first, kept, nch;
        rev_size(s, j, first, kept, nch);
        pk += kept;
        pc += nch;
    }
    const int2 pre = block_scan2_256(pk, pc, wtot);
    const int j = j0 + tid;
    int first = 0, kept = 0, nch = 0;
    if (j < nrev) rev_size(s, j, first, kept, nch);
    int a = kept, b = nch;
    const int2 tot = block_scan2_256(a, b, wtot);
    const int pt0 = pre.x + a - kept, ch0 = pre.y + b - nch;  // exclusive offsets
    if (j < nrev) {
        s.rev_info[j] = make_int4(first, kept, pt0, 0);
        if (j < o.cap_scans) o.scan_chunk_off[j] = ch0;
        for (int t = 0; t < nch; t++)
            if (ch0 + t < o.cap_chunks) o.chunk_pt_off[ch0 + t] = pt0 + t * EXP_CHUNK;
    }
    // the workgroup holding the last revolution (or 0 when there is none) closes the CSR
    if (tid == 0 && (nrev == 0 || (j0 < nrev && nrev <= j0 + 256))) {
        const int npt = pre.x + tot.x, nchk = pre.y + tot.y;
        if (nrev <= o.cap_scans) o.scan_chunk_off[nrev] = nchk;
        if (nchk <= o.cap_chunks) o.chunk_pt_off[nchk] = npt;
        s.counts[0] = nrev;
        s.counts[1] = nchk;
        s.counts[2] = npt;
        s.counts[3] = nrev ? s.rev_end[nrev - 1].y : -1;
    }
}

// Decode + A1 + scatter: lane (q, k) = cabin k of packets p0 + q + 8r, each
// written at its place in its revolution's kept points (dropped remainders and
// the open revolution write nothing).
__global__ __launch_bounds__(256) void express_scatter_kernel(const uint8_t *__restrict__ pk, int64_t M, int skip,
                                                              ExpressScratch s, ExpressScans o) {
    __shared__ __attribute__((aligned(16))) uint8_t st[(EXP_DEC_PER_WG + 1) * EXP_PKT + 32];
    const int64_t p0 = (int64_t)blockIdx.x * EXP_DEC_PER_WG;
    const int tid = (int)threadIdx.x;
    const int k = tid & 31;
    // the revolution lookups do not depend on the packet bytes: issue them
    // first, so their two dependent loads overlap the staging loads
    int64_t dst[EXP_ROWS];
    const int nrev = s.counts[0];
#pragma unroll
    for (int r = 0; r < EXP_ROWS; r++) {
        const int64_t p = p0 + (tid >> 5) + 8 * r;
        dst[r] = -1;
        if (p < M - 1) {
            const uint8_t f = s.pkt_flags[p];
            const int sk = p == 0 ? skip : 0;
            const int2 rr = s.pkt_rank[p];
            const int rev = (k == 0 && (f & EXP_NEW)) ? rr.y - 1 : rr.y;
            if ((f & EXP_OK) && k >= sk && rev < nrev) {  // not invalid, skipped or the open revolution
                const int4 ri = s.rev_info[rev];
                const int l = rr.x + k - sk - ri.x;
                if (l < ri.y) dst[r] = (int64_t)ri.z + l;  // else a remainder of <= 2 points
            }
        }
    }
    const int64_t npk = min((int64_t)(EXP_DEC_PER_WG + 1), M - p0);
    const uint8_t *sp = st + stage_packets(st, pk, p0, npk);
    __syncthreads();
#pragma unroll
    for (int r = 0; r < EXP_ROWS; r++) {
        if (dst[r] < 0 || dst[r] >= o.cap_points) continue;
        const uint8_t *b = sp + ((tid >> 5) + 8 * r) * EXP_PKT;
        int dist, corr;
        cabin(b, k, dist, corr);
        o.xy[dst[r]] = polar_xy_q11(measure_angle_q11(start_q6(b), start_q6(b + EXP_PKT), k, corr), (double)dist);
    }
}

}  // namespace lslam
