// lslam_ransac.h — one RANSAC call per chunk on one wave.
//
// Arithmetic is the reference's, op for op (compile with -ffp-contract=off):
//   LineModelND.estimate on 2 points   fit.py:84-91
//     o = (p0 + p1) / 2 ; d = (p1 - o) - (p0 - o) ; n = sqrt(fma(dy,dy, dx*dx))
//     u = d / n  (n != 0), else u = d
//   LineModelND.residuals               fit.py:19-21,129-132
//     t = fma(ex,ux, ey*uy)  [OpenBLAS dgemv_t rounding]
//     r^2 = (ex - t*ux)^2 + (ey - t*uy)^2   [einsum, no FMA]
//   inlier <=> sqrt(r^2) < thr  <=>  r^2 < ecut   (ecut = lslam_inlier_cutoff(thr))
//   tie-break sum = numpy pairwise_sum of RN(sqrt(r^2))^2 over all N points
//   selection fit.py:850-869, stop_residuals_sum=0 stop, final refit fit.py:871-875
// Layout: the chunk's points are staged in LDS as double2; pass 1 puts one
// hypothesis per lane and streams the points as LDS broadcasts (no bank
// conflicts, points stay uniform, every lane runs the same FP64 chain).
#pragma once
#include "lslam_wave.h"

namespace lslam {

// single-wave workgroups: LDS ordering across lanes needs only a compiler barrier
__device__ __forceinline__ void wave_lds_sync_rt() {
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
}

struct Model {
    double ox, oy, ux, uy;
};

__device__ __forceinline__ Model model2(double2 p0, double2 p1) {
    Model m;
    m.ox = (p0.x + p1.x) / 2.0;
    m.oy = (p0.y + p1.y) / 2.0;
    const double d0x = p0.x - m.ox, d0y = p0.y - m.oy;
    const double d1x = p1.x - m.ox, d1y = p1.y - m.oy;
    double dx = d1x - d0x, dy = d1y - d0y;
    const double nrm = cr_sqrt(__builtin_fma(dy, dy, dx * dx));
    if (nrm != 0.0) {
        dx = dx / nrm;
        dy = dy / nrm;
    }
    m.ux = dx;
    m.uy = dy;
    return m;
}

__device__ __forceinline__ double resid2(double2 p, const Model &m) {
    const double ex = p.x - m.ox, ey = p.y - m.oy;
    const double t = __builtin_fma(ex, m.ux, ey * m.uy);
    const double rx = ex - t * m.ux, ry = ey - t * m.uy;
    return rx * rx + ry * ry;
}

__device__ __forceinline__ double r2sq(double2 p, const Model &m) {
    const double r = cr_sqrt(resid2(p, m));
    return r * r;
}

// numpy pairwise_sum leaf (n <= 128) of r^2 over P[start .. start+n)
__device__ __forceinline__ double pw_leaf(const double2 *P, int start, int n, const Model &m) {
    if (n < 8) {
        double res = 0.0;
        for (int i = 0; i < n; i++) res += r2sq(P[start + i], m);
        return res;
    }
    double r0 = r2sq(P[start + 0], m), r1 = r2sq(P[start + 1], m), r2 = r2sq(P[start + 2], m),
           r3 = r2sq(P[start + 3], m), r4 = r2sq(P[start + 4], m), r5 = r2sq(P[start + 5], m),
           r6 = r2sq(P[start + 6], m), r7 = r2sq(P[start + 7], m);
    int i = 8;
    const int lim = n - (n % 8);
    for (; i < lim; i += 8) {
        r0 += r2sq(P[start + i + 0], m);
        r1 += r2sq(P[start + i + 1], m);
        r2 += r2sq(P[start + i + 2], m);
        r3 += r2sq(P[start + i + 3], m);
        r4 += r2sq(P[start + i + 4], m);
        r5 += r2sq(P[start + i + 5], m);
        r6 += r2sq(P[start + i + 6], m);
        r7 += r2sq(P[start + i + 7], m);
    }
    double res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
    for (; i < n; i++) res += r2sq(P[start + i], m);
    return res;
}

// numpy pairwise_sum for any n: the recursion (n2 = n/2 - (n/2)%8) is walked
// iteratively; the node stack is wave-uniform (same n for every lane) and the
// per-lane partial sums live in an LDS stack vstack[depth*64 + lane];
// nstack (LDS, 3*24 ints) holds the uniform node stack (all lanes write the
// same values).  Depth <= 24 covers any n < 2^30.
__device__ __forceinline__ double pw_sum(const double2 *P, int n, const Model &m, double *vstack,
                                         int *nstack, int lane) {
    if (n <= 128) return pw_leaf(P, 0, n, m);
    // explicit DFS: node = (start, len, state); state 0 = descend left, 1 = descend right, 2 = combine
    int *st_start = nstack, *st_len = nstack + 24, *st_state = nstack + 48;
    int sp = 0;
    st_start[0] = 0; st_len[0] = n; st_state[0] = 0;
    int vsp = 0;
    while (sp >= 0) {
        const int s0 = st_start[sp], ln = st_len[sp];
        if (ln <= 128) {
            vstack[vsp * 64 + lane] = pw_leaf(P, s0, ln, m);
            vsp++;
            sp--;
            continue;
        }
        int n2 = ln / 2;
        n2 -= n2 % 8;
        if (st_state[sp] == 0) {
            st_state[sp] = 1;
            sp++;
            st_start[sp] = s0; st_len[sp] = n2; st_state[sp] = 0;
        } else if (st_state[sp] == 1) {
            st_state[sp] = 2;
            sp++;
            st_start[sp] = s0 + n2; st_len[sp] = ln - n2; st_state[sp] = 0;
        } else {
            const double right = vstack[(vsp - 1) * 64 + lane];
            const double left = vstack[(vsp - 2) * 64 + lane];
            vsp -= 2;
            vstack[vsp * 64 + lane] = left + right;
            vsp++;
            sp--;
        }
    }
    return vstack[lane];
}

// largest x >= 0 with fl(x*x) < e (-1 if none), smallest x with fl(x*x) > e
__device__ __forceinline__ double sq_floor_lt(double e) {
    if (!(e > 0.0)) return -1.0;
    double x = sqrt(e);
    while (x > 0.0 && x * x >= e) x = __longlong_as_double(__double_as_longlong(x) - 1);
    for (;;) {
        const double y = __longlong_as_double(__double_as_longlong(x) + 1);
        if (y * y < e) x = y;
        else break;
    }
    return x;
}
__device__ __forceinline__ double sq_ceil_gt(double e) {
    if (!(e >= 0.0)) return 0.0;
    double x = sqrt(e);
    while (x * x <= e) x = __longlong_as_double(__double_as_longlong(x) + 1);
    for (;;) {
        if (x == 0.0) break;
        const double y = __longlong_as_double(__double_as_longlong(x) - 1);
        if (y * y > e) x = y;
        else break;
    }
    return x;
}

// closed-form principal direction of the centred inliers (replaces dgesdd's
// v[0], fit.py:94); identical formula in oracle/ransac_oracle.c
__device__ __forceinline__ void tls_direction(double sxx, double sxy, double syy, double &ux, double &uy) {
    const double h = (sxx - syy) * 0.5;
    const double r = cr_sqrt(h * h + sxy * sxy);
    double vx, vy;
    if (sxx >= syy) { vx = h + r; vy = sxy; }
    else { vx = sxy; vy = r - h; }
    const double nv = cr_sqrt(vx * vx + vy * vy);
    if (!(nv > 0.0)) { ux = 1.0; uy = 0.0; return; }
    ux = vx / nv;
    uy = vy / nv;
}

__device__ __forceinline__ double wave_min_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ double wave_max_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
    return v;
}

// Final refit on the inliers P[0..nin) (compacted in data order by chunk_finish_fit), nin >= 3
// (fit.py:84-95).  The mean is numpy's axis-0 add.reduce: sequential, done by every lane.  The
// scatter matrix for the closed-form direction is our own quantity: inlier k goes to lane
// k % 64 (ascending k), then an xor butterfly (32, 16, ..., 1) leaves the same sums in every
// lane.  oracle/ransac_oracle.c:scatter2 restates this order.
__device__ __forceinline__ Model refit_line(const double2 *P, int nin, int lane) {
    Model f;
    // The two sequential sums run side by side: even lanes accumulate x, odd lanes y (same
    // additions, same order), so one v_add per inlier carries both chains; the inliers are
    // contiguous, so each load is an immediate offset from one base.
    const double *Pc = (const double *)P + (lane & 1);
    double acc = Pc[0];
    int i = 1;
    for (; i + 8 <= nin; i += 8) {
        double v[8];
#pragma unroll
        for (int j = 0; j < 8; j++) v[j] = Pc[2 * (i + j)];
#pragma unroll
        for (int j = 0; j < 8; j++) acc += v[j];
    }
    for (; i < nin; i++) acc += Pc[2 * i];
    const double sx = unid(acc);                      // lane 0
    const double sy = __shfl(acc, 1);                 // lane 1
    f.ox = sx / (double)nin;
    f.oy = sy / (double)nin;
    double sxx = 0.0, sxy = 0.0, syy = 0.0;
    for (int k = lane; k < nin; k += 64) {
        const double2 q = P[k];
        const double cx = q.x - f.ox, cy = q.y - f.oy;
        sxx += cx * cx;
        sxy += cx * cy;
        syy += cy * cy;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        sxx += __shfl_xor(sxx, o);
        sxy += __shfl_xor(sxy, o);
        syy += __shfl_xor(syy, o);
    }
    tls_direction(sxx, sxy, syy, f.ux, f.uy);
    return f;
}

// numpy pairwise_sum of RN(sqrt(r^2))^2 over P[0..N), N <= 128, lanes over
// points (pw_leaf's order): v_i by lane i % 64 into vtmp, accumulators
// r_j = v_j + v_{j+8} + ... (lane j < 8, sequential), the fixed tree
// ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) by xor shuffles, then the tail.
__device__ __forceinline__ double pw_sum_lanes(const double2 *P, int N, const Model &m, double *vtmp, int lane) {
    wave_lds_sync_rt();
    if (lane < N) vtmp[lane] = r2sq(P[lane], m);
    if (lane + 64 < N) vtmp[lane + 64] = r2sq(P[lane + 64], m);
    wave_lds_sync_rt();
    double res;
    if (N < 8) {
        res = 0.0;
        for (int i = 0; i < N; i++) res += vtmp[i];
        return res;
    }
    const int lim = N - (N % 8);
    double r = 0.0;
    if (lane < 8) {
        r = vtmp[lane];
        for (int i = lane + 8; i < lim; i += 8) r += vtmp[i];
    }
    r += __shfl_xor(r, 1);
    r += __shfl_xor(r, 2);
    r += __shfl_xor(r, 4);
    res = unid(r);
    for (int i = lim; i < N; i++) res += vtmp[i];
    return res;
}

// The same sum without the LDS scratch (chunk_consensus: beside the producer every KiB of LDS
// is residency): the squared residuals stay in the lanes (point p in lane p, p + 64 in lane p's
// second register) and the accumulators read them by shuffles, in the same order and with the
// same tree, so the result is bit-identical to pw_sum_lanes.
__device__ __forceinline__ double pw_sum_regs(const double2 *P, int N, const Model &m, int lane) {
    const double v0 = lane < N ? r2sq(P[lane], m) : 0.0;
    const double v1 = lane + 64 < N ? r2sq(P[lane + 64], m) : 0.0;
    if (N < 8) {
        double res = 0.0;
        for (int i = 0; i < N; i++) res += __shfl(v0, i);
        return res;
    }
    const int lim = N - (N % 8);
    const int j = lane & 7;
    double r = __shfl(v0, j);  // lanes 0..7: r_j = v_j + v_{j+8} + ... (i < lim), in order
    for (int t = 1; 8 * t < lim; t++) {
        const int i = j + 8 * t;
        const double vi = (t < 8) ? __shfl(v0, i) : __shfl(v1, i - 64);  // t < 8 <=> i < 64 for every j
        r += (i < lim) ? vi : 0.0;  // + 0.0 is exact (r >= 0)
    }
    r += __shfl_xor(r, 1);
    r += __shfl_xor(r, 2);
    r += __shfl_xor(r, 4);
    double res = unid(r);
    for (int i = lim; i < N; i++) res += (i < 64) ? __shfl(v0, i) : __shfl(v1, i - 64);
    return res;
}

// pw_sum for any n with lanes over points: the leaves (<= 128 points) by
// pw_sum_lanes, combined in numpy's recursion order (n2 = n/2 - (n/2)%8).
// The node stack (nstack, 3*24 ints) and the partial sums (vst, 24 doubles)
// are uniform: every lane writes and reads the same values.
__device__ __forceinline__ double pw_sum_lanes_any(const double2 *P, int n, const Model &m, double *vtmp, double *vst,
                                                   int *nstack, int lane) {
    if (n <= 128) return pw_sum_lanes(P, n, m, vtmp, lane);
    int *st_start = nstack, *st_len = nstack + 24, *st_state = nstack + 48;
    int sp = 0, vsp = 0;
    st_start[0] = 0; st_len[0] = n; st_state[0] = 0;
    while (sp >= 0) {
        const int s0 = st_start[sp], ln = st_len[sp];
        if (ln <= 128) {
            vst[vsp++] = pw_sum_lanes(P + s0, ln, m, vtmp, lane);
            sp--;
            continue;
        }
        int n2 = ln / 2;
        n2 -= n2 % 8;
        if (st_state[sp] == 0) {
            st_state[sp] = 1;
            sp++;
            st_start[sp] = s0; st_len[sp] = n2; st_state[sp] = 0;
        } else if (st_state[sp] == 1) {
            st_state[sp] = 2;
            sp++;
            st_start[sp] = s0 + n2; st_len[sp] = ln - n2; st_state[sp] = 0;
        } else {
            const double right = vst[vsp - 1], left = vst[vsp - 2];
            vsp -= 2;
            vst[vsp++] = left + right;
            sp--;
        }
    }
    return vst[0];
}

}  // namespace lslam
