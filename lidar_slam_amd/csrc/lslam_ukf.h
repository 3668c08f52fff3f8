// lslam_ukf.h — one UKF predict/update per scan on one wave.
//
// Semantics: the INTENT of UKFMethods.py:10-71 + systemClass.py:7-29 (both files
// fail to parse in the reference) run through filterpy 1.4.5's
// UnscentedKalmanFilter (absent from the container; restated).  PARITY
// UNPINNED — checked per component against a 50-digit evaluation of the same
// algorithm (oracle/ukf_exact.py, tests/test_gpu_ukf_exact.py) and against the
// NumPy restatement in oracle/ukf.py.
//
//   sigma points  MerweScaled: U = chol_upper((lambda+n) P); s0 = x,
//                 s_{1+k} = x + U[k], s_{4+k} = x - U[k]
//   fx            x + dt * B(theta) u,  B = [[R/2 c, R/2 c],[R/2 s, R/2 s],[-R/L, R/L]]
//   hx            per landmark j: [sqrt(dx^2+dy^2), wrap(atan2(dy,dx) - theta)]
//   means         linear weighted sums; angles by atan2(sum W sin, sum W cos),
//                 both evaluated about sigma point 0 (centred_mean): with
//                 alpha = 1e-4 the float64 weights (~-1e8, 1.7e7) sum to
//                 1 - 1.1e-8, so filterpy's literal sum sum(W s) is biased by
//                 1.1e-8 |s| (3e-5 mm at 3 m), which reaches P as ~1e-5 relative
//                 through the (Wc0 - Wm0) term.  s_0 + sum W (s - s_0) is the same
//                 value in exact arithmetic and carries no such bias.
//   residuals     differences with angle components wrapped to (-pi, pi]
//   predict       x, P = UT(fx(sigmas)) + Q; sigmas_f re-drawn from (x, P)
//   update        S = sum Wc rz rz^T + R, Pxz = sum Wc rx rz^T, K = Pxz S^-1,
//                 x += K y, P -= K S K^T
// The update is evaluated in its exact rank-7 (Woodbury) form, so no 2L x 2L
// matrix is ever formed (L = 200 -> dim_z = 400 stays a 7x7 solve):
//   with Y = [rz_k] (7 x m), Dx = [rx_k] (7 x 3), W = diag(Wc), G = Y R^-1 Y^T,
//   M = W^-1 + G:   K y = Dx^T M^-1 (Y R^-1 y),   K S K^T = Dx^T (W - M^-1) Dx.
// Work split: lane k < 7 owns sigma point k (fx), lanes own landmarks for hx,
// lanes own G entries for the 7x7 products, lanes own matrix entries in the
// Gauss-Jordan solve; small uniform values are exchanged through LDS.
#pragma once
#include "lslam_wave.h"

namespace lslam {

constexpr double LS_PI = 3.141592653589793;
constexpr double LS_TWO_PI = 6.283185307179586;

// UKFMethods.py:10-14 normalize_angle: Python float % (floor-mod), then -2pi above pi
// fmod(a, 2pi) is exact; for |a| < 4pi it is a itself or a -+ 2pi (Sterbenz: exact
// too), so the library call is only needed for far-out angles.
__device__ __forceinline__ double fmod_two_pi(double a) {
    const double x = fabs(a);
    if (x < LS_TWO_PI) return a;
    if (x < 2.0 * LS_TWO_PI) return a < 0.0 ? a + LS_TWO_PI : a - LS_TWO_PI;
    return fmod(a, LS_TWO_PI);
}

__device__ __forceinline__ double wrap_angle(double a) {
    double m = fmod_two_pi(a);
    if (m != 0.0) {
        if (m < 0.0) m += LS_TWO_PI;
    } else {
        m = 0.0;
    }
    if (m > LS_PI) m -= LS_TWO_PI;
    return m;
}

// The library's FP64 sin / cos / atan2 inline a large-argument reduction each;
// inlined at every UKF call site they pushed the scan kernels past 256 VGPRs
// (occupancy 1, scratch spills).  Out of line, each is one call.
__device__ __attribute__((noinline)) double ukf_sin(double x) { return sin(x); }
__device__ __attribute__((noinline)) double ukf_cos(double x) { return cos(x); }
__device__ __attribute__((noinline)) double ukf_atan2(double y, double x) { return atan2(y, x); }
// sin and cos of one argument share its reduction (one call instead of two); returned by
// value (.x = sin, .y = cos) so the results come back in registers, not through scratch
__device__ __attribute__((noinline)) double2 ukf_sincos(double x) {
    double s, c;
    sincos(x, &s, &c);
    return make_double2(s, c);
}

struct UkfConst {
    double Wm[7], Wc[7];
    double cfac;  // lambda + n
    double dt, wr, wb;
    double Q[9];
    int L;
    int flags;
};

// LDS scratch layout for one wave's UKF step (doubles)
struct UkfLds {
    double *sig;   // [7][3]
    double *Dx;    // [7][3]
    double *aug;   // [7][14]  [M | I] -> [I | M^-1]
    double *G;     // [28]
    double *bv;    // [7]
    double *xv;    // [16] misc: M^-1 b (7), K y (3)
    double *tw;    // [7][2] predict: Wm_k ukf_sin(theta_k), Wm_k ukf_cos(theta_k)
    double *T;     // [7][3] (W - M^-1) Dx
    double *Y;     // [7][2L] measurement sigmas, then residuals rz_k
    double *yr;    // [2L] innovation residual_h(z, zp)
    double *wsc;   // [7][2L] Wm_k ukf_sin(phi_kj), Wm_k ukf_cos(phi_kj)
    double *rinv;  // [2L] 1 / R_diag
    static __host__ __device__ int doubles(int L) {
        return 21 + 21 + 98 + 28 + 7 + 16 + 14 + 21 + 7 * 2 * L + 2 * L + 7 * 2 * L + 2 * L;
    }
    __device__ void carve(double *base, int L) {
        sig = base; Dx = sig + 21; aug = Dx + 21; G = aug + 98; bv = G + 28; xv = bv + 7; tw = xv + 16;
        T = tw + 14; Y = T + 21; yr = Y + 7 * 2 * L; wsc = yr + 2 * L; rinv = wsc + 7 * 2 * L;
    }
};

// LAPACK dpotrf('U') on a 3x3 SPD matrix (recursive dpotrf2 order)
__device__ __forceinline__ void chol3_upper(const double A[9], double U[9]) {
    U[0] = cr_sqrt(A[0]);
    U[1] = A[1] / U[0];
    U[2] = A[2] / U[0];
    U[3] = 0.0;
    U[4] = cr_sqrt(A[4] - U[1] * U[1]);
    U[5] = (A[5] - U[1] * U[2]) / U[4];
    U[6] = 0.0;
    U[7] = 0.0;
    U[8] = cr_sqrt((A[8] - U[2] * U[2]) - U[5] * U[5]);
}

// sigma point k of MerweScaledSigmaPoints.sigma_points(x, P)
__device__ __forceinline__ void sigma_point(int k, const double x[3], const double U[9], double o[3]) {
    for (int j = 0; j < 3; j++) {
        if (k == 0) o[j] = x[j];
        else if (k <= 3) o[j] = x[j] - (-U[3 * (k - 1) + j]);
        else o[j] = x[j] - U[3 * (k - 4) + j];
    }
}

// UKFMethods.py:17-24 transition_function (intended form)
__device__ __forceinline__ void fx(const double s[3], double dt, double u0, double u1, double wr, double wb,
                                   double o[3]) {
    const double2 scv = ukf_sincos(s[2]);
    const double c = (wr / 2.0) * scv.y;
    const double sn = (wr / 2.0) * scv.x;
    const double k0 = (-1.0 * wr) / wb, k1 = (1.0 * wr) / wb;
    const double b0 = c * u0 + c * u1;
    const double b1 = sn * u0 + sn * u1;
    const double b2 = k0 * u0 + k1 * u1;
    o[0] = s[0] + dt * b0;
    o[1] = s[1] + dt * b1;
    o[2] = s[2] + dt * b2;
}

// One UKF step for one scan; x[3], P[9] in/out (uniform).  `flags` = the
// predict (1) / update (2) bits to run.  lmk(j, px, py) gives landmark j's
// position and returns whether measurement slot j is active: an inactive slot's
// rows of Y and y are zero, so it adds exactly nothing to G = Y R^-1 Y^T and
// b = Y R^-1 y (the update equals one over the active measurements alone).
// Returns false if a factorisation failed (non-SPD P or singular M).
//
// Work is spread over lanes and exchanged through LDS (one wave per scan is
// latency-bound): sigma points on lanes 0..6, hx on (sigma, landmark) pairs,
// per-landmark means on landmark lanes, the 7x7 products on entry lanes.  Loops
// stay rolled so the kernel keeps a few waves per SIMD resident.  Every sum runs
// in the sigma index order k = 0..6 of the sequential form.
template <typename LmkFn>
__device__ bool ukf_step(double x[3], double P[9], double u0, double u1, const double *z, const double *Rd,
                         LmkFn lmk, const UkfConst &C, int flags, UkfLds &S, int lane) {
    bool ok = true;
    double U[9];
    if (flags & 1) {  // ---- predict (filterpy UKF.predict)
        {
            double A[9];
            for (int i = 0; i < 9; i++) A[i] = C.cfac * P[i];
            chol3_upper(A, U);
        }
        if (lane < 7) {
            double sg[3], o[3];
            sigma_point(lane, x, U, sg);
            fx(sg, C.dt, u0, u1, C.wr, C.wb, o);
            S.sig[3 * lane] = o[0];
            S.sig[3 * lane + 1] = o[1];
            S.sig[3 * lane + 2] = o[2];
        }
        __syncthreads();
        if (lane < 7) {
            const double d = S.sig[3 * lane + 2] - S.sig[2];
            const double2 scv = ukf_sincos(d);
            S.tw[2 * lane] = scv.x * C.Wm[lane];
            S.tw[2 * lane + 1] = scv.y * C.Wm[lane];
        }
        __syncthreads();
        // UKFMethods.py:37-45 state_mean (intended form), evaluated about sigma point 0 (see
        // centred_mean): sum Wm s = s_0 + sum Wm (s - s_0) and
        // atan2(sum Wm sin a, sum Wm cos a) = a_0 + atan2(sum Wm sin(a - a_0), sum Wm cos(a - a_0))
        double s0 = 0.0, s1 = 0.0, ss = 0.0, sc = 0.0;
#pragma unroll 1
        for (int k = 0; k < 7; k++) {
            s0 += (S.sig[3 * k] - S.sig[0]) * C.Wm[k];
            s1 += (S.sig[3 * k + 1] - S.sig[1]) * C.Wm[k];
            ss += S.tw[2 * k];
            sc += S.tw[2 * k + 1];
        }
        const double xm0 = S.sig[0] + s0, xm1 = S.sig[1] + s1;
        const double xm2 = wrap_angle(S.sig[2] + ukf_atan2(ss, sc));
        // unscented_transform with residual_x (loop form) + Q
        double Pn[9];
        for (int i = 0; i < 9; i++) Pn[i] = 0.0;
#pragma unroll 1
        for (int k = 0; k < 7; k++) {
            const double y0 = S.sig[3 * k] - xm0, y1 = S.sig[3 * k + 1] - xm1;
            const double y2 = wrap_angle(S.sig[3 * k + 2] - xm2);
            const double y[3] = {y0, y1, y2};
            const double w = C.Wc[k];
            for (int i = 0; i < 3; i++)
                for (int j = 0; j < 3; j++) Pn[3 * i + j] = Pn[3 * i + j] + w * (y[i] * y[j]);
        }
        for (int i = 0; i < 9; i++) P[i] = Pn[i] + C.Q[i];
        x[0] = xm0;
        x[1] = xm1;
        x[2] = xm2;
        __syncthreads();
    }
    if (!(flags & 2)) return ok;
    // ---- sigmas_f re-drawn from (x, P) (end of predict; also the update-only case)
    {
        double A[9];
        for (int i = 0; i < 9; i++) A[i] = C.cfac * P[i];
        chol3_upper(A, U);
        if (!(U[0] > 0.0) || !(U[4] > 0.0) || !(U[8] > 0.0)) ok = false;
    }
    if (lane < 7) {
        double sg[3];
        sigma_point(lane, x, U, sg);
        S.sig[3 * lane] = sg[0];
        S.sig[3 * lane + 1] = sg[1];
        S.sig[3 * lane + 2] = sg[2];
        S.Dx[3 * lane] = sg[0] - x[0];
        S.Dx[3 * lane + 1] = sg[1] - x[1];
        S.Dx[3 * lane + 2] = wrap_angle(sg[2] - x[2]);
    }
    __syncthreads();
    const int m2 = 2 * C.L;
    const int npair = 7 * C.L;
    // ---- hx on (sigma k, landmark j) pairs: distance, bearing, Wm-weighted sin/cos
#pragma unroll 1
    for (int e = lane; e < npair; e += 64) {
        const int k = e / C.L, j = e - k * C.L;
        double px, py;
        double d = 0.0, ph = 0.0;
        if (lmk(j, px, py)) {
            const double dx = px - S.sig[3 * k], dy = py - S.sig[3 * k + 1];
            d = cr_sqrt(dx * dx + dy * dy);
            ph = wrap_angle(ukf_atan2(dy, dx) - S.sig[3 * k + 2]);
        }
        S.Y[k * m2 + 2 * j] = d;
        S.Y[k * m2 + 2 * j + 1] = ph;
    }
    __syncthreads();
    // Wm-weighted sin / cos of each bearing about sigma 0's (the centred z_mean, below)
#pragma unroll 1
    for (int e = lane; e < npair; e += 64) {
        const int k = e / C.L, j = e - k * C.L;
        const double dph = S.Y[k * m2 + 2 * j + 1] - S.Y[2 * j + 1];
        const double2 scv = ukf_sincos(dph);
        S.wsc[k * m2 + 2 * j] = scv.x * C.Wm[k];
        S.wsc[k * m2 + 2 * j + 1] = scv.y * C.Wm[k];
    }
    __syncthreads();
    // ---- z_mean per landmark (lanes), innovation; means kept in yr until the residuals.
    // UKFMethods.py:47-57 about sigma 0 (as state_mean above): dm = d_0 + sum Wm (d - d_0),
    // pm = phi_0 + atan2(sum Wm sin(phi - phi_0), sum Wm cos(phi - phi_0)).
#pragma unroll 1
    for (int j = lane; j < C.L; j += 64) {
        double px, py;
        if (!lmk(j, px, py)) {
            S.yr[2 * j] = 0.0;
            S.yr[2 * j + 1] = 0.0;
            continue;
        }
        double dm = 0.0, ss = 0.0, sc = 0.0;
        for (int k = 0; k < 7; k++) {
            dm += (S.Y[k * m2 + 2 * j] - S.Y[2 * j]) * C.Wm[k];
            ss += S.wsc[k * m2 + 2 * j];
            sc += S.wsc[k * m2 + 2 * j + 1];
        }
        dm = S.Y[2 * j] + dm;
        const double pm = wrap_angle(S.Y[2 * j + 1] + ukf_atan2(ss, sc));
        S.wsc[2 * j] = dm;  // row 0 of wsc is consumed: (dm, pm) per landmark
        S.wsc[2 * j + 1] = pm;
        S.yr[2 * j] = z[2 * j] - dm;
        S.yr[2 * j + 1] = wrap_angle(z[2 * j + 1] - pm);
    }
    __syncthreads();
    for (int m = lane; m < m2; m += 64) S.rinv[m] = 1.0 / Rd[m];
    // ---- residuals rz_k on the pairs (inactive slots -> 0)
#pragma unroll 1
    for (int e = lane; e < npair; e += 64) {
        const int k = e / C.L, j = e - k * C.L;
        double px, py;
        double r0 = 0.0, r1 = 0.0;
        if (lmk(j, px, py)) {
            r0 = S.Y[k * m2 + 2 * j] - S.wsc[2 * j];
            r1 = wrap_angle(S.Y[k * m2 + 2 * j + 1] - S.wsc[2 * j + 1]);
        }
        S.Y[k * m2 + 2 * j] = r0;
        S.Y[k * m2 + 2 * j + 1] = r1;
    }
    __syncthreads();
    // ---- G = Y R^-1 Y^T (28 upper entries, lanes 0..27), b = Y R^-1 y (lanes 28..34)
    if (lane < 35) {
        int k, l;
        if (lane < 28) {
            int e = lane;
            k = 0;
            while (e >= 7 - k) { e -= 7 - k; k++; }
            l = k + e;
        } else {
            k = lane - 28;
            l = -1;
        }
        // four partial sums over m (ILP for the dependent FMA chain), then summed in order
        double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
        const double *yk = S.Y + k * m2;
        const double *yl = (l >= 0) ? S.Y + l * m2 : S.yr;
        int m = 0;
        for (; m + 4 <= m2; m += 4) {
            a0 = __builtin_fma(yk[m] * S.rinv[m], yl[m], a0);
            a1 = __builtin_fma(yk[m + 1] * S.rinv[m + 1], yl[m + 1], a1);
            a2 = __builtin_fma(yk[m + 2] * S.rinv[m + 2], yl[m + 2], a2);
            a3 = __builtin_fma(yk[m + 3] * S.rinv[m + 3], yl[m + 3], a3);
        }
        for (; m < m2; m++) a0 = __builtin_fma(yk[m] * S.rinv[m], yl[m], a0);
        const double acc = (a0 + a1) + (a2 + a3);
        if (lane < 28) S.G[lane] = acc;
        else S.bv[lane - 28] = acc;
    }
    __syncthreads();
    // ---- M = W^-1 + G ; [M | I] in LDS
    for (int e = lane; e < 98; e += 64) {
        const int r = e / 14, cc = e % 14;
        double v;
        if (cc < 7) {
            const int k = min(r, cc), l = max(r, cc);
            const int idx = k * 7 - (k * (k - 1)) / 2 + (l - k);
            v = S.G[idx];
            if (r == cc) v += 1.0 / C.Wc[r];
        } else {
            v = (cc - 7 == r) ? 1.0 : 0.0;
        }
        S.aug[e] = v;
    }
    __syncthreads();
    // ---- Gauss-Jordan with partial pivoting, lanes over entries
#pragma unroll 1
    for (int c = 0; c < 7; c++) {
        int piv = c;
        double best = fabs(S.aug[c * 14 + c]);
        for (int r = c + 1; r < 7; r++) {
            const double v = fabs(S.aug[r * 14 + c]);
            if (v > best) { best = v; piv = r; }
        }
        if (!(best > 0.0)) ok = false;
        if (piv != c) {
            double t0 = 0.0, t1 = 0.0;
            if (lane < 14) { t0 = S.aug[c * 14 + lane]; t1 = S.aug[piv * 14 + lane]; }
            __syncthreads();
            if (lane < 14) { S.aug[c * 14 + lane] = t1; S.aug[piv * 14 + lane] = t0; }
            __syncthreads();
        }
        const double dpiv = S.aug[c * 14 + c];
        double rowc = 0.0;
        if (lane < 14) rowc = S.aug[c * 14 + lane] / dpiv;
        __syncthreads();
        if (lane < 14) S.aug[c * 14 + lane] = rowc;
        __syncthreads();
        // eliminate column c from the other rows (lanes own entries e and e+64)
        const int e0 = lane, e1 = lane + 64;
        double v0, v1 = 0.0;
        {
            const int r = e0 / 14, cc = e0 % 14;
            v0 = S.aug[e0];
            if (r != c) {
                const double f = S.aug[r * 14 + c];
                if (f != 0.0) v0 = v0 - f * S.aug[c * 14 + cc];
            }
        }
        if (e1 < 98) {
            const int r = e1 / 14, cc = e1 % 14;
            v1 = S.aug[e1];
            if (r != c) {
                const double f = S.aug[r * 14 + c];
                if (f != 0.0) v1 = v1 - f * S.aug[c * 14 + cc];
            }
        }
        __syncthreads();
        S.aug[e0] = v0;
        if (e1 < 98) S.aug[e1] = v1;
        __syncthreads();
    }
    // Minv[k][l] = aug[k*14 + 7 + l]
    // ---- x += Dx^T M^-1 b ;  P -= Dx^T (W - M^-1) Dx  (entry lanes, LDS exchange)
    if (lane < 7) {  // mb[k] = sum_l Minv[k][l] b[l]
        double sacc = 0.0;
        for (int l = 0; l < 7; l++) sacc += S.aug[lane * 14 + 7 + l] * S.bv[l];
        S.xv[lane] = sacc;
    } else if (lane >= 32 && lane < 32 + 21) {  // T[k][j] = sum_l (W - Minv)[k][l] Dx[l][j]
        const int e = lane - 32, k = e / 3, j = e - 3 * k;
        double t = 0.0;
        for (int l = 0; l < 7; l++) {
            const double wml = ((k == l) ? C.Wc[k] : 0.0) - S.aug[k * 14 + 7 + l];
            t += wml * S.Dx[3 * l + j];
        }
        S.T[e] = t;
    }
    __syncthreads();
    double dxn[3], KSK[9];
    for (int i = 0; i < 3; i++) {
        double sacc = 0.0;
        for (int k = 0; k < 7; k++) sacc += S.Dx[3 * k + i] * S.xv[k];
        dxn[i] = sacc;
    }
#pragma unroll 1
    for (int e = 0; e < 9; e++) {
        const int i = e / 3, j = e - 3 * i;
        double sacc = 0.0;
        for (int k = 0; k < 7; k++) sacc += S.Dx[3 * k + i] * S.T[3 * k + j];
        KSK[e] = sacc;
    }
    for (int i = 0; i < 3; i++) x[i] = x[i] + dxn[i];
    for (int i = 0; i < 9; i++) P[i] = P[i] - KSK[i];
    __syncthreads();
    return ok;
}

// The same step for one scan on a GROUP of Pg lanes (Pg a power of two <= 64; 64 / Pg scans
// per wave): registers only, no LDS and no barriers.  Every lane of the group runs the predict,
// the sigma points and the final solve redundantly (identical inputs give identical results);
// the measurement work is split by landmark (lane g takes j = g, g + Pg, ...), each lane
// accumulates its landmarks' share of G = Y R^-1 Y^T and b = Y R^-1 y, and an xor butterfly over
// the group sums them (commutative pairs: every lane ends with the same G and b).  The sums keep
// the sigma order k = 0..6; M X = [b | Dx] is solved directly (Gauss-Jordan, partial pivoting)
// instead of forming M^-1, so the last bits differ from ukf_step; both are held to the 50-digit
// evaluation per component (tests/test_gpu_ukf_exact.py).
//
// VAR (lslam_ukf_step only; the pipeline's kernels run VAR = 0): bit UKF_VAR_SIGMAS reads and
// writes filterpy's cached sigma points through `sio` ([7][3], the scan's ukf_sigmas): a predict
// stores the re-drawn sigmas_f there, and an update without a predict in the same call
// (LSLAM_UKF_SIGMAS_IN) takes them from there instead of drawing them from (x, P), as
// filterpy's update uses self.sigmas_f with the current self.x and self.P.  Bit UKF_VAR_TRACE
// writes the step's intermediate values to `tr` (layout UKF_TR_*; the lane that owns a
// landmark writes its entries), so tests can read hx and the wrapped residuals.
enum { UKF_VAR_TRACE = 1, UKF_VAR_SIGMAS = 2 };
__host__ __device__ constexpr int ukf_tr_doubles(int L) { return 42 + 16 * 2 * L; }
// per-scan trace layout (doubles, m = 2L): update's sigma points [7][3], Dx = residual_x(sigma_k, x)
// [7][3], hx(sigma_k) [7][m], zp [m], y = residual_h(z, zp) [m], rz_k = residual_h(hx(sigma_k), zp) [7][m]
__host__ __device__ constexpr int ukf_tr_hx(int L) { return 42; }
__host__ __device__ constexpr int ukf_tr_zp(int L) { return 42 + 7 * 2 * L; }
__host__ __device__ constexpr int ukf_tr_yr(int L) { return 42 + 8 * 2 * L; }
__host__ __device__ constexpr int ukf_tr_rz(int L) { return 42 + 9 * 2 * L; }

template <int VAR = 0, typename LmkFn>
__device__ bool ukf_step_group(double x[3], double P[9], double u0, double u1, const double *z, const double *Rd,
                               LmkFn lmk, const UkfConst &C, int flags, int g, int Pg, double *sio = nullptr,
                               double *tr = nullptr) {
    constexpr bool kTrace = (VAR & UKF_VAR_TRACE) != 0, kSig = (VAR & UKF_VAR_SIGMAS) != 0;
    bool ok = true;
    double U[9];
    double sig[21];
    if (flags & 1) {  // ---- predict
        {
            double A[9];
#pragma unroll
            for (int i = 0; i < 9; i++) A[i] = C.cfac * P[i];
            chol3_upper(A, U);
        }
#pragma unroll
        for (int k = 0; k < 7; k++) {
            double sg[3];
            sigma_point(k, x, U, sg);
            fx(sg, C.dt, u0, u1, C.wr, C.wb, sig + 3 * k);
        }
        double s0 = 0.0, s1 = 0.0, ss = 0.0, sc = 0.0;
#pragma unroll
        for (int k = 0; k < 7; k++) {
            const double2 scv = ukf_sincos(sig[3 * k + 2] - sig[2]);
            s0 += (sig[3 * k] - sig[0]) * C.Wm[k];
            s1 += (sig[3 * k + 1] - sig[1]) * C.Wm[k];
            ss += scv.x * C.Wm[k];
            sc += scv.y * C.Wm[k];
        }
        const double xm0 = sig[0] + s0, xm1 = sig[1] + s1;
        const double xm2 = wrap_angle(sig[2] + ukf_atan2(ss, sc));
        double Pn[9];
#pragma unroll
        for (int i = 0; i < 9; i++) Pn[i] = 0.0;
#pragma unroll
        for (int k = 0; k < 7; k++) {
            const double y[3] = {sig[3 * k] - xm0, sig[3 * k + 1] - xm1, wrap_angle(sig[3 * k + 2] - xm2)};
            const double w = C.Wc[k];
#pragma unroll
            for (int i = 0; i < 3; i++)
#pragma unroll
                for (int j = 0; j < 3; j++) Pn[3 * i + j] = Pn[3 * i + j] + w * (y[i] * y[j]);
        }
#pragma unroll
        for (int i = 0; i < 9; i++) P[i] = Pn[i] + C.Q[i];
        x[0] = xm0;
        x[1] = xm1;
        x[2] = xm2;
    }
    const bool sig_in = kSig && !(flags & 1) && (flags & LSLAM_UKF_SIGMAS_IN);
    if (!(flags & 2) && !(kSig && (flags & 1))) return ok;
    if (!sig_in) {
        double A[9];
#pragma unroll
        for (int i = 0; i < 9; i++) A[i] = C.cfac * P[i];
        chol3_upper(A, U);
        if (!(U[0] > 0.0) || !(U[4] > 0.0) || !(U[8] > 0.0)) ok = false;
    }
    double Dx[21];
#pragma unroll
    for (int k = 0; k < 7; k++) {
        if (sig_in) {
            sig[3 * k] = sio[3 * k];
            sig[3 * k + 1] = sio[3 * k + 1];
            sig[3 * k + 2] = sio[3 * k + 2];
        } else {
            sigma_point(k, x, U, sig + 3 * k);
        }
        Dx[3 * k] = sig[3 * k] - x[0];
        Dx[3 * k + 1] = sig[3 * k + 1] - x[1];
        Dx[3 * k + 2] = wrap_angle(sig[3 * k + 2] - x[2]);
    }
    if constexpr (kSig) {
        if ((flags & 1) && g == 0)
            for (int e = 0; e < 21; e++) sio[e] = sig[e];  // filterpy's sigmas_f after predict
        if (!(flags & 2)) return ok;
    }
    if constexpr (kTrace) {
        if (g == 0)
            for (int e = 0; e < 21; e++) {
                tr[e] = sig[e];
                tr[21 + e] = Dx[e];
            }
    }
    // G = Y R^-1 Y^T (upper triangle, row-major k <= l) and b = Y R^-1 y over the landmarks
    double G[28], bv[7];
#pragma unroll
    for (int e = 0; e < 28; e++) G[e] = 0.0;
#pragma unroll
    for (int k = 0; k < 7; k++) bv[k] = 0.0;
#pragma unroll 1
    for (int j = g; j < C.L; j += Pg) {
        double px, py;
        if (!lmk(j, px, py)) continue;  // an inactive slot adds exactly nothing
        double d[7], ph[7];
#pragma unroll
        for (int k = 0; k < 7; k++) {
            const double dx = px - sig[3 * k], dy = py - sig[3 * k + 1];
            d[k] = cr_sqrt(dx * dx + dy * dy);
            ph[k] = wrap_angle(ukf_atan2(dy, dx) - sig[3 * k + 2]);
        }
        // z_mean about sigma 0 (as in ukf_step)
        double dm = 0.0, ss = 0.0, sc = 0.0;
#pragma unroll
        for (int k = 0; k < 7; k++) {
            const double2 scv = ukf_sincos(ph[k] - ph[0]);
            dm += (d[k] - d[0]) * C.Wm[k];
            ss += scv.x * C.Wm[k];
            sc += scv.y * C.Wm[k];
        }
        dm = d[0] + dm;
        const double pm = wrap_angle(ph[0] + ukf_atan2(ss, sc));
        const double yr0 = z[2 * j] - dm, yr1 = wrap_angle(z[2 * j + 1] - pm);
        const double ri0 = 1.0 / Rd[2 * j], ri1 = 1.0 / Rd[2 * j + 1];
        double r0[7], r1[7];
#pragma unroll
        for (int k = 0; k < 7; k++) {
            r0[k] = d[k] - dm;
            r1[k] = wrap_angle(ph[k] - pm);
        }
        if constexpr (kTrace) {
            const int m = 2 * C.L;
            for (int k = 0; k < 7; k++) {
                tr[ukf_tr_hx(C.L) + k * m + 2 * j] = d[k];
                tr[ukf_tr_hx(C.L) + k * m + 2 * j + 1] = ph[k];
                tr[ukf_tr_rz(C.L) + k * m + 2 * j] = r0[k];
                tr[ukf_tr_rz(C.L) + k * m + 2 * j + 1] = r1[k];
            }
            tr[ukf_tr_zp(C.L) + 2 * j] = dm;
            tr[ukf_tr_zp(C.L) + 2 * j + 1] = pm;
            tr[ukf_tr_yr(C.L) + 2 * j] = yr0;
            tr[ukf_tr_yr(C.L) + 2 * j + 1] = yr1;
        }
        int e = 0;
#pragma unroll
        for (int k = 0; k < 7; k++) {
            const double w0 = r0[k] * ri0, w1 = r1[k] * ri1;
#pragma unroll
            for (int l = k; l < 7; l++, e++) {
                G[e] = __builtin_fma(w0, r0[l], G[e]);
                G[e] = __builtin_fma(w1, r1[l], G[e]);
            }
            bv[k] = __builtin_fma(w0, yr0, bv[k]);
            bv[k] = __builtin_fma(w1, yr1, bv[k]);
        }
    }
    // the group's sum of G and b
#pragma unroll 1
    for (int o = 1; o < Pg; o <<= 1) {
#pragma unroll
        for (int e = 0; e < 28; e++) G[e] += __shfl_xor(G[e], o);
#pragma unroll
        for (int k = 0; k < 7; k++) bv[k] += __shfl_xor(bv[k], o);
    }
    // [M | b | Dx], M = W^-1 + G; Gauss-Jordan with partial pivoting (first largest |pivot|)
    double A[7][11];
#pragma unroll
    for (int r = 0; r < 7; r++) {
#pragma unroll
        for (int cc = 0; cc < 7; cc++) {
            const int k = r < cc ? r : cc, l = r < cc ? cc : r;
            double v = G[k * 7 - (k * (k - 1)) / 2 + (l - k)];
            if (r == cc) v += 1.0 / C.Wc[r];
            A[r][cc] = v;
        }
        A[r][7] = bv[r];
#pragma unroll
        for (int j = 0; j < 3; j++) A[r][8 + j] = Dx[3 * r + j];
    }
#pragma unroll
    for (int c = 0; c < 7; c++) {
        int piv = c;
        double best = fabs(A[c][c]);
#pragma unroll
        for (int r = c + 1; r < 7; r++) {
            const double v = fabs(A[r][c]);
            if (v > best) {
                best = v;
                piv = r;
            }
        }
        if (!(best > 0.0)) ok = false;
#pragma unroll
        for (int r = c + 1; r < 7; r++) {
            if (piv == r) {
#pragma unroll
                for (int cc = 0; cc < 11; cc++) {
                    const double t = A[c][cc];
                    A[c][cc] = A[r][cc];
                    A[r][cc] = t;
                }
            }
        }
        const double dpiv = A[c][c];
#pragma unroll
        for (int cc = 0; cc < 11; cc++) A[c][cc] = A[c][cc] / dpiv;
#pragma unroll
        for (int r = 0; r < 7; r++) {
            if (r == c) continue;
            const double f = A[r][c];
            if (f != 0.0) {
#pragma unroll
                for (int cc = 0; cc < 11; cc++) A[r][cc] = A[r][cc] - f * A[c][cc];
            }
        }
    }
    // x += Dx^T M^-1 b ;  P -= Dx^T (W Dx - M^-1 Dx)
    double dxn[3], KSK[9];
#pragma unroll
    for (int i = 0; i < 3; i++) {
        double sacc = 0.0;
#pragma unroll
        for (int k = 0; k < 7; k++) sacc += Dx[3 * k + i] * A[k][7];
        dxn[i] = sacc;
    }
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++) {
            double sacc = 0.0;
#pragma unroll
            for (int k = 0; k < 7; k++) sacc += Dx[3 * k + i] * (C.Wc[k] * Dx[3 * k + j] - A[k][8 + j]);
            KSK[3 * i + j] = sacc;
        }
#pragma unroll
    for (int i = 0; i < 3; i++) x[i] = x[i] + dxn[i];
#pragma unroll
    for (int i = 0; i < 9; i++) P[i] = P[i] - KSK[i];
    return ok;
}

}  // namespace lslam
