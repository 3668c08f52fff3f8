/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Never linked into, loaded by, or called
 * from the product path (lidar_slam_amd/).  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may use it, and only as the checker.
 *
 * Plain-C CPU restatement of the reference's per-chunk RANSAC/landmark path,
 * bit-exact by construction (compile with -ffp-contract=off; every FMA that
 * the reference's native code performs is written out with fma()).
 *
 * What it restates (file:line):
 *   - ransac_functions.py:15-59   landmark_extraction (line params, tip,
 *                                  association walk incl. skip-after-remove)
 *   - landmarking.py:3-6,48-77    LIFE/TOLERANCE constants, decrease_life,
 *                                  reset_life, is_equal, distance_* (np.linalg.norm)
 *   - skimage 0.18.3 measure/fit.py:581-881 `ransac` (hypothesis loop, best
 *     selection, stop_residuals_sum stop, final refit) and fit.py:19-132
 *     LineModelND.estimate/residuals; _shared/utils.py:323-341 (global RNG).
 *     scikit-image is a third-party dependency NOT vendored in the reference;
 *     its 0.18.3 algorithm is restated here.
 *   - numpy 1.26 legacy RandomState: MT19937 init_genrand seeding, genrand_int32
 *     tempering, `random_interval` masked rejection, `_shuffle_raw`
 *     Fisher-Yates, `choice(n, 2, replace=False) == permutation(n)[:2]`.
 *   - numpy `pairwise_sum` (8 accumulators, 128-element leaves) behind
 *     `np.sum(r**2)`; sequential axis-0 `add.reduce` behind `data.mean(0)`.
 *   - OpenBLAS rounding measured on the fixture host: `(d-o) @ u` rounds as
 *     fma(dx,ux, dy*uy); `np.linalg.norm(v)` as sqrt(fma(vy,vy, vx*vx));
 *     einsum('ij,ij->i') as plain rx*rx + ry*ry.
 *   - LAPACK dgesdd (final TLS refit, fit.py:94) is replaced by the closed-form
 *     principal eigenvector of the 2x2 scatter matrix (tls_direction below,
 *     scatter matrix summed in the kernel's lane order, scatter2),
 *     the SAME formula the HIP kernel uses; vs LAPACK it agrees to ~1e-14
 *     relative (checked against the golden vectors), with the sign of the
 *     direction normalised by nothing (a, b are sign-invariant).
 *
 * Parity is pinned against the tests/golden .npz vectors produced by importing the
 * reference (tests/golden/make_golden.py).
 */
#include <math.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>

#define MT_N 624
#define MT_M 397

/* ---------------- legacy MT19937 (numpy randomkit / mt19937.c) ---------- */
void or_mt_seed(uint32_t seed, uint32_t *key, int32_t *pos) {
    for (int i = 0; i < MT_N; i++) {
        key[i] = seed;
        seed = 1812433253u * (seed ^ (seed >> 30)) + (uint32_t)(i + 1);
    }
    *pos = MT_N;
}

static void mt_gen(uint32_t *key) {
    const uint32_t UP = 0x80000000u, LO = 0x7fffffffu, MA = 0x9908b0dfu;
    int i;
    uint32_t y;
    for (i = 0; i < MT_N - MT_M; i++) {
        y = (key[i] & UP) | (key[i + 1] & LO);
        key[i] = key[i + MT_M] ^ (y >> 1) ^ ((uint32_t)(-(int32_t)(y & 1)) & MA);
    }
    for (; i < MT_N - 1; i++) {
        y = (key[i] & UP) | (key[i + 1] & LO);
        key[i] = key[i + (MT_M - MT_N)] ^ (y >> 1) ^ ((uint32_t)(-(int32_t)(y & 1)) & MA);
    }
    y = (key[MT_N - 1] & UP) | (key[0] & LO);
    key[MT_N - 1] = key[MT_M - 1] ^ (y >> 1) ^ ((uint32_t)(-(int32_t)(y & 1)) & MA);
}

uint32_t or_mt_next(uint32_t *key, int32_t *pos) {
    if (*pos >= MT_N) { mt_gen(key); *pos = 0; }
    uint32_t y = key[(*pos)++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

static uint32_t random_interval(uint32_t *key, int32_t *pos, uint32_t max) {
    if (max == 0) return 0;
    uint32_t mask = max;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
    uint32_t v;
    while ((v = (or_mt_next(key, pos) & mask)) > max) {}
    return v;
}

/* choice(n, 2, replace=False) = permutation(n)[:2]; `perm` is scratch of n ints. */
void or_choice2(uint32_t *key, int32_t *pos, int32_t n, int32_t *perm, int32_t *out2) {
    for (int32_t i = 0; i < n; i++) perm[i] = i;
    for (int32_t i = n - 1; i >= 1; i--) {
        int32_t j = (int32_t)random_interval(key, pos, (uint32_t)i);
        int32_t t = perm[j]; perm[j] = perm[i]; perm[i] = t;
    }
    out2[0] = perm[0];
    out2[1] = perm[1];
}

/* ---------------- numeric helpers ----------------------------------------- */
/* smallest e with RN(sqrt(e)) >= thr, so that  (sqrt(e) < thr)  <=>  (e < ecut) */
double or_ecut(double thr) {
    if (isnan(thr)) return NAN;
    if (!(thr > 0)) return 0.0;
    if (isinf(thr)) return INFINITY;
    double e = thr * thr;
    while (e > 0 && sqrt(e) >= thr) e = nextafter(e, 0.0);
    while (sqrt(e) < thr) e = nextafter(e, INFINITY);
    return e;
}

/* numpy pairwise_sum over a[0..n) (numpy/core/src/umath/loops_utils.h.src) */
static double pairwise_sum(const double *a, int64_t n) {
    if (n < 8) {
        double res = 0.;
        for (int64_t i = 0; i < n; i++) res += a[i];
        return res;
    } else if (n <= 128) {
        double r[8], res;
        int64_t i;
        for (int k = 0; k < 8; k++) r[k] = a[k];
        for (i = 8; i < n - (n % 8); i += 8)
            for (int k = 0; k < 8; k++) r[k] += a[i + k];
        res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; i++) res += a[i];
        return res;
    } else {
        int64_t n2 = n / 2;
        n2 -= n2 % 8;
        return pairwise_sum(a, n2) + pairwise_sum(a + n2, n - n2);
    }
}

/* LineModelND.estimate on exactly two points (fit.py:84-91) */
static void model2(double x0, double y0, double x1, double y1, double *m) {
    double ox = (x0 + x1) / 2.0, oy = (y0 + y1) / 2.0;
    double d0x = x0 - ox, d0y = y0 - oy, d1x = x1 - ox, d1y = y1 - oy;
    double dx = d1x - d0x, dy = d1y - d0y;
    double nrm = sqrt(fma(dy, dy, dx * dx));
    if (nrm != 0) { dx = dx / nrm; dy = dy / nrm; }
    m[0] = ox; m[1] = oy; m[2] = dx; m[3] = dy;
}

/* squared residual of (x,y) to model m, in the reference's rounding (fit.py:129-132) */
static inline double resid2(double x, double y, const double *m) {
    double ex = x - m[0], ey = y - m[1];
    double t = fma(ex, m[2], ey * m[3]);
    double rx = ex - t * m[2], ry = ey - t * m[3];
    return rx * rx + ry * ry;
}

/* closed-form replacement for dgesdd's v[0] on centred data (shared with HIP) */
static void tls_direction(double sxx, double sxy, double syy, double *ux, double *uy) {
    double h = (sxx - syy) * 0.5;
    double r = sqrt(h * h + sxy * sxy);
    double vx, vy;
    if (sxx >= syy) { vx = h + r; vy = sxy; }
    else { vx = sxy; vy = r - h; }
    double nv = sqrt(vx * vx + vy * vy);
    if (!(nv > 0)) { *ux = 1.0; *uy = 0.0; return; }
    *ux = vx / nv;
    *uy = vy / nv;
}

/* ---------------- ransac (fit.py:581-881) + line parameters ------------- */
enum {
    OR_VALID = 1, OR_N_TOO_SMALL = 2, OR_NO_INLIERS = 4, OR_EST_FAIL = 8, OR_EARLY_STOP = 16,
    OR_VERTICAL = 32, OR_NEW_LANDMARK = 64, OR_MATCHED = 128
};

/* chunk model record, same field order as the C-ABI's lslam_chunk_model */
typedef struct {
    double ox, oy, ux, uy, a, b, tip_x, tip_y, proj_a, proj_b;
    int32_t n_inliers, best_trial, n_draws, flags;
    int32_t match_index, landmark_id, n_points, reserved;
} or_chunk_model;

/*
 * One ransac call on xy[n][2] with min_samples=2.
 * key/pos: legacy MT19937 state (in/out).  If hyp != NULL, draws are taken from
 * hyp[(T+1)][2] instead of the RNG (explicit-hypothesis mode).
 * mask[n] out.  draws_out[(T+1)*2] optional.  cnt_out[T]/sum_out[T] optional
 * (sums only for trials whose count equals the maximum; others NaN).
 */
/* Scatter matrix of the centred inliers for tls_direction, in the HIP
 * kernel's order (lslam_ransac.h:refit_line): inlier k (data order) is added
 * into partial sum k % 64 in ascending k, then the 64 partials are combined by
 * an xor butterfly with offsets 32, 16, ..., 1 (every lane ends with the same
 * value; lane 0's is returned). */
static void scatter2(const double *xy, const uint8_t *mask, int32_t n, double ox, double oy,
                     double *sxx_o, double *sxy_o, double *syy_o) {
    double sxx[64], sxy[64], syy[64], t0[64], t1[64], t2[64];
    for (int l = 0; l < 64; l++) sxx[l] = sxy[l] = syy[l] = 0.0;
    int32_t k = 0;
    for (int32_t p = 0; p < n; p++) if (mask[p]) {
        double cx = xy[2 * p] - ox, cy = xy[2 * p + 1] - oy;
        int l = k % 64;
        sxx[l] += cx * cx; sxy[l] += cx * cy; syy[l] += cy * cy;
        k++;
    }
    for (int off = 32; off >= 1; off >>= 1) {
        for (int l = 0; l < 64; l++) {
            t0[l] = sxx[l] + sxx[l ^ off];
            t1[l] = sxy[l] + sxy[l ^ off];
            t2[l] = syy[l] + syy[l ^ off];
        }
        for (int l = 0; l < 64; l++) { sxx[l] = t0[l]; sxy[l] = t1[l]; syy[l] = t2[l]; }
    }
    *sxx_o = sxx[0]; *sxy_o = sxy[0]; *syy_o = syy[0];
}

int or_ransac(const double *xy, int32_t n, double thr, int32_t T, uint32_t *key, int32_t *pos,
              const int32_t *hyp, uint8_t *mask, or_chunk_model *out, int32_t *draws_out,
              int32_t *cnt_out, double *sum_out) {
    memset(out, 0, sizeof(*out));
    out->best_trial = -1;
    out->match_index = -1;
    out->n_points = n;
    for (int32_t i = 0; i < n; i++) mask[i] = 0;
    if (!(2 < n)) { out->flags = OR_N_TOO_SMALL; return 0; }  /* fit.py:798-799 */
    if (thr < 0 || T < 0) return -1;                             /* fit.py:801-805 */
    double ecut = or_ecut(thr);
    int32_t *perm = (int32_t *)malloc(sizeof(int32_t) * (size_t)n);
    int32_t *draws = (int32_t *)malloc(sizeof(int32_t) * 2 * (size_t)(T + 1));
    int32_t *cnt = (int32_t *)malloc(sizeof(int32_t) * (size_t)(T > 0 ? T : 1));
    double *r2 = (double *)malloc(sizeof(double) * (size_t)n);
    /* fit.py:819: first draw before the loop, then one per trial (draw t+1 in trial t) */
    int32_t ndraw = 0;
    int32_t best = -1, bcnt = 0, stop = 0;
    double bsum = INFINITY;
    for (int32_t d = 0; d <= T; d++) {
        if (hyp) { draws[2 * d] = hyp[2 * d]; draws[2 * d + 1] = hyp[2 * d + 1]; }
        else or_choice2(key, pos, n, perm, draws + 2 * d);
    }
    /* counts for every trial (draws are data-independent); then the sequential
       selection with the stop test, exactly fit.py:822-869 */
    int32_t M = 0;
    for (int32_t t = 0; t < T; t++) {
        double m[4];
        int32_t i0 = draws[2 * t], i1 = draws[2 * t + 1];
        model2(xy[2 * i0], xy[2 * i0 + 1], xy[2 * i1], xy[2 * i1 + 1], m);
        int32_t c = 0;
        for (int32_t p = 0; p < n; p++) c += resid2(xy[2 * p], xy[2 * p + 1], m) < ecut;
        cnt[t] = c;
        if (c > M) M = c;
        if (cnt_out) cnt_out[t] = c;
        if (sum_out) sum_out[t] = NAN;
    }
    for (int32_t t = 0; t < T && !stop; t++) {
        if (cnt[t] != M) continue;  /* only max-count trials can end up best */
        double m[4];
        int32_t i0 = draws[2 * t], i1 = draws[2 * t + 1];
        model2(xy[2 * i0], xy[2 * i0 + 1], xy[2 * i1], xy[2 * i1 + 1], m);
        for (int32_t p = 0; p < n; p++) {
            double r = sqrt(resid2(xy[2 * p], xy[2 * p + 1], m));
            r2[p] = r * r;
        }
        double s = pairwise_sum(r2, n);
        if (sum_out) sum_out[t] = s;
        if (cnt[t] > bcnt || (cnt[t] == bcnt && s < bsum)) {
            best = t; bcnt = cnt[t]; bsum = s;
            if (bsum <= 0) { stop = 1; ndraw = t + 2; }
        }
    }
    if (!stop) ndraw = T + 1;
    if (draws_out) memcpy(draws_out, draws, sizeof(int32_t) * 2 * (size_t)(T + 1));
    out->n_draws = ndraw;
    out->best_trial = best;
    if (stop) out->flags |= OR_EARLY_STOP;
    int32_t nin = 0, last = -1;
    if (best >= 0) {
        double m[4];
        int32_t i0 = draws[2 * best], i1 = draws[2 * best + 1];
        model2(xy[2 * i0], xy[2 * i0 + 1], xy[2 * i1], xy[2 * i1 + 1], m);
        for (int32_t p = 0; p < n; p++) {
            mask[p] = resid2(xy[2 * p], xy[2 * p + 1], m) < ecut;
            if (mask[p]) { nin++; last = p; }
        }
    }
    out->n_inliers = nin;
    free(perm); free(draws); free(cnt); free(r2);
    if (nin == 0) {  /* fit.py:877-879: warn, (None, None) */
        for (int32_t p = 0; p < n; p++) mask[p] = 0;
        out->flags |= OR_NO_INLIERS;
        return 0;
    }
    if (nin == 1) { out->flags |= OR_EST_FAIL; return 0; }  /* fit.py:96-97 ValueError */
    /* final refit on inliers in data order (fit.py:871-875 -> 84-95) */
    double ox, oy, ux, uy;
    if (nin == 2) {
        int32_t a = -1, b = -1;
        for (int32_t p = 0; p < n; p++) if (mask[p]) { if (a < 0) a = p; else b = p; }
        double m[4];
        model2(xy[2 * a], xy[2 * a + 1], xy[2 * b], xy[2 * b + 1], m);
        ox = m[0]; oy = m[1]; ux = m[2]; uy = m[3];
    } else {
        double sx = 0, sy = 0;
        int first = 1;
        for (int32_t p = 0; p < n; p++) if (mask[p]) {
            if (first) { sx = xy[2 * p]; sy = xy[2 * p + 1]; first = 0; }
            else { sx += xy[2 * p]; sy += xy[2 * p + 1]; }
        }
        ox = sx / (double)nin; oy = sy / (double)nin;
        double sxx, sxy, syy;
        scatter2(xy, mask, n, ox, oy, &sxx, &sxy, &syy);
        tls_direction(sxx, sxy, syy, &ux, &uy);
    }
    out->ox = ox; out->oy = oy; out->ux = ux; out->uy = uy;
    /* ransac_functions.py:26-30 */
    double a = uy / ux;
    double b = oy - a * ox;
    out->a = a; out->b = b;
    out->tip_x = xy[2 * last];
    out->tip_y = out->tip_x * a + b;
    out->proj_a = a; out->proj_b = b;
    out->flags |= OR_VALID;
    if (ux == 0) out->flags |= OR_VERTICAL;
    return 0;
}

/* advance (key,pos) by exactly `ndraw` choice(n,2) draws */
void or_skip_draws(uint32_t *key, int32_t *pos, int32_t n, int32_t ndraw) {
    int32_t *perm = (int32_t *)malloc(sizeof(int32_t) * (size_t)n);
    int32_t o[2];
    for (int32_t d = 0; d < ndraw; d++) or_choice2(key, pos, n, perm, o);
    free(perm);
}

/* ransac with the RNG state advanced by the draws the reference actually made */
int or_ransac_chained(const double *xy, int32_t n, double thr, int32_t T, uint32_t *key, int32_t *pos,
                      uint8_t *mask, or_chunk_model *out, int32_t *draws_out, int32_t *cnt_out,
                      double *sum_out) {
    uint32_t k0[MT_N];
    int32_t p0 = *pos;
    memcpy(k0, key, sizeof(k0));
    int rc = or_ransac(xy, n, thr, T, key, pos, NULL, mask, out, draws_out, cnt_out, sum_out);
    if (rc == 0 && n > 2 && out->n_draws < T + 1) {
        memcpy(key, k0, sizeof(k0));
        *pos = p0;
        or_skip_draws(key, pos, n, out->n_draws);
    }
    return rc;
}

/* ---------------- landmarks (landmarking.py, ransac_functions.py:34-54) -- */
typedef struct {
    double a, b, px, py, ex, ey;
    int32_t id, life;
} or_landmark;

#define OR_LIFE 40
/* landmarking.py:4-6 TOLERANCE_A / TOLERANCE_B / TOLERANCE (module constants;
 * settable like lslam_ransac_params.tol_* for the map tests) */
static double OR_TOL_A = 0.1, OR_TOL_B = 10.0, OR_TOL = 100.0;
void or_set_tolerances(double tol_a, double tol_b, double tol_dist) {
    OR_TOL_A = tol_a; OR_TOL_B = tol_b; OR_TOL = tol_dist;
}

static inline double norm2(double vx, double vy) { return sqrt(fma(vy, vy, vx * vx)); }

/* landmarking.py:66-77: self=old landmark L, other=new F */
int or_is_equal(const or_landmark *L, const or_landmark *F) {
    double distA = fabs(L->a - F->a);
    double distB = fabs(L->b - F->b);
    double dEO = norm2(L->ex - F->px, L->ey - F->py);
    double dOE = norm2(L->px - F->ex, L->py - F->ey);
    if (distA <= OR_TOL_A && distB <= OR_TOL_B) return (dEO <= OR_TOL || dOE <= OR_TOL);
    return 0;
}

/*
 * ransac_functions.py:34-54 association walk + check_ransac's append (:75-76).
 * list[0..*count) in/out (capacity cap).  Returns matched original index or -1;
 * *new_flag = 1 if F was appended.
 */
int32_t or_associate(or_landmark *list, int32_t *count, int32_t cap, const or_landmark *F, int32_t *new_flag,
                     double *proj_a, double *proj_b) {
    int32_t L = *count, k = 0, match = -1;
    uint8_t *dead = (uint8_t *)calloc((size_t)(L > 0 ? L : 1), 1);
    while (k < L) {
        if (or_is_equal(&list[k], F)) { match = k; break; }
        /* decrease_life (landmarking.py:48-52) */
        if (list[k].life > 0) list[k].life -= 1;
        if (list[k].life == 0) { dead[k] = 1; k += 2; }  /* removal + i+=1 skips the next one */
        else k += 1;
    }
    *proj_a = F->a; *proj_b = F->b;
    if (match >= 0) {  /* reset_life; yBase uses the matched landmark's line (ransac_functions.py:44-47) */
        list[match].life = OR_LIFE;
        *proj_a = list[match].a; *proj_b = list[match].b;
    }
    int32_t w = 0;
    for (int32_t i = 0; i < L; i++) if (!dead[i]) list[w++] = list[i];
    free(dead);
    *new_flag = match < 0;
    if (match < 0) {
        if (w < cap) { list[w] = *F; list[w].life = OR_LIFE; w++; }
        else { *count = w; return -2; }
    }
    *count = w;
    return match;
}

/*
 * Whole landmark_extraction (ransac_functions.py:15-59) for one chunk, chained
 * RNG, plus check_ransac's append.  yproj[n]: y of the projected inliers
 * (0 for outliers).  Returns 0, or the flags in `out` describe the failure.
 */
int or_landmark_extraction(const double *xy, int32_t n, int32_t landmark_number, double thr, int32_t T,
                           uint32_t *key, int32_t *pos, or_landmark *list, int32_t *count, int32_t cap,
                           uint8_t *mask, double *yproj, or_chunk_model *out) {
    int rc = or_ransac_chained(xy, n, thr, T, key, pos, mask, out, NULL, NULL, NULL);
    if (rc) return rc;
    out->landmark_id = landmark_number;
    if (!(out->flags & OR_VALID)) return 0;
    or_landmark F = {out->a, out->b, out->ox, out->oy, out->tip_x, out->tip_y, landmark_number, OR_LIFE};
    int32_t nf = 0;
    int32_t m = or_associate(list, count, cap, &F, &nf, &out->proj_a, &out->proj_b);
    if (m == -2) return -2;
    out->match_index = m;
    out->flags |= (m >= 0) ? OR_MATCHED : OR_NEW_LANDMARK;
    if (yproj) for (int32_t p = 0; p < n; p++) yproj[p] = mask[p] ? (out->proj_a * xy[2 * p] + out->proj_b) : 0.0;
    return 0;
}

/* projection helper: y of inliers with the line that landmark_extraction uses */
void or_project(const double *xy, int32_t n, const uint8_t *mask, double a, double b, double *yproj) {
    for (int32_t p = 0; p < n; p++) yproj[p] = mask[p] ? (a * xy[2 * p] + b) : 0.0;
}
