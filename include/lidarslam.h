/*
 * lidarslam.h — C ABI of the MI355X-native per-scan hot path of
 * Farofeiro231/LiDAR_SLAM (RANSAC line/landmark extraction + UKF step).
 *
 * Plain pointers and sizes only; no torch, no C++ types.  Every function
 * returns an int status (LSLAM_OK = 0, < 0 on error) and never aborts.
 * Device pointers are HIP device memory (lslam_malloc or any hipMalloc'd
 * buffer); work is enqueued on the context's own HIP streams and is
 * asynchronous unless stated otherwise (lslam_sync waits for all of them).
 * lslam_h2d / lslam_d2h / lslam_memset are ordered after every earlier call
 * on the context (a pipeline call may finish on a side stream).
 *
 * Reference interfaces each entry point replaces (reference = /root/reference,
 * fit.py = scikit-image 0.18.3 skimage/measure/fit.py, the third-party code the
 * reference calls):
 *   lslam_polar_to_xy     functions.py:59-60   (dX, dY of each measure)
 *   lslam_express_decode  lidar.py:55-91 ExpressPacket.decode + :179-187
 *                         _process_express_scan over the :327-338 measure stream
 *   lslam_express_scans   the above + functions.py:56-76 (A1 + the A2 chunking of
 *                         each revolution fed to rawPoints)
 *   lslam_hyp_mt19937     fit.py:819-826 random_state.choice(N, 2, replace=False)
 *                         on the global np.random legacy MT19937 stream
 *   lslam_ransac          ransac_functions.py:23-31  ransac(data, LineModelND, 2, 20,
 *                         max_trials=100) + a, b, tip (fit.py:581-881, 19-132)
 *   lslam_landmarks       ransac_functions.py:34-54 association walk +
 *                         landmarking.py:48-77 + check_ransac append (:75-76)
 *   lslam_scan_pipeline   ransac_functions.py:63-93 check_ransac over the chunks
 *                         of many scans (landmark_extraction per chunk), fused with
 *                         the UKF step below
 *   lslam_ukf_step        systemClass.py:12-29 System.ukf.predict(u=..) +
 *                         .update(z, landmarks=..) with UKFMethods.py:10-71
 *                         callbacks (filterpy 1.4.5 UnscentedKalmanFilter semantics)
 *   lslam_ukf_trace       the same, exposing UKFMethods.py:26-34 hx and :60-71
 *                         residuals for the reference-pinned tests
 */
#ifndef LIDARSLAM_H
#define LIDARSLAM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LSLAM_ABI_VERSION 4

/* ---- status codes ---- */
enum {
    LSLAM_OK = 0,
    LSLAM_ERR_ARG = -1,         /* invalid argument (ValueError in the reference) */
    LSLAM_ERR_HIP = -2,         /* HIP runtime error (message: lslam_last_error) */
    LSLAM_ERR_NOMEM = -3,
    LSLAM_ERR_CAPACITY = -4,    /* a landmark list or chunk count exceeded its capacity */
    LSLAM_ERR_UNSUPPORTED = -5  /* e.g. min_samples != 2 */
};

/* ---- per-chunk flags (lslam_chunk_model.flags) ---- */
enum {
    LSLAM_VALID = 1,          /* model fitted; landmark_extraction returned normally */
    LSLAM_N_TOO_SMALL = 2,    /* N < 3: fit.py:798-799 ValueError, no RNG consumed */
    LSLAM_NO_INLIERS = 4,     /* fit.py:877-879 (None, None) -> AttributeError at ransac_functions.py:25 */
    LSLAM_EST_FAIL = 8,       /* 1 final inlier: fit.py:96-97 ValueError */
    LSLAM_EARLY_STOP = 16,    /* stop_residuals_sum hit (sum of squared residuals == 0) */
    LSLAM_VERTICAL = 32,      /* final direction x == 0: a = +-inf/nan (ransac_functions.py:26) */
    LSLAM_NEW_LANDMARK = 64,  /* no landmark matched: the chunk's Landmark was appended */
    LSLAM_MATCHED = 128,      /* an existing landmark matched (its life reset to LIFE) */
    LSLAM_CAPACITY = 256,     /* no match and the list was full: the new landmark was dropped */
    LSLAM_CHUNK_BOUND = 512   /* LSLAM_UKF_MAP only: a matched chunk at index >= max_scan_chunks of its
                                 scan (an understated max_scan_chunks) has no measurement slot, so the
                                 UKF update does not use it; association and outputs are unaffected */
};

/* ---- hypothesis sources ---- */
enum {
    LSLAM_HYP_MT19937 = 0,  /* numpy legacy RandomState stream, bit-exact with the reference */
    LSLAM_HYP_PHILOX = 1,   /* counter-based Philox4x32-10, statistically equivalent only */
    LSLAM_HYP_EXPLICIT = 2  /* caller-provided draws (lslam_scan_batch.hyp) */
};

/* ---- UKF flags ---- */
enum {
    LSLAM_UKF_PREDICT = 1,
    LSLAM_UKF_UPDATE = 2,
    LSLAM_UKF_LMK_FROM_RANSAC = 4, /* landmark slot c <- chunk c's Landmark.pos (fused pipeline) */
    /* Landmark MAP mode (lslam_scan_pipeline with landmarks only): each scan's
     * landmark list is a persistent WORLD-frame map.  Per scan: predict (if PREDICT); every fitted
     * chunk line (ransac_functions.py:25-31, robot frame) is moved into the world frame by the
     * predicted pose x = [tx, ty, th] (p_w = R(th) p + t; a, b from the rotated direction); the
     * association walk (ransac_functions.py:34-54) runs on the map; each chunk that MATCHED a map
     * landmark j becomes one range/bearing measurement against hx(x, pos_j) (UKFMethods.py:26-34):
     * z_c = [|f|, atan2(f_y, f_x)], f = the foot of pos_j (moved into the robot frame by the
     * predicted pose) on the chunk's fitted line (is_equal matches any segment continuing the same
     * wall, so the chunk's own origin is not pos_j's re-observation); update (if UPDATE and >= 1
     * match) with those measurements only.  ukf_z / ukf_lmk are not read; n_landmarks = measurement slots, one per
     * chunk of a scan (>= max_scan_chunks); R_diag[2c], R_diag[2c+1] is slot c's noise.
     * models[c] keeps the robot-frame fit; proj_a/proj_b (y_proj) stay the chunk's own line.
     * id_base (if given) is in/out in this mode: advanced by the scan's chunk count, as
     * check_ransac's landmarkNumber (ransac_functions.py:77), so steps chain without host syncs. */
    LSLAM_UKF_MAP = 8,
    /* lslam_ukf_step, an UPDATE without PREDICT in the same call: the sigma points are read from
     * lslam_scan_batch.ukf_sigmas (filterpy's self.sigmas_f, cached by the last predict) instead of
     * being drawn from (x, P); x and P are the current ones (filterpy UKF.update: cross_variance(self.x,
     * zp, self.sigmas_f, ...), self.P - K S K^T).  Not supported by lslam_scan_pipeline. */
    LSLAM_UKF_SIGMAS_IN = 16
};

/* One RANSAC call's result (one chunk), 112 bytes. */
typedef struct lslam_chunk_model {
    double ox, oy;          /* final model origin   (model_robust.params[0]) */
    double ux, uy;          /* final model direction (params[1]; sign arbitrary) */
    double a, b;            /* y = a*x + b         (ransac_functions.py:26-27) */
    double tip_x, tip_y;    /* Landmark.end        (ransac_functions.py:29-30) */
    double proj_a, proj_b;  /* line used for yBase: matched landmark's or own (:46,:49,:53) */
    int32_t n_inliers;      /* popcount of the inlier mask */
    int32_t best_trial;     /* winning hypothesis index (-1 if none) */
    int32_t n_draws;        /* choice() draws consumed: T+1, or stop_trial+2 on early stop */
    int32_t flags;          /* LSLAM_* flags above */
    int32_t match_index;    /* index of the matched landmark in the pre-call list, -1 if none */
    int32_t landmark_id;    /* landmarkNumber given to this chunk's Landmark */
    int32_t n_points;       /* chunk size N */
    int32_t reserved;
} lslam_chunk_model;

/* landmarking.Landmark (landmarking.py:12-19), 56 bytes. */
typedef struct lslam_landmark {
    double a, b;
    double pos_x, pos_y;   /* Landmark.pos = final model origin */
    double end_x, end_y;   /* Landmark.end = (tipX, tipY) */
    int32_t id;
    int32_t life;
} lslam_landmark;

typedef struct lslam_ransac_params {
    double residual_threshold;  /* ransac_functions.py:9  THRESHOLD = 20 */
    int32_t max_trials;         /* ransac_functions.py:10 MAX_TRIALS = 100 */
    int32_t min_samples;        /* ransac_functions.py:11 MIN_SAMPLES = 2 (only 2 supported) */
    int32_t hyp_source;         /* LSLAM_HYP_* */
    int32_t life;               /* landmarking.py:3 LIFE = 40 */
    double tol_a;               /* landmarking.py:4 TOLERANCE_A = 0.1 */
    double tol_b;               /* landmarking.py:5 TOLERANCE_B = 10 */
    double tol_dist;            /* landmarking.py:6 TOLERANCE = 100 */
    uint64_t philox_seed;       /* LSLAM_HYP_PHILOX key */
} lslam_ransac_params;

typedef struct lslam_ukf_params {
    int32_t n_landmarks;     /* L; dim_z = 2L (systemClass.py:7 LANDMARK_NUMBER = 8) */
    int32_t flags;           /* LSLAM_UKF_* */
    double dt;               /* systemClass.py:10 DT = 0.005 */
    double wheel_radius;     /* UKFMethods.py:6 R = 50 (mm) */
    double wheel_base;       /* UKFMethods.py:7 L = 200 (mm) */
    double alpha, beta, kappa; /* systemClass.py:20 MerweScaledSigmaPoints(3, 1e-4, 2, 0) */
    double Q[9];             /* systemClass.py:29 Q = 1e-3 * I3 */
} lslam_ukf_params;

/* A batch of scans, all pointers DEVICE memory (NULL = absent where optional). */
typedef struct lslam_scan_batch {
    int32_t n_scans;
    int32_t n_chunks;               /* = scan_chunk_off[n_scans] */
    int64_t n_points;               /* = chunk_pt_off[n_chunks] */
    int32_t max_chunk_points;       /* max chunk size N over the batch */
    int32_t max_scan_chunks;        /* max chunks per scan: sizes the post pass's LDS staging.  A scan with
                                       more chunks gets the same results through the unstaged paths (a
                                       rewind snapshot per chunk, records walked in place); only
                                       LSLAM_UKF_MAP's measurement slots stop there (LSLAM_CHUNK_BOUND) */
    int32_t lmk_capacity;           /* per-scan landmark list capacity */
    int32_t reserved;
    /* inputs */
    const double *xy;               /* [n_points][2] fp64 Cartesian points (AoS); NULL: theta_deg / dist_mm */
    const int32_t *scan_chunk_off;  /* [n_scans+1] CSR scan -> chunks */
    const int32_t *chunk_pt_off;    /* [n_chunks+1] CSR chunk -> points */
    const uint32_t *seeds;          /* [n_scans] np.random.seed(seed) per scan (MT19937 mode) */
    const uint32_t *mt_state_in;    /* [n_scans][625] key[624] + pos, overrides seeds */
    uint32_t *mt_state_out;         /* [n_scans][625] state after the scan (optional) */
    const int32_t *hyp;             /* [n_chunks][max_trials+1][2] (LSLAM_HYP_EXPLICIT) */
    const int32_t *id_base;         /* [n_scans] landmarkNumber of the first chunk (optional, 0) */
    lslam_landmark *landmarks;      /* [n_scans][lmk_capacity] in/out (optional) */
    int32_t *lmk_count;             /* [n_scans] in/out (required with landmarks) */
    int32_t *lmk_walk;              /* [n_scans][lmk_capacity] out (optional): life of each entry of the
                                       list as it was before the scan's LAST chunk, after that chunk's
                                       association walk (0 = removed); lets a caller holding its own
                                       list objects apply the walk (the drop-in shim) */
    /* outputs */
    uint8_t *inlier_mask;           /* [n_points] */
    lslam_chunk_model *models;      /* [n_chunks] */
    double *y_proj;                 /* [n_points] projected y of inliers, 0 elsewhere (optional) */
    int32_t *draws_out;             /* [n_chunks][max_trials+1][2] (optional, parity/debug) */
    int32_t *trial_cnt_out;         /* [n_chunks][max_trials] (optional, parity/debug; zero rows
                                       for chunks of fewer than 3 points) */
    /* UKF, per scan */
    double *ukf_x;                  /* [n_scans][3] in/out */
    double *ukf_P;                  /* [n_scans][3][3] in/out */
    const double *ukf_u;            /* [n_scans][2]  [vl, vr] */
    const double *ukf_z;            /* [n_scans][2L] interleaved [d0, phi0, d1, phi1, ...] (not in MAP mode) */
    const double *ukf_lmk;          /* [n_scans][L][2] landmark positions (not in MAP mode) */
    const double *ukf_R_diag;       /* [2L] measurement noise diagonal (systemClass.py:28) */
    /* A1 fused into the point loads (ABI 2): with xy == NULL the points are
     * the raw measures and every kernel that reads a point converts it as functions.py:59-60 does,
     * x = d cos(-th * pi/180 + pi/2), y = d sin(...), bit-identical to lslam_polar_to_xy. */
    const double *theta_deg;        /* [n_points] */
    const double *dist_mm;          /* [n_points] */
    /* ABI 4: filterpy's sigmas_f per scan, [n_scans][7][3] (optional; lslam_ukf_step only): a PREDICT
     * writes the sigma points re-drawn from the predicted (x, P); an UPDATE with LSLAM_UKF_SIGMAS_IN
     * reads them.  NULL: not written, and an update draws its sigma points from (x, P). */
    double *ukf_sigmas;
} lslam_scan_batch;

/* Express-scan measures (lslam_express_decode): device arrays, NULL = not written.
 * Packet p (< M-1) yields measures 32p .. 32p+31 (trame 1..32, using packet p+1's start angle). */
typedef struct lslam_express_measures {
    double *angle_deg;    /* [(M-1)*32] lidar.py:185 (0 where invalid) */
    double *dist_mm;      /* [(M-1)*32] ExpressPacket.distance (0 where invalid) */
    uint8_t *new_scan;    /* [(M-1)*32] lidar.py:181-184 */
    uint8_t *valid;       /* [(M-1)*32] packets p and p+1 both decode */
    double *xy;           /* [(M-1)*32][2] functions.py:59-60 (A1 fused) */
    uint8_t *pkt_valid;   /* [M] ExpressPacket.decode would not raise */
} lslam_express_measures;

/* Express-scan revolutions (lslam_express_scans): device arrays sized by the caller.
 * Safe capacities for M packets: cap_points = 32(M-1), cap_scans = M-1,
 * cap_chunks = 32(M-1)/100 + M-1.  counts (device, int32[4]) receives
 * n_scans, n_chunks, n_points, and the packet holding the last new-revolution
 * flag (-1 if none): resume the stream from that packet with skip = 1. */
typedef struct lslam_express_revs {
    double *xy;                 /* [cap_points][2] */
    int32_t *scan_chunk_off;    /* [cap_scans + 1] CSR revolution -> chunks */
    int32_t *chunk_pt_off;      /* [cap_chunks + 1] CSR chunk -> points */
    int32_t *counts;            /* [4] */
    int64_t cap_points;
    int32_t cap_scans, cap_chunks;
} lslam_express_revs;

typedef struct lslam_ctx lslam_ctx;  /* opaque: device, stream, events, scratch */

/* ---- library / context ---- */
const char *lslam_version(void);
const char *lslam_status_string(int status);
const char *lslam_last_error(void);  /* thread-local message of the last error */
int lslam_device_count(int *n);
int lslam_ctx_create(int device, lslam_ctx **out);
int lslam_ctx_destroy(lslam_ctx *ctx);
int lslam_sync(lslam_ctx *ctx);
int lslam_malloc(lslam_ctx *ctx, size_t bytes, void **dptr);
int lslam_free(lslam_ctx *ctx, void *dptr);
int lslam_host_alloc(size_t bytes, void **hptr);  /* pinned host memory */
int lslam_host_free(void *hptr);
int lslam_h2d(lslam_ctx *ctx, void *dst, const void *src, size_t bytes);  /* async */
int lslam_d2h(lslam_ctx *ctx, void *dst, const void *src, size_t bytes);  /* async */
int lslam_d2d(lslam_ctx *ctx, void *dst, const void *src, size_t bytes);  /* async */
int lslam_memset(lslam_ctx *ctx, void *dst, int value, size_t bytes);     /* async */
/* Page-lock existing host memory (hipHostRegister), e.g. a host batch shared between the
 * ranks of one node (the reference's mp.Queue hand-off, SLAM.py:13,18-23, done as shared
 * memory + per-rank H2D of a shard): lslam_h2d / lslam_d2h from it then run at PCIe rate. */
int lslam_host_register(void *hptr, size_t bytes);
int lslam_host_unregister(void *hptr);
/* The context's main HIP stream (a hipStream_t).  Work a caller enqueues on it, e.g. an RCCL
 * gather of a pipeline call's outputs (lidar_slam_amd/collective.py), runs after every call made
 * on the context so far and before later ones.  It must not write a buffer a later call's MT
 * producer reads (seeds, CSR offsets, mt_state_in) unless followed by lslam_sync. */
int lslam_ctx_stream(lslam_ctx *ctx, void **stream);
/* sizes (bytes) of the ABI structs as compiled into the library, in this order:
 * lslam_chunk_model, lslam_landmark, lslam_ransac_params, lslam_ukf_params, lslam_scan_batch,
 * lslam_express_measures, lslam_express_revs.  Writes min(n, 7) entries, returns 7. */
int lslam_abi_sizes(int64_t *sizes, int n);
/* per-kernel HIP-event timing on the ctx stream (kernel ids: LSLAM_K_*) */
enum { LSLAM_K_POLAR = 0, LSLAM_K_HYP = 1, LSLAM_K_PIPELINE = 2, LSLAM_K_LANDMARK = 3, LSLAM_K_UKF = 4,
       LSLAM_K_RNG = 5 /* parity-stream producer */, LSLAM_K_CONSENSUS = 6 /* per-chunk A4-A8 */,
       LSLAM_K_EXPRESS = 7 /* a whole express decode / scans call */,
       LSLAM_K_EXPRESS_SCATTER = 8 /* its decode + A1 + scatter kernel */, LSLAM_K_COUNT = 9 };
int lslam_set_timing(lslam_ctx *ctx, int enable);
/* which kernel ids are timed while timing is on (bit k = LSLAM_K_k; default all).  Timing
 * events between the producer and consumer kernels change how the two streams overlap,
 * so a throughput measurement should time only the kernel it reports. */
int lslam_set_timing_mask(lslam_ctx *ctx, uint32_t mask);
int lslam_timing(lslam_ctx *ctx, int kernel, double *total_ms, int64_t *launches);  /* syncs */
int lslam_timing_reset(lslam_ctx *ctx);
/* Bytes of Fisher-Yates steps scratch per producer slot (two slots; default 2 GiB, or the
 * LSLAM_STEPS_BUDGET environment variable).  A parity-mode call whose scans are one chunk each
 * (C5) and whose steps exceed it runs the producer in epochs of as many draws as fit, each
 * resolved before its slot is reused.  bytes <= 0 restores the default.  Syncs. */
int lslam_set_steps_budget(lslam_ctx *ctx, int64_t bytes);

/* ---- host helpers ---- */
int lslam_ransac_params_default(lslam_ransac_params *p);
int lslam_ukf_params_default(lslam_ukf_params *p, int32_t n_landmarks);
/* smallest e with RN(sqrt(e)) >= thr: (residual < thr) <=> (squared residual < cutoff) */
double lslam_inlier_cutoff(double thr);
/* MerweScaledSigmaPoints weights (filterpy _compute_weights) for n = 3 */
int lslam_ukf_weights(const lslam_ukf_params *p, double *Wm7, double *Wc7, double *lambda_plus_n);
/* numpy RandomState(seed) state: key[624] + pos (host memory, 625 words) */
int lslam_mt_seed_state(uint32_t seed, uint32_t *state625);

/* ---- hot path (device pointers, async on the ctx stream) ---- */
/* A1: xy[i] = (d cos(-th*pi/180 + pi/2), d sin(...)); n measures */
int lslam_polar_to_xy(lslam_ctx *ctx, const double *theta_deg, const double *dist, double *xy, int64_t n);
/* E1: RPLidar express packets (M x 84 bytes, 4-byte aligned) -> measure stream */
int lslam_express_decode(lslam_ctx *ctx, const uint8_t *packets, int64_t n_packets, const lslam_express_measures *out);
/* E1 + A1 + A2: packets -> revolutions of chunked xy (functions.py:56-76); the first
 * `skip` measures of packet 0 are dropped (a resumed stream).  Writes are clipped
 * to the capacities; counts always holds the required sizes. */
int lslam_express_scans(lslam_ctx *ctx, const uint8_t *packets, int64_t n_packets, int32_t skip,
                        const lslam_express_revs *out);
/* A3: the draws each chunk's ransac would make, assuming no early stop
 * (draws_out [n_chunks][max_trials+1][2]).  Uses b->seeds/mt_state_in/mt_state_out. */
int lslam_hyp_mt19937(lslam_ctx *ctx, const lslam_scan_batch *b, int32_t max_trials);
/* A3-A8: ransac per chunk (chained RNG per scan), masks, models */
int lslam_ransac(lslam_ctx *ctx, const lslam_scan_batch *b, const lslam_ransac_params *p);
/* A9-A10: association over b->models (already fitted) + y_proj */
int lslam_landmarks(lslam_ctx *ctx, const lslam_scan_batch *b, const lslam_ransac_params *p);
/* U1-U8: one predict and/or update per scan */
int lslam_ukf_step(lslam_ctx *ctx, const lslam_scan_batch *b, const lslam_ukf_params *u);
/* Test / diagnostic: lslam_ukf_step (the same kernel code, lane-group form) that also writes the
 * update's intermediate values per scan to trace (device, [n_scans][42 + 32 L] doubles, m = 2L):
 *   [0, 21)            sigma points sigma_k (k = 0..6, [x, y, theta])
 *   [21, 42)           residual_x(sigma_k, x)                           UKFMethods.py:60-63
 *   [42, 42 + 7m)      hx(sigma_k) = transfer_function(sigma_k, lmk)    UKFMethods.py:26-34
 *   [42 + 7m, +m)      zp (z_mean about sigma 0)
 *   [42 + 8m, +m)      residual_h(z, zp)                                UKFMethods.py:66-71
 *   [42 + 9m, +7m)     residual_h(hx(sigma_k), zp)
 * Entries of inactive landmark slots are not written.  Needs LSLAM_UKF_UPDATE; not in MAP mode. */
int lslam_ukf_trace(lslam_ctx *ctx, const lslam_scan_batch *b, const lslam_ukf_params *u, double *trace);
/* A3-A10 (+ U1-U8 if u != NULL) for every scan of the batch in one call: MT19937 producer (its
 * own stream, overlapping the previous call's consumers), resolve, consensus, fix-up, then the
 * association / UKF post pass */
int lslam_scan_pipeline(lslam_ctx *ctx, const lslam_scan_batch *b, const lslam_ransac_params *p,
                        const lslam_ukf_params *u);

#ifdef __cplusplus
}
#endif
#endif /* LIDARSLAM_H */
