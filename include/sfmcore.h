/*
 * sfmcore.h -- C-ABI of libsfmcore.so, the MI355X (gfx950) numerical core
 * that replaces the reference's hot path
 *   EstimateFundamentalMatrix -> GetInliersRANSAC -> LinearTriangulation
 *   -> BundleAdjustment       (pvrohin/Structure-from-Motion-, "Phase 1/").
 *
 * Plain C types only: caller-owned, row-major, C-contiguous host buffers,
 * int return codes (0 = OK, < 0 = error; message via sfm_last_error()).
 * No C++ exception crosses this line.  Every entry point is reentrant: each
 * host thread gets its own HIP stream and scratch buffers per device.
 *
 * The Python drop-in modules in structure-from-motion-_amd/ bind these with
 * ctypes (_sfmcore.py); INTEGRATION.md shows the binding.
 */
#ifndef SFMCORE_H
#define SFMCORE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SFM_ABI_VERSION 1

enum {
    SFM_OK = 0,
    SFM_ERR_ARG = -1,     /* bad argument (shape, null pointer, range)   */
    SFM_ERR_HIP = -2,     /* HIP runtime error                           */
    SFM_ERR_NOMEM = -3,   /* device allocation failed                    */
    SFM_ERR_SOLVE = -4,   /* reduced camera system not positive definite */
    SFM_ERR_COMM = -5     /* RCCL error                                  */
};

int sfm_version(void);
/* last error message of the calling thread ("" if none) */
const char *sfm_last_error(void);
int sfm_device_count(void);
/* per-call phase timings of the calling thread's last call (ms):
 * [0] host->device upload, [1] kernels, [2] device->host download,
 * [3] kernel-only time of the dominant kernel.  Returns the count written. */
int sfm_last_timings(double *out, int n);
/* device-side timings (HIP events) in the in-call-sampling and shard RANSAC
 * calls; off by default (host sampling time is always reported) */
int sfm_set_call_timing(int on);

/* ---------------------------------------------------------------------
 * Python `random` replay (host code, no GPU).
 * Replaces the n_max calls of random.sample(range(n), k) made by
 * GetInliersRANSAC.py:55 on the *global* MT19937 instance.  `mt_state`
 * is random.getstate()[1] (624 words + position) and is advanced in place
 * exactly as CPython 3.10 would (random.py:_randbelow_with_getrandbits and
 * sample()'s pool / set branches), so random.setstate() afterwards leaves
 * the global stream where the reference leaves it.  out: H x k int32.
 * ------------------------------------------------------------------- */
int sfm_pyrandom_sample_table(uint32_t *mt_state /* 625 in/out */, int64_t n, int32_t k,
                              int64_t H, int32_t *out);

/* ---------------------------------------------------------------------
 * EstimateFundamentalMatrix (EstimateFundamentalMatrix.py:3-83)
 * ------------------------------------------------------------------- */
/* H independent 8-point estimates: x1s, x2s are H x 8 x 2; F is H x 9. */
int sfm_f8_batch(const double *x1s, const double *x2s, int64_t H, double *F, int device);
/* one estimate from N >= 8 correspondences (least-squares null vector). */
int sfm_f8_general(const double *x1, const double *x2, int64_t N, double *F, int device);

/* ---------------------------------------------------------------------
 * GetInliersRANSAC (GetInliersRANSAC.py:5-106)
 * x1, x2: N x 2; samples: H x 8 indices (host-drawn, see above).
 * counts_out (H, nullable): inliers per hypothesis.  *best_iter: first
 * hypothesis with the strictly largest positive count, or -1 if every
 * count is 0 (the reference's "F_best is None").  F_best (9) and
 * best_mask (N, 1 = inlier) are written only when *best_iter >= 0.
 * ------------------------------------------------------------------- */
int sfm_ransac_f8(const double *x1, const double *x2, int64_t N, const int32_t *samples, int64_t H,
                  double thr, int32_t *counts_out, int64_t *best_iter, double *F_best,
                  uint8_t *best_mask, int device);
/* The same call with the H x 8 samples drawn inside it from the CPython
 * random state st[625] (random.getstate()[1]: 624 MT19937 words + position;
 * advanced in place exactly as H calls of random.sample(range(N), 8) would
 * advance it).  The draw is replayed on the host in chunks and each chunk's
 * upload / fit / score is enqueued as soon as it is drawn, so the GPU works
 * while the host draws.  samples_out (H x 8, nullable) receives the table. */
int sfm_ransac_f8_pyrandom(const double *x1, const double *x2, int64_t N, uint32_t *st, int64_t H,
                           double thr, int32_t *counts_out, int64_t *best_iter, double *F_best,
                           uint8_t *best_mask, int32_t *samples_out, int device);
/* GetInliersRANSAC's whole call (GetInliersRANSAC.py:53-106) as the drop-in
 * needs it: sfm_ransac_f8_pyrandom with the winner's inlier positions
 * (ascending) in split[0, *n_inliers) and the outliers' positions in
 * split[*n_inliers, N) (split: N entries) in place of the mask;
 * *n_inliers = 0 when *best_iter is -1. */
int sfm_ransac_f8_dropin(const double *x1, const double *x2, int64_t N, uint32_t *st, int64_t H, double thr,
                         int64_t *best_iter, double *F_best, int64_t *split, int64_t *n_inliers, int device);

/* ---------------------------------------------------------------------
 * Homography (GetHomographyInliers.py)
 * sfm_h4_batch: find_homography (:4-85) on H independent 4-point samples
 *   (x1s, x2s: H x 4 x 2) -> Hout (H x 9), each normalised by H[2,2].
 * sfm_homography_general: find_homography on N >= 4 points -> Hout (9).
 * sfm_ransac_h4: get_homography_inliers' loop (:124-157) over a host-drawn
 *   H x 4 sample table: per hypothesis the transfer error
 *   |H x1 / (t2 + 1e-8) - x2| < thr is counted; the winner is the first
 *   hypothesis with the strictly largest positive count (-1 if none);
 *   H_best (9) and best_mask (N) are written when *best_iter >= 0.
 * ------------------------------------------------------------------- */
int sfm_h4_batch(const double *x1s, const double *x2s, int64_t H, double *Hout, int device);
int sfm_homography_general(const double *x1, const double *x2, int64_t N, double *Hout, int device);
int sfm_ransac_h4(const double *x1, const double *x2, int64_t N, const int32_t *samples, int64_t H,
                  double thr, int32_t *counts_out, int64_t *best_iter, double *H_best,
                  uint8_t *best_mask, int device);
/* sfm_ransac_h4 with in-call sampling (H x 4), as sfm_ransac_f8_pyrandom. */
int sfm_ransac_h4_pyrandom(const double *x1, const double *x2, int64_t N, uint32_t *st, int64_t H,
                           double thr, int32_t *counts_out, int64_t *best_iter, double *H_best,
                           uint8_t *best_mask, int32_t *samples_out, int device);

/* ---------------------------------------------------------------------
 * PnP (LinearPnP.py, PnPRANSAC.py, NonlinearPnP.py); K is 3x3 row-major.
 * sfm_linear_pnp: LinearPnP on N >= 4 points (X: N x 3, x: N x 2) ->
 *   C (3), R (9); *branch (nullable) = 1 where R's final orthogonalisation
 *   is the LAPACK-noise-defined case (det(R) < 0).
 * sfm_pnp_ransac: PnPRANSAC's loop (:48-80) over a host-drawn H x 4 sample
 *   table: LinearPnP per hypothesis, reprojection error < thr counted;
 *   *best_iter = first strict maximum (-1 if every count is 0) and
 *   *best_count its count -- the caller applies the reference's fallback
 *   (:82-87, LinearPnP on all points when best_count < 4).
 * sfm_nonlinear_pnp: NonlinearPnP (:47-123), scipy 'lm' semantics with
 *   max_nfev on the 2N-residual loss (:5-44); info: MINPACK info, 0 for the
 *   N < 4 early return, -1 where the reference's except keeps (C0, R0); a
 *   non-negative info carries the CholeskyQR flags in bits 8-9 (1: the
 *   Jacobian's Gram factor needed a shift and a third pass ran; 2: a later
 *   Gram factor failed) -- info & 0xff is MINPACK's code.
 * ------------------------------------------------------------------- */
int sfm_linear_pnp(const double *X, const double *x, int64_t N, const double *K, double *C_out,
                   double *R_out, int32_t *branch, int device);
int sfm_pnp_ransac(const double *X, const double *x, int64_t N, const double *K, const int32_t *samples,
                   int64_t H, double thr, int32_t *counts_out, int32_t *branch_out, int64_t *best_iter,
                   int64_t *best_count, double *C_best, double *R_best, int device);
int sfm_nonlinear_pnp(const double *X, const double *x, int64_t N, const double *K, const double *C0,
                      const double *R0, int32_t max_nfev, double *C_out, double *R_out, int32_t *info,
                      int device);

/* ---------------------------------------------------------------------
 * Matching files (Utils.py:8-64 get_data) -> COO observation store.
 * sfm_matching_parse: reads data_path/matching1..(no_of_images-1).txt with
 *   get_data's semantics (header skipped; primary x, y as floats; match
 *   coordinates int()-truncated; last write per image wins) using
 *   n_threads host threads (0 = up to 16); returns an opaque store with
 *   n_features rows and n_obs observations (feature-major, image ascending).
 * sfm_matching_read: copies the COO arrays (feature, image 0-based, x, y).
 * ------------------------------------------------------------------- */
int sfm_matching_parse(const char *data_path, int32_t no_of_images, int32_t n_threads, void **handle,
                       int64_t *n_features, int64_t *n_obs);
int sfm_matching_read(void *handle, int32_t *feature, int32_t *image, double *x, double *y);
int sfm_matching_free(void *handle);

/* ---------------------------------------------------------------------
 * Dense visibility -> COO observations (BundleAdjustment.py:164-169, the
 * drop-in's np.where over filtered_feature_flags[valid_point_indices]
 * [:, :n_cameras] == 1 and the feature_x / feature_y gathers at the hits).
 * sfm_dense_obs_scan: rows[i] (i < n_rows) are the valid feature rows, each
 *   in [0, n_matrix_rows) (SFM_ERR_ARG otherwise: the matrices' row count,
 *   where the reference's indexing raises IndexError); a row r of the flag matrix starts at flags + r * flag_row_bytes (dtype
 *   0 f64, 1 f32, 2 i64, 3 i32, 4 u8/bool; "== 1" in that dtype), of the
 *   coordinate matrices at fx / fy + r * xy_row_bytes (f64); n_threads
 *   row jobs on the library's host threads (0 = its default).  Returns a
 *   store of n_obs observations in np.where's order (point-major, camera
 *   ascending), kept by the library for the next scan once freed.
 * sfm_dense_obs_read: copies (camera, point i, (x, y)).
 * sfm_ba_lm_dense (below) solves from the store without these copies.
 * ------------------------------------------------------------------- */
int sfm_dense_obs_scan(const void *flags, int32_t dtype, int64_t flag_row_bytes, int64_t n_matrix_rows,
                       const int64_t *rows, int64_t n_rows, int32_t n_cams, const double *fx, const double *fy,
                       int64_t xy_row_bytes, int32_t n_threads, void **handle, int64_t *n_obs);
int sfm_dense_obs_read(void *handle, int32_t *cam, int32_t *pt, double *obs);
int sfm_dense_obs_free(void *handle);
/* perform_bundle_adjustment's x0 points (BundleAdjustment.py:196-197):
 * dst[i] = src[rows[i]] for 3-double rows (rows NULL: src[i]), on the host
 * thread pool; SFM_ERR_ARG for a row outside [0, src_rows). */
int sfm_gather_rows3(const double *src, int64_t src_rows, const int64_t *rows, int64_t n, double *dst);
/* The camera parameter conversions around the solve (BundleAdjustment.py:
 * 183-193 and 220-228), scipy's Rotation with its bits (csrc/rotations.cpp):
 * sfm_matrix_to_rotvec = from_matrix(R).as_rotvec() for n row-major 3 x 3
 * matrices, returning how many are not orthogonal to within 1e-13 (scipy
 * orthogonalises those first: nothing is written for them, the caller
 * converts the batch with scipy), -1 for a null pointer / negative n;
 * sfm_rotvec_to_matrix = from_rotvec(w).as_matrix(). */
int64_t sfm_matrix_to_rotvec(const double *R, int64_t n, double *w);
int sfm_rotvec_to_matrix(const double *w, int64_t n, double *R);

/* ---------------------------------------------------------------------
 * LinearTriangulation (LinearTriangulation.py:3-92)
 * P1, P2: 3 x 4 projection matrices K[R | -RC]; x1, x2: N x 2; X: N x 3.
 * ------------------------------------------------------------------- */
int sfm_triangulate_dlt(const double *P1, const double *P2, const double *x1, const double *x2,
                        int64_t N, double *X, int device);

/* ---------------------------------------------------------------------
 * NonLinearTriangulation (NonLinearTriangulation.py:53-121): per point,
 * scipy least_squares(method='lm', max_nfev) of the 4-residual Loss
 * (:5-50) from X0[i]; MINPACK lmdif semantics (diag = ones, factor 100,
 * forward differences, ftol = xtol = gtol = 1e-8).  Rows where the
 * reference's try/except keeps X0 (x0 with a NaN, non-finite residuals at
 * x0) are copied through.  info (N, nullable): MINPACK info 1..8, or -1
 * for a copied-through row.
 * ------------------------------------------------------------------- */
int sfm_triangulate_nonlinear(const double *P1, const double *P2, const double *x1, const double *x2,
                              const double *X0, int64_t N, int32_t max_nfev, double *X, int32_t *info,
                              int device);

/* ---------------------------------------------------------------------
 * BundleAdjustment (BundleAdjustment.py:8-242)
 * Camera parameters are the reference's: [rotvec(3), t(3)] with
 * x_cam = R(rotvec) X + t, proj = K x_cam [:2] / (K x_cam [2] + 1e-8),
 * residual r = obs - proj (BundleAdjustment.py:73-110).
 * ------------------------------------------------------------------- */
/* project_points (BundleAdjustment.py:8-40) for one camera P = K[R|-RC]:
 * P is 3 x 4, X is M x 3, out M x 2. */
int sfm_project_points(const double *P, const double *X, int64_t M, double *out, int device);
/* bundle_adjustment_residuals: r (2 * n_obs), interleaved [rx0, ry0, ...]. */
int sfm_ba_residuals(int32_t n_cams, int64_t n_pts, int64_t n_obs, const int32_t *cam_idx,
                     const int32_t *pt_idx, const double *obs, const double *K,
                     const double *cam_params, const double *points, double *r, int device);

typedef struct {
    int32_t max_iterations;      /* LM iterations (damped solve + trial)        */
    int32_t fixed_iterations;    /* 1: run exactly max_iterations (benchmark)   */
    double function_tolerance;   /* stop: accepted step with dcost < ftol*cost  */
    double gradient_tolerance;   /* stop after a linearisation when max |J^T r| < gtol
                                    (status 2; 0 = off; < 0 is SFM_ERR_ARG)      */
    double parameter_tolerance;  /* stop: |dx| < xtol (|x| + xtol)               */
    double initial_lambda;       /* Marquardt damping on clamp(diag(J^T J))      */
} sfm_ba_opts;

typedef struct {
    int32_t iterations;  /* LM iterations performed                             */
    int32_t accepted;    /* accepted steps (re-linearisations)                  */
    int32_t status;      /* 1 ftol, 2 gtol, 3 xtol, 4 max_iterations, 5 lambda,
                            6 cost at x0 not finite (no step taken)             */
    int32_t n_ranks;
    double cost0, cost;  /* 0.5 sum r^2 before / after                          */
    double t_setup_ms;   /* host prep + uploads                                 */
    double t_loop_ms;    /* LM loop wall time                                   */
    double t_download_ms;
    double lambda;
} sfm_ba_report;

/* Observations must be point-major (sorted by pt_idx, as the reference
 * assembles them: BundleAdjustment.py:164-169).  cam_params (n_cams x 6)
 * and points (n_pts x 3) are updated in place. */
int sfm_ba_lm(int32_t n_cams, int64_t n_pts, int64_t n_obs, const int32_t *cam_idx,
              const int32_t *pt_idx, const double *obs, const double *K, double *cam_params,
              double *points, const sfm_ba_opts *opts, sfm_ba_report *report, int device);

/* sfm_ba_lm with the observations of a dense scan (sfm_dense_obs_scan's
 * handle, not freed here; its rows are the n_pts points, its cameras at
 * most n_cams): perform_bundle_adjustment's whole path
 * (BundleAdjustment.py:156-242) from the dense matrices, the observations
 * copied from the scan straight into the pinned upload buffer. */
int sfm_ba_lm_dense(void *obs_handle, int32_t n_cams, int64_t n_pts, const double *K, double *cam_params,
                    double *points, const sfm_ba_opts *opts, sfm_ba_report *report, int device);

/* ---- device-resident BA session (bench / multi-GPU) -------------------
 * A problem is uploaded once and iterated many times.  With a communicator
 * each rank holds a disjoint subset of the points (and all of their
 * observations) and every camera; one RCCL all-reduce (sum, fp64) of the
 * partial reduced camera system per LM iteration + one of the trial cost. */
typedef struct sfm_comm sfm_comm;
typedef struct sfm_ba_problem sfm_ba_problem;

int sfm_comm_unique_id(char out[128]);
int sfm_comm_init(const char id[128], int nranks, int rank, int device, sfm_comm **out);
/* in-process group of nranks communicators (one host thread per rank, any
 * devices, the same device allowed): out receives nranks handles */
int sfm_comm_init_local(int nranks, sfm_comm **out);
int sfm_comm_destroy(sfm_comm *comm);

/* ---- hypothesis-sharded RANSAC: the loop of
 * GetInliersRANSAC.py:53-92 (and GetHomographyInliers.py:124-156) split into
 * contiguous hypothesis ranges [h0, h1), one per rank.
 * Shard key = (count << 32) | (0xFFFFFFFF - iteration), 0 when no hypothesis
 * of the shard has an inlier: the max over ranks is the reference's winner
 * (max count, earliest iteration: the strict '>' update at :85-88).
 * _pyrandom_range draws ALL H rows from the CPython MT19937 state st[625]
 * (in/out) in the reference's order, so st ends where the unsharded call
 * leaves it, and fits/scores only [h0, h1).  counts_out: h1 - h0 entries
 * (nullable).  F_best/H_best: the shard winner's model (untouched when the
 * key is 0).  Requires H < 2^32. */
int sfm_ransac_f8_range(const double *x1, const double *x2, int64_t N, const int32_t *samples /* H x 8 */,
                        int64_t H, int64_t h0, int64_t h1, double thr, int32_t *counts_out,
                        uint64_t *best_key, double *F_best, int device);
int sfm_ransac_f8_pyrandom_range(const double *x1, const double *x2, int64_t N, uint32_t *st, int64_t H,
                                 int64_t h0, int64_t h1, double thr, int32_t *counts_out,
                                 uint64_t *best_key, double *F_best, int device);
int sfm_ransac_h4_pyrandom_range(const double *x1, const double *x2, int64_t N, uint32_t *st, int64_t H,
                                 int64_t h0, int64_t h1, double thr, int32_t *counts_out,
                                 uint64_t *best_key, double *H_best, int device);
/* max of the ranks' keys (in/out) and the winner's model (in/out, 9) over
 * comm: RCCL all-reduce(max, u64) then a sum in which only the winner
 * contributes; or the in-process group.  Every rank returns the same. */
int sfm_ransac_combine(sfm_comm *comm, uint64_t *key, double *model);
/* inlier mask of one model (GetInliersRANSAC.py:67-81 /
 * GetHomographyInliers.py:135-146): the winner's emit after the combine */
int sfm_ransac_f8_mask(const double *x1, const double *x2, int64_t N, const double *F, double thr,
                       uint8_t *mask, int device);
int sfm_ransac_h4_mask(const double *x1, const double *x2, int64_t N, const double *Hm, double thr,
                       uint8_t *mask, int device);

int sfm_ba_create(int32_t n_cams, int64_t n_pts, int64_t n_obs, const int32_t *cam_idx,
                  const int32_t *pt_idx, const double *obs, const double *K,
                  const double *cam_params, const double *points, int device, sfm_comm *comm,
                  sfm_ba_problem **out);
int sfm_ba_solve(sfm_ba_problem *p, const sfm_ba_opts *opts, sfm_ba_report *report);
/* digest of the Schur sweep plan built at create (set only when the
 * environment has SFM_PLAN_DIGEST=1, else 0): the device planner and the
 * host planner (SFM_PLAN_HOST=1) must produce the same plan */
int sfm_ba_plan_digest(sfm_ba_problem *p, uint64_t *out);
/* reset the device state to the initial parameters given at create time */
int sfm_ba_reset(sfm_ba_problem *p);
int sfm_ba_download(sfm_ba_problem *p, double *cam_params, double *points);
/* per-phase HIP events in the following solves (off by default: each event
 * record costs the stream a few microseconds) */
int sfm_ba_set_timing(sfm_ba_problem *p, int on);
/* average device time per LM iteration of each kernel family over the
 * last solve with timing on (ms; zeros otherwise): names are written
 * ';'-separated into `names`. */
int sfm_ba_kernel_times(sfm_ba_problem *p, double *ms, int n, char *names, int names_len);
/* Diagnostic: x = S^-1 rhs for an SPD n x n S (row-major) with the reduced
 * camera system solver of sfm_ba_solve (the scipy 'lm' reference solves the
 * same normal equations inside least_squares, BundleAdjustment.py:205-213).
 * SFM_ERR_SOLVE if a pivot is not positive. */
int sfm_reduced_solve(const double *S, const double *rhs, int32_t n, double *x, int device);
int sfm_ba_destroy(sfm_ba_problem *p);

/* single-process multi-GPU BA: points split over `devices` (n_ranks
 * entries; repeats allowed), one host thread per rank, reduced camera
 * system summed every LM iteration.  Same arguments as sfm_ba_lm. */
int sfm_ba_lm_multi(int32_t n_cams, int64_t n_pts, int64_t n_obs, const int32_t *cam_idx,
                    const int32_t *pt_idx, const double *obs, const double *K, double *cam_params,
                    double *points, const sfm_ba_opts *opts, sfm_ba_report *report, const int *devices,
                    int n_ranks);

#ifdef __cplusplus
}
#endif
#endif /* SFMCORE_H */
