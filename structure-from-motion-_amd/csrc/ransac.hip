// Fundamental-matrix RANSAC entry points (GetInliersRANSAC.py:5-106,
// EstimateFundamentalMatrix.py:3-83) on the engine in ransac_engine.hpp.
#include "ransac_engine.hpp"

using namespace sfm;

extern "C" int sfm_f8_batch(const double *x1s, const double *x2s, int64_t H, double *F, int device) {
    SFM_CHECK_ARG(H >= 0, "H < 0");
    if (H == 0) return 0;
    SFM_CHECK_ARG(x1s && x2s && F, "null pointer");
    ThreadCtx *c = thread_ctx(device);
    if (!c) return SFM_ERR_HIP;
    const size_t pb = (size_t)H * 8 * sizeof(double2);
    int rc;
    if ((rc = c->buf[0].reserve(pb)) || (rc = c->buf[1].reserve(pb)) ||
        (rc = c->buf[2].reserve((size_t)H * 9 * sizeof(double))))
        return rc;
    SFM_HIP(hipMemcpyAsync(c->buf[0].p, x1s, pb, hipMemcpyHostToDevice, c->stream));
    SFM_HIP(hipMemcpyAsync(c->buf[1].p, x2s, pb, hipMemcpyHostToDevice, c->stream));
    hipLaunchKernelGGL(k_fit_points<EpiModel>, dim3(ceil_div(H, 256)), dim3(256), 0, c->stream, c->buf[0].as<double2>(),
                       c->buf[1].as<double2>(), H, c->buf[2].as<double>());
    SFM_HIP(hipGetLastError());
    SFM_HIP(hipMemcpyAsync(F, c->buf[2].p, (size_t)H * 9 * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    SFM_HIP(hipStreamSynchronize(c->stream));
    return 0;
}

extern "C" int sfm_ransac_f8(const double *x1, const double *x2, int64_t N, const int32_t *samples, int64_t H,
                             double thr, int32_t *counts_out, int64_t *best_iter, double *F_best,
                             uint8_t *best_mask, int device) {
    return ransac_run<EpiModel>(x1, x2, N, samples, H, thr, counts_out, best_iter, F_best, best_mask, device);
}

// sfm_ransac_f8 with the samples drawn inside the call from the CPython
// random state st[625] (in/out), pipelined with the GPU work.
extern "C" int sfm_ransac_f8_pyrandom(const double *x1, const double *x2, int64_t N, uint32_t *st, int64_t H,
                                      double thr, int32_t *counts_out, int64_t *best_iter, double *F_best,
                                      uint8_t *best_mask, int32_t *samples_out, int device) {
    return ransac_run_pysample<EpiModel>(x1, x2, N, st, H, thr, counts_out, best_iter, F_best, best_mask,
                                         samples_out, device);
}

// The drop-in's form of sfm_ransac_f8_pyrandom: the winner's inlier
// positions (ascending) in split[0, n_inliers) and the outliers' in
// split[n_inliers, N) instead of a mask -- GetInliersRANSAC.py:95-106's
// np.where(inlier_mask)[0] and index[~inlier_mask] without a pass over the
// mask in numpy.  n_inliers = 0 when no hypothesis wins (split untouched).
extern "C" int sfm_ransac_f8_dropin(const double *x1, const double *x2, int64_t N, uint32_t *st, int64_t H,
                                    double thr, int64_t *best_iter, double *F_best, int64_t *split,
                                    int64_t *n_inliers, int device) {
    SFM_CHECK_ARG(split && n_inliers, "null pointer");
    return ransac_run_pysample<EpiModel>(x1, x2, N, st, H, thr, nullptr, best_iter, F_best, nullptr, nullptr,
                                         device, split, n_inliers);
}

// One hypothesis shard [h0, h1) of sfm_ransac_f8 / sfm_ransac_f8_pyrandom
// (SURVEY §8(e)): the shard's key (count << 32 | 0xFFFFFFFF - iteration,
// 0 = none) and model.  Ranks combine keys with max (sfm_ransac_combine);
// the winner's model gives the mask (sfm_ransac_f8_mask).  The _pyrandom
// form draws all H rows from st, so every rank's stream ends where the
// unsharded call leaves it.
extern "C" int sfm_ransac_f8_range(const double *x1, const double *x2, int64_t N, const int32_t *samples, int64_t H,
                                   int64_t h0, int64_t h1, double thr, int32_t *counts_out, uint64_t *best_key,
                                   double *F_best, int device) {
    return ransac_run_range<EpiModel>(x1, x2, N, samples, nullptr, H, h0, h1, thr, counts_out, best_key, F_best,
                                      device);
}

extern "C" int sfm_ransac_f8_pyrandom_range(const double *x1, const double *x2, int64_t N, uint32_t *st, int64_t H,
                                            int64_t h0, int64_t h1, double thr, int32_t *counts_out,
                                            uint64_t *best_key, double *F_best, int device) {
    SFM_CHECK_ARG(st, "null MT19937 state");
    return ransac_run_range<EpiModel>(x1, x2, N, nullptr, st, H, h0, h1, thr, counts_out, best_key, F_best, device);
}

extern "C" int sfm_ransac_f8_mask(const double *x1, const double *x2, int64_t N, const double *F, double thr,
                                  uint8_t *mask, int device) {
    return ransac_mask_run<EpiModel>(x1, x2, N, F, thr, mask, device);
}
