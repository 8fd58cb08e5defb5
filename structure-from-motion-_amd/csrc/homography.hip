// Homography RANSAC (GetHomographyInliers.py:4-165)
// on the RANSAC engine: 4-point DLT per hypothesis (one thread), transfer
// error sweep (one wave per hypothesis), strict-max select + winner mask.
#include "dlt_general.hpp"
#include "ransac_engine.hpp"

using namespace sfm;

extern "C" int sfm_h4_batch(const double *x1s, const double *x2s, int64_t H, double *Hout, int device) {
    SFM_CHECK_ARG(H >= 0, "H < 0");
    if (H == 0) return 0;
    SFM_CHECK_ARG(x1s && x2s && Hout, "null pointer");
    ThreadCtx *c = thread_ctx(device);
    if (!c) return SFM_ERR_HIP;
    const size_t pb = (size_t)H * HomModel::K * sizeof(double2);
    int rc;
    if ((rc = c->buf[0].reserve(pb)) || (rc = c->buf[1].reserve(pb)) ||
        (rc = c->buf[2].reserve((size_t)H * 9 * sizeof(double))))
        return rc;
    SFM_HIP(hipMemcpyAsync(c->buf[0].p, x1s, pb, hipMemcpyHostToDevice, c->stream));
    SFM_HIP(hipMemcpyAsync(c->buf[1].p, x2s, pb, hipMemcpyHostToDevice, c->stream));
    hipLaunchKernelGGL(k_fit_points<HomModel>, dim3(ceil_div(H, 256)), dim3(256), 0, c->stream,
                       c->buf[0].as<double2>(), c->buf[1].as<double2>(), H, c->buf[2].as<double>());
    SFM_HIP(hipGetLastError());
    SFM_HIP(hipMemcpyAsync(Hout, c->buf[2].p, (size_t)H * 9 * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    SFM_HIP(hipStreamSynchronize(c->stream));
    return 0;
}

extern "C" int sfm_homography_general(const double *x1, const double *x2, int64_t N, double *Hout, int device) {
    SFM_CHECK_ARG(N >= 4, "need N >= 4 correspondences");
    SFM_CHECK_ARG(x1 && x2 && Hout, "null pointer");
    ThreadCtx *c = thread_ctx(device);
    if (!c) return SFM_ERR_HIP;
    const size_t pb = (size_t)N * sizeof(double2);
    int rc;
    if ((rc = c->buf[0].reserve(pb)) || (rc = c->buf[1].reserve(pb)) || (rc = c->buf[2].reserve(9 * sizeof(double))))
        return rc;
    SFM_HIP(hipMemcpyAsync(c->buf[0].p, x1, pb, hipMemcpyHostToDevice, c->stream));
    SFM_HIP(hipMemcpyAsync(c->buf[1].p, x2, pb, hipMemcpyHostToDevice, c->stream));
    hipLaunchKernelGGL(k_dlt_general<HDesign>, dim3(1), dim3(FG_THREADS), 0, c->stream, c->buf[0].as<double2>(),
                       c->buf[1].as<double2>(), N, c->buf[2].as<double>());
    SFM_HIP(hipGetLastError());
    SFM_HIP(hipMemcpyAsync(Hout, c->buf[2].p, 9 * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    SFM_HIP(hipStreamSynchronize(c->stream));
    return 0;
}

extern "C" int sfm_ransac_h4(const double *x1, const double *x2, int64_t N, const int32_t *samples, int64_t H,
                             double thr, int32_t *counts_out, int64_t *best_iter, double *H_best, uint8_t *best_mask,
                             int device) {
    return ransac_run<HomModel>(x1, x2, N, samples, H, thr, counts_out, best_iter, H_best, best_mask, device);
}

// sfm_ransac_h4 with the samples drawn inside the call from the CPython
// random state st[625] (in/out), pipelined with the GPU work.
extern "C" int sfm_ransac_h4_pyrandom(const double *x1, const double *x2, int64_t N, uint32_t *st, int64_t H,
                                      double thr, int32_t *counts_out, int64_t *best_iter, double *H_best,
                                      uint8_t *best_mask, int32_t *samples_out, int device) {
    return ransac_run_pysample<HomModel>(x1, x2, N, st, H, thr, counts_out, best_iter, H_best, best_mask,
                                         samples_out, device);
}

// Hypothesis shard [h0, h1) of the homography RANSAC (as sfm_ransac_f8_range).
extern "C" int sfm_ransac_h4_pyrandom_range(const double *x1, const double *x2, int64_t N, uint32_t *st, int64_t H,
                                            int64_t h0, int64_t h1, double thr, int32_t *counts_out,
                                            uint64_t *best_key, double *H_best, int device) {
    SFM_CHECK_ARG(st, "null MT19937 state");
    return ransac_run_range<HomModel>(x1, x2, N, nullptr, st, H, h0, h1, thr, counts_out, best_key, H_best, device);
}

extern "C" int sfm_ransac_h4_mask(const double *x1, const double *x2, int64_t N, const double *Hm, double thr,
                                  uint8_t *mask, int device) {
    return ransac_mask_run<HomModel>(x1, x2, N, Hm, thr, mask, device);
}
