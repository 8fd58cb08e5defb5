// Non-linear triangulation: the reference refines
// every linearly-triangulated point with its own scipy least_squares
// (method='lm', max_nfev=50) on a 4-residual reprojection loss
// (Phase 1/NonLinearTriangulation.py:5-50 Loss, :53-121 the per-point loop).
// Here one thread owns one point and runs the same MINPACK lmdif
// (lm_small.hpp) in registers; points are independent, so the launch is a
// flat grid over N.  Work per point is ~O(100) residual evaluations of 60
// flops; the kernel is FP64-VALU / latency bound, its HBM traffic (56 B in,
// 28 B out per point) is negligible.
#include <cstring>

#include "lm_small.hpp"
#include "sfm_common.hpp"

#pragma clang fp contract(off)

namespace sfm {

struct NlTriCams {
    double p[24];  // P1 (3x4 row-major) | P2
};

struct NlTriLoss {
    const double *P1, *P2;
    double u1, v1, u2, v2;
    // Loss (NonLinearTriangulation.py:5-50).  numpy's 3x4 @ 4 mat-vec sums
    // pairwise, (p0 x0 + p2 x2) + (p1 x1 + p3 * 1); a view whose depth is
    // below 1e-8 in magnitude falls back to the observation (residual 0).
    __device__ __forceinline__ void view(const double *P, const double (&X)[3], double u, double v, double &fu,
                                         double &fv) const {
        const double h0 = (P[0] * X[0] + P[2] * X[2]) + (P[1] * X[1] + P[3]);
        const double h1 = (P[4] * X[0] + P[6] * X[2]) + (P[5] * X[1] + P[7]);
        const double h2 = (P[8] * X[0] + P[10] * X[2]) + (P[9] * X[1] + P[11]);
        double px = u, py = v;
        if (!(fabs(h2) < 1e-8)) {
            px = h0 / h2;
            py = h1 / h2;
        }
        fu = u - px;
        fv = v - py;
    }
    __device__ __forceinline__ void operator()(const double (&X)[3], double (&f)[4]) const {
        view(P1, X, u1, v1, f[0], f[1]);
        view(P2, X, u2, v2, f[2], f[3]);
    }
};

// info[i]: MINPACK info (1..8), or -1 where the reference's try/except keeps
// x0 (x0 has a NaN -> scipy's bounds check raises; residuals at x0 are not
// finite -> "Residuals are not finite in the initial point").
__global__ void __launch_bounds__(256) k_nltri(NlTriCams cams, const double2 *__restrict__ x1,
                                               const double2 *__restrict__ x2, const double *__restrict__ X0,
                                               int64_t n, int32_t max_nfev, double *__restrict__ X,
                                               int32_t *__restrict__ info_out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double2 a = x1[i], b = x2[i];
    NlTriLoss loss{cams.p, cams.p + 12, a.x, a.y, b.x, b.y};
    double x[3] = {X0[3 * i], X0[3 * i + 1], X0[3 * i + 2]};
    bool ok = !(isnan(x[0]) || isnan(x[1]) || isnan(x[2]));
    if (ok) {
        double f0[4];
        loss(x, f0);
#pragma unroll
        for (int k = 0; k < 4; ++k) ok = ok && isfinite(f0[k]);
    }
    int info = -1;
    if (ok) info = lm::lmdif<4, 3>(loss, x, 1e-8, 1e-8, 1e-8, max_nfev);
    X[3 * i] = x[0];
    X[3 * i + 1] = x[1];
    X[3 * i + 2] = x[2];
    if (info_out) info_out[i] = info;
}

}  // namespace sfm

using namespace sfm;

extern "C" int sfm_triangulate_nonlinear(const double *P1, const double *P2, const double *x1, const double *x2,
                                         const double *X0, int64_t N, int32_t max_nfev, double *X, int32_t *info,
                                         int device) {
    SFM_CHECK_ARG(N >= 0, "N < 0");
    SFM_CHECK_ARG(max_nfev > 0, "max_nfev must be positive");
    if (N == 0) return 0;
    SFM_CHECK_ARG(P1 && P2 && x1 && x2 && X0 && X, "null pointer");
    ThreadCtx *c = thread_ctx(device);
    if (!c) return SFM_ERR_HIP;
    const size_t pb = (size_t)N * sizeof(double2), xb = (size_t)N * 3 * sizeof(double);
    int rc;
    if ((rc = c->buf[0].reserve(pb)) || (rc = c->buf[1].reserve(pb)) || (rc = c->buf[2].reserve(xb)) ||
        (rc = c->buf[3].reserve(xb)) || (rc = c->buf[4].reserve((size_t)N * sizeof(int32_t))))
        return rc;
    NlTriCams cams;
    std::memcpy(cams.p, P1, 12 * sizeof(double));
    std::memcpy(cams.p + 12, P2, 12 * sizeof(double));
    hipStream_t s = c->stream;
    const bool tm = call_timing();  // HIP events only when asked (each costs the stream us)
    if (tm) SFM_HIP(hipEventRecord(c->ev[0], s));
    SFM_HIP(hipMemcpyAsync(c->buf[0].p, x1, pb, hipMemcpyHostToDevice, s));
    SFM_HIP(hipMemcpyAsync(c->buf[1].p, x2, pb, hipMemcpyHostToDevice, s));
    SFM_HIP(hipMemcpyAsync(c->buf[2].p, X0, xb, hipMemcpyHostToDevice, s));
    if (tm) SFM_HIP(hipEventRecord(c->ev[1], s));
    hipLaunchKernelGGL(k_nltri, dim3(ceil_div(N, 256)), dim3(256), 0, s, cams, c->buf[0].as<double2>(),
                       c->buf[1].as<double2>(), c->buf[2].as<double>(), N, max_nfev, c->buf[3].as<double>(),
                       c->buf[4].as<int32_t>());
    SFM_HIP(hipGetLastError());
    if (tm) SFM_HIP(hipEventRecord(c->ev[2], s));
    SFM_HIP(hipMemcpyAsync(X, c->buf[3].p, xb, hipMemcpyDeviceToHost, s));
    if (info) SFM_HIP(hipMemcpyAsync(info, c->buf[4].p, (size_t)N * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    if (tm) SFM_HIP(hipEventRecord(c->ev[3], s));
    SFM_HIP(hipStreamSynchronize(s));
    float a = 0, b = 0, d = 0;
    if (tm) (void)hipEventElapsedTime(&a, c->ev[0], c->ev[1]);
    if (tm) (void)hipEventElapsedTime(&b, c->ev[1], c->ev[2]);
    if (tm) (void)hipEventElapsedTime(&d, c->ev[2], c->ev[3]);
    const double t[4] = {a, b, d, b};
    set_timings(t, 4);
    return 0;
}
