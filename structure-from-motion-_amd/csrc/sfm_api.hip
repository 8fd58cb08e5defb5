// libsfmcore: C-ABI plumbing + the small entry points
// (EstimateFundamentalMatrix general-N, LinearTriangulation, project_points,
// bundle_adjustment_residuals) and the host-side CPython random replay.
#include <atomic>
#include <cmath>
#include <cstring>
#include <memory>
#include <unordered_map>

#include "sfm_common.hpp"
#include "sfm_geom.hpp"
#include "dlt_general.hpp"
#include "pyrandom.hpp"

namespace sfm {

static thread_local std::string g_err;
static thread_local double g_timings[12];
static thread_local int g_ntimings = 0;

void set_error(const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
}
void clear_error() { g_err.clear(); }
static std::atomic<int> g_call_timing{0};
bool call_timing() { return g_call_timing.load(std::memory_order_relaxed) != 0; }
void set_timings(const double *t, int n) {
    g_ntimings = n < 12 ? n : 12;
    for (int i = 0; i < g_ntimings; ++i) g_timings[i] = t[i];
}

ThreadCtx *thread_ctx(int device) {
    static thread_local std::unordered_map<int, std::unique_ptr<ThreadCtx>> ctxs;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        set_error("no HIP device visible (hipGetDeviceCount=%d)", ndev);
        return nullptr;
    }
    if (device < 0 || device >= ndev) {
        set_error("device %d out of range (%d devices)", device, ndev);
        return nullptr;
    }
    if (hipSetDevice(device) != hipSuccess) {
        set_error("hipSetDevice(%d) failed", device);
        return nullptr;
    }
    (void)hipGetLastError();  // launches are checked with hipGetLastError: start clean
    auto &slot = ctxs[device];
    if (!slot) {
        auto c = std::make_unique<ThreadCtx>();
        c->device = device;
        if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
            set_error("hipStreamCreate failed on device %d", device);
            return nullptr;
        }
        for (auto &e : c->ev)
            if (hipEventCreate(&e) != hipSuccess) {
                set_error("hipEventCreate failed");
                return nullptr;
            }
        slot = std::move(c);
    }
    return slot.get();
}

// ---------------------------------------------------------------- kernels

// LinearTriangulation.py:54-90: one thread per point, 4x4 DLT system,
// right singular vector of the smallest singular value by one-sided Jacobi.
struct P2 {
    double p[24];
};

__global__ void __launch_bounds__(256) k_triangulate(P2 P, const double2 *__restrict__ x1,
                                                     const double2 *__restrict__ x2, int64_t N,
                                                     double *__restrict__ X) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const double *P1 = P.p, *Q = P.p + 12;
    const double2 u = x1[i], v = x2[i];
    double a[4][4], V[4][4];  // a[col][row]
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        a[c][0] = u.y * P1[8 + c] - P1[4 + c];
        a[c][1] = P1[c] - u.x * P1[8 + c];
        a[c][2] = v.y * Q[8 + c] - Q[4 + c];
        a[c][3] = Q[c] - v.x * Q[8 + c];
    }
    jacobi_onesided<4, 4, 40>(a, V);
    const int j = weakest_column<4, 4>(a);
    const double h0 = V[0][j], h1 = V[1][j], h2 = V[2][j], h3 = V[3][j];
    if (fabs(h3) > 1e-8) {
        X[3 * i] = h0 / h3; X[3 * i + 1] = h1 / h3; X[3 * i + 2] = h2 / h3;
    } else {
        X[3 * i] = h0; X[3 * i + 1] = h1; X[3 * i + 2] = h2;
    }
}

// project_points (BundleAdjustment.py:29-38)
struct P1s {
    double p[12];
};
__global__ void __launch_bounds__(256) k_project(P1s P, const double *__restrict__ X, int64_t M,
                                                 double *__restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= M) return;
    const double x = X[3 * i], y = X[3 * i + 1], z = X[3 * i + 2];
    const double *p = P.p;
    const double u = p[0] * x + p[1] * y + p[2] * z + p[3];
    const double v = p[4] * x + p[5] * y + p[6] * z + p[7];
    const double w = p[8] * x + p[9] * y + p[10] * z + p[11];
    out[2 * i] = u / (w + 1e-8);
    out[2 * i + 1] = v / (w + 1e-8);
}

// bundle_adjustment_residuals (BundleAdjustment.py:73-110): per camera
// R = from_rotvec, C = -R^T t, P = K [R | -R C]; per observation obs - proj.
__global__ void k_camera_P(int32_t nc, const double *__restrict__ cams, const double *__restrict__ Kd,
                           double *__restrict__ P) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= nc) return;
    double R[9];
    const double *w = cams + 6 * c;
    rotvec_to_R(w[0], w[1], w[2], R);
    double C[3], tt[3];
    for (int i = 0; i < 3; ++i) C[i] = -(R[i] * w[3] + R[3 + i] * w[4] + R[6 + i] * w[5]);
    for (int i = 0; i < 3; ++i) tt[i] = -(R[3 * i] * C[0] + R[3 * i + 1] * C[1] + R[3 * i + 2] * C[2]);
    for (int r = 0; r < 3; ++r) {
        for (int k = 0; k < 3; ++k)
            P[12 * c + 4 * r + k] = Kd[3 * r] * R[k] + Kd[3 * r + 1] * R[3 + k] + Kd[3 * r + 2] * R[6 + k];
        P[12 * c + 4 * r + 3] = Kd[3 * r] * tt[0] + Kd[3 * r + 1] * tt[1] + Kd[3 * r + 2] * tt[2];
    }
}

__global__ void __launch_bounds__(256) k_ba_residuals(int64_t n_obs, const int32_t *__restrict__ cam,
                                                      const int32_t *__restrict__ pt,
                                                      const double2 *__restrict__ obs,
                                                      const double *__restrict__ P,
                                                      const double *__restrict__ X, double2 *__restrict__ r) {
    const int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (o >= n_obs) return;
    const double *p = P + 12 * cam[o];
    const double *x = X + 3 * (int64_t)pt[o];
    const double u = p[0] * x[0] + p[1] * x[1] + p[2] * x[2] + p[3];
    const double v = p[4] * x[0] + p[5] * x[1] + p[6] * x[2] + p[7];
    const double w = p[8] * x[0] + p[9] * x[1] + p[10] * x[2] + p[11];
    const double2 ob = obs[o];
    r[o] = make_double2(ob.x - u / (w + 1e-8), ob.y - v / (w + 1e-8));
}

}  // namespace sfm

using namespace sfm;

extern "C" int sfm_version(void) { return SFM_ABI_VERSION; }
extern "C" const char *sfm_last_error(void) { return g_err.c_str(); }
extern "C" int sfm_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}
extern "C" int sfm_set_call_timing(int on) {
    g_call_timing.store(on != 0, std::memory_order_relaxed);
    return 0;
}
extern "C" int sfm_last_timings(double *out, int n) {
    const int m = n < g_ntimings ? n : g_ntimings;
    for (int i = 0; i < m; ++i) out[i] = g_timings[i];
    return m;
}

extern "C" int sfm_pyrandom_sample_table(uint32_t *st, int64_t n, int32_t k, int64_t H, int32_t *out) {
    SFM_CHECK_ARG(st && (out || H == 0), "null pointer");
    SFM_CHECK_ARG(k >= 0 && k <= n && n < (int64_t)1 << 31, "need 0 <= k <= n < 2^31");
    SFM_CHECK_ARG(st[624] <= 624, "bad MT19937 position");
    PySampler ps(st, n, k);
    ps.draw(0, H, out);
    ps.save(st);
    return 0;
}

extern "C" int sfm_f8_general(const double *x1, const double *x2, int64_t N, double *F, int device) {
    SFM_CHECK_ARG(N >= 1, "need N >= 1 correspondences");
    SFM_CHECK_ARG(x1 && x2 && F, "null pointer");
    ThreadCtx *c = thread_ctx(device);
    if (!c) return SFM_ERR_HIP;
    const size_t pb = (size_t)N * sizeof(double2);
    int rc;
    if ((rc = c->buf[0].reserve(pb)) || (rc = c->buf[1].reserve(pb)) || (rc = c->buf[2].reserve(9 * sizeof(double))))
        return rc;
    SFM_HIP(hipMemcpyAsync(c->buf[0].p, x1, pb, hipMemcpyHostToDevice, c->stream));
    SFM_HIP(hipMemcpyAsync(c->buf[1].p, x2, pb, hipMemcpyHostToDevice, c->stream));
    hipLaunchKernelGGL(k_dlt_general<FDesign>, dim3(1), dim3(FG_THREADS), 0, c->stream, c->buf[0].as<double2>(),
                       c->buf[1].as<double2>(), N, c->buf[2].as<double>());
    SFM_HIP(hipGetLastError());
    SFM_HIP(hipMemcpyAsync(F, c->buf[2].p, 9 * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    SFM_HIP(hipStreamSynchronize(c->stream));
    return 0;
}

extern "C" int sfm_triangulate_dlt(const double *P1, const double *P2_, const double *x1, const double *x2,
                                   int64_t N, double *X, int device) {
    SFM_CHECK_ARG(N >= 0, "N < 0");
    if (N == 0) return 0;
    SFM_CHECK_ARG(P1 && P2_ && x1 && x2 && X, "null pointer");
    ThreadCtx *c = thread_ctx(device);
    if (!c) return SFM_ERR_HIP;
    const size_t pb = (size_t)N * sizeof(double2);
    int rc;
    if ((rc = c->buf[0].reserve(pb)) || (rc = c->buf[1].reserve(pb)) || (rc = c->buf[2].reserve((size_t)N * 24)))
        return rc;
    P2 P;
    std::memcpy(P.p, P1, 12 * sizeof(double));
    std::memcpy(P.p + 12, P2_, 12 * sizeof(double));
    hipStream_t s = c->stream;
    const bool tm = call_timing();  // HIP events only when asked (each costs the stream us)
    if (tm) SFM_HIP(hipEventRecord(c->ev[0], s));
    SFM_HIP(hipMemcpyAsync(c->buf[0].p, x1, pb, hipMemcpyHostToDevice, s));
    SFM_HIP(hipMemcpyAsync(c->buf[1].p, x2, pb, hipMemcpyHostToDevice, s));
    if (tm) SFM_HIP(hipEventRecord(c->ev[1], s));
    hipLaunchKernelGGL(k_triangulate, dim3(ceil_div(N, 256)), dim3(256), 0, s, P, c->buf[0].as<double2>(),
                       c->buf[1].as<double2>(), N, c->buf[2].as<double>());
    SFM_HIP(hipGetLastError());
    if (tm) SFM_HIP(hipEventRecord(c->ev[2], s));
    SFM_HIP(hipMemcpyAsync(X, c->buf[2].p, (size_t)N * 24, hipMemcpyDeviceToHost, s));
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

extern "C" int sfm_project_points(const double *P, const double *X, int64_t M, double *out, int device) {
    SFM_CHECK_ARG(M >= 0, "M < 0");
    if (M == 0) return 0;
    SFM_CHECK_ARG(P && X && out, "null pointer");
    ThreadCtx *c = thread_ctx(device);
    if (!c) return SFM_ERR_HIP;
    int rc;
    if ((rc = c->buf[0].reserve((size_t)M * 24)) || (rc = c->buf[1].reserve((size_t)M * 16))) return rc;
    P1s p;
    std::memcpy(p.p, P, sizeof p.p);
    SFM_HIP(hipMemcpyAsync(c->buf[0].p, X, (size_t)M * 24, hipMemcpyHostToDevice, c->stream));
    hipLaunchKernelGGL(k_project, dim3(ceil_div(M, 256)), dim3(256), 0, c->stream, p, c->buf[0].as<double>(), M,
                       c->buf[1].as<double>());
    SFM_HIP(hipGetLastError());
    SFM_HIP(hipMemcpyAsync(out, c->buf[1].p, (size_t)M * 16, hipMemcpyDeviceToHost, c->stream));
    SFM_HIP(hipStreamSynchronize(c->stream));
    return 0;
}

extern "C" int sfm_ba_residuals(int32_t nc, int64_t np_, int64_t no, const int32_t *cam, const int32_t *pt,
                                const double *obs, const double *K, const double *cams, const double *pts,
                                double *r, int device) {
    SFM_CHECK_ARG(nc >= 0 && np_ >= 0 && no >= 0, "negative size");
    if (no == 0) return 0;
    SFM_CHECK_ARG(cam && pt && obs && K && cams && pts && r, "null pointer");
    for (int64_t o = 0; o < no; ++o)
        SFM_CHECK_ARG(cam[o] >= 0 && cam[o] < nc && pt[o] >= 0 && pt[o] < np_, "index out of range");
    ThreadCtx *c = thread_ctx(device);
    if (!c) return SFM_ERR_HIP;
    int rc;
    if ((rc = c->buf[0].reserve((size_t)no * 8)) || (rc = c->buf[1].reserve((size_t)no * 16)) ||
        (rc = c->buf[2].reserve((size_t)nc * 48 + 72)) || (rc = c->buf[3].reserve((size_t)np_ * 24)) ||
        (rc = c->buf[4].reserve((size_t)nc * 96)) || (rc = c->buf[5].reserve((size_t)no * 16)))
        return rc;
    hipStream_t s = c->stream;
    int32_t *dcam = c->buf[0].as<int32_t>(), *dpt = dcam + no;
    double *dK = c->buf[2].as<double>(), *dcams = dK + 9;
    SFM_HIP(hipMemcpyAsync(dcam, cam, (size_t)no * 4, hipMemcpyHostToDevice, s));
    SFM_HIP(hipMemcpyAsync(dpt, pt, (size_t)no * 4, hipMemcpyHostToDevice, s));
    SFM_HIP(hipMemcpyAsync(c->buf[1].p, obs, (size_t)no * 16, hipMemcpyHostToDevice, s));
    SFM_HIP(hipMemcpyAsync(dK, K, 72, hipMemcpyHostToDevice, s));
    SFM_HIP(hipMemcpyAsync(dcams, cams, (size_t)nc * 48, hipMemcpyHostToDevice, s));
    SFM_HIP(hipMemcpyAsync(c->buf[3].p, pts, (size_t)np_ * 24, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_camera_P, dim3(ceil_div(nc, 64)), dim3(64), 0, s, nc, dcams, dK, c->buf[4].as<double>());
    SFM_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_ba_residuals, dim3(ceil_div(no, 256)), dim3(256), 0, s, no, dcam, dpt,
                       c->buf[1].as<double2>(), c->buf[4].as<double>(), c->buf[3].as<double>(),
                       c->buf[5].as<double2>());
    SFM_HIP(hipGetLastError());
    SFM_HIP(hipMemcpyAsync(r, c->buf[5].p, (size_t)no * 16, hipMemcpyDeviceToHost, s));
    SFM_HIP(hipStreamSynchronize(s));
    return 0;
}
