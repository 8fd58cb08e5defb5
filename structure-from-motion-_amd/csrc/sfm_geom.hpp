// Device-side fp64 geometry shared by the kernels.  All loops have
// compile-time trip counts so every matrix lives in VGPRs (no scratch).
#pragma once
#include <hip/hip_runtime.h>

namespace sfm {

// --------------------------------------------------------------------
// Symmetric epipolar distance test of GetInliersRANSAC.py:64-81.
// Same operation order as the reference expression; strict '<'.
// --------------------------------------------------------------------
__device__ __forceinline__ bool epi_inlier(const double *F, double x, double y, double u, double v,
                                           double thr) {
    const double a0 = F[0] * x + F[1] * y + F[2];
    const double a1 = F[3] * x + F[4] * y + F[5];
    const double a2 = F[6] * x + F[7] * y + F[8];
    const double b0 = F[0] * u + F[3] * v + F[6];
    const double b1 = F[1] * u + F[4] * v + F[7];
    const double e = u * a0 + v * a1 + a2;
    const double ae = fabs(e);
    const double d1 = ae / (sqrt(a0 * a0 + a1 * a1) + 1e-8);
    const double d2 = ae / (sqrt(b0 * b0 + b1 * b1) + 1e-8);
    return (d1 + d2) * 0.5 < thr;
}

// Same decision, cheaper: approximate sqrt / reciprocal (v_rsq_f64,
// v_rcp_f64, ~1e-7 relative) decide every pair whose approximate error is
// farther than 1e-4 relative from the threshold; the rest (and any
// non-finite / tiny operand) take the exact expression above.  The
// decision is therefore always the exact one.
__device__ __forceinline__ bool epi_inlier_fast(const double *F, double x, double y, double u, double v,
                                                double thr, double thr_lo, double thr_hi) {
    const double a0 = F[0] * x + F[1] * y + F[2];
    const double a1 = F[3] * x + F[4] * y + F[5];
    const double a2 = F[6] * x + F[7] * y + F[8];
    const double b0 = F[0] * u + F[3] * v + F[6];
    const double b1 = F[1] * u + F[4] * v + F[7];
    const double e = u * a0 + v * a1 + a2;
    const double ae = fabs(e);
    const double qa = a0 * a0 + a1 * a1, qb = b0 * b0 + b1 * b1;
    const double sa = qa * __builtin_amdgcn_rsq(qa), sb = qb * __builtin_amdgcn_rsq(qb);
    const double ap = (ae * __builtin_amdgcn_rcp(sa + 1e-8) + ae * __builtin_amdgcn_rcp(sb + 1e-8)) * 0.5;
    const bool sure_in = ap < thr_lo && qa > 1e-280 && qb > 1e-280;
    const bool sure_out = ap > thr_hi && qa > 1e-280 && qb > 1e-280 && qa < 1e280 && qb < 1e280;
    if (sure_in) return true;
    if (sure_out) return false;
    const double d1 = ae / (sqrt(qa) + 1e-8);
    const double d2 = ae / (sqrt(qb) + 1e-8);
    return (d1 + d2) * 0.5 < thr;
}

// --------------------------------------------------------------------
// One-sided (Hestenes) Jacobi on an M x N matrix held column-major in
// registers: a[j][i] = column j, row i.  V (N x N) accumulates rotations,
// column j of V is the right singular vector for column j of a.
// Same rotation rule as the oracle (oracle/sfm_oracle.c:jacobi_svd).
// --------------------------------------------------------------------
template <int M, int N, int SWEEPS>
__device__ __forceinline__ void jacobi_onesided(double (&a)[N][M], double (&V)[N][N]) {
#pragma unroll
    for (int i = 0; i < N; ++i)
#pragma unroll
        for (int j = 0; j < N; ++j) V[i][j] = (i == j) ? 1.0 : 0.0;
    for (int sweep = 0; sweep < SWEEPS; ++sweep) {
        double off = 0.0;
#pragma unroll
        for (int p = 0; p < N - 1; ++p) {
#pragma unroll
            for (int q = p + 1; q < N; ++q) {
                double al = 0, be = 0, ga = 0;
#pragma unroll
                for (int k = 0; k < M; ++k) {
                    al += a[p][k] * a[p][k];
                    be += a[q][k] * a[q][k];
                    ga += a[p][k] * a[q][k];
                }
                const double r = fabs(ga) / sqrt(al * be);
                if (ga != 0.0 && r > 1e-15) {
                    off = fmax(off, r);
                    const double zeta = (be - al) / (2.0 * ga);
                    const double t = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
                    const double cs = 1.0 / sqrt(1.0 + t * t), sn = cs * t;
#pragma unroll
                    for (int k = 0; k < M; ++k) {
                        const double x = a[p][k], y = a[q][k];
                        a[p][k] = cs * x - sn * y;
                        a[q][k] = sn * x + cs * y;
                    }
#pragma unroll
                    for (int k = 0; k < N; ++k) {
                        const double x = V[k][p], y = V[k][q];
                        V[k][p] = cs * x - sn * y;
                        V[k][q] = sn * x + cs * y;
                    }
                }
            }
        }
        if (off < 1e-15) break;
    }
}

template <int M, int N>
__device__ __forceinline__ int weakest_column(const double (&a)[N][M]) {
    int best = 0;
    double bn = 0;
#pragma unroll
    for (int k = 0; k < M; ++k) bn += a[0][k] * a[0][k];
#pragma unroll
    for (int j = 1; j < N; ++j) {
        double n = 0;
#pragma unroll
        for (int k = 0; k < M; ++k) n += a[j][k] * a[j][k];
        if (n < bn) { bn = n; best = j; }
    }
    return best;
}

// Hartley normalisation (EstimateFundamentalMatrix.py:30-55) of 8 points.
struct Hartley {
    double s, ox, oy;  // x' = s*x + ox
};

__device__ __forceinline__ Hartley hartley8(const double (&x)[8], const double (&y)[8]) {
    double mx = 0, my = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) { mx += x[i]; my += y[i]; }
    mx = mx / 8.0;
    my = my / 8.0;
    double d = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const double ax = x[i] - mx, ay = y[i] - my;
        d += sqrt(ax * ax + ay * ay);
    }
    Hartley h;
    h.s = 1.4142135623730951 / (d / 8.0 + 1e-8);
    h.ox = -h.s * mx;
    h.oy = -h.s * my;
    return h;
}

// Rank-2 projection (EstimateFundamentalMatrix.py:70-72), denormalisation
// F = T2^T F T1 (:75, as shipped) and F / F[2,2] (:78).
// f: normalised null vector, row-major 3x3.
__device__ __forceinline__ void f8_finish(const double (&f)[9], const Hartley &h1, const Hartley &h2,
                                          double *F_out) {
    double b[3][3], W[3][3];  // b[col][row]
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int r = 0; r < 3; ++r) b[c][r] = f[r * 3 + c];
    jacobi_onesided<3, 3, 24>(b, W);
    const int z = weakest_column<3, 3>(b);
    double F2[3][3];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            double acc = 0;
#pragma unroll
            for (int k = 0; k < 3; ++k)
                if (k != z) acc += b[k][r] * W[c][k];
            F2[r][c] = acc;
        }
    // T = [[s,0,ox],[0,s,oy],[0,0,1]] ; G = T2^T F2 T1
    const double T1[3][3] = {{h1.s, 0, h1.ox}, {0, h1.s, h1.oy}, {0, 0, 1}};
    const double T2[3][3] = {{h2.s, 0, h2.ox}, {0, h2.s, h2.oy}, {0, 0, 1}};
    double tmp[3][3], G[3][3];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            double acc = 0;
#pragma unroll
            for (int k = 0; k < 3; ++k) acc += T2[k][r] * F2[k][c];
            tmp[r][c] = acc;
        }
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            double acc = 0;
#pragma unroll
            for (int k = 0; k < 3; ++k) acc += tmp[r][k] * T1[k][c];
            G[r][c] = acc;
        }
    const double d = G[2][2];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) F_out[r * 3 + c] = G[r][c] / d;
}

// 8-point F (EstimateFundamentalMatrix.py:21-83).  The null vector of the
// 8 x 9 design matrix A (:58-67) is obtained from a Householder LQ of A:
// A Q_0..Q_7 = [L 0], so n = Q_0 ... Q_7 e_8 spans null(A) whenever
// rank(A) = 8 -- the same vector as Vt[-1] of the reference's SVD up to
// sign, which F / F[2,2] removes.  ~0.6 kflop instead of a 9-column SVD.
__device__ __forceinline__ void f8_points(const double (&x1)[8], const double (&y1)[8],
                                          const double (&x2)[8], const double (&y2)[8], double *F_out) {
    const Hartley h1 = hartley8(x1, y1), h2 = hartley8(x2, y2);
    double A[8][9];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const double a = h1.s * x1[i] + h1.ox, b = h1.s * y1[i] + h1.oy;
        const double c = h2.s * x2[i] + h2.ox, d = h2.s * y2[i] + h2.oy;
        A[i][0] = a * c; A[i][1] = a * d; A[i][2] = a;
        A[i][3] = b * c; A[i][4] = b * d; A[i][5] = b;
        A[i][6] = c; A[i][7] = d; A[i][8] = 1.0;
    }
    double tau[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        // reflector zeroing A[k][k+1..8]; v overwrites A[k][k..8]
        double nrm2 = 0;
#pragma unroll
        for (int j = k; j < 9; ++j) nrm2 += A[k][j] * A[k][j];
        const double nrm = sqrt(nrm2);
        const double alpha = A[k][k] > 0 ? -nrm : nrm;
        A[k][k] -= alpha;
        double vtv = 0;
#pragma unroll
        for (int j = k; j < 9; ++j) vtv += A[k][j] * A[k][j];
        tau[k] = nrm2 > 0 ? 2.0 / vtv : 0.0;
#pragma unroll
        for (int i = k + 1; i < 8; ++i) {
            double d = 0;
#pragma unroll
            for (int j = k; j < 9; ++j) d += A[i][j] * A[k][j];
            d *= tau[k];
#pragma unroll
            for (int j = k; j < 9; ++j) A[i][j] -= d * A[k][j];
        }
    }
    double n[9];
#pragma unroll
    for (int j = 0; j < 9; ++j) n[j] = (j == 8) ? 1.0 : 0.0;
#pragma unroll
    for (int k = 7; k >= 0; --k) {
        double d = 0;
#pragma unroll
        for (int j = k; j < 9; ++j) d += A[k][j] * n[j];
        d *= tau[k];
#pragma unroll
        for (int j = k; j < 9; ++j) n[j] -= d * A[k][j];
    }
    f8_finish(n, h1, h2, F_out);
}

// Rodrigues (scipy Rotation.from_rotvec(...).as_matrix()), row-major.
__device__ __forceinline__ void rotvec_to_R(double wx, double wy, double wz, double *R) {
    const double th2 = wx * wx + wy * wy + wz * wz;
    const double th = sqrt(th2);
    double a, b;
    if (th < 1e-6) {
        a = 1.0 - th2 / 6.0 + th2 * th2 / 120.0;
        b = 0.5 - th2 / 24.0 + th2 * th2 / 720.0;
    } else {
        double s, c;
        sincos(th, &s, &c);
        a = s / th;
        b = (1.0 - c) / th2;
    }
    R[0] = 1.0 - b * (wy * wy + wz * wz); R[1] = -a * wz + b * wx * wy;        R[2] = a * wy + b * wx * wz;
    R[3] = a * wz + b * wx * wy;          R[4] = 1.0 - b * (wx * wx + wz * wz); R[5] = -a * wx + b * wy * wz;
    R[6] = -a * wy + b * wx * wz;         R[7] = a * wx + b * wy * wz;          R[8] = 1.0 - b * (wx * wx + wy * wy);
}

}  // namespace sfm
