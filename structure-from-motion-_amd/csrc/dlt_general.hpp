// Least-squares DLT fits on N correspondences (one workgroup), shared by
// the F (sfm_api.hip) and H (homography.hip) entry points.
#pragma once
#include "sfm_common.hpp"
#include "sfm_geom.hpp"

namespace sfm {

// Least-squares DLT fit of a 3x3 model to N correspondences in ONE
// workgroup: F for N >= 8 (EstimateFundamentalMatrix.py:21-83, one design
// row per correspondence) and H for N >= 4 (GetHomographyInliers.py:4-85,
// two rows).  Hartley statistics by block reduction; the N x 9 design
// matrix is reduced to a 9 x 9 triangular factor by per-thread Givens QR
// plus a binary tree merge in LDS (same right singular vectors as A);
// thread 0 then runs a 9-column one-sided Jacobi SVD for the null vector.
constexpr int FG_THREADS = 128;

__device__ __forceinline__ void givens_absorb(double (&R)[9][9], double (&a)[9]) {
#pragma unroll
    for (int j = 0; j < 9; ++j) {
        if (a[j] != 0.0) {
            const double r = sqrt(R[j][j] * R[j][j] + a[j] * a[j]);
            const double c = R[j][j] / r, s = a[j] / r;
#pragma unroll
            for (int k = j; k < 9; ++k) {
                const double u = R[j][k], v = a[k];
                R[j][k] = c * u + s * v;
                a[k] = -s * u + c * v;
            }
        }
    }
}

struct FDesign {
    static constexpr int ROWS = 1;
    __device__ static void rows(double a, double b, double c, double d, double (&r)[ROWS][9]) {
        r[0][0] = a * c; r[0][1] = a * d; r[0][2] = a;
        r[0][3] = b * c; r[0][4] = b * d; r[0][5] = b;
        r[0][6] = c; r[0][7] = d; r[0][8] = 1.0;
    }
    __device__ static void finish(const double (&f)[9], const Hartley &h1, const Hartley &h2, double *out) {
        f8_finish(f, h1, h2, out);
    }
};

struct HDesign {
    static constexpr int ROWS = 2;
    __device__ static void rows(double a, double b, double c, double d, double (&r)[ROWS][9]) {
        h_rows(a, b, c, d, r[0], r[1]);
    }
    __device__ static void finish(const double (&f)[9], const Hartley &h1, const Hartley &h2, double *out) {
        h_finish(f, h1, h2, out);
    }
};

template <class D>
__global__ void __launch_bounds__(FG_THREADS) k_dlt_general(const double2 *__restrict__ x1,
                                                           const double2 *__restrict__ x2, int64_t N,
                                                           double *__restrict__ F) {
    __shared__ double red[4][FG_THREADS];
    __shared__ double Rs[FG_THREADS][45];
    const int t = threadIdx.x;
    double s0 = 0, s1 = 0, s2 = 0, s3 = 0;
    for (int64_t i = t; i < N; i += FG_THREADS) {
        const double2 p = x1[i], q = x2[i];
        s0 += p.x; s1 += p.y; s2 += q.x; s3 += q.y;
    }
    red[0][t] = s0; red[1][t] = s1; red[2][t] = s2; red[3][t] = s3;
    __syncthreads();
    for (int w = FG_THREADS / 2; w > 0; w >>= 1) {
        if (t < w)
            for (int k = 0; k < 4; ++k) red[k][t] += red[k][t + w];
        __syncthreads();
    }
    const double m1x = red[0][0] / (double)N, m1y = red[1][0] / (double)N;
    const double m2x = red[2][0] / (double)N, m2y = red[3][0] / (double)N;
    __syncthreads();
    double d1 = 0, d2 = 0;
    for (int64_t i = t; i < N; i += FG_THREADS) {
        const double2 p = x1[i], q = x2[i];
        const double ax = p.x - m1x, ay = p.y - m1y, bx = q.x - m2x, by = q.y - m2y;
        d1 += sqrt(ax * ax + ay * ay);
        d2 += sqrt(bx * bx + by * by);
    }
    red[0][t] = d1; red[1][t] = d2;
    __syncthreads();
    for (int w = FG_THREADS / 2; w > 0; w >>= 1) {
        if (t < w) { red[0][t] += red[0][t + w]; red[1][t] += red[1][t + w]; }
        __syncthreads();
    }
    Hartley h1, h2;
    h1.s = 1.4142135623730951 / (red[0][0] / (double)N + 1e-8);
    h2.s = 1.4142135623730951 / (red[1][0] / (double)N + 1e-8);
    h1.ox = -h1.s * m1x; h1.oy = -h1.s * m1y; h2.ox = -h2.s * m2x; h2.oy = -h2.s * m2y;
    double R[9][9];
#pragma unroll
    for (int i = 0; i < 9; ++i)
#pragma unroll
        for (int j = 0; j < 9; ++j) R[i][j] = 0.0;
    for (int64_t i = t; i < N; i += FG_THREADS) {
        const double2 p = x1[i], q = x2[i];
        const double a = h1.s * p.x + h1.ox, b = h1.s * p.y + h1.oy;
        const double c = h2.s * q.x + h2.ox, d = h2.s * q.y + h2.oy;
        double rows[D::ROWS][9];
        D::rows(a, b, c, d, rows);
#pragma unroll
        for (int q = 0; q < D::ROWS; ++q) givens_absorb(R, rows[q]);
    }
    for (int w = FG_THREADS / 2; w > 0; w >>= 1) {
        if (t >= w && t < 2 * w) {
            int k = 0;
#pragma unroll
            for (int i = 0; i < 9; ++i)
#pragma unroll
                for (int j = i; j < 9; ++j) Rs[t][k++] = R[i][j];
        }
        __syncthreads();
        if (t < w) {
#pragma unroll
            for (int i = 0; i < 9; ++i) {
                double row[9];
#pragma unroll
                for (int j = 0; j < 9; ++j) row[j] = 0.0;
#pragma unroll
                for (int j = i; j < 9; ++j) row[j] = Rs[t + w][i * 9 - i * (i - 1) / 2 + (j - i)];
                givens_absorb(R, row);
            }
        }
        __syncthreads();
    }
    if (t != 0) return;
    double a[9][9], V[9][9];  // a[col][row]
#pragma unroll
    for (int c = 0; c < 9; ++c)
#pragma unroll
        for (int r = 0; r < 9; ++r) a[c][r] = R[r][c];
    jacobi_onesided<9, 9, 40>(a, V);
    const int j = weakest_column<9, 9>(a);
    double f[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) f[k] = V[k][j];
    D::finish(f, h1, h2, F);
}

}  // namespace sfm
