// Device-side fp64 geometry shared by the kernels.  All loops have
// compile-time trip counts so every matrix lives in VGPRs (no scratch).
#pragma once
#include <hip/hip_runtime.h>

namespace sfm {

// --------------------------------------------------------------------
// Symmetric epipolar distance test of GetInliersRANSAC.py:64-81.
// Same operation order as the reference expression; strict '<'.  Every
// function of the F path (the epipolar tests and the 8-point fit below) is
// compiled with contraction off and states numpy's FMAs explicitly: Fx1 =
// F @ x1h and FTx2 are OpenBLAS dgemm products (a0 b0, then fma), the row
// sum of x2h * Fx1 and the squares are plain products and sums.  The C
// oracle uses the same expression (equal to numpy's bit for bit,
// tests/test_oracle.py), so the decisions match at the threshold itself.
// --------------------------------------------------------------------
__device__ __forceinline__ bool epi_inlier(const double *F, double x, double y, double u, double v,
                                           double thr) {
#pragma clang fp contract(off)
    const double a0 = fma(F[1], y, F[0] * x) + F[2];  // F @ x1h: OpenBLAS dgemm's order
    const double a1 = fma(F[4], y, F[3] * x) + F[5];
    const double a2 = fma(F[7], y, F[6] * x) + F[8];
    const double b0 = fma(F[3], v, F[0] * u) + F[6];  // F.T @ x2h
    const double b1 = fma(F[4], v, F[1] * u) + F[7];
    const double e = u * a0 + v * a1 + a2;
    const double ae = fabs(e);
    const double d1 = ae / (sqrt(a0 * a0 + a1 * a1) + 1e-8);
    const double d2 = ae / (sqrt(b0 * b0 + b1 * b1) + 1e-8);
    return (d1 + d2) * 0.5 < thr;
}

// Same decision, cheaper: approximate sqrt / reciprocal (v_rsq_f64, ~1e-7
// relative) decide every pair whose approximate error is farther than 1e-4
// relative from the threshold; the rest (and any non-finite / tiny
// operand) take the exact expression (epi_exact).  The decision is
// therefore always the exact one.  Split in two so a caller can run the
// fast part of several pairs before any branch to the exact tail.
struct EpiPart {
    double ae, qa, qb;  // |x2^T F x1|, |Fx1|_xy^2, |F^T x2|_xy^2
    bool in, unsure;    // fast decision; unsure: take epi_exact
};

__device__ __forceinline__ EpiPart epi_fast(const double *F, double x, double y, double u, double v, double thr_lo2,
                                            double thr_hi2) {
#pragma clang fp contract(off)
    const double a0 = fma(F[1], y, F[0] * x) + F[2];  // F @ x1h: OpenBLAS dgemm's order
    const double a1 = fma(F[4], y, F[3] * x) + F[5];
    const double a2 = fma(F[7], y, F[6] * x) + F[8];
    const double b0 = fma(F[3], v, F[0] * u) + F[6];  // F.T @ x2h
    const double b1 = fma(F[4], v, F[1] * u) + F[7];
    const double e = u * a0 + v * a1 + a2;
    EpiPart r;
    r.ae = fabs(e);
    r.qa = a0 * a0 + a1 * a1;
    r.qb = b0 * b0 + b1 * b1;
    // 1 / (sqrt(q) + 1e-8) = r (1 - 1e-8 r + ...), r = rsq(q): first order,
    // whose error (1e-8 r)^2 <= 1e-6 relative while r < 1e5 (q > 1e-10) --
    // no v_rcp.  ok = ra + rb < 1e5 holds exactly when both r are finite and
    // below 1e5 (a NaN fails it), so it also guards q = 0 / NaN; q = inf
    // gives r = 0, the exact limit.  thr_lo2 / thr_hi2 are the band around
    // 2 thr (the 1/2 of the mean is folded in).
    const double ra = __builtin_amdgcn_rsq(r.qa), rb = __builtin_amdgcn_rsq(r.qb);
    const double srr = ra + rb;
    const double ap2 = r.ae * fma(-1e-8, fma(ra, ra, rb * rb), srr);  // ae (ia + ib)
    const bool ok = srr < 1e5;
    const bool sure_in = ap2 < thr_lo2 && ok;
    const bool sure_out = ap2 > thr_hi2 && ok;
    r.in = sure_in;
    r.unsure = !(sure_in || sure_out);
    return r;
}

// epi_fast in two stages, the same operations: stage A (the first image's
// line, e and |Fx1|^2) already proves "outlier" for most pairs --
// the mean is at least half the first distance, so a first distance above the
// band's upper edge decides it; the score kernel skips stage B for a wave
// whose pairs are all decided that way.  epi_fast_b(epi_fast_a(...)) equals
// epi_fast(...) in every field.
struct EpiPartA {
    double ae, qa;
    bool out;  // decided: outlier
};

__device__ __forceinline__ EpiPartA epi_fast_a(const double *F, double x, double y, double u, double v,
                                               double thr_hi2) {
#pragma clang fp contract(off)
    const double a0 = fma(F[1], y, F[0] * x) + F[2];  // F @ x1h: OpenBLAS dgemm's order
    const double a1 = fma(F[4], y, F[3] * x) + F[5];
    const double a2 = fma(F[7], y, F[6] * x) + F[8];
    const double e = u * a0 + v * a1 + a2;
    EpiPartA r;
    r.ae = fabs(e);
    r.qa = a0 * a0 + a1 * a1;
    // d1 = ae / (sqrt(qa) + 1e-8) > thr_hi2 without a square root:
    // (sqrt(qa) + 1e-8)^2 <= qa (1 + 1e-8) + 1e-8 + 1e-16 (sqrt(qa) <= (qa + 1) / 2),
    // so ae^2 > thr_hi2^2 (qa (1 + 1e-8) + 1.00000001e-8) proves it; the band
    // (thr_hi2 = 2 thr (1 + 1e-4)) absorbs the rounding of these few
    // operations.  The magnitude guards keep ae^2 and the right side finite;
    // NaN fails every comparison (stage B decides those pairs)
    const double rhs = thr_hi2 * thr_hi2 * fma(r.qa, 1.0 + 1e-8, 1.00000001e-8);
    // thr_hi2 > 1e-150: below it thr_hi2^2 underflows and rhs would prove
    // pairs "out" that the exact mean keeps (stage B decides those)
    r.out = r.ae * r.ae > rhs && r.ae < 1e150 && r.qa < 1e290 && thr_hi2 > 1e-150;
    return r;
}

__device__ __forceinline__ EpiPart epi_fast_b(const EpiPartA &a, const double *F, double u, double v,
                                              double thr_lo2, double thr_hi2) {
#pragma clang fp contract(off)
    const double b0 = fma(F[3], v, F[0] * u) + F[6];  // F.T @ x2h
    const double b1 = fma(F[4], v, F[1] * u) + F[7];
    EpiPart r;
    r.ae = a.ae;
    r.qa = a.qa;
    r.qb = b0 * b0 + b1 * b1;
    const double ra = __builtin_amdgcn_rsq(a.qa), rb = __builtin_amdgcn_rsq(r.qb);
    const double srr = ra + rb;
    const double ap2 = r.ae * fma(-1e-8, fma(ra, ra, rb * rb), srr);
    const bool ok = srr < 1e5;
    const bool sure_in = ap2 < thr_lo2 && ok;
    const bool sure_out = ap2 > thr_hi2 && ok;
    r.in = sure_in;
    r.unsure = !(sure_in || sure_out);
    return r;
}

// A float prefilter ahead of stage A (round 5): two pairs per packed FP32
// instruction (v_pk_fma_f32), seven instructions a pair against stage A's
// ~20 FP64 ones, proving "outlier" for the pairs far from the threshold.
// The proof is rigorous, not a tolerance.  Per hypothesis F is scaled by a
// power of two g = s F (max |g| in [0.5, 1), exact; the reference's d1 is
// then |e'| / (sqrt(qa') + s 1e-8) in the scaled terms) and rounded to
// float.  With the point coordinates bounded by the slice's maxima X, Y, U, V
// (<= 2^24, k_stage_tiles), the float evaluation
//   a_k = fma(g_k1, y, fma(g_k0, x, g_k2)),  e = fma(u, a0, fma(v, a1, a2))
// (at most 4 + 3 roundings per term, inputs included) obeys
//   |e_ref| >= |e~| - E,  E = 5e-7 Mt + 2^-70,  Mt = (U, V, 1) |g| (X, Y, 1)
//   sqrt(qa_ref) <= (1 + 1e-6) sqrt(qa~) + 3e-7 At + 2^-60,
//   At = |((|g0| X + |g1| Y + |g2|), (|g3| X + |g4| Y + |g5|))|
// (a_k carries at most 4 roundings a term, gamma_4 = 2.4e-7 of A_k; e adds
// 3, 7u = 4.2e-7 of Mt; the reference's own FP64 rounding and float
// underflow of tiny g or coordinates fit in the absolute terms).  Stage
// A's condition |e_ref| > thr_hi2 (sqrt(qa_ref) + s 1e-8) therefore holds when
//   |e~| > K1 sqrt(qa~) + K0,   K1 = thr_hi2 (1 + 1e-6),
//   K0 = thr_hi2 (3e-7 At + 2^-60 + s 1e-8) + E,
// and, squared with (a + b)^2 <= (1 + d) a^2 + (1 + 1/d) b^2 (d = 2^-8), when
//   e~^2 > q1 qa~ + q0,  q1 = (1 + d) K1^2, q0 = (1 + 1/d) K0^2,
// both rounded up to float after a (1 + 2^-20) factor that covers the three
// roundings of evaluating this test in float.  Inf / NaN anywhere makes the
// comparison false: the pair is simply not proven (stage A decides it).
struct EpiPre {
    float g[9];
    float q1, q0;
    bool on;  // the prefilter applies to this hypothesis and coordinate range
};

// per hypothesis f (finite) and slice bounds b = (X, Y, U, V)
__device__ __forceinline__ EpiPre epi_pre_setup(const double *f, double thr_hi2, float4 b) {
    EpiPre r;
    r.on = false;
    double m = 0.0;
#pragma unroll
    for (int k = 0; k < 9; ++k) m = fmax(m, fabs(f[k]));
    const float lim = 0x1p24f;
    if (!(m > 0.0) || !(b.x <= lim && b.y <= lim && b.z <= lim && b.w <= lim)) return r;
    if (!(thr_hi2 >= 0x1p-60 && thr_hi2 <= 0x1p60)) return r;
    const int ex = ilogb(m);
    // |scale| <= 2^400 both ways: the reference's own FP64 evaluation then
    // neither overflows (a non-finite qa would make its d1 0) nor loses more
    // than 2^-270 to underflow in the scaled terms
    if (ex < -399 || ex > 398) return r;
    double g[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) g[k] = ldexp(f[k], -ex - 1);
    const double c = ldexp(1e-8, -ex - 1);
    const double X = b.x, Y = b.y, U = b.z, V = b.w;
    const double A0 = fabs(g[0]) * X + fabs(g[1]) * Y + fabs(g[2]);
    const double A1 = fabs(g[3]) * X + fabs(g[4]) * Y + fabs(g[5]);
    const double A2 = fabs(g[6]) * X + fabs(g[7]) * Y + fabs(g[8]);
    const double Mt = U * A0 + V * A1 + A2;
    const double At = sqrt(A0 * A0 + A1 * A1);
    const double E = 5e-7 * Mt + 0x1p-70;
    const double K1 = thr_hi2 * (1.0 + 1e-6);
    const double K0 = thr_hi2 * (3e-7 * At + 0x1p-60 + c) + E;
    const double d = 0x1p-8;
    r.q1 = __double2float_ru((1.0 + d) * K1 * K1 * (1.0 + 0x1p-20));
    r.q0 = __double2float_ru((1.0 + 1.0 / d) * K0 * K0 * (1.0 + 0x1p-20));
#pragma unroll
    for (int k = 0; k < 9; ++k) r.g[k] = (float)g[k];
    r.on = true;
    return r;
}
typedef float epi_f2 __attribute__((ext_vector_type(2)));

// the prefilter's constants as broadcast pairs (both halves equal), the
// operands the packed instructions take as they are (from single floats the
// compiler copied each into an aligned register pair per hypothesis)
struct EpiPk {
    epi_f2 q1, q0, g[9];
};

// two pairs: pa = (x_0, x_1, y_0, y_1), pb = (u_0, u_1, v_0, v_1) (pair 0 in
// the low halves); out0 / out1: proven outliers
__device__ __forceinline__ void epi_pre_test(const EpiPk &p, float4 pa, float4 pb, bool &out0, bool &out1) {
    const epi_f2 x = {pa.x, pa.y}, y = {pa.z, pa.w}, u = {pb.x, pb.y}, v = {pb.z, pb.w};
    const epi_f2 a0 = __builtin_elementwise_fma(p.g[1], y, __builtin_elementwise_fma(p.g[0], x, p.g[2]));
    const epi_f2 a1 = __builtin_elementwise_fma(p.g[4], y, __builtin_elementwise_fma(p.g[3], x, p.g[5]));
    const epi_f2 a2 = __builtin_elementwise_fma(p.g[7], y, __builtin_elementwise_fma(p.g[6], x, p.g[8]));
    const epi_f2 e = __builtin_elementwise_fma(u, a0, __builtin_elementwise_fma(v, a1, a2));
    const epi_f2 qa = __builtin_elementwise_fma(a0, a0, a1 * a1);
    const epi_f2 rhs = __builtin_elementwise_fma(p.q1, qa, p.q0);
    const epi_f2 e2 = e * e;
    out0 = e2.x > rhs.x;
    out1 = e2.y > rhs.y;
}

// the exact tail of epi_inlier from epi_fast's terms (same operations)
__device__ __forceinline__ bool epi_exact(const EpiPart &r, double thr) {
#pragma clang fp contract(off)
    const double d1 = r.ae / (sqrt(r.qa) + 1e-8);
    const double d2 = r.ae / (sqrt(r.qb) + 1e-8);
    return (d1 + d2) * 0.5 < thr;
}

__device__ __forceinline__ bool epi_inlier_fast(const double *F, double x, double y, double u, double v,
                                                double thr, double thr_lo2, double thr_hi2) {
    const EpiPart r = epi_fast(F, x, y, u, v, thr_lo2, thr_hi2);
    return r.unsure ? epi_exact(r, thr) : r.in;
}

// --------------------------------------------------------------------
// One-sided (Hestenes) Jacobi on an M x N matrix held column-major in
// registers: a[j][i] = column j, row i.  V (N x N) accumulates rotations,
// column j of V is the right singular vector for column j of a.
// Same rotation rule as the oracle (oracle/sfm_oracle.c:jacobi_svd).
// --------------------------------------------------------------------
template <int M, int N, int SWEEPS>
__device__ __forceinline__ void jacobi_onesided(double (&a)[N][M], double (&V)[N][N]) {
#pragma clang fp contract(off)
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
#pragma clang fp contract(off)
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
#pragma clang fp contract(off)
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
// Unit right singular vector of F (3x3, row-major) for its smallest singular
// value: the eigenvector of A = F^T F for its smallest eigenvalue, from the
// closed-form (trigonometric) eigenvalue and the largest cross product of
// two rows of A - lambda I.  Its error is ~eps * lambda_1 / (lambda_2 -
// lambda_3), i.e. ~eps unless F is nearly rank 1 (false: use Jacobi).
__device__ __forceinline__ bool smallest_right_sv(const double (&f)[9], double (&v)[3]) {
#pragma clang fp contract(off)
    double a[3][3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) a[i][j] = f[i] * f[j] + f[3 + i] * f[3 + j] + f[6 + i] * f[6 + j];
    const double p1 = a[0][1] * a[0][1] + a[0][2] * a[0][2] + a[1][2] * a[1][2];
    const double q = (a[0][0] + a[1][1] + a[2][2]) / 3.0;
    const double b0 = a[0][0] - q, b1 = a[1][1] - q, b2 = a[2][2] - q;
    const double p2 = b0 * b0 + b1 * b1 + b2 * b2 + 2.0 * p1;
    if (!(p2 > 0.0)) return false;
    const double pp = sqrt(p2 / 6.0), ip = 1.0 / pp;
    const double B00 = b0 * ip, B11 = b1 * ip, B22 = b2 * ip;
    const double B01 = a[0][1] * ip, B02 = a[0][2] * ip, B12 = a[1][2] * ip;
    double r = 0.5 * (B00 * (B11 * B22 - B12 * B12) - B01 * (B01 * B22 - B12 * B02) + B02 * (B01 * B12 - B11 * B02));
    r = fmin(1.0, fmax(-1.0, r));
    const double phi = acos(r) / 3.0;
    const double lam = q + 2.0 * pp * cos(phi + 2.0943951023931957);  // the smallest eigenvalue
    const double m[3][3] = {{a[0][0] - lam, a[0][1], a[0][2]},
                            {a[0][1], a[1][1] - lam, a[1][2]},
                            {a[0][2], a[1][2], a[2][2] - lam}};
    double c[3][3];  // cross products of row pairs (0,1), (0,2), (1,2)
    const int pr[3][2] = {{0, 1}, {0, 2}, {1, 2}};
    double best = -1.0;
    int bi = 0;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const double *u = m[pr[k][0]], *w = m[pr[k][1]];
        c[k][0] = u[1] * w[2] - u[2] * w[1];
        c[k][1] = u[2] * w[0] - u[0] * w[2];
        c[k][2] = u[0] * w[1] - u[1] * w[0];
        const double n = c[k][0] * c[k][0] + c[k][1] * c[k][1] + c[k][2] * c[k][2];
        if (n > best) { best = n; bi = k; }
    }
    // nearly rank 1 (two eigenvalues meet the smallest): leave it to Jacobi
    if (!(best > 1e-20 * p2 * p2)) return false;
    const double in = 1.0 / sqrt(best);
#pragma unroll
    for (int i = 0; i < 3; ++i) v[i] = (bi == 0 ? c[0][i] : bi == 1 ? c[1][i] : c[2][i]) * in;
    return true;
}

// lane < 0: one thread writes all of F.  lane in [0, 8): the 8 lanes of a
// group run it together on the same inputs (the same bits) and lane i
// divides and writes entry i, lane 0 entry 8 as well: two divisions in
// flight per lane instead of nine on one.
__device__ __forceinline__ void f8_finish(const double (&f)[9], const Hartley &h1, const Hartley &h2,
                                          double *F_out, int lane = -1) {
#pragma clang fp contract(off)
    // rank 2 (EstimateFundamentalMatrix.py:70-72): U diag(s1, s2, 0) V^T =
    // F - (F v3) v3^T with v3 the smallest right singular vector
    double F2[3][3];
    double v3[3];
    if (smallest_right_sv(f, v3)) {
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            const double fv = f[r * 3] * v3[0] + f[r * 3 + 1] * v3[1] + f[r * 3 + 2] * v3[2];
#pragma unroll
            for (int c = 0; c < 3; ++c) F2[r][c] = f[r * 3 + c] - fv * v3[c];
        }
    } else {
        double b[3][3], W[3][3];  // b[col][row]
#pragma unroll
        for (int c = 0; c < 3; ++c)
#pragma unroll
            for (int r = 0; r < 3; ++r) b[c][r] = f[r * 3 + c];
        jacobi_onesided<3, 3, 24>(b, W);
        const int z = weakest_column<3, 3>(b);
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
    if (lane >= 0) {
        double num = G[0][0];
#pragma unroll
        for (int k = 1; k < 8; ++k) num = lane == k ? G[k / 3][k % 3] : num;
        F_out[lane] = num / d;
        if (lane == 0) F_out[8] = G[2][2] / d;
        return;
    }
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) F_out[r * 3 + c] = G[r][c] / d;
}

// Null vector of an 8 x 9 matrix A (rank 8) from a Householder LQ:
// A Q_0..Q_7 = [L 0], so n = Q_0 ... Q_7 e_8 spans null(A) -- the same vector
// as Vt[-1] of the reference's SVD up to sign (both the F and the H paths
// divide by the [2,2] entry, which removes it).  ~0.6 kflop instead of a
// 9-column SVD.  A is destroyed.
__device__ __forceinline__ void null_vector_8x9(double (&A)[8][9], double (&n)[9]) {
#pragma clang fp contract(off)
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
}

// 8-point F (EstimateFundamentalMatrix.py:21-83): Hartley-normalised design
// matrix (:58-62), its null vector, rank 2 and denormalisation (f8_finish).
__device__ __forceinline__ void f8_points(const double (&x1)[8], const double (&y1)[8],
                                          const double (&x2)[8], const double (&y2)[8], double *F_out) {
#pragma clang fp contract(off)
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
    double n[9];
    null_vector_8x9(A, n);
    f8_finish(n, h1, h2, F_out);
}

// f8_points on a group of 8 consecutive lanes, lane i of the group holding
// sample point i: the same operations in the same order, with one
// design-matrix row per lane.  The compiler contracts some products into
// FMAs differently in the two forms, so F can differ from f8_points in the
// last bits (tools/fit_group_check.hip); every RANSAC path therefore fits F
// with this one, and the batch entry (sfm_f8_batch) with f8_points.  The Hartley sums gather the group's
// values by shuffles in point order; reflector k (row k's lane) and its tau
// are broadcast to the group for the rows below and again for the
// back-substitution, which every lane runs on its own copy of n.  ~60 VGPRs
// against the one-thread fit's 136, so it can share a launch with the score.
// Every lane of the group runs the rank-2 step (the same bits: the lanes'
// n, h1 and h2 are equal) and writes one entry of F_out (lane 0 two).
__device__ __forceinline__ double hartley_sum8(double v) {
#pragma clang fp contract(off)
    double s = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += __shfl(v, k, 8);
    return s;
}

__device__ __forceinline__ Hartley hartley8_group(double x, double y) {
#pragma clang fp contract(off)
    const double mx = hartley_sum8(x) / 8.0, my = hartley_sum8(y) / 8.0;
    const double ax = x - mx, ay = y - my;
    const double d = hartley_sum8(sqrt(ax * ax + ay * ay));
    Hartley h;
    h.s = 1.4142135623730951 / (d / 8.0 + 1e-8);
    h.ox = -h.s * mx;
    h.oy = -h.s * my;
    return h;
}

__device__ __forceinline__ void f8_points_group8(double px, double py, double qx, double qy, double *F_out) {
#pragma clang fp contract(off)
    const int i = threadIdx.x & 7;
    const Hartley h1 = hartley8_group(px, py), h2 = hartley8_group(qx, qy);
    double A[9];
    {
        const double a = h1.s * px + h1.ox, b = h1.s * py + h1.oy;
        const double c = h2.s * qx + h2.ox, d = h2.s * qy + h2.oy;
        A[0] = a * c; A[1] = a * d; A[2] = a;
        A[3] = b * c; A[4] = b * d; A[5] = b;
        A[6] = c; A[7] = d; A[8] = 1.0;
    }
    double tau = 0;  // this lane's reflector (row i)
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        if (i == k) {
            double nrm2 = 0;
#pragma unroll
            for (int j = k; j < 9; ++j) nrm2 += A[j] * A[j];
            const double nrm = sqrt(nrm2);
            const double alpha = A[k] > 0 ? -nrm : nrm;
            A[k] -= alpha;
            double vtv = 0;
#pragma unroll
            for (int j = k; j < 9; ++j) vtv += A[j] * A[j];
            tau = nrm2 > 0 ? 2.0 / vtv : 0.0;
        }
        double v[9];
#pragma unroll
        for (int j = k; j < 9; ++j) v[j] = __shfl(A[j], k, 8);
        const double tk = __shfl(tau, k, 8);
        if (i > k) {
            double d = 0;
#pragma unroll
            for (int j = k; j < 9; ++j) d += A[j] * v[j];
            d *= tk;
#pragma unroll
            for (int j = k; j < 9; ++j) A[j] -= d * v[j];
        }
    }
    double n[9];
#pragma unroll
    for (int j = 0; j < 9; ++j) n[j] = (j == 8) ? 1.0 : 0.0;
#pragma unroll
    for (int k = 7; k >= 0; --k) {
        double v[9];
#pragma unroll
        for (int j = k; j < 9; ++j) v[j] = __shfl(A[j], k, 8);
        const double tk = __shfl(tau, k, 8);
        double d = 0;
#pragma unroll
        for (int j = k; j < 9; ++j) d += v[j] * n[j];
        d *= tk;
#pragma unroll
        for (int j = k; j < 9; ++j) n[j] -= d * v[j];
    }
    f8_finish(n, h1, h2, F_out, i);
}

// ------------------------------------------------------------ homography
// find_homography (GetHomographyInliers.py:4-85).  numpy's 3x3 @ 3xN and
// 3x3 @ 3x3 products run through OpenBLAS dgemm, whose accumulation is an
// FMA chain acc = a0*b0; acc = fma(a1, b1, acc); acc = fma(a2, b2, acc)
// (measured against exact arithmetic, see tests/golden/make_golden.py);
// the code below states those fma() calls explicitly and keeps every other
// operation uncontracted.

// Hartley-style normalisation of K points (:27-42): centroid, then
// scale = sqrt(2) / (mean distance + 1e-8); x' = s x + ox
template <int K>
__device__ __forceinline__ Hartley hartley_k(const double (&x)[K], const double (&y)[K]) {
#pragma clang fp contract(off)
    double mx = 0, my = 0;
#pragma unroll
    for (int i = 0; i < K; ++i) { mx += x[i]; my += y[i]; }
    mx = mx / (double)K;
    my = my / (double)K;
    double d = 0;
#pragma unroll
    for (int i = 0; i < K; ++i) {
        const double ax = x[i] - mx, ay = y[i] - my;
        d += sqrt(ax * ax + ay * ay);
    }
    Hartley h;
    h.s = 1.4142135623730951 / (d / (double)K + 1e-8);
    h.ox = -h.s * mx;
    h.oy = -h.s * my;
    return h;
}

// C = A @ B, 3x3 row-major, dgemm accumulation order
__device__ __forceinline__ void mm3_blas(const double (&A)[3][3], const double (&B)[3][3], double (&C)[3][3]) {
#pragma clang fp contract(off)
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) C[r][c] = fma(A[r][2], B[2][c], fma(A[r][1], B[1][c], A[r][0] * B[0][c]));
}

// H = inv(T2) @ Hn @ T1, H / H[2,2] (:79-83).  inv(T2) as LAPACK getri
// forms it for this upper-triangular T2: 1/s on the diagonal and
// -(o * (1/s)) in the last column.
__device__ __forceinline__ void h_finish(const double (&n)[9], const Hartley &h1, const Hartley &h2, double *H_out) {
#pragma clang fp contract(off)
    const double is = 1.0 / h2.s;
    const double Ti[3][3] = {{is, -0.0, -(h2.ox * is)}, {0.0, is, -(h2.oy * is)}, {0.0, 0.0, 1.0}};
    const double Hn[3][3] = {{n[0], n[1], n[2]}, {n[3], n[4], n[5]}, {n[6], n[7], n[8]}};
    const double T1[3][3] = {{h1.s, 0.0, h1.ox}, {0.0, h1.s, h1.oy}, {0.0, 0.0, 1.0}};
    double M[3][3], G[3][3];
    mm3_blas(Ti, Hn, M);
    mm3_blas(M, T1, G);
    const double d = G[2][2];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) H_out[r * 3 + c] = G[r][c] / d;
}

// The two DLT rows of one normalised correspondence (:59-71)
__device__ __forceinline__ void h_rows(double a, double b, double c, double d, double (&r0)[9], double (&r1)[9]) {
#pragma clang fp contract(off)
    r0[0] = 0.0; r0[1] = 0.0; r0[2] = 0.0; r0[3] = -a; r0[4] = -b; r0[5] = -1.0;
    r0[6] = d * a; r0[7] = d * b; r0[8] = d;
    r1[0] = a; r1[1] = b; r1[2] = 1.0; r1[3] = 0.0; r1[4] = 0.0; r1[5] = 0.0;
    r1[6] = -c * a; r1[7] = -c * b; r1[8] = -c;
}

// 4-point homography: 8 x 9 DLT system, LQ null vector, denormalisation
__device__ __forceinline__ void h4_points(const double (&x1)[4], const double (&y1)[4], const double (&x2)[4],
                                          const double (&y2)[4], double *H_out) {
#pragma clang fp contract(off)
    const Hartley h1 = hartley_k<4>(x1, y1), h2 = hartley_k<4>(x2, y2);
    double A[8][9];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const double a = h1.s * x1[i] + h1.ox, b = h1.s * y1[i] + h1.oy;
        const double c = h2.s * x2[i] + h2.ox, d = h2.s * y2[i] + h2.oy;
        h_rows(a, b, c, d, A[2 * i], A[2 * i + 1]);
    }
    double n[9];
    null_vector_8x9(A, n);
    h_finish(n, h1, h2, H_out);
}

// get_homography_inliers' test (GetHomographyInliers.py:134-146):
// t = H [x y 1]^T; (u, v) = t[:2] / (t[2] + 1e-8); |(u, v) - x2| < thr
__device__ __forceinline__ bool hom_inlier(const double *H, double x, double y, double u, double v, double thr) {
#pragma clang fp contract(off)
    const double t0 = fma(H[1], y, H[0] * x) + H[2];
    const double t1 = fma(H[4], y, H[3] * x) + H[5];
    const double t2 = fma(H[7], y, H[6] * x) + H[8];
    const double w = t2 + 1e-8;
    const double d0 = t0 / w - u, d1 = t1 / w - v;
    return sqrt(d0 * d0 + d1 * d1) < thr;
}

// The same decision, cheaper: 1/w from v_rcp_f64 and two Newton steps
// (relative error far below 1e-12), the transfer error squared without the
// two IEEE divides and the square root, compared against the threshold
// widened by a bound E on how far the exact expression can sit from this one
// (|d - d_fast| <= (|t/w| + |u|) 3e-12 per coordinate, plus 1e-9 relative for
// the exact path's own rounding).  Pairs inside that band, and any NaN, take
// the exact expression (hom_exact on the same t0, t1, w): every decision is
// the reference's.
struct HomPart {
    double t0, t1, w;
    bool in, unsure;
};

__device__ __forceinline__ HomPart hom_fast(const double *H, double x, double y, double u, double v, double thr) {
    HomPart r;
    {
#pragma clang fp contract(off)
        r.t0 = fma(H[1], y, H[0] * x) + H[2];
        r.t1 = fma(H[4], y, H[3] * x) + H[5];
        const double t2 = fma(H[7], y, H[6] * x) + H[8];
        r.w = t2 + 1e-8;
    }
    double iw = __builtin_amdgcn_rcp(r.w);
    iw = fma(iw, fma(-r.w, iw, 1.0), iw);
    iw = fma(iw, fma(-r.w, iw, 1.0), iw);
    const double ua = r.t0 * iw, va = r.t1 * iw;
    const double d0 = ua - u, d1 = va - v;
    const double s2 = d0 * d0 + d1 * d1;
    const double E = (fabs(ua) + fabs(u) + fabs(va) + fabs(v)) * 3e-12;
    const double lo = thr * (1.0 - 1e-9) - E, hi = thr * (1.0 + 1e-9) + E;
    const bool sure_in = lo > 0.0 && s2 < lo * lo;
    const bool sure_out = hi > 0.0 && s2 > hi * hi;
    r.in = sure_in;
    r.unsure = !(sure_in || sure_out) || thr < 0.0;
    return r;
}

__device__ __forceinline__ bool hom_exact(const HomPart &r, double u, double v, double thr) {
#pragma clang fp contract(off)
    const double d0 = r.t0 / r.w - u, d1 = r.t1 / r.w - v;
    return sqrt(d0 * d0 + d1 * d1) < thr;
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
