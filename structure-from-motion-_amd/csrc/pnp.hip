// PnP on gfx950: LinearPnP (LinearPnP.py:3-96),
// PnPRANSAC (PnPRANSAC.py:6-89) and NonlinearPnP (NonlinearPnP.py:5-151).
//
//   k_pnp_fit      one thread per 4-point hypothesis: the 8 x 12 DLT system
//                  and the null vector np.linalg.svd returns for it (its
//                  4-D null space makes Vt[-1] a property of LAPACK dgesdd's
//                  path: the product of dgebd2's right reflectors applied to
//                  e_12 -- emulated here in registers), then LinearPnP's
//                  post-processing (det sign, QR of M^T, scale, orthogonal
//                  projection), the pose and its 3x4 projection.
//   k_pnp_score    one wave per hypothesis; correspondences (X, Y, Z, u, v)
//                  staged in LDS tiles; ballot popcount of err < thr.
//   k_pnp_select   strict-max / earliest-iteration winner.
//   k_pnp_general  LinearPnP on all N points (one wave): Givens QR of the
//                  2N x 12 system to 12 x 12, Jacobi SVD for the (unique,
//                  N >= 6) null vector; N = 4, 5 take the dgebd2 path.
//   k_nonlinear_pnp one 512-thread workgroup per problem: MINPACK lmdif
//                  (scipy 'lm', forward differences, max_nfev) on the
//                  2N-residual loss; the Jacobian rows stay in registers and
//                  are reduced to their 6 x 6 R factor by CholeskyQR2, then
//                  qrfac (column pivoting) and lmpar run on lane 0.
//
// numpy evaluates the small products through OpenBLAS; the operation orders
// used here are the measured ones (oracle/sfm_oracle_pnp.c header), with FP
// contraction off (lm_small.hpp) and explicit fma() where BLAS fuses.
#include <cstring>

#include "lm_small.hpp"
#include "sfm_common.hpp"
#include "select.hpp"

namespace sfm {

struct Cam3 {
    double k[9];
};

// ------------------------------------------------------------ LAPACK bits
__device__ __forceinline__ double dlapy2_d(double x, double y) {
    const double xa = fabs(x), ya = fabs(y);
    const double w = xa > ya ? xa : ya, z = xa < ya ? xa : ya;
    if (z == 0.0) return w;
    const double q = z / w;
    return w * sqrt(1.0 + q * q);
}

// dlarfg on (alpha; x[0..n-2]) held in registers; returns tau, rewrites
// alpha := beta and x := v tail
template <int L>
__device__ __forceinline__ double dlarfg_d(int n, double &alpha, double (&x)[L], int lo) {
    // x[lo .. lo+n-2] is the vector below/right of alpha
    if (n <= 1) return 0.0;
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < L; ++i)
        if (i >= lo && i < lo + n - 1) s += x[i] * x[i];
    const double xnorm = sqrt(s);
    if (xnorm == 0.0) return 0.0;
    const double beta = -copysign(dlapy2_d(alpha, xnorm), alpha);
    const double tau = (beta - alpha) / beta;
    const double sc = 1.0 / (alpha - beta);
#pragma unroll
    for (int i = 0; i < L; ++i)
        if (i >= lo && i < lo + n - 1) x[i] *= sc;
    alpha = beta;
    return tau;
}

// ----------------------------------------------- LinearPnP post-processing
__device__ __forceinline__ double det3_d(const double (&M)[9]) {
    return M[0] * (M[4] * M[8] - M[5] * M[7]) - M[1] * (M[3] * M[8] - M[5] * M[6]) +
           M[2] * (M[3] * M[7] - M[4] * M[6]);
}

// column-major 3x3 Householder step on column i of a[col][row]
__device__ __forceinline__ double house_col(double (&a)[3][3], int i) {
    double alpha = a[i][i];
    double x[3] = {a[i][0], a[i][1], a[i][2]};
    const double tau = dlarfg_d<3>(3 - i, alpha, x, i + 1);
    a[i][i] = alpha;
#pragma unroll
    for (int r = 0; r < 3; ++r)
        if (r > i) a[i][r] = x[r];
    return tau;
}

// apply (I - tau v v^T), v = (.., 1 at i, a[i][i+1..]), to columns c > i
__device__ __forceinline__ void house_apply_left(double (&a)[3][3], int i, double tau) {
    const double aii = a[i][i];
    a[i][i] = 1.0;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        if (c <= i) continue;
        double w = 0;
#pragma unroll
        for (int r = 0; r < 3; ++r)
            if (r >= i) w += a[i][r] * a[c][r];
#pragma unroll
        for (int r = 0; r < 3; ++r)
            if (r >= i) a[c][r] -= tau * a[i][r] * w;
    }
    a[i][i] = aii;
}

// LAPACK-path emulation of R := U diag(1,1,-1) Vt for an orthogonal R with
// det < 0 (LinearPnP.py:84-87); see oracle/sfm_oracle_pnp.c flip_last_singular
__device__ void flip_last_singular_d(double (&R)[9]) {
    double a[3][3];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) a[c][r] = R[r * 3 + c];
    double tauq[3], d[3], taup0 = 0.0;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        tauq[i] = house_col(a, i);
        d[i] = a[i][i];
        house_apply_left(a, i, tauq[i]);
        if (i == 0) {  // G(0) on row 0, columns 1..2
            double alpha = a[1][0];
            double x[3] = {0.0, 0.0, a[2][0]};
            taup0 = dlarfg_d<3>(2, alpha, x, 2);
            a[1][0] = alpha;
            a[2][0] = x[2];
            const double e = a[1][0];
            a[1][0] = 1.0;
#pragma unroll
            for (int r = 1; r < 3; ++r) {
                double w = 0;
#pragma unroll
                for (int c = 1; c < 3; ++c) w += a[c][r] * a[c][0];
#pragma unroll
                for (int c = 1; c < 3; ++c) a[c][r] -= taup0 * w * a[c][0];
            }
            a[1][0] = e;
        }
    }
    double U[3][3], P[3][3];
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int r = 0; r < 3; ++r) { U[c][r] = r == c ? 1.0 : 0.0; P[c][r] = r == c ? 1.0 : 0.0; }
#pragma unroll
    for (int i = 1; i >= 0; --i) {
        double v[3] = {0, 0, 0};
        v[i] = 1.0;
#pragma unroll
        for (int r = 0; r < 3; ++r)
            if (r > i) v[r] = a[i][r];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            double w = 0;
#pragma unroll
            for (int r = 0; r < 3; ++r)
                if (r >= i) w += v[r] * U[c][r];
#pragma unroll
            for (int r = 0; r < 3; ++r)
                if (r >= i) U[c][r] -= tauq[i] * v[r] * w;
        }
    }
    {
        const double v[3] = {0.0, 1.0, a[2][0]};
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            double w = 0;
#pragma unroll
            for (int r = 1; r < 3; ++r) w += v[r] * P[c][r];
#pragma unroll
            for (int r = 1; r < 3; ++r) P[c][r] -= taup0 * v[r] * w;
        }
    }
    int ord[3] = {0, 1, 2};
    double sv[3], sg[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) { sg[i] = d[i] < 0 ? -1.0 : 1.0; sv[i] = fabs(d[i]); }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        int isub = 0;
        double smin = sv[ord[0]];
        for (int j = 1; j < 3 - i; ++j)
            if (sv[ord[j]] <= smin) { isub = j; smin = sv[ord[j]]; }
        if (isub != 2 - i) { const int t = ord[isub]; ord[isub] = ord[2 - i]; ord[2 - i] = t; }
    }
    const int k = ord[2];
    double u[3], w[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        u[r] = k == 0 ? U[0][r] : (k == 1 ? U[1][r] : U[2][r]);
        w[r] = sg[k] * (k == 0 ? P[0][r] : (k == 1 ? P[1][r] : P[2][r]));
    }
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) R[r * 3 + c] -= 2.0 * u[r] * w[c];
}

// LinearPnP.py:61-96 from the null vector p (P = p.reshape(3, 4)).
// Returns the LAPACK-noise branch flag.
__device__ int pnp_post(const double (&p)[12], double (&C)[3], double (&R)[9]) {
    double M[9] = {p[0], p[1], p[2], p[4], p[5], p[6], p[8], p[9], p[10]};
    double t[3] = {p[3], p[7], p[11]};
    if (det3_d(M) < 0) {
#pragma unroll
        for (int k = 0; k < 9; ++k) M[k] = -M[k];
#pragma unroll
        for (int k = 0; k < 3; ++k) t[k] = -t[k];
    }
    double a[3][3];  // M^T, column-major: a[c][r] = M^T[r][c] = M[c][r]
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int r = 0; r < 3; ++r) a[c][r] = M[c * 3 + r];
    double tau[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        tau[i] = house_col(a, i);
        house_apply_left(a, i, tau[i]);
    }
    double q[3][3];  // Q = H0 H1 H2 I, q[col][row]
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int r = 0; r < 3; ++r) q[c][r] = r == c ? 1.0 : 0.0;
#pragma unroll
    for (int i = 2; i >= 0; --i) {
        double v[3] = {0, 0, 0};
        v[i] = 1.0;
#pragma unroll
        for (int r = 0; r < 3; ++r)
            if (r > i) v[r] = a[i][r];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            double w = 0;
#pragma unroll
            for (int r = 0; r < 3; ++r)
                if (r >= i) w += v[r] * q[c][r];
#pragma unroll
            for (int r = 0; r < 3; ++r)
                if (r >= i) q[c][r] -= tau[i] * v[r] * w;
        }
    }
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) R[r * 3 + c] = q[r][c];  // R = Q.T
    double scale = ((a[0][0] + a[1][1]) + a[2][2]) / 3.0;
    if (scale < 0) {
#pragma unroll
        for (int k = 0; k < 9; ++k) R[k] = -R[k];
        scale = -scale;
    }
    int branch = 0;
    if (det3_d(R) < 0) {
        flip_last_singular_d(R);
        branch = 1;
    }
    const double tn[3] = {t[0] / scale, t[1] / scale, t[2] / scale};
#pragma unroll
    for (int i = 0; i < 3; ++i) C[i] = fma(-R[6 + i], tn[2], fma(-R[3 + i], tn[1], (-R[i]) * tn[0]));
    return branch;
}

// normalised image point: inv(K) @ [u, v, 1] (LinearPnP.py:36-39)
__device__ __forceinline__ void pnp_xn(const Cam3 &K, double u, double v, double &xn, double &yn) {
    const double i0 = 1.0 / K.k[0], i4 = 1.0 / K.k[4];
    const double k02 = -(K.k[2] * i0), k12 = -(K.k[5] * i4);
    xn = fma(k02, 1.0, fma(-0.0, v, i0 * u));
    yn = fma(k12, 1.0, fma(i4, v, 0.0 * u));
}

__device__ __forceinline__ void pnp_rows(double Xw, double Yw, double Zw, double xn, double yn, double (&r0)[12],
                                         double (&r1)[12]) {
    r0[0] = Xw; r0[1] = Yw; r0[2] = Zw; r0[3] = 1.0; r0[4] = 0.0; r0[5] = 0.0; r0[6] = 0.0; r0[7] = 0.0;
    r0[8] = -xn * Xw; r0[9] = -xn * Yw; r0[10] = -xn * Zw; r0[11] = -xn;
    r1[0] = 0.0; r1[1] = 0.0; r1[2] = 0.0; r1[3] = 0.0; r1[4] = Xw; r1[5] = Yw; r1[6] = Zw; r1[7] = 1.0;
    r1[8] = -yn * Xw; r1[9] = -yn * Yw; r1[10] = -yn * Zw; r1[11] = -yn;
}

// Vt[-1] of np.linalg.svd for an MR x 12 system, MR < 12 (dgesdd path 5t)
template <int MR>
__device__ void pnp_null_small(double (&A)[MR][12], double (&v)[12]) {
    double taup[MR];
#pragma unroll
    for (int i = 0; i < MR; ++i) {
        // G(i): annihilate A[i][i+1..11]
        double alpha = A[i][i];
        taup[i] = dlarfg_d<12>(12 - i, alpha, A[i], i + 1);
        const double d = alpha;
        A[i][i] = 1.0;
#pragma unroll
        for (int r = i + 1; r < MR; ++r) {
            double w = 0;
#pragma unroll
            for (int j = i; j < 12; ++j) w += A[r][j] * A[i][j];
#pragma unroll
            for (int j = i; j < 12; ++j) A[r][j] -= taup[i] * w * A[i][j];
        }
        A[i][i] = d;
        if (i < MR - 1) {
            // H(i): annihilate A[i+2..MR-1][i]
            double col[MR];
#pragma unroll
            for (int r = 0; r < MR; ++r) col[r] = A[r][i];
            double alpha2 = col[i + 1];
            const double tauq = dlarfg_d<MR>(MR - i - 1, alpha2, col, i + 2);
            const double e = alpha2;
#pragma unroll
            for (int r = i + 2; r < MR; ++r) A[r][i] = col[r];
            A[i + 1][i] = 1.0;
#pragma unroll
            for (int c = i + 1; c < 12; ++c) {
                double w = 0;
#pragma unroll
                for (int r = i + 1; r < MR; ++r) w += A[r][i] * A[r][c];
#pragma unroll
                for (int r = i + 1; r < MR; ++r) A[r][c] -= tauq * A[r][i] * w;
            }
            A[i + 1][i] = e;
        }
    }
#pragma unroll
    for (int j = 0; j < 12; ++j) v[j] = j == 11 ? 1.0 : 0.0;
#pragma unroll
    for (int i = MR - 1; i >= 0; --i) {
        double w = v[i];
#pragma unroll
        for (int j = i + 1; j < 12; ++j) w += A[i][j] * v[j];
        v[i] -= taup[i] * w;
#pragma unroll
        for (int j = i + 1; j < 12; ++j) v[j] -= taup[i] * w * A[i][j];
    }
}

template <int NP>
__device__ int pnp_small(const double (&Xw)[NP][3], const double (&xs)[NP][2], const Cam3 &K, double (&C)[3],
                         double (&R)[9]) {
    double A[2 * NP][12];
#pragma unroll
    for (int i = 0; i < NP; ++i) {
        double xn, yn;
        pnp_xn(K, xs[i][0], xs[i][1], xn, yn);
        pnp_rows(Xw[i][0], Xw[i][1], Xw[i][2], xn, yn, A[2 * i], A[2 * i + 1]);
    }
    double p[12];
    pnp_null_small<2 * NP>(A, p);
    return pnp_post(p, C, R);
}

// P = K @ hstack([R, -R @ C.reshape(3, 1)]) in numpy's orders
__device__ __forceinline__ void pnp_projection(const Cam3 &K, const double (&C)[3], const double (&R)[9],
                                               double *P) {
    double B[12];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        const double a0 = -R[r * 3], a1 = -R[r * 3 + 1], a2 = -R[r * 3 + 2];
        B[r * 4 + 3] = fma(a2, C[2], fma(a0, C[0], a1 * C[1]));
#pragma unroll
        for (int c = 0; c < 3; ++c) B[r * 4 + c] = R[r * 3 + c];
    }
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c)
            P[r * 4 + c] = fma(K.k[r * 3 + 2], B[8 + c], fma(K.k[r * 3 + 1], B[4 + c], K.k[r * 3] * B[c]));
}

__device__ __forceinline__ void pnp_project(const double *P, double X, double Y, double Z, double &u, double &v) {
    const double h0 = fma(P[3], 1.0, fma(P[2], Z, fma(P[1], Y, P[0] * X)));
    const double h1 = fma(P[7], 1.0, fma(P[6], Z, fma(P[5], Y, P[4] * X)));
    const double h2 = fma(P[11], 1.0, fma(P[10], Z, fma(P[9], Y, P[8] * X)));
    const double w = h2 + 1e-8;
    u = h0 / w;
    v = h1 / w;
}

// --------------------------------------------------------------- RANSAC
constexpr int PNP_MODEL = 24;  // P (12) | C (3) | R (9)
constexpr int PNP_WAVES = 8;
constexpr int PNP_TILE = 1024;

__global__ void __launch_bounds__(64) k_pnp_fit(const double *__restrict__ X, const double2 *__restrict__ x,
                                                const int32_t *__restrict__ samples, int64_t H, Cam3 K,
                                                double *__restrict__ models, int32_t *__restrict__ branch) {
    const int64_t h = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (h >= H) return;
    double Xw[4][3], xs[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int32_t s = samples[h * 4 + i];
        Xw[i][0] = X[3 * s]; Xw[i][1] = X[3 * s + 1]; Xw[i][2] = X[3 * s + 2];
        const double2 q = x[s];
        xs[i][0] = q.x; xs[i][1] = q.y;
    }
    double C[3], R[9];
    const int br = pnp_small<4>(Xw, xs, K, C, R);
    double *m = models + PNP_MODEL * h;
    pnp_projection(K, C, R, m);
#pragma unroll
    for (int k = 0; k < 3; ++k) m[12 + k] = C[k];
#pragma unroll
    for (int k = 0; k < 9; ++k) m[15 + k] = R[k];
    if (branch) branch[h] = br;
}

__device__ __forceinline__ bool pnp_inlier(const double *P, double X, double Y, double Z, double u, double v,
                                           double thr) {
    double pu, pv;
    pnp_project(P, X, Y, Z, pu, pv);
    const double du = u - pu, dv = v - pv;
    return sqrt(du * du + dv * dv) < thr;
}

// The same decision, cheaper (as hom_fast, sfm_geom.hpp): 1/w by v_rcp_f64
// and two Newton steps, the squared reprojection error against the threshold
// widened by E = (|h0/w| + |u| + |h1/w| + |v|) 3e-12 and 1e-9 relative; the
// band, NaN and thr < 0 take pnp_exact, pnp_inlier's expression on the same
// h0, h1, w.
struct PnpPart {
    double h0, h1, w;
    bool in, unsure;
};

__device__ __forceinline__ PnpPart pnp_fast(const double *P, double X, double Y, double Z, double u, double v,
                                            double thr) {
    PnpPart r;
    r.h0 = fma(P[3], 1.0, fma(P[2], Z, fma(P[1], Y, P[0] * X)));
    r.h1 = fma(P[7], 1.0, fma(P[6], Z, fma(P[5], Y, P[4] * X)));
    const double h2 = fma(P[11], 1.0, fma(P[10], Z, fma(P[9], Y, P[8] * X)));
    r.w = h2 + 1e-8;
    double iw = __builtin_amdgcn_rcp(r.w);
    iw = fma(iw, fma(-r.w, iw, 1.0), iw);
    iw = fma(iw, fma(-r.w, iw, 1.0), iw);
    const double pu = r.h0 * iw, pv = r.h1 * iw;
    const double du = u - pu, dv = v - pv;
    const double s2 = du * du + dv * dv;
    const double E = (fabs(pu) + fabs(u) + fabs(pv) + fabs(v)) * 3e-12;
    const double lo = thr * (1.0 - 1e-9) - E, hi = thr * (1.0 + 1e-9) + E;
    const bool sure_in = lo > 0.0 && s2 < lo * lo;
    const bool sure_out = hi > 0.0 && s2 > hi * hi;
    r.in = sure_in;
    r.unsure = !(sure_in || sure_out) || thr < 0.0;
    return r;
}

__device__ __forceinline__ bool pnp_exact(const PnpPart &r, double u, double v, double thr) {
    const double pu = r.h0 / r.w, pv = r.h1 / r.w;
    const double du = u - pu, dv = v - pv;
    return sqrt(du * du + dv * dv) < thr;
}

__global__ void __launch_bounds__(64 * PNP_WAVES) k_pnp_score(const double *__restrict__ X,
                                                              const double2 *__restrict__ x, int64_t N,
                                                              const double *__restrict__ models, int64_t H,
                                                              double thr, int32_t *__restrict__ counts) {
    __shared__ double sX[PNP_TILE * 3];
    __shared__ double2 sx[PNP_TILE];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t h = (int64_t)blockIdx.x * PNP_WAVES + wave;
    const bool active = h < H;
    double P[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) P[k] = active ? models[PNP_MODEL * h + k] : 0.0;
    int cnt = 0;
    for (int64_t base = 0; base < N; base += PNP_TILE) {
        const int n = (int)min<int64_t>(PNP_TILE, N - base);
        for (int i = threadIdx.x; i < 3 * n; i += blockDim.x) sX[i] = X[3 * base + i];
        for (int i = threadIdx.x; i < n; i += blockDim.x) sx[i] = x[base + i];
        __syncthreads();
        if (active) {
            int j = 0;
            for (; j + 128 <= n; j += 128) {  // two points per lane per pass: independent FP64 chains
                const int i0 = j + lane, i1 = i0 + 64;
                const double2 q0 = sx[i0], q1 = sx[i1];
                // both fast decisions before either branch to the exact tail
                const PnpPart r0 = pnp_fast(P, sX[3 * i0], sX[3 * i0 + 1], sX[3 * i0 + 2], q0.x, q0.y, thr);
                const PnpPart r1 = pnp_fast(P, sX[3 * i1], sX[3 * i1 + 1], sX[3 * i1 + 2], q1.x, q1.y, thr);
                bool in0 = r0.in, in1 = r1.in;
                if (r0.unsure) in0 = pnp_exact(r0, q0.x, q0.y, thr);
                if (r1.unsure) in1 = pnp_exact(r1, q1.x, q1.y, thr);
                cnt += __popcll(__ballot(in0)) + __popcll(__ballot(in1));
            }
            for (; j < n; j += 64) {
                const int i = j + lane;
                bool inl = false;
                if (i < n) {
                    const double2 q = sx[i];
                    inl = pnp_inlier(P, sX[3 * i], sX[3 * i + 1], sX[3 * i + 2], q.x, q.y, thr);
                }
                cnt += __popcll(__ballot(inl));
            }
        }
        __syncthreads();
    }
    if (active && lane == 0) counts[h] = cnt;
}

__global__ void __launch_bounds__(1024) k_pnp_select(const double *__restrict__ models,
                                                     const int32_t *__restrict__ counts, int64_t H,
                                                     int64_t *__restrict__ best_out, double *__restrict__ best_model) {
    __shared__ int32_t sc[1024 / 64];
    __shared__ int64_t sh[1024 / 64];
    int32_t bc;
    int64_t best;
    wg_select_best<1024>(counts, H, sc, sh, bc, best);
    if (threadIdx.x == 0) best_out[0] = best, best_out[1] = bc;
    if (best >= 0 && threadIdx.x < PNP_MODEL) best_model[threadIdx.x] = models[PNP_MODEL * best + threadIdx.x];
}

// ------------------------------------------------------ LinearPnP, all N
constexpr int PG_THREADS = 64;

__device__ __forceinline__ void givens_absorb12(double (&R)[12][12], double (&a)[12]) {
#pragma unroll
    for (int j = 0; j < 12; ++j) {
        if (a[j] != 0.0) {
            const double r = sqrt(R[j][j] * R[j][j] + a[j] * a[j]);
            const double c = R[j][j] / r, s = a[j] / r;
#pragma unroll
            for (int k = j; k < 12; ++k) {
                const double u = R[j][k], v = a[k];
                R[j][k] = c * u + s * v;
                a[k] = -s * u + c * v;
            }
        }
    }
}

// out: C (3) | R (9) | branch (as double)
__global__ void __launch_bounds__(PG_THREADS) k_pnp_general(const double *__restrict__ X,
                                                            const double2 *__restrict__ x, int64_t N, Cam3 K,
                                                            double *__restrict__ out) {
    __shared__ double Rs[PG_THREADS][78];
    __shared__ double Aj[12][12], Vj[12][12];
    const int t = threadIdx.x;
    double C[3], R[9];
    int br = 0;
    if (N < 6) {  // 8 or 10 rows: LAPACK's rank-deficient path, one lane
        if (t != 0) return;
        if (N == 4) {
            double Xw[4][3], xs[4][2];
            for (int i = 0; i < 4; ++i) {
                Xw[i][0] = X[3 * i]; Xw[i][1] = X[3 * i + 1]; Xw[i][2] = X[3 * i + 2];
                xs[i][0] = x[i].x; xs[i][1] = x[i].y;
            }
            br = pnp_small<4>(Xw, xs, K, C, R);
        } else {
            double Xw[5][3], xs[5][2];
            for (int i = 0; i < 5; ++i) {
                Xw[i][0] = X[3 * i]; Xw[i][1] = X[3 * i + 1]; Xw[i][2] = X[3 * i + 2];
                xs[i][0] = x[i].x; xs[i][1] = x[i].y;
            }
            br = pnp_small<5>(Xw, xs, K, C, R);
        }
    } else {
        double Rt[12][12];
#pragma unroll
        for (int i = 0; i < 12; ++i)
#pragma unroll
            for (int j = 0; j < 12; ++j) Rt[i][j] = 0.0;
        for (int64_t i = t; i < N; i += PG_THREADS) {
            double xn, yn, r0[12], r1[12];
            const double2 q = x[i];
            pnp_xn(K, q.x, q.y, xn, yn);
            pnp_rows(X[3 * i], X[3 * i + 1], X[3 * i + 2], xn, yn, r0, r1);
            givens_absorb12(Rt, r0);
            givens_absorb12(Rt, r1);
        }
        for (int w = PG_THREADS / 2; w > 0; w >>= 1) {
            if (t >= w && t < 2 * w) {
                int k = 0;
#pragma unroll
                for (int i = 0; i < 12; ++i)
#pragma unroll
                    for (int j = i; j < 12; ++j) Rs[t][k++] = Rt[i][j];
            }
            __syncthreads();
            if (t < w) {
#pragma unroll
                for (int i = 0; i < 12; ++i) {
                    double row[12];
#pragma unroll
                    for (int j = 0; j < 12; ++j) row[j] = j >= i ? Rs[t + w][i * 12 - i * (i - 1) / 2 + (j - i)] : 0.0;
                    givens_absorb12(Rt, row);
                }
            }
            __syncthreads();
        }
        if (t != 0) return;
        // one-sided Jacobi on the 12 x 12 factor (columns of Aj), in LDS
        for (int i = 0; i < 12; ++i)
            for (int j = 0; j < 12; ++j) { Aj[j][i] = Rt[i][j]; Vj[i][j] = i == j ? 1.0 : 0.0; }
        for (int sweep = 0; sweep < 60; ++sweep) {
            double off = 0.0;
            for (int pp = 0; pp < 11; ++pp)
                for (int qq = pp + 1; qq < 12; ++qq) {
                    double al = 0, be = 0, ga = 0;
                    for (int k = 0; k < 12; ++k) {
                        al += Aj[pp][k] * Aj[pp][k];
                        be += Aj[qq][k] * Aj[qq][k];
                        ga += Aj[pp][k] * Aj[qq][k];
                    }
                    if (ga == 0.0) continue;
                    const double rr = fabs(ga) / sqrt(al * be);
                    if (!(rr > 1e-15)) continue;
                    off = fmax(off, rr);
                    const double zeta = (be - al) / (2.0 * ga);
                    const double tt = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
                    const double cs = 1.0 / sqrt(1.0 + tt * tt), sn = cs * tt;
                    for (int k = 0; k < 12; ++k) {
                        const double a1 = Aj[pp][k], a2 = Aj[qq][k];
                        Aj[pp][k] = cs * a1 - sn * a2;
                        Aj[qq][k] = sn * a1 + cs * a2;
                        const double v1 = Vj[k][pp], v2 = Vj[k][qq];
                        Vj[k][pp] = cs * v1 - sn * v2;
                        Vj[k][qq] = sn * v1 + cs * v2;
                    }
                }
            if (off < 1e-15) break;
        }
        int b = 0;
        double bn = 1e300;
        for (int j = 0; j < 12; ++j) {
            double s = 0;
            for (int k = 0; k < 12; ++k) s += Aj[j][k] * Aj[j][k];
            if (s < bn) { bn = s; b = j; }
        }
        double p[12];
        for (int k = 0; k < 12; ++k) p[k] = Vj[k][b];
        br = pnp_post(p, C, R);
    }
    for (int k = 0; k < 3; ++k) out[k] = C[k];
    for (int k = 0; k < 9; ++k) out[3 + k] = R[k];
    out[12] = (double)br;
}

// ---------------------------------------------------------- NonlinearPnP
// scipy Rotation.from_rotvec(...).as_matrix() (quaternion path)
__device__ __forceinline__ void scipy_rotvec_to_R(const double *rv, double (&R)[9]) {
    const double x = rv[0], y = rv[1], z = rv[2];
    const double ang = sqrt(x * x + y * y + z * z);
    double sc;
    if (ang <= 1e-3) {
        const double a2 = ang * ang;
        sc = 0.5 - a2 / 48 + a2 * a2 / 3840;
    } else {
        sc = sin(ang / 2) / ang;
    }
    const double qx = sc * x, qy = sc * y, qz = sc * z, qw = cos(ang / 2);
    const double x2 = qx * qx, y2 = qy * qy, z2 = qz * qz, w2 = qw * qw;
    const double xy = qx * qy, zw = qz * qw, xz = qx * qz, yw = qy * qw, yz = qy * qz, xw = qx * qw;
    R[0] = x2 - y2 - z2 + w2; R[1] = 2 * (xy - zw);       R[2] = 2 * (xz + yw);
    R[3] = 2 * (xy + zw);     R[4] = -x2 + y2 - z2 + w2;  R[5] = 2 * (yz - xw);
    R[6] = 2 * (xz - yw);     R[7] = 2 * (yz + xw);       R[8] = -x2 - y2 + z2 + w2;
}

// scipy Rotation.from_matrix(R).as_rotvec()
__device__ __forceinline__ void scipy_R_to_rotvec(const double *R, double *w) {
    const double tr = R[0] + R[4] + R[8];
    double q[4];
    if (tr > R[0] && tr > R[4] && tr > R[8]) {
        q[3] = 1.0 + tr;
        q[0] = R[7] - R[5]; q[1] = R[2] - R[6]; q[2] = R[3] - R[1];
    } else {
        const int i = (R[0] >= R[4] && R[0] >= R[8]) ? 0 : (R[4] >= R[8] ? 1 : 2);
        const int j = (i + 1) % 3, k = (j + 1) % 3;
        double qq[3];
        qq[i] = 1.0 - tr + 2.0 * R[i * 4];
        qq[j] = R[j * 3 + i] + R[i * 3 + j];
        qq[k] = R[k * 3 + i] + R[i * 3 + k];
        q[0] = qq[0]; q[1] = qq[1]; q[2] = qq[2];
        q[3] = R[k * 3 + j] - R[j * 3 + k];
    }
    const double nq = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    for (int i = 0; i < 4; ++i) q[i] /= nq;
    if (q[3] < 0)
        for (int i = 0; i < 4; ++i) q[i] = -q[i];
    const double vn = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2]);
    const double ang = 2.0 * atan2(vn, q[3]);
    double sc;
    if (ang <= 1e-3) {
        const double a2 = ang * ang;
        sc = 2.0 + a2 / 12.0 + 7.0 * a2 * a2 / 2880.0;
    } else {
        sc = ang / sin(ang / 2.0);
    }
    w[0] = sc * q[0]; w[1] = sc * q[1]; w[2] = sc * q[2];
}

// pose parameters (rotvec, t) -> projection, NonLinearPnPLoss (:30-38)
__device__ void nlpnp_projection(const Cam3 &K, const double *p, double *P) {
    double R[9], C[3];
    scipy_rotvec_to_R(p, R);
#pragma unroll
    for (int i = 0; i < 3; ++i) C[i] = fma(-R[6 + i], p[5], fma(-R[3 + i], p[4], (-R[i]) * p[3]));
    pnp_projection(K, C, R, P);
}

// ---- NonlinearPnP: MINPACK lmdif (NonlinearPnP.py:98-123 via scipy 'lm')
// in one 512-thread workgroup.  The m = 2N residual rows never leave
// registers: each forward-difference Jacobian (fdjac2: the base and the six
// perturbed projections of every point, in one pass) is reduced to its
// 6 x 6 R factor and Q^T f by CholeskyQR2 -- pass 1 sums the Gram matrix
// J^T J (fixed-order block sums), R1 = chol; pass 2 recomputes the rows,
// q = J R1^-1, sums q^T q and q^T f, R2 = chol, R = R2 R1, Q^T f = R2^-T q^T f
// (orthogonal to working precision for cond(J) up to ~1e8).  When pass 1's
// Gram factor needs a diagonal shift (J numerically rank-deficient), a
// third pass runs (shifted CholeskyQR3); a shift, and a later pass whose
// Gram factor still fails (its factor kept as the identity), are reported
// in bits 8 and 9 of info (sfm_nonlinear_pnp).  MINPACK's
// qrfac with column pivoting then runs on R (6 x 6, lane 0): the trailing
// column norms it pivots on are invariant under Q, so it picks the pivots
// qrfac would pick on J.  lmpar, the trust region and the stopping tests are
// lmdif's (the same code as before), one trial evaluation per inner
// iteration (one pass + a block sum).
constexpr int NL2_THREADS = 512;  // 256 VGPRs per lane: the row pass holds 27 sums + two Jacobian rows
constexpr int NL2_WAVES = NL2_THREADS / 64;

// fixed-order block sum of NV values per thread; every thread gets the totals
template <int NV>
__device__ __forceinline__ void nl2_sum(double (&v)[NV], double (*red)[NV]) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        double x = v[k];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
        v[k] = x;
    }
    __syncthreads();  // the previous sum's readers are done with red
    if (lane == 0)
#pragma unroll
        for (int k = 0; k < NV; ++k) red[w][k] = v[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        double x = 0;
#pragma unroll
        for (int i = 0; i < NL2_WAVES; ++i) x += red[i][k];
        v[k] = x;
    }
}

// Several workgroups per problem (round 3): the rows are cut into nb
// contiguous slices, one per workgroup, and every workgroup runs the whole
// lmdif control flow itself on the same totals (the same operations on the
// same values, so the same decisions and bits everywhere; only block 0
// writes the result).  A row pass ends in a cross-workgroup all-gather of
// the per-workgroup sums: each block stores its totals (write-through, the
// parity-`seq` buffer), drains them, raises its flag to (epoch << 32) | seq;
// wave 0 polls the nb flags (one lane each), and every block sums the nb
// partials in block order.  Double buffering by the parity of seq is enough:
// a block reaches pass seq + 2 only after every block published seq + 1,
// i.e. after every block finished reading seq.  Polls are bounded (200 ms);
// a timeout raises the abort word and every block returns (info -2, the host
// reports an error) -- no wait can outlive it.
struct NlX {
    double *part;                // [2][NL_MAXWG][32] per-block totals by seq parity
    unsigned long long *flag;    // [NL_MAXWG] (epoch << 32) | seq of the block's last publication
    unsigned long long *abort_;  // = epoch once a poll has timed out
    unsigned long long epoch;
    long long limit;             // poll bound in s_memrealtime ticks; < 0: time out at once (test hook)
    int nb;
};
constexpr int NL_MAXWG = 64;
constexpr long long NL_POLL_LIMIT = 20000000;  // s_memrealtime ticks (100 MHz): 200 ms

__device__ __forceinline__ double nl_ldag(const double *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// nl2_sum, then (nb > 1) the all-gather over the blocks; false on an abort
template <int NV>
__device__ __forceinline__ bool nlx_sum(double (&v)[NV], double (*red)[NV], const NlX &X, unsigned &seq,
                                        double *xtot, int *xok) {
    nl2_sum<NV>(v, red);
    if (X.nb == 1) return true;
    ++seq;
    const int slot = seq & 1, lane = threadIdx.x & 63;
    const unsigned long long want = (X.epoch << 32) | seq;
    if (threadIdx.x == 0) {
        double *mine = X.part + ((size_t)slot * NL_MAXWG + blockIdx.x) * 32;
#pragma unroll
        for (int k = 0; k < NV; ++k) __hip_atomic_store(mine + k, v[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(X.flag + blockIdx.x, want, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (threadIdx.x < 64) {
        auto seen = [&]() {
            return lane >= X.nb ||
                   __hip_atomic_load(X.flag + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= want;
        };
        bool done = seen(), ab = false;
        long long t0 = -1;
        if (X.limit < 0) {  // SFM_NLPNP_FORCE_TIMEOUT: this hand-off times out
            if (lane == 0) __hip_atomic_store(X.abort_, X.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            ab = true;
            done = true;
        }
        for (unsigned it = 1; !__all(done); ++it) {  // wave-uniform loop
            __builtin_amdgcn_s_sleep(1);
            if (!done) done = seen();
            if (it % 128 == 0) {
                bool a = __hip_atomic_load(X.abort_, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == X.epoch;
                const long long t = __builtin_amdgcn_s_memrealtime();
                if (t0 < 0) t0 = t;
                else if (t - t0 > X.limit) {
                    a = true;
                    if (lane == 0)
                        __hip_atomic_store(X.abort_, X.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                if (__any(a)) {
                    ab = true;
                    break;
                }
            }
        }
        if (lane == 0) *xok = !ab;
    }
    __syncthreads();
    if (!*xok) return false;
    if (threadIdx.x < NV) {
        const double *col = X.part + (size_t)slot * NL_MAXWG * 32 + threadIdx.x;
        double s = 0.0;
        for (int w = 0; w < X.nb; ++w) s += nl_ldag(col + w * 32);
        xtot[threadIdx.x] = s;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] = xtot[k];
    return true;
}

// Cholesky of a 6 x 6 SPD matrix given as its upper triangle (21, row-major
// packed); R upper with R^T R = G.  false on a non-positive pivot.
__device__ __forceinline__ bool chol6(const double *G, double (&R)[6][6]) {
    double A[6][6];
    int u = 0;
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
        for (int j = i; j < 6; ++j) { A[i][j] = G[u++]; A[j][i] = A[i][j]; }
    bool ok = true;
#pragma unroll
    for (int j = 0; j < 6; ++j) {
        double d = A[j][j];
#pragma unroll
        for (int k = 0; k < j; ++k) d -= R[k][j] * R[k][j];
        ok = ok && d > 0.0;
        d = sqrt(d);
        R[j][j] = d;
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            if (i < j) R[j][i] = 0.0;
            if (i <= j) continue;
            double v = A[j][i];
#pragma unroll
            for (int k = 0; k < j; ++k) v -= R[k][j] * R[k][i];
            R[j][i] = v / d;
        }
    }
    return ok;
}

struct NlShared {
    double p[6], pt[6], sP[7][12], R1[6][6];
    double g[28];  // Gram sums; [21..27) pass 2's 1 / R1[j][j]
    double rdiag[6], acnorm[6], wa1[6], wa3[6], qtf[6];
    double r6[6][6];  // upper triangle of the pivoted QR factor, column-major r6[col][row]
    double par, delta, xnorm, fnorm, gnorm, ratio, temp;
    int ipvt[6], info, nfev, iter, flag, npass, qrflags;
};

// Residual rows of point i under projection P: f = (x - proj).flatten()
// (one reciprocal of w instead of two divides: the rows are within an ulp
// of numpy's, and the row passes are FP64-throughput bound on one CU)
__device__ __forceinline__ void nl2_res(const double *P, double X, double Y, double Z, double2 q, double &f0,
                                        double &f1) {
    const double h0 = fma(P[3], 1.0, fma(P[2], Z, fma(P[1], Y, P[0] * X)));
    const double h1 = fma(P[7], 1.0, fma(P[6], Z, fma(P[5], Y, P[4] * X)));
    const double h2 = fma(P[11], 1.0, fma(P[10], Z, fma(P[9], Y, P[8] * X)));
    const double iw = 1.0 / (h2 + 1e-8);
    f0 = q.x - h0 * iw;
    f1 = q.y - h1 * iw;
}
__device__ __forceinline__ void nl2_res(const double *P, const double *X, const double2 *x, int64_t i, double &f0,
                                        double &f1) {
    nl2_res(P, X[3 * i], X[3 * i + 1], X[3 * i + 2], x[i], f0, f1);
}

// nb = gridDim.x workgroups per problem (NlX above).  out: C (3) | R (9) |
// info (as double) | CholeskyQR flags, written by block 0
__global__ void __launch_bounds__(NL2_THREADS) k_nonlinear_pnp(const double *__restrict__ X,
                                                               const double2 *__restrict__ x, int64_t n, Cam3 K,
                                                               const double *__restrict__ C0,
                                                               const double *__restrict__ R0, int32_t maxfev,
                                                               double *__restrict__ out, NlX XG) {
    __shared__ NlShared S;
    __shared__ double red27[NL2_WAVES][27];
    __shared__ double red2[NL2_WAVES][2];
    __shared__ double red1[NL2_WAVES][1];
    __shared__ double xtot[32];
    __shared__ int xok;
    const int t = threadIdx.x;
    const bool lead = blockIdx.x == 0;
    const int64_t lo = n * blockIdx.x / gridDim.x, hi = n * (blockIdx.x + 1) / gridDim.x;  // this block's rows
    unsigned seq = 0;
    auto fail = [&]() {  // a cross-block hand-off timed out
        if (lead && t == 0) out[12] = -2.0;
    };
    if (t == 0) {
        if (lead) {
            for (int k = 0; k < 3; ++k) out[k] = C0[k];
            for (int k = 0; k < 9; ++k) out[3 + k] = R0[k];
            out[12] = 0.0;
            out[13] = 0.0;
        }
        S.flag = 0;
        S.qrflags = 0;
        if (n >= 4) {
            scipy_R_to_rotvec(R0, S.p);
            for (int i = 0; i < 3; ++i)
                S.p[3 + i] = fma(-R0[i * 3 + 2], C0[2], fma(-R0[i * 3], C0[0], (-R0[i * 3 + 1]) * C0[1]));
            for (int k = 0; k < 6; ++k)
                if (isnan(S.p[k])) S.flag = 1;
            nlpnp_projection(K, S.p, S.sP[0]);
        } else {
            S.flag = 2;
        }
    }
    __syncthreads();
    if (S.flag == 2) return;                                              // n < 4: C, R unchanged
    if (S.flag == 1) { if (lead && t == 0) out[12] = -1.0; return; }      // except path
    // initial residual norm and finiteness (one sum: {non-finite, |f|^2})
    {
        double v[2] = {0.0, 0.0};
        int fin = 1;
        for (int64_t i = lo + t; i < hi; i += NL2_THREADS) {
            double f0, f1;
            nl2_res(S.sP[0], X, x, i, f0, f1);
            fin &= (isfinite(f0) && isfinite(f1)) ? 1 : 0;
            v[1] += f0 * f0 + f1 * f1;
        }
        v[0] = (double)(1 - fin);
        if (!nlx_sum<2>(v, red2, XG, seq, xtot, &xok)) return fail();
        if (v[0] != 0.0) { if (lead && t == 0) out[12] = -1.0; return; }
        if (t == 0) {
            S.fnorm = sqrt(v[1]); S.par = 0.0; S.delta = 0.0; S.xnorm = 0.0; S.iter = 1; S.nfev = 1; S.info = 0;
        }
    }
    __syncthreads();
    const double eps = 1.4901161193847656e-08;
    for (;;) {
        // ---- fdjac2's seven projections: the base and p + h_j e_j
        double h[6], ih[6];
#pragma unroll
        for (int j = 0; j < 6; ++j) {
            h[j] = eps * fabs(S.p[j]);
            if (h[j] == 0.0) h[j] = eps;
            ih[j] = 1.0 / h[j];
        }
        if (t < 7) {
            double pp[6];
            for (int k = 0; k < 6; ++k) pp[k] = S.p[k];
            if (t > 0) pp[t - 1] = S.p[t - 1] + h[t - 1];
            nlpnp_projection(K, pp, S.sP[t]);
        }
        __syncthreads();
        // ---- pass 1: Gram matrix of the Jacobian rows
        double gsum[27];
#pragma unroll
        for (int k = 0; k < 27; ++k) gsum[k] = 0.0;
        for (int64_t i = lo + t; i < hi; i += NL2_THREADS) {
            double b0, b1, J0[6], J1[6];
            const double Xi = X[3 * i], Yi = X[3 * i + 1], Zi = X[3 * i + 2];
            const double2 qi = x[i];
            nl2_res(S.sP[0], Xi, Yi, Zi, qi, b0, b1);
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                double w0, w1;
                nl2_res(S.sP[1 + j], Xi, Yi, Zi, qi, w0, w1);
                J0[j] = (w0 - b0) * ih[j];
                J1[j] = (w1 - b1) * ih[j];
            }
            int u = 0;
#pragma unroll
            for (int a2 = 0; a2 < 6; ++a2)
#pragma unroll
                for (int c2 = a2; c2 < 6; ++c2) gsum[u++] += J0[a2] * J0[c2] + J1[a2] * J1[c2];
        }
        if (!nlx_sum<27>(gsum, red27, XG, seq, xtot, &xok)) return fail();
        if (t == 0) {
#pragma unroll
            for (int k = 0; k < 21; ++k) S.g[k] = gsum[k];
            double R1[6][6];
            S.npass = 2;
            if (!chol6(S.g, R1)) {  // numerically rank-deficient: shifted factor, passes 2 and 3 correct
                S.npass = 3;
                S.qrflags |= 1;
                double tr = 0;
                int u = 0;
                for (int a2 = 0; a2 < 6; ++a2)
                    for (int c2 = a2; c2 < 6; ++c2, ++u)
                        if (a2 == c2) tr += S.g[u];
                u = 0;
                for (int a2 = 0; a2 < 6; ++a2)
                    for (int c2 = a2; c2 < 6; ++c2, ++u)
                        if (a2 == c2) S.g[u] += 1e-12 * tr + 1e-300;
                if (!chol6(S.g, R1)) S.qrflags |= 2;
            }
#pragma unroll
            for (int a2 = 0; a2 < 6; ++a2) {
#pragma unroll
                for (int c2 = 0; c2 < 6; ++c2) S.R1[a2][c2] = R1[a2][c2];
                S.g[21 + a2] = 1.0 / R1[a2][a2];  // pivot reciprocals for pass 2
            }
        }
        __syncthreads();
        const int npass = S.npass;
        for (int pass = 2; pass <= npass; ++pass) {
        // ---- pass 2 (3): q = J R1^-1 rows (R1 read from LDS): q^T q and q^T f
#pragma unroll
        for (int k = 0; k < 27; ++k) gsum[k] = 0.0;
        for (int64_t i = lo + t; i < hi; i += NL2_THREADS) {
            double b0, b1, J0[6], J1[6];
            const double Xi = X[3 * i], Yi = X[3 * i + 1], Zi = X[3 * i + 2];
            const double2 qi = x[i];
            nl2_res(S.sP[0], Xi, Yi, Zi, qi, b0, b1);
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                double w0, w1;
                nl2_res(S.sP[1 + j], Xi, Yi, Zi, qi, w0, w1);
                J0[j] = (w0 - b0) * ih[j];
                J1[j] = (w1 - b1) * ih[j];
            }
            double q0[6], q1[6];
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                double a0 = J0[j], a1 = J1[j];
#pragma unroll
                for (int k = 0; k < j; ++k) { a0 -= q0[k] * S.R1[k][j]; a1 -= q1[k] * S.R1[k][j]; }
                q0[j] = a0 * S.g[21 + j];
                q1[j] = a1 * S.g[21 + j];
            }
            int u = 0;
#pragma unroll
            for (int a2 = 0; a2 < 6; ++a2)
#pragma unroll
                for (int c2 = a2; c2 < 6; ++c2) gsum[u++] += q0[a2] * q0[c2] + q1[a2] * q1[c2];
#pragma unroll
            for (int a2 = 0; a2 < 6; ++a2) gsum[21 + a2] += q0[a2] * b0 + q1[a2] * b1;
        }
        if (!nlx_sum<27>(gsum, red27, XG, seq, xtot, &xok)) return fail();
        if (t == 0 && pass < npass) {  // an intermediate pass: R1 <- R2 R1, then the next pass
            double R2[6][6];
            if (!chol6(gsum, R2)) {
                S.qrflags |= 2;
                for (int a2 = 0; a2 < 6; ++a2)
                    for (int c2 = 0; c2 < 6; ++c2) R2[a2][c2] = a2 == c2 ? 1.0 : 0.0;
            }
            double Rn[6][6];
            for (int i = 0; i < 6; ++i)
                for (int j = 0; j < 6; ++j) {
                    double v = 0;
                    for (int k = i; k <= j; ++k) v += R2[i][k] * S.R1[k][j];
                    Rn[i][j] = i <= j ? v : 0.0;
                }
            for (int i = 0; i < 6; ++i) {
                for (int j = 0; j < 6; ++j) S.R1[i][j] = Rn[i][j];
                S.g[21 + i] = 1.0 / Rn[i][i];
            }
        }
        if (pass < npass) {
            __syncthreads();
            continue;
        }
        if (t == 0) {
            double R2[6][6];
            if (!chol6(gsum, R2)) {  // cannot happen for a full-rank J; keep R1 (reported)
                S.qrflags |= 2;
                for (int a2 = 0; a2 < 6; ++a2)
                    for (int c2 = 0; c2 < 6; ++c2) R2[a2][c2] = a2 == c2 ? 1.0 : 0.0;
            }
            // R = R2 R1 (column-major a[col][row] for qrfac), Q^T f = R2^-T (q^T f)
            double a[6][6], qtu[6];
#pragma unroll
            for (int i = 0; i < 6; ++i)
#pragma unroll
                for (int j = 0; j < 6; ++j) {
                    double v = 0;
#pragma unroll
                    for (int k = 0; k < 6; ++k)
                        if (k >= i && k <= j) v += R2[i][k] * S.R1[k][j];
                    a[j][i] = i <= j ? v : 0.0;
                }
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                double v = gsum[21 + i];
#pragma unroll
                for (int k = 0; k < i; ++k) v -= R2[k][i] * qtu[k];
                qtu[i] = v / R2[i][i];
            }
            // ---- qrfac with column pivoting on R, Q'^T applied to Q^T f (lmdif's qtf loop)
            int ipvt[6];
            double rdiag[6], acnorm[6];
            lm::qrfac<6, 6>(a, ipvt, rdiag, acnorm);
            if (S.iter == 1) {
                double s3 = 0;
                for (int k = 0; k < 6; ++k) s3 += S.p[k] * S.p[k];
                S.xnorm = sqrt(s3);
                S.delta = 100.0 * S.xnorm;
                if (S.delta == 0.0) S.delta = 100.0;
            }
            double wa4[6];
            for (int i = 0; i < 6; ++i) wa4[i] = qtu[i];
            for (int j = 0; j < 6; ++j) {
                if (a[j][j] != 0.0) {
                    double sum = 0.0;
                    for (int i = j; i < 6; ++i) sum += a[j][i] * wa4[i];
                    const double temp = -sum / a[j][j];
                    for (int i = j; i < 6; ++i) wa4[i] += a[j][i] * temp;
                }
                a[j][j] = rdiag[j];
                S.qtf[j] = wa4[j];
            }
            for (int j = 0; j < 6; ++j) {
                S.ipvt[j] = ipvt[j];
                S.acnorm[j] = acnorm[j];
                for (int i = 0; i < 6; ++i) S.r6[j][i] = a[j][i];
            }
            S.nfev += 6;
            double gnorm = 0.0;
            if (S.fnorm != 0.0)
                for (int j = 0; j < 6; ++j) {
                    const double cn = S.acnorm[S.ipvt[j]];
                    if (cn != 0.0) {
                        double sum = 0.0;
                        for (int i = 0; i <= j; ++i) sum += S.r6[j][i] * (S.qtf[i] / S.fnorm);
                        const double g = fabs(sum / cn);
                        if (g > gnorm) gnorm = g;
                    }
                }
            S.gnorm = gnorm;
            if (gnorm <= 1e-8) S.info = 4;
        }
        }  // passes
        __syncthreads();
        if (S.info != 0) break;
        // ---- inner loop
        for (;;) {
            if (t == 0) {
                double r[6][6], qtb[6], xs[6], sd[6];
                int ipvt[6];
                for (int j = 0; j < 6; ++j) {
                    for (int i = 0; i < 6; ++i) r[j][i] = S.r6[j][i];
                    qtb[j] = S.qtf[j];
                    ipvt[j] = S.ipvt[j];
                }
                double par = S.par;
                lm::lmpar<6, 6>(r, ipvt, qtb, S.delta, par, xs, sd);
                S.par = par;
                for (int j = 0; j < 6; ++j) {
                    S.wa1[j] = -xs[j];
                    S.pt[j] = S.p[j] + S.wa1[j];
                    S.wa3[j] = S.wa1[j];
                }
                double s3 = 0;
                for (int j = 0; j < 6; ++j) s3 += S.wa3[j] * S.wa3[j];
                S.temp = sqrt(s3);  // pnorm
                if (S.iter == 1 && S.temp < S.delta) S.delta = S.temp;
                nlpnp_projection(K, S.pt, S.sP[0]);
            }
            __syncthreads();
            double v[1] = {0.0};
            for (int64_t i = lo + t; i < hi; i += NL2_THREADS) {
                double f0, f1;
                nl2_res(S.sP[0], X, x, i, f0, f1);
                v[0] += f0 * f0 + f1 * f1;
            }
            if (!nlx_sum<1>(v, red1, XG, seq, xtot, &xok)) return fail();
            const double fnorm1 = sqrt(v[0]);
            if (t == 0) {
                S.nfev += 1;
                const double pnorm = S.temp, fnorm = S.fnorm;
                double actred = -1.0;
                if (0.1 * fnorm1 < fnorm) {
                    const double tq = fnorm1 / fnorm;
                    actred = 1.0 - tq * tq;
                }
                double w3[6];
                for (int j = 0; j < 6; ++j) {
                    w3[j] = 0.0;
                    const double temp = S.wa1[S.ipvt[j]];
                    for (int i = 0; i <= j; ++i) w3[i] += S.r6[j][i] * temp;
                }
                double s5 = 0;
                for (int j = 0; j < 6; ++j) s5 += w3[j] * w3[j];
                const double temp1 = sqrt(s5) / fnorm;
                const double temp2 = (sqrt(S.par) * pnorm) / fnorm;
                const double prered = temp1 * temp1 + temp2 * temp2 / 0.5;
                const double dirder = -(temp1 * temp1 + temp2 * temp2);
                double ratio = 0.0;
                if (prered != 0.0) ratio = actred / prered;
                if (ratio <= 0.25) {
                    double temp;
                    if (actred >= 0.0) temp = 0.5;
                    else temp = 0.5 * dirder / (dirder + 0.5 * actred);
                    if (0.1 * fnorm1 >= fnorm || temp < 0.1) temp = 0.1;
                    const double dm = S.delta < pnorm / 0.1 ? S.delta : pnorm / 0.1;
                    S.delta = temp * dm;
                    S.par = S.par / temp;
                } else if (S.par == 0.0 || ratio >= 0.75) {
                    S.delta = pnorm / 0.5;
                    S.par = 0.5 * S.par;
                }
                if (ratio >= 1e-4) {
                    for (int j = 0; j < 6; ++j) S.p[j] = S.pt[j];
                    double s6 = 0;
                    for (int j = 0; j < 6; ++j) s6 += S.p[j] * S.p[j];
                    S.xnorm = sqrt(s6);
                    S.fnorm = fnorm1;
                    S.iter += 1;
                }
                int info = 0;
                if (fabs(actred) <= 1e-8 && prered <= 1e-8 && 0.5 * ratio <= 1.0) info = 1;
                if (S.delta <= 1e-8 * S.xnorm) info = 2;
                if (fabs(actred) <= 1e-8 && prered <= 1e-8 && 0.5 * ratio <= 1.0 && info == 2) info = 3;
                if (info == 0) {
                    if (S.nfev >= maxfev) info = 5;
                    if (fabs(actred) <= lm::EPSMCH && prered <= lm::EPSMCH && 0.5 * ratio <= 1.0) info = 6;
                    if (S.delta <= lm::EPSMCH * S.xnorm) info = 7;
                    if (S.gnorm <= lm::EPSMCH) info = 8;
                }
                S.info = info;
                S.ratio = ratio;
            }
            __syncthreads();
            if (S.info != 0 || S.ratio >= 1e-4) break;
        }
        if (S.info != 0) break;
    }
    if (lead && t == 0) {
        double R[9];
        scipy_rotvec_to_R(S.p, R);
        for (int i = 0; i < 3; ++i) out[i] = fma(-R[6 + i], S.p[5], fma(-R[3 + i], S.p[4], (-R[i]) * S.p[3]));
        for (int k = 0; k < 9; ++k) out[3 + k] = R[k];
        out[12] = (double)S.info;
        out[13] = (double)S.qrflags;
    }
}

}  // namespace sfm

using namespace sfm;

static int env_int(const char *name, int dflt) {
    const char *v = getenv(name);
    return v && *v ? atoi(v) : dflt;
}

static int load_cam(const double *K, Cam3 &c) {
    std::memcpy(c.k, K, sizeof c.k);
    return 0;
}

extern "C" int sfm_linear_pnp(const double *X, const double *x, int64_t N, const double *K, double *C_out,
                              double *R_out, int32_t *branch, int device) {
    SFM_CHECK_ARG(N >= 4, "At least 4 point correspondences are required for PnP");
    SFM_CHECK_ARG(X && x && K && C_out && R_out, "null pointer");
    ThreadCtx *c = thread_ctx(device);
    if (!c) return SFM_ERR_HIP;
    int rc;
    if ((rc = c->buf[0].reserve((size_t)N * 24)) || (rc = c->buf[1].reserve((size_t)N * 16)) ||
        (rc = c->buf[2].reserve(16 * sizeof(double))))
        return rc;
    Cam3 cam;
    load_cam(K, cam);
    hipStream_t s = c->stream;
    SFM_HIP(hipMemcpyAsync(c->buf[0].p, X, (size_t)N * 24, hipMemcpyHostToDevice, s));
    SFM_HIP(hipMemcpyAsync(c->buf[1].p, x, (size_t)N * 16, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_pnp_general, dim3(1), dim3(PG_THREADS), 0, s, c->buf[0].as<double>(),
                       c->buf[1].as<double2>(), N, cam, c->buf[2].as<double>());
    SFM_HIP(hipGetLastError());
    double out[13];
    SFM_HIP(hipMemcpyAsync(out, c->buf[2].p, sizeof out, hipMemcpyDeviceToHost, s));
    SFM_HIP(hipStreamSynchronize(s));
    std::memcpy(C_out, out, 3 * sizeof(double));
    std::memcpy(R_out, out + 3, 9 * sizeof(double));
    if (branch) *branch = (int32_t)out[12];
    return 0;
}

extern "C" int sfm_pnp_ransac(const double *X, const double *x, int64_t N, const double *K, const int32_t *samples,
                              int64_t H, double thr, int32_t *counts_out, int32_t *branch_out, int64_t *best_iter,
                              int64_t *best_count, double *C_best, double *R_best, int device) {
    SFM_CHECK_ARG(N >= 4 && H >= 0, "need N >= 4 and H >= 0");
    SFM_CHECK_ARG(X && x && K && best_iter && C_best && R_best && (samples || H == 0), "null pointer");
    for (int64_t i = 0; i < H * 4; ++i)
        SFM_CHECK_ARG(samples[i] >= 0 && samples[i] < N, "sample index out of range");
    *best_iter = -1;
    if (best_count) *best_count = 0;
    if (H == 0) return 0;
    ThreadCtx *c = thread_ctx(device);
    if (!c) return SFM_ERR_HIP;
    int rc;
    if ((rc = c->buf[0].reserve((size_t)N * 24)) || (rc = c->buf[1].reserve((size_t)N * 16)) ||
        (rc = c->buf[2].reserve((size_t)H * 4 * sizeof(int32_t))) ||
        (rc = c->buf[3].reserve((size_t)H * PNP_MODEL * sizeof(double))) ||
        (rc = c->buf[4].reserve((size_t)H * sizeof(int32_t))) || (rc = c->buf[5].reserve((size_t)H * sizeof(int32_t))) ||
        (rc = c->buf[6].reserve(32 * sizeof(double))))
        return rc;
    Cam3 cam;
    load_cam(K, cam);
    double *dX = c->buf[0].as<double>(), *dM = c->buf[3].as<double>(), *dOut = c->buf[6].as<double>();
    double2 *dx = c->buf[1].as<double2>();
    int32_t *ds = c->buf[2].as<int32_t>(), *dcnt = c->buf[4].as<int32_t>(), *dbr = c->buf[5].as<int32_t>();
    int64_t *dbest = reinterpret_cast<int64_t *>(dOut + 24);
    hipStream_t s = c->stream;
    const bool tm = call_timing();  // HIP events only when asked (each costs the stream us)
    if (tm) SFM_HIP(hipEventRecord(c->ev[0], s));
    SFM_HIP(hipMemcpyAsync(dX, X, (size_t)N * 24, hipMemcpyHostToDevice, s));
    SFM_HIP(hipMemcpyAsync(dx, x, (size_t)N * 16, hipMemcpyHostToDevice, s));
    SFM_HIP(hipMemcpyAsync(ds, samples, (size_t)H * 4 * sizeof(int32_t), hipMemcpyHostToDevice, s));
    if (tm) SFM_HIP(hipEventRecord(c->ev[1], s));
    hipLaunchKernelGGL(k_pnp_fit, dim3(ceil_div(H, 64)), dim3(64), 0, s, dX, dx, ds, H, cam, dM, dbr);
    SFM_HIP(hipGetLastError());
    if (tm) SFM_HIP(hipEventRecord(c->ev[2], s));
    hipLaunchKernelGGL(k_pnp_score, dim3(ceil_div(H, PNP_WAVES)), dim3(64 * PNP_WAVES), 0, s, dX, dx, N, dM, H, thr,
                       dcnt);
    SFM_HIP(hipGetLastError());
    if (tm) SFM_HIP(hipEventRecord(c->ev[3], s));
    hipLaunchKernelGGL(k_pnp_select, dim3(1), dim3(1024), 0, s, dM, dcnt, H, dbest, dOut);
    SFM_HIP(hipGetLastError());
    if (tm) SFM_HIP(hipEventRecord(c->ev[4], s));
    double out[24];
    int64_t best[2];
    SFM_HIP(hipMemcpyAsync(out, dOut, sizeof out, hipMemcpyDeviceToHost, s));
    SFM_HIP(hipMemcpyAsync(best, dbest, sizeof best, hipMemcpyDeviceToHost, s));
    if (counts_out) SFM_HIP(hipMemcpyAsync(counts_out, dcnt, (size_t)H * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    if (branch_out) SFM_HIP(hipMemcpyAsync(branch_out, dbr, (size_t)H * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    if (tm) SFM_HIP(hipEventRecord(c->ev[5], s));
    SFM_HIP(hipStreamSynchronize(s));
    *best_iter = best[0];
    if (best_count) *best_count = best[1];
    if (best[0] >= 0) {
        std::memcpy(C_best, out + 12, 3 * sizeof(double));
        std::memcpy(R_best, out + 15, 9 * sizeof(double));
    }
    float a = 0, b = 0, d = 0, e = 0, f = 0;
    if (tm) (void)hipEventElapsedTime(&a, c->ev[0], c->ev[1]);
    if (tm) (void)hipEventElapsedTime(&b, c->ev[1], c->ev[4]);
    if (tm) (void)hipEventElapsedTime(&d, c->ev[4], c->ev[5]);
    if (tm) (void)hipEventElapsedTime(&e, c->ev[2], c->ev[3]);
    if (tm) (void)hipEventElapsedTime(&f, c->ev[1], c->ev[2]);
    const double t[5] = {a, b, d, e, f};
    set_timings(t, 5);
    return 0;
}

// NonlinearPnP inputs from the pinned staging buffer [C0 R0 | pad | X | x]
static __global__ void __launch_bounds__(256) k_stage_pnp(const double *__restrict__ h, int64_t N,
                                                          double *__restrict__ dIn, double *__restrict__ dX,
                                                          double *__restrict__ dx) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < 12) dIn[i] = h[i];
    if (i < N) {
#pragma unroll
        for (int k = 0; k < 3; ++k) dX[3 * i + k] = h[16 + 3 * i + k];
        dx[2 * i] = h[16 + 3 * N + 2 * i];
        dx[2 * i + 1] = h[16 + 3 * N + 2 * i + 1];
    }
}

extern "C" int sfm_nonlinear_pnp(const double *X, const double *x, int64_t N, const double *K, const double *C0,
                                 const double *R0, int32_t max_nfev, double *C_out, double *R_out, int32_t *info,
                                 int device) {
    SFM_CHECK_ARG(N >= 0 && max_nfev > 0, "need N >= 0 and max_nfev > 0");
    SFM_CHECK_ARG(K && C0 && R0 && C_out && R_out && (N == 0 || (X && x)), "null pointer");
    if (N < 4) {  // NonlinearPnP.py:96-98: not enough points, initial estimate
        std::memcpy(C_out, C0, 3 * sizeof(double));
        std::memcpy(R_out, R0, 9 * sizeof(double));
        if (info) *info = 0;
        return 0;
    }
    ThreadCtx *c = thread_ctx(device);
    if (!c) return SFM_ERR_HIP;
    int rc;
    // inputs [C0 R0 (12) | pad | X (3N) | x (2N)] and the result (13) go
    // through pinned memory: one staging kernel on the compute queue instead
    // of pageable copies, the result stored by the kernel straight to the
    // host (each SDMA copy or event record costs the stream microseconds)
    const size_t nin = 16 + 5 * (size_t)N;
    if ((rc = c->buf[0].reserve((size_t)N * 24)) || (rc = c->buf[1].reserve((size_t)N * 16)) ||
        (rc = c->buf[2].reserve(32 * sizeof(double))) || (rc = c->pinned.reserve((nin + 16) * sizeof(double))))
        return rc;
    Cam3 cam;
    load_cam(K, cam);
    double *dIn = c->buf[2].as<double>();
    double *hp = c->pinned.as<double>(), *hres = hp + nin;
    std::memcpy(hp, C0, 3 * sizeof(double));
    std::memcpy(hp + 3, R0, 9 * sizeof(double));
    std::memcpy(hp + 16, X, (size_t)N * 24);
    std::memcpy(hp + 16 + 3 * (size_t)N, x, (size_t)N * 16);
    hres[12] = -1.0;
    hres[13] = 0.0;
    hipStream_t s = c->stream;
    const bool tm = call_timing();
    if (tm) SFM_HIP(hipEventRecord(c->ev[0], s));
    hipLaunchKernelGGL(k_stage_pnp, dim3(ceil_div((int64_t)N, 256)), dim3(256), 0, s, hp, (int64_t)N, dIn,
                       c->buf[0].as<double>(), c->buf[1].as<double>());
    SFM_HIP(hipGetLastError());
    if (tm) SFM_HIP(hipEventRecord(c->ev[1], s));
    // workgroups: ~1024 rows each (SFM_NLPNP_WGS overrides), at most NL_MAXWG,
    // and never more than can be resident at once (the workgroups wait on
    // each other's sums)
    int nb = std::max(1, std::min(NL_MAXWG, env_int("SFM_NLPNP_WGS", ceil_div((int64_t)N, 1024))));
    if (c->nl_resident < 0) {  // per thread context (device): no shared state between host threads
        int per_cu = 0, ncu = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_nonlinear_pnp, NL2_THREADS, 0) != hipSuccess ||
            hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess)
            per_cu = ncu = 0;
        (void)hipGetLastError();
        c->nl_resident = std::max(1, per_cu * ncu);
    }
    nb = std::min(nb, c->nl_resident);
    // SFM_NLPNP_FORCE_TIMEOUT=1 (tests): the first multi-workgroup launch's
    // first hand-off times out, so the one-workgroup retry below runs
    const bool force_timeout = env_int("SFM_NLPNP_FORCE_TIMEOUT", 0) != 0;
    for (int attempt = 0;; ++attempt) {
    NlX xg{};
    xg.nb = nb;
    if (nb > 1) {
        const size_t sync_bytes = (2 * NL_MAXWG * 32 + NL_MAXWG + 1) * sizeof(double);
        if (!c->nl_sync) {
            SFM_HIP(hipMalloc(&c->nl_sync, sync_bytes));
            SFM_HIP(hipMemsetAsync(c->nl_sync, 0, sync_bytes, s));
        }
        xg.part = static_cast<double *>(c->nl_sync);
        xg.flag = reinterpret_cast<unsigned long long *>(xg.part + 2 * NL_MAXWG * 32);
        xg.abort_ = xg.flag + NL_MAXWG;
        xg.epoch = ++c->nl_epoch;
        xg.limit = force_timeout && attempt == 0 ? -1 : NL_POLL_LIMIT;
    }
    hipLaunchKernelGGL(k_nonlinear_pnp, dim3(nb), dim3(NL2_THREADS), 0, s, c->buf[0].as<double>(),
                       c->buf[1].as<double2>(), (int64_t)N, cam, dIn, dIn + 3, max_nfev, hres, xg);
    SFM_HIP(hipGetLastError());
    if (tm) SFM_HIP(hipEventRecord(c->ev[2], s));
    SFM_HIP(hipStreamSynchronize(s));
    if (hres[12] == -2.0) {
        // a hand-off timed out (other work held the CUs the workgroups wait
        // on): the same solve again on one workgroup, which waits on nobody
        if (nb > 1 && attempt == 0) {
            nb = 1;
            hres[12] = -1.0;
            hres[13] = 0.0;
            continue;
        }
        set_error("NonlinearPnP: a cross-workgroup hand-off timed out (%d workgroups)", nb);
        return SFM_ERR_HIP;
    }
    break;
    }
    std::memcpy(C_out, hres, 3 * sizeof(double));
    std::memcpy(R_out, hres + 3, 9 * sizeof(double));
    // info: MINPACK's code; bits 8-9 (non-negative info only): the CholeskyQR
    // flags (1: pass 1's Gram factor needed a shift, a third pass ran; 2: a
    // later Gram factor failed and was kept as the identity)
    if (info) *info = (int32_t)hres[12] >= 0 ? (int32_t)hres[12] | ((int32_t)hres[13] << 8) : (int32_t)hres[12];
    double t[4] = {0, 0, 0, 0};
    if (tm) {
        float a = 0, b = 0;
        (void)hipEventElapsedTime(&a, c->ev[0], c->ev[1]);
        (void)hipEventElapsedTime(&b, c->ev[1], c->ev[2]);
        t[0] = a; t[1] = b; t[3] = b;
    }
    set_timings(t, 4);
    return 0;
}
