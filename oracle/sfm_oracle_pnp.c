/* TEST INFRASTRUCTURE ONLY: the checker for the HIP path, never shipped or
 * measured as the product.
 *
 * CPU restatement of the reference's PnP path:
 *   orc_linear_pnp     LinearPnP.py:3-96
 *   orc_pnp_count      PnPRANSAC.py:60-70 (scoring of one pose)
 *   orc_pnp_ransac     PnPRANSAC.py:48-87 (strict '>' update, fallback flag)
 *   orc_nonlinear_pnp  NonlinearPnP.py:5-44 loss, :47-123 least_squares 'lm'
 *
 * numpy's small products are restated in the order OpenBLAS evaluates them
 * (measured against exact arithmetic; tests/golden/make_golden.py notes):
 *   3x3 @ 3x3 / 3x3 @ 3x4 / 3x4 @ 4xN (dgemm): acc = a0 b0, then fma chain
 *   C-order 3x3 @ 3 (dgemv_t tail):  fma(a2, x2, fma(a0, x0, a1 x1))
 *   F-order 3x3 @ 3 (-R.T @ t, dgemv_n): fma chain
 *   inv(K) (gesv through trsm with reciprocal diagonal): -(c * (1/f))
 *   Rotation.from_rotvec / as_matrix / from_matrix / as_rotvec (scipy 1.15.3,
 *   quaternion path) -- reproduced bit for bit.
 *
 * np.linalg.svd on the 2N x 12 DLT matrix: for N >= 6 the null vector is
 * unique and any SVD gives it (QR + Jacobi here).  For N = 4, 5 (the RANSAC
 * samples) the null space is 4-/2-dimensional and Vt[-1] is whatever
 * LAPACK dgesdd's path 5t produces: bidiagonalisation dgebd2 without LQ,
 * then VT = blockdiag(VT_bd, I) P^T, so Vt[-1] = P e_12 with P the product
 * of dgebd2's right reflectors.  That path is emulated below (dlarfg / dlarf
 * semantics), so the chosen null vector agrees up to rounding.
 *
 * LinearPnP's final orthogonalisation R = U @ Vt of an (already orthogonal)
 * R is well defined when det(R) > 0.  When det(R) < 0 (scale < 0 flipped R,
 * ~25 % of 4-point samples) the reference negates U[:, -1] for the singular
 * triplet LAPACK sorts last among three EQUAL singular values -- decided by
 * rounding noise inside OpenBLAS.  The emulation (dgebd2 on R, dbdsqr's sign
 * fix and selection sort on the computed |d|) is deterministic but that
 * branch is parity-unpinned; *branch reports it.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

void orc_jacobi_svd(double *A, int m, int n, double *V, double *s);
int orc_lmdif(void (*fcn)(const double *, double *, const void *), const void *ctx, int m, int n, double *x,
              double ftol, double xtol, double gtol, int maxfev, int *nfev_out);
void orc_R_to_rotvec(const double *R, double *w);

/* ---------------------------------------------------------- LAPACK bits */
static double dlapy2(double x, double y) {
    double xa = fabs(x), ya = fabs(y);
    double w = xa > ya ? xa : ya, z = xa < ya ? xa : ya;
    if (z == 0.0) return w;
    double q = z / w;
    return w * sqrt(1.0 + q * q);
}

static double nrm2(int n, const double *x, int inc) {
    double s = 0;
    for (int i = 0; i < n; ++i) s += x[i * inc] * x[i * inc];
    return sqrt(s);
}

/* dlarfg: H (alpha; x) = (beta; 0), H = I - tau v v^T, v = (1; x') */
static void dlarfg(int n, double *alpha, double *x, int inc, double *tau) {
    if (n <= 1) { *tau = 0.0; return; }
    double xnorm = nrm2(n - 1, x, inc);
    if (xnorm == 0.0) { *tau = 0.0; return; }
    double beta = -copysign(dlapy2(*alpha, xnorm), *alpha);
    *tau = (beta - *alpha) / beta;
    double sc = 1.0 / (*alpha - beta);
    for (int i = 0; i < n - 1; ++i) x[i * inc] *= sc;
    *alpha = beta;
}

/* ------------------------------------------------ DLT null vector (12) */
/* A: m x 12 row-major, destroyed.  v: the 12-vector np.linalg.svd's
 * Vt[-1] would be (see the header). */
static void pnp_null_vector(double *A, int m, double *v) {
    const int n = 12;
    if (m < n) {
        /* dgebd2, m < n: lower bidiagonal; right reflectors G(i) in rows */
        double taup[12];
        for (int i = 0; i < m; ++i) {
            double *row = A + i * n;
            dlarfg(n - i, &row[i], &row[i + 1 < n ? i + 1 : n - 1], 1, &taup[i]);
            double d = row[i];
            row[i] = 1.0;
            /* apply G(i) from the right to A(i+1:m, i:n) */
            for (int r = i + 1; r < m; ++r) {
                double *ar = A + r * n, w = 0;
                for (int j = i; j < n; ++j) w += ar[j] * row[j];
                for (int j = i; j < n; ++j) ar[j] -= taup[i] * w * row[j];
            }
            row[i] = d;
            if (i < m - 1) {
                double tauq;
                double *col = A + (i + 1) * n + i;
                dlarfg(m - i - 1, col, (i + 2 < m) ? A + (i + 2) * n + i : col, n, &tauq);
                double e = *col;
                *col = 1.0;
                /* apply H(i) from the left to A(i+1:m, i+1:n) */
                for (int c = i + 1; c < n; ++c) {
                    double w = 0;
                    for (int r = i + 1; r < m; ++r) w += A[r * n + i] * A[r * n + c];
                    for (int r = i + 1; r < m; ++r) A[r * n + c] -= tauq * A[r * n + i] * w;
                }
                *col = e;
            }
        }
        /* Vt[-1] = (G(0) G(1) ... G(m-1) e_{n-1})^T */
        for (int j = 0; j < n; ++j) v[j] = j == n - 1 ? 1.0 : 0.0;
        for (int i = m - 1; i >= 0; --i) {
            const double *u = A + i * n;  /* u[i] = 1, u[i+1:] stored, u[:i] = 0 */
            double w = v[i];
            for (int j = i + 1; j < n; ++j) w += u[j] * v[j];
            v[i] -= taup[i] * w;
            for (int j = i + 1; j < n; ++j) v[j] -= taup[i] * w * u[j];
        }
        return;
    }
    /* unique null vector: Householder QR to 12 rows, then Jacobi */
    for (int k = 0; k < n && m > n; ++k) {
        double nrm = 0;
        for (int i = k; i < m; ++i) nrm += A[i * n + k] * A[i * n + k];
        nrm = sqrt(nrm);
        if (nrm == 0) continue;
        double alpha = A[k * n + k] > 0 ? -nrm : nrm;
        double v0 = A[k * n + k] - alpha, vtv = v0 * v0;
        for (int i = k + 1; i < m; ++i) vtv += A[i * n + k] * A[i * n + k];
        for (int j = k + 1; j < n; ++j) {
            double d = v0 * A[k * n + j];
            for (int i = k + 1; i < m; ++i) d += A[i * n + k] * A[i * n + j];
            double f = 2.0 * d / vtv;
            A[k * n + j] -= f * v0;
            for (int i = k + 1; i < m; ++i) A[i * n + j] -= f * A[i * n + k];
        }
        A[k * n + k] = alpha;
        for (int i = k + 1; i < m; ++i) A[i * n + k] = 0.0;
    }
    double V[144], s[12];
    orc_jacobi_svd(A, m > n ? n : m, n, V, s);
    int b = 0;
    for (int j = 1; j < n; ++j) if (s[j] < s[b]) b = j;
    for (int k = 0; k < n; ++k) v[k] = V[k * n + b];
}

/* ------------------------------------------ 3x3 helpers (numpy orders) */
static double det3(const double *M) {
    return M[0] * (M[4] * M[8] - M[5] * M[7]) - M[1] * (M[3] * M[8] - M[5] * M[6]) +
           M[2] * (M[3] * M[7] - M[4] * M[6]);
}

/* np.linalg.qr(A) for 3x3 A (row-major): dgeqr2 + dorg2r.  Q, Rq row-major. */
static void qr3(const double *Ain, double *Q, double *Rq) {
    double a[3][3];  /* a[col][row] */
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) a[c][r] = Ain[r * 3 + c];
    double tau[3];
    for (int i = 0; i < 3; ++i) {
        dlarfg(3 - i, &a[i][i], i + 1 < 3 ? &a[i][i + 1] : &a[i][i], 1, &tau[i]);
        double aii = a[i][i];
        a[i][i] = 1.0;
        for (int c = i + 1; c < 3; ++c) {
            double w = 0;
            for (int r = i; r < 3; ++r) w += a[i][r] * a[c][r];
            for (int r = i; r < 3; ++r) a[c][r] -= tau[i] * a[i][r] * w;
        }
        a[i][i] = aii;
    }
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) Rq[r * 3 + c] = r <= c ? a[c][r] : 0.0;
    /* Q = H0 H1 H2 applied to I (dorg2r, backwards) */
    double q[3][3];  /* q[col][row] */
    for (int c = 0; c < 3; ++c)
        for (int r = 0; r < 3; ++r) q[c][r] = r == c ? 1.0 : 0.0;
    for (int i = 2; i >= 0; --i) {
        double v[3] = {0, 0, 0};
        v[i] = 1.0;
        for (int r = i + 1; r < 3; ++r) v[r] = a[i][r];
        for (int c = 0; c < 3; ++c) {
            double w = 0;
            for (int r = i; r < 3; ++r) w += v[r] * q[c][r];
            for (int r = i; r < 3; ++r) q[c][r] -= tau[i] * v[r] * w;
        }
    }
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) Q[r * 3 + c] = q[c][r];
}

/* R - 2 u w^T for the singular pair dgesdd sorts last (see header) */
static void flip_last_singular(double *R) {
    double a[3][3];  /* a[col][row] */
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) a[c][r] = R[r * 3 + c];
    double tauq[3], taup[3], d[3];
    for (int i = 0; i < 3; ++i) {
        /* H(i): column i below the diagonal */
        dlarfg(3 - i, &a[i][i], i + 1 < 3 ? &a[i][i + 1] : &a[i][i], 1, &tauq[i]);
        d[i] = a[i][i];
        a[i][i] = 1.0;
        for (int c = i + 1; c < 3; ++c) {
            double w = 0;
            for (int r = i; r < 3; ++r) w += a[i][r] * a[c][r];
            for (int r = i; r < 3; ++r) a[c][r] -= tauq[i] * a[i][r] * w;
        }
        a[i][i] = d[i];
        taup[i] = 0.0;
        if (i < 1) {  /* G(i): row i right of the superdiagonal (n - i - 1 = 2 entries) */
            dlarfg(2, &a[i + 1][i], &a[i + 2][i], 3, &taup[i]);
            double e = a[i + 1][i];
            a[i + 1][i] = 1.0;
            for (int r = i + 1; r < 3; ++r) {
                double w = 0;
                for (int c = i + 1; c < 3; ++c) w += a[c][r] * a[c][i];
                for (int c = i + 1; c < 3; ++c) a[c][r] -= taup[i] * w * a[c][i];
            }
            a[i + 1][i] = e;
        }
    }
    /* U = H0 H1 (columns), P = G0; singular values |d|, sign into VT rows */
    double U[3][3], P[3][3];  /* [col][row] */
    for (int c = 0; c < 3; ++c)
        for (int r = 0; r < 3; ++r) { U[c][r] = r == c; P[c][r] = r == c; }
    for (int i = 1; i >= 0; --i) {
        double v[3] = {0, 0, 0};
        v[i] = 1.0;
        for (int r = i + 1; r < 3; ++r) v[r] = a[i][r];
        for (int c = 0; c < 3; ++c) {
            double w = 0;
            for (int r = i; r < 3; ++r) w += v[r] * U[c][r];
            for (int r = i; r < 3; ++r) U[c][r] -= tauq[i] * v[r] * w;
        }
    }
    {
        double v[3] = {0, 1.0, a[2][0]};
        for (int c = 0; c < 3; ++c) {
            double w = 0;
            for (int r = 1; r < 3; ++r) w += v[r] * P[c][r];
            for (int r = 1; r < 3; ++r) P[c][r] -= taup[0] * v[r] * w;
        }
    }
    int ord[3] = {0, 1, 2};
    double sv[3], sg[3];
    for (int i = 0; i < 3; ++i) { sg[i] = d[i] < 0 ? -1.0 : 1.0; sv[i] = fabs(d[i]); }
    for (int i = 0; i < 2; ++i) {  /* dbdsqr's selection sort (LE scan) */
        int isub = 0;
        double smin = sv[ord[0]];
        for (int j = 1; j < 3 - i; ++j)
            if (sv[ord[j]] <= smin) { isub = j; smin = sv[ord[j]]; }
        if (isub != 2 - i) { int t = ord[isub]; ord[isub] = ord[2 - i]; ord[2 - i] = t; }
    }
    const int k = ord[2];
    double u[3], w[3];
    for (int r = 0; r < 3; ++r) { u[r] = U[k][r]; w[r] = sg[k] * P[k][r]; }
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) R[r * 3 + c] -= 2.0 * u[r] * w[c];
}

/* LinearPnP.py:3-96.  X: n x 3, x: n x 2, K: 3x3 row-major.
 * Returns 0, or -1 for n < 4 (ValueError in the reference).
 * *branch = 1 where the final orthogonalisation is LAPACK-noise defined. */
int orc_linear_pnp(const double *X, const double *x, int64_t n, const double *K, double *C_out, double *R_out,
                   int *branch) {
    if (n < 4) return -1;
    const double i0 = 1.0 / K[0], i4 = 1.0 / K[4];
    const double Ki[9] = {i0, -0.0, -(K[2] * i0), 0.0, i4, -(K[5] * i4), 0.0, 0.0, 1.0};
    double *A = (double *)malloc(sizeof(double) * (size_t)(2 * n) * 12);
    for (int64_t i = 0; i < n; ++i) {
        const double px = x[2 * i], py = x[2 * i + 1];
        const double xn = fma(Ki[2], 1.0, fma(Ki[1], py, Ki[0] * px));
        const double yn = fma(Ki[5], 1.0, fma(Ki[4], py, Ki[3] * px));
        const double Xw = X[3 * i], Yw = X[3 * i + 1], Zw = X[3 * i + 2];
        double *r0 = A + (2 * i) * 12, *r1 = r0 + 12;
        const double r0v[12] = {Xw, Yw, Zw, 1, 0, 0, 0, 0, -xn * Xw, -xn * Yw, -xn * Zw, -xn};
        const double r1v[12] = {0, 0, 0, 0, Xw, Yw, Zw, 1, -yn * Xw, -yn * Yw, -yn * Zw, -yn};
        memcpy(r0, r0v, sizeof r0v);
        memcpy(r1, r1v, sizeof r1v);
    }
    double p[12];
    pnp_null_vector(A, (int)(2 * n), p);
    free(A);
    double M[9] = {p[0], p[1], p[2], p[4], p[5], p[6], p[8], p[9], p[10]};
    double t[3] = {p[3], p[7], p[11]};
    if (det3(M) < 0) {
        for (int k = 0; k < 9; ++k) M[k] = -M[k];
        for (int k = 0; k < 3; ++k) t[k] = -t[k];
    }
    const double MT[9] = {M[0], M[3], M[6], M[1], M[4], M[7], M[2], M[5], M[8]};
    double Q[9], Rq[9], R[9];
    qr3(MT, Q, Rq);
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) R[r * 3 + c] = Q[c * 3 + r];  /* R = Q.T */
    double scale = ((Rq[0] + Rq[4]) + Rq[8]) / 3.0;
    if (scale < 0) {
        for (int k = 0; k < 9; ++k) R[k] = -R[k];
        scale = -scale;
    }
    int br = 0;
    if (det3(R) < 0) {  /* U[:, -1] *= -1; R = U @ Vt */
        flip_last_singular(R);
        br = 1;
    }
    if (branch) *branch = br;
    const double tn[3] = {t[0] / scale, t[1] / scale, t[2] / scale};
    for (int i = 0; i < 3; ++i)  /* C = -R.T @ t_n (F-order dgemv: fma chain) */
        C_out[i] = fma(-R[6 + i], tn[2], fma(-R[3 + i], tn[1], (-R[i]) * tn[0]));
    memcpy(R_out, R, sizeof R);
    return 0;
}

/* P = K @ hstack([R, -R @ C.reshape(3, 1)]) with numpy's orders */
static void pnp_projection(const double *K, const double *C, const double *R, double *P) {
    double B[12];
    for (int r = 0; r < 3; ++r) {
        const double a0 = -R[r * 3], a1 = -R[r * 3 + 1], a2 = -R[r * 3 + 2];
        B[r * 4 + 3] = fma(a2, C[2], fma(a0, C[0], a1 * C[1]));
        for (int c = 0; c < 3; ++c) B[r * 4 + c] = R[r * 3 + c];
    }
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 4; ++c)
            P[r * 4 + c] = fma(K[r * 3 + 2], B[8 + c], fma(K[r * 3 + 1], B[4 + c], K[r * 3] * B[c]));
}

static inline void pnp_project(const double *P, const double *Xw, double *u, double *v) {
    double h[3];
    for (int r = 0; r < 3; ++r)
        h[r] = fma(P[r * 4 + 3], 1.0, fma(P[r * 4 + 2], Xw[2], fma(P[r * 4 + 1], Xw[1], P[r * 4] * Xw[0])));
    const double w = h[2] + 1e-8;
    *u = h[0] / w;
    *v = h[1] / w;
}

/* PnPRANSAC.py:60-68: the reprojection error of every point for one pose */
void orc_pnp_err(const double *X, const double *x, int64_t n, const double *K, const double *C, const double *R,
                 double *err) {
    double P[12];
    pnp_projection(K, C, R, P);
    for (int64_t i = 0; i < n; ++i) {
        double u, v;
        pnp_project(P, X + 3 * i, &u, &v);
        const double du = x[2 * i] - u, dv = x[2 * i + 1] - v;
        err[i] = sqrt(du * du + dv * dv);
    }
}

/* PnPRANSAC.py:60-70 for one pose */
int64_t orc_pnp_count(const double *X, const double *x, int64_t n, const double *K, const double *C,
                      const double *R, double thr) {
    double P[12];
    pnp_projection(K, C, R, P);
    int64_t c = 0;
    for (int64_t i = 0; i < n; ++i) {
        double u, v;
        pnp_project(P, X + 3 * i, &u, &v);
        const double du = x[2 * i] - u, dv = x[2 * i + 1] - v;
        c += sqrt(du * du + dv * dv) < thr;
    }
    return c;
}

/* PnPRANSAC.py:48-87 over a host-drawn H x 4 sample table.  Returns the
 * winning iteration, -1 when the all-point LinearPnP fallback applies
 * (no winner or best count < 4); counts/branches per hypothesis (nullable). */
int64_t orc_pnp_ransac(const double *X, const double *x, int64_t n, const double *K, const int32_t *samples,
                       int64_t H, double thr, int32_t *counts, int32_t *branches, double *C_best, double *R_best) {
    int64_t best = -1, best_c = 0;
    for (int64_t h = 0; h < H; ++h) {
        double Xs[12], xs[8], C[3], R[9];
        for (int j = 0; j < 4; ++j) {
            const int32_t s = samples[h * 4 + j];
            memcpy(Xs + 3 * j, X + 3 * s, 3 * sizeof(double));
            memcpy(xs + 2 * j, x + 2 * s, 2 * sizeof(double));
        }
        int br = 0;
        orc_linear_pnp(Xs, xs, 4, K, C, R, &br);
        const int64_t c = orc_pnp_count(X, x, n, K, C, R, thr);
        if (counts) counts[h] = (int32_t)c;
        if (branches) branches[h] = br;
        if (c > best_c) {
            best_c = c;
            best = h;
            memcpy(C_best, C, sizeof C);
            memcpy(R_best, R, sizeof R);
        }
    }
    if (best < 0 || best_c < 4) return -1;
    return best;
}

/* ---------------------------------------------------------- NonlinearPnP */
/* scipy Rotation.from_rotvec(...).as_matrix(), bit for bit (quaternion path) */
static void scipy_rotvec_to_R(const double *rv, double *R) {
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

typedef struct {
    const double *X, *x, *K;
    int64_t n;
} pnp_ctx;

/* NonLinearPnPLoss (NonlinearPnP.py:5-44): (x - proj).flatten() */
static void pnp_loss(const double *p, double *f, const void *vctx) {
    const pnp_ctx *c = (const pnp_ctx *)vctx;
    double R[9], C[3], P[12];
    scipy_rotvec_to_R(p, R);
    for (int i = 0; i < 3; ++i) C[i] = fma(-R[6 + i], p[5], fma(-R[3 + i], p[4], (-R[i]) * p[3]));
    pnp_projection(c->K, C, R, P);
    for (int64_t i = 0; i < c->n; ++i) {
        double u, v;
        pnp_project(P, c->X + 3 * i, &u, &v);
        f[2 * i] = c->x[2 * i] - u;
        f[2 * i + 1] = c->x[2 * i + 1] - v;
    }
}

/* NonlinearPnP.py:47-123.  Returns MINPACK info, 0 for the n < 4 early
 * return (C, R unchanged), -1 where the reference's except path keeps them. */
int orc_nonlinear_pnp(const double *X, const double *x, int64_t n, const double *K, const double *C0,
                      const double *R0, int32_t max_nfev, double *C_out, double *R_out) {
    memcpy(C_out, C0, 3 * sizeof(double));
    memcpy(R_out, R0, 9 * sizeof(double));
    if (n < 4) return 0;
    double p[6];
    orc_R_to_rotvec(R0, p);
    for (int i = 0; i < 3; ++i)  /* tvec = -R @ C (C-order dgemv tail) */
        p[3 + i] = fma(-R0[i * 3 + 2], C0[2], fma(-R0[i * 3], C0[0], (-R0[i * 3 + 1]) * C0[1]));
    for (int k = 0; k < 6; ++k)
        if (isnan(p[k])) return -1;
    pnp_ctx c = {X, x, K, n};
    double *f0 = (double *)malloc(sizeof(double) * (size_t)(2 * n));
    pnp_loss(p, f0, &c);
    int finite = 1;
    for (int64_t i = 0; i < 2 * n; ++i) finite &= isfinite(f0[i]) ? 1 : 0;
    free(f0);
    if (!finite) return -1;
    int nfev = 0;
    const int info = orc_lmdif(pnp_loss, &c, (int)(2 * n), 6, p, 1e-8, 1e-8, 1e-8, max_nfev, &nfev);
    double R[9];
    scipy_rotvec_to_R(p, R);
    for (int i = 0; i < 3; ++i) C_out[i] = fma(-R[6 + i], p[5], fma(-R[3 + i], p[4], (-R[i]) * p[3]));
    memcpy(R_out, R, sizeof R);
    return info;
}
