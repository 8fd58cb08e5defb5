// Per-thread MINPACK lmdif for tiny problems (M residuals, N parameters,
// both compile-time), exactly as scipy.optimize.least_squares(method='lm')
// drives it (scipy 1.15.3 least_squares.py:40-78 call_minpack): diag = ones
// (x_scale = 1, mode 2), factor = 100, forward differences with
// epsfcn = EPS, ftol = xtol = gtol given.  Same operations in the same order
// as the published MINPACK-1 routines (lmdif, fdjac2, qrfac with column
// pivoting, lmpar, qrsolv, enorm); with FP contraction off every result
// rounds like the CPU build, which makes the kernels bit-comparable with the
// reference's own outputs (tests/golden/nltri.npz).
//
// Every loop has a compile-time trip count and is fully unrolled, so the
// matrices live in VGPRs; the data-dependent pivot permutation is applied
// with unrolled selects (gather/scatter below) instead of indexed scratch.
#pragma once
#include <hip/hip_runtime.h>

#pragma clang fp contract(off)

namespace sfm {
namespace lm {

constexpr double EPSMCH = 2.220446049250313e-16;
constexpr double DWARF = 2.2250738585072014e-308;

// enorm over x[lo..hi) of a length-L array (MINPACK enorm: three sums)
template <int L>
__device__ __forceinline__ double enorm_range(const double (&x)[L], int lo, int hi) {
    const double rdwarf = 3.834e-20, rgiant = 1.304e19;
    double s1 = 0, s2 = 0, s3 = 0, x1max = 0, x3max = 0;
    const double agiant = rgiant / (double)(hi - lo);
#pragma unroll
    for (int i = 0; i < L; ++i) {
        if (i < lo || i >= hi) continue;
        const double xabs = fabs(x[i]);
        if (xabs > rdwarf && xabs < agiant) {
            s2 += xabs * xabs;
        } else if (xabs > rdwarf) {
            if (xabs > x1max) {
                const double t = x1max / xabs;
                s1 = 1.0 + s1 * t * t;
                x1max = xabs;
            } else {
                const double t = xabs / x1max;
                s1 += t * t;
            }
        } else {
            if (xabs > x3max) {
                const double t = x3max / xabs;
                s3 = 1.0 + s3 * t * t;
                x3max = xabs;
            } else if (xabs != 0.0) {
                const double t = xabs / x3max;
                s3 += t * t;
            }
        }
    }
    if (s1 != 0.0) return x1max * sqrt(s1 + (s2 / x1max) / x1max);
    if (s2 != 0.0) {
        if (s2 >= x3max) return sqrt(s2 * (1.0 + (x3max / s2) * (x3max * s3)));
        return sqrt(x3max * ((s2 / x3max) + (x3max * s3)));
    }
    return x3max * sqrt(s3);
}

template <int L>
__device__ __forceinline__ double gather(const double (&a)[L], int idx) {
    double v = a[0];
#pragma unroll
    for (int k = 1; k < L; ++k)
        if (idx == k) v = a[k];
    return v;
}

template <int L>
__device__ __forceinline__ void scatter(double (&a)[L], int idx, double v) {
#pragma unroll
    for (int k = 0; k < L; ++k)
        if (idx == k) a[k] = v;
}

// a[j][i] = A(i, j): M x N column-major
template <int M, int N>
__device__ __forceinline__ void qrfac(double (&a)[N][M], int (&ipvt)[N], double (&rdiag)[N], double (&acnorm)[N]) {
    double wa[N];
#pragma unroll
    for (int j = 0; j < N; ++j) {
        acnorm[j] = enorm_range<M>(a[j], 0, M);
        rdiag[j] = acnorm[j];
        wa[j] = rdiag[j];
        ipvt[j] = j;
    }
    constexpr int MINMN = M < N ? M : N;
#pragma unroll
    for (int j = 0; j < MINMN; ++j) {
        int kmax = j;
#pragma unroll
        for (int k = j; k < N; ++k)
            if (rdiag[k] > gather<N>(rdiag, kmax)) kmax = k;
#pragma unroll
        for (int k = j + 1; k < N; ++k) {
            if (kmax == k) {
#pragma unroll
                for (int i = 0; i < M; ++i) {
                    const double t = a[j][i];
                    a[j][i] = a[k][i];
                    a[k][i] = t;
                }
                rdiag[k] = rdiag[j];
                wa[k] = wa[j];
                const int tp = ipvt[j];
                ipvt[j] = ipvt[k];
                ipvt[k] = tp;
            }
        }
        double ajnorm = enorm_range<M>(a[j], j, M);
        if (ajnorm != 0.0) {
            if (a[j][j] < 0.0) ajnorm = -ajnorm;
#pragma unroll
            for (int i = j; i < M; ++i) a[j][i] /= ajnorm;
            a[j][j] += 1.0;
#pragma unroll
            for (int k = j + 1; k < N; ++k) {
                double sum = 0.0;
#pragma unroll
                for (int i = j; i < M; ++i) sum += a[j][i] * a[k][i];
                const double temp = sum / a[j][j];
#pragma unroll
                for (int i = j; i < M; ++i) a[k][i] -= temp * a[j][i];
                if (rdiag[k] != 0.0) {
                    const double t = a[k][j] / rdiag[k];
                    const double t2 = 1.0 - t * t;
                    rdiag[k] *= sqrt(t2 > 0.0 ? t2 : 0.0);
                    const double q = rdiag[k] / wa[k];
                    if (0.05 * (q * q) <= EPSMCH) {
                        rdiag[k] = enorm_range<M>(a[k], j + 1, M);
                        wa[k] = rdiag[k];
                    }
                }
            }
        }
        rdiag[j] = -ajnorm;
    }
}

// qrsolv with diag(l) = dval for every l (scipy's diag = ones scaled by sqrt(par))
template <int M, int N>
__device__ __forceinline__ void qrsolv(double (&r)[N][M], const int (&ipvt)[N], double dval, const double (&qtb)[N],
                                       double (&x)[N], double (&sdiag)[N]) {
    double wa[N];
#pragma unroll
    for (int j = 0; j < N; ++j) {
#pragma unroll
        for (int i = j; i < N; ++i) r[j][i] = r[i][j];
        x[j] = r[j][j];
        wa[j] = qtb[j];
    }
#pragma unroll
    for (int j = 0; j < N; ++j) {
        if (dval != 0.0) {
#pragma unroll
            for (int k = j; k < N; ++k) sdiag[k] = 0.0;
            sdiag[j] = dval;
            double qtbpj = 0.0;
#pragma unroll
            for (int k = j; k < N; ++k) {
                if (sdiag[k] == 0.0) continue;
                double sn, cs;
                if (fabs(r[k][k]) < fabs(sdiag[k])) {
                    const double cotan = r[k][k] / sdiag[k];
                    sn = 0.5 / sqrt(0.25 + 0.25 * cotan * cotan);
                    cs = sn * cotan;
                } else {
                    const double tn = sdiag[k] / r[k][k];
                    cs = 0.5 / sqrt(0.25 + 0.25 * tn * tn);
                    sn = cs * tn;
                }
                r[k][k] = cs * r[k][k] + sn * sdiag[k];
                const double temp = cs * wa[k] + sn * qtbpj;
                qtbpj = -sn * wa[k] + cs * qtbpj;
                wa[k] = temp;
#pragma unroll
                for (int i = k + 1; i < N; ++i) {
                    const double t = cs * r[k][i] + sn * sdiag[i];
                    sdiag[i] = -sn * r[k][i] + cs * sdiag[i];
                    r[k][i] = t;
                }
            }
        }
        sdiag[j] = r[j][j];
        r[j][j] = x[j];
    }
    int nsing = N;
#pragma unroll
    for (int j = 0; j < N; ++j) {
        if (sdiag[j] == 0.0 && nsing == N) nsing = j;
        if (nsing < N) wa[j] = 0.0;
    }
#pragma unroll
    for (int j = N - 1; j >= 0; --j) {
        if (j >= nsing) continue;
        double sum = 0.0;
#pragma unroll
        for (int i = j + 1; i < N; ++i)
            if (i < nsing) sum += r[j][i] * wa[i];
        wa[j] = (wa[j] - sum) / sdiag[j];
    }
#pragma unroll
    for (int j = 0; j < N; ++j) scatter<N>(x, ipvt[j], wa[j]);
}

template <int M, int N>
__device__ __forceinline__ void lmpar(double (&r)[N][M], const int (&ipvt)[N], const double (&qtb)[N], double delta,
                                      double &par, double (&x)[N], double (&sdiag)[N]) {
    double wa1[N], wa2[N];
    int nsing = N;
#pragma unroll
    for (int j = 0; j < N; ++j) {
        wa1[j] = qtb[j];
        if (r[j][j] == 0.0 && nsing == N) nsing = j;
        if (nsing < N) wa1[j] = 0.0;
    }
#pragma unroll
    for (int j = N - 1; j >= 0; --j) {
        if (j >= nsing) continue;
        wa1[j] /= r[j][j];
        const double temp = wa1[j];
#pragma unroll
        for (int i = 0; i < j; ++i) wa1[i] -= r[j][i] * temp;
    }
#pragma unroll
    for (int j = 0; j < N; ++j) scatter<N>(x, ipvt[j], wa1[j]);
    int iter = 0;
#pragma unroll
    for (int j = 0; j < N; ++j) wa2[j] = x[j];  // diag = 1
    double dxnorm = enorm_range<N>(wa2, 0, N);
    double fp = dxnorm - delta;
    if (fp <= 0.1 * delta) {
        par = 0.0;
        return;
    }
    double parl = 0.0;
    if (nsing >= N) {
#pragma unroll
        for (int j = 0; j < N; ++j) wa1[j] = 1.0 * (gather<N>(wa2, ipvt[j]) / dxnorm);
#pragma unroll
        for (int j = 0; j < N; ++j) {
            double sum = 0.0;
#pragma unroll
            for (int i = 0; i < j; ++i) sum += r[j][i] * wa1[i];
            wa1[j] = (wa1[j] - sum) / r[j][j];
        }
        const double temp = enorm_range<N>(wa1, 0, N);
        parl = ((fp / delta) / temp) / temp;
    }
#pragma unroll
    for (int j = 0; j < N; ++j) {
        double sum = 0.0;
#pragma unroll
        for (int i = 0; i <= j; ++i) sum += r[j][i] * qtb[i];
        wa1[j] = sum / 1.0;
    }
    const double gnorm = enorm_range<N>(wa1, 0, N);
    double paru = gnorm / delta;
    if (paru == 0.0) paru = DWARF / (delta < 0.1 ? delta : 0.1);
    if (par < parl) par = parl;
    if (par > paru) par = paru;
    if (par == 0.0) par = gnorm / dxnorm;
    for (;;) {
        ++iter;
        if (par == 0.0) par = DWARF > 0.001 * paru ? DWARF : 0.001 * paru;
        const double temp = sqrt(par);
        qrsolv<M, N>(r, ipvt, temp * 1.0, qtb, x, sdiag);
#pragma unroll
        for (int j = 0; j < N; ++j) wa2[j] = x[j];
        dxnorm = enorm_range<N>(wa2, 0, N);
        const double fp_old = fp;
        fp = dxnorm - delta;
        if (fabs(fp) <= 0.1 * delta || (parl == 0.0 && fp <= fp_old && fp_old < 0.0) || iter == 10) break;
#pragma unroll
        for (int j = 0; j < N; ++j) wa1[j] = 1.0 * (gather<N>(wa2, ipvt[j]) / dxnorm);
#pragma unroll
        for (int j = 0; j < N; ++j) {
            wa1[j] /= sdiag[j];
            const double t = wa1[j];
#pragma unroll
            for (int i = j + 1; i < N; ++i) wa1[i] -= r[j][i] * t;
        }
        const double t = enorm_range<N>(wa1, 0, N);
        const double parc = ((fp / delta) / t) / t;
        if (fp > 0.0 && parl < par) parl = par;
        if (fp < 0.0 && paru > par) paru = par;
        par = parl > par + parc ? parl : par + parc;
    }
    if (iter == 0) par = 0.0;
}

// lmdif as called by scipy (mode 2, diag = ones, factor = 100, epsfcn = EPS).
// fcn(x, f) evaluates the residuals.  Returns MINPACK's info.
template <int M, int N, class Fcn>
__device__ int lmdif(const Fcn &fcn, double (&x)[N], double ftol, double xtol, double gtol, int maxfev) {
    double fvec[M], fjac[N][M], qtf[N], wa1[N], wa2[N], wa3[N], wa4[M];
    int ipvt[N];
    const double factor = 100.0;
    int info = 0;
    fcn(x, fvec);
    int nfev = 1;
    double fnorm = enorm_range<M>(fvec, 0, M);
    double par = 0.0, delta = 0.0, xnorm = 0.0;
    int iter = 1;
    const double eps = 1.4901161193847656e-08;  // sqrt(max(epsfcn, epsmch)) = sqrt(EPS)
    for (;;) {
#pragma unroll
        for (int j = 0; j < N; ++j) {
            const double temp = x[j];
            double h = eps * fabs(temp);
            if (h == 0.0) h = eps;
            x[j] = temp + h;
            double wf[M];
            fcn(x, wf);
            x[j] = temp;
#pragma unroll
            for (int i = 0; i < M; ++i) fjac[j][i] = (wf[i] - fvec[i]) / h;
        }
        nfev += N;
        qrfac<M, N>(fjac, ipvt, wa1, wa2);
        if (iter == 1) {
#pragma unroll
            for (int j = 0; j < N; ++j) wa3[j] = x[j];
            xnorm = enorm_range<N>(wa3, 0, N);
            delta = factor * xnorm;
            if (delta == 0.0) delta = factor;
        }
#pragma unroll
        for (int i = 0; i < M; ++i) wa4[i] = fvec[i];
#pragma unroll
        for (int j = 0; j < N; ++j) {
            if (fjac[j][j] != 0.0) {
                double sum = 0.0;
#pragma unroll
                for (int i = j; i < M; ++i) sum += fjac[j][i] * wa4[i];
                const double temp = -sum / fjac[j][j];
#pragma unroll
                for (int i = j; i < M; ++i) wa4[i] += fjac[j][i] * temp;
            }
            fjac[j][j] = wa1[j];
            qtf[j] = wa4[j];
        }
        double gnorm = 0.0;
        if (fnorm != 0.0) {
#pragma unroll
            for (int j = 0; j < N; ++j) {
                const double cn = gather<N>(wa2, ipvt[j]);
                if (cn != 0.0) {
                    double sum = 0.0;
#pragma unroll
                    for (int i = 0; i <= j; ++i) sum += fjac[j][i] * (qtf[i] / fnorm);
                    const double g = fabs(sum / cn);
                    if (g > gnorm) gnorm = g;
                }
            }
        }
        if (gnorm <= gtol) info = 4;
        if (info != 0) break;
        double ratio;
        do {
            lmpar<M, N>(fjac, ipvt, qtf, delta, par, wa1, wa2);
#pragma unroll
            for (int j = 0; j < N; ++j) {
                wa1[j] = -wa1[j];
                wa2[j] = x[j] + wa1[j];
                wa3[j] = wa1[j];
            }
            const double pnorm = enorm_range<N>(wa3, 0, N);
            if (iter == 1 && pnorm < delta) delta = pnorm;
            fcn(wa2, wa4);
            nfev += 1;
            const double fnorm1 = enorm_range<M>(wa4, 0, M);
            double actred = -1.0;
            if (0.1 * fnorm1 < fnorm) {
                const double t = fnorm1 / fnorm;
                actred = 1.0 - t * t;
            }
#pragma unroll
            for (int j = 0; j < N; ++j) {
                wa3[j] = 0.0;
                const double temp = gather<N>(wa1, ipvt[j]);
#pragma unroll
                for (int i = 0; i <= j; ++i) wa3[i] += fjac[j][i] * temp;
            }
            const double temp1 = enorm_range<N>(wa3, 0, N) / fnorm;
            const double temp2 = (sqrt(par) * pnorm) / fnorm;
            const double prered = temp1 * temp1 + temp2 * temp2 / 0.5;
            const double dirder = -(temp1 * temp1 + temp2 * temp2);
            ratio = 0.0;
            if (prered != 0.0) ratio = actred / prered;
            if (ratio <= 0.25) {
                double temp;
                if (actred >= 0.0) temp = 0.5;
                else temp = 0.5 * dirder / (dirder + 0.5 * actred);
                if (0.1 * fnorm1 >= fnorm || temp < 0.1) temp = 0.1;
                const double dm = delta < pnorm / 0.1 ? delta : pnorm / 0.1;
                delta = temp * dm;
                par = par / temp;
            } else if (par == 0.0 || ratio >= 0.75) {
                delta = pnorm / 0.5;
                par = 0.5 * par;
            }
            if (ratio >= 1e-4) {
#pragma unroll
                for (int j = 0; j < N; ++j) {
                    x[j] = wa2[j];
                    wa2[j] = x[j];
                }
#pragma unroll
                for (int i = 0; i < M; ++i) fvec[i] = wa4[i];
                xnorm = enorm_range<N>(wa2, 0, N);
                fnorm = fnorm1;
                ++iter;
            }
            if (fabs(actred) <= ftol && prered <= ftol && 0.5 * ratio <= 1.0) info = 1;
            if (delta <= xtol * xnorm) info = 2;
            if (fabs(actred) <= ftol && prered <= ftol && 0.5 * ratio <= 1.0 && info == 2) info = 3;
            if (info != 0) break;
            if (nfev >= maxfev) info = 5;
            if (fabs(actred) <= EPSMCH && prered <= EPSMCH && 0.5 * ratio <= 1.0) info = 6;
            if (delta <= EPSMCH * xnorm) info = 7;
            if (gnorm <= EPSMCH) info = 8;
            if (info != 0) break;
        } while (ratio < 1e-4);
        if (info != 0) break;
    }
    return info;
}

}  // namespace lm
}  // namespace sfm
