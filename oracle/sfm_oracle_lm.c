/* TEST INFRASTRUCTURE ONLY: the checker for the HIP path, never shipped or
 * measured as the product.
 *
 * CPU restatement of the reference's per-point non-linear triangulation
 * (Phase 1/NonLinearTriangulation.py:5-50 Loss, :53-121 the per-point
 * least_squares loop).  The optimiser the reference calls is
 * scipy.optimize.least_squares(method='lm', max_nfev=50) from scipy 1.15.3
 * (not vendored in the reference): least_squares.py:40-78 call_minpack with
 * diag = 1/x_scale = ones (mode 2), factor = 100, epsfcn = EPS,
 * ftol = xtol = gtol = 1e-8, i.e. MINPACK-1 lmdif (Moré, Garbow, Hillstrom
 * 1980).  lmdif, fdjac2, qrfac, lmpar, qrsolv and enorm are restated below
 * from that published algorithm; parity is pinned by tests/golden/nltri.npz
 * (outputs of the reference itself).
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <stdlib.h>

#define LM_MAXN 8  /* parameters; residual count m is dynamic */

typedef void (*lm_fcn)(const double *x, double *f, const void *ctx);

static const double EPSMCH = 2.220446049250313e-16;
static const double DWARF = 2.2250738585072014e-308;

/* MINPACK enorm: scaled Euclidean norm (small / intermediate / large sums) */
static double enorm(int n, const double *x) {
    const double rdwarf = 3.834e-20, rgiant = 1.304e19;
    double s1 = 0, s2 = 0, s3 = 0, x1max = 0, x3max = 0;
    const double agiant = rgiant / n;
    for (int i = 0; i < n; ++i) {
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

/* column-major with leading dimension lda: COL(a, j)[i] = A(i, j) */
#define COL(a, j) ((a) + (size_t)(j) * lda)

static void qrfac(int m, int n, double *a, int lda, int *ipvt, double *rdiag, double *acnorm) {
    double wa[LM_MAXN];
    for (int j = 0; j < n; ++j) {
        acnorm[j] = enorm(m, COL(a, j));
        rdiag[j] = acnorm[j];
        wa[j] = rdiag[j];
        ipvt[j] = j;
    }
    const int minmn = m < n ? m : n;
    for (int j = 0; j < minmn; ++j) {
        int kmax = j;
        for (int k = j; k < n; ++k)
            if (rdiag[k] > rdiag[kmax]) kmax = k;
        if (kmax != j) {
            for (int i = 0; i < m; ++i) {
                const double t = COL(a, j)[i];
                COL(a, j)[i] = COL(a, kmax)[i];
                COL(a, kmax)[i] = t;
            }
            rdiag[kmax] = rdiag[j];
            wa[kmax] = wa[j];
            const int k = ipvt[j];
            ipvt[j] = ipvt[kmax];
            ipvt[kmax] = k;
        }
        double ajnorm = enorm(m - j, COL(a, j) + j);
        if (ajnorm != 0.0) {
            if (COL(a, j)[j] < 0.0) ajnorm = -ajnorm;
            for (int i = j; i < m; ++i) COL(a, j)[i] /= ajnorm;
            COL(a, j)[j] += 1.0;
            for (int k = j + 1; k < n; ++k) {
                double sum = 0.0;
                for (int i = j; i < m; ++i) sum += COL(a, j)[i] * COL(a, k)[i];
                const double temp = sum / COL(a, j)[j];
                for (int i = j; i < m; ++i) COL(a, k)[i] -= temp * COL(a, j)[i];
                if (rdiag[k] != 0.0) {
                    const double t = COL(a, k)[j] / rdiag[k];
                    const double t2 = 1.0 - t * t;
                    rdiag[k] *= sqrt(t2 > 0.0 ? t2 : 0.0);
                    const double q = rdiag[k] / wa[k];
                    if (0.05 * (q * q) <= EPSMCH) {
                        rdiag[k] = enorm(m - j - 1, COL(a, k) + j + 1);
                        wa[k] = rdiag[k];
                    }
                }
            }
        }
        rdiag[j] = -ajnorm;
    }
}

static void qrsolv(int n, double *r, int lda, const int *ipvt, const double *diag, const double *qtb,
                   double *x, double *sdiag) {
    double wa[LM_MAXN];
    for (int j = 0; j < n; ++j) {
        for (int i = j; i < n; ++i) COL(r, j)[i] = COL(r, i)[j];
        x[j] = COL(r, j)[j];
        wa[j] = qtb[j];
    }
    for (int j = 0; j < n; ++j) {
        const int l = ipvt[j];
        if (diag[l] != 0.0) {
            for (int k = j; k < n; ++k) sdiag[k] = 0.0;
            sdiag[j] = diag[l];
            double qtbpj = 0.0;
            for (int k = j; k < n; ++k) {
                if (sdiag[k] == 0.0) continue;
                double sn, cs;
                if (fabs(COL(r, k)[k]) < fabs(sdiag[k])) {
                    const double cotan = COL(r, k)[k] / sdiag[k];
                    sn = 0.5 / sqrt(0.25 + 0.25 * cotan * cotan);
                    cs = sn * cotan;
                } else {
                    const double tn = sdiag[k] / COL(r, k)[k];
                    cs = 0.5 / sqrt(0.25 + 0.25 * tn * tn);
                    sn = cs * tn;
                }
                COL(r, k)[k] = cs * COL(r, k)[k] + sn * sdiag[k];
                const double temp = cs * wa[k] + sn * qtbpj;
                qtbpj = -sn * wa[k] + cs * qtbpj;
                wa[k] = temp;
                for (int i = k + 1; i < n; ++i) {
                    const double t = cs * COL(r, k)[i] + sn * sdiag[i];
                    sdiag[i] = -sn * COL(r, k)[i] + cs * sdiag[i];
                    COL(r, k)[i] = t;
                }
            }
        }
        sdiag[j] = COL(r, j)[j];
        COL(r, j)[j] = x[j];
    }
    int nsing = n;
    for (int j = 0; j < n; ++j) {
        if (sdiag[j] == 0.0 && nsing == n) nsing = j;
        if (nsing < n) wa[j] = 0.0;
    }
    for (int j = nsing - 1; j >= 0; --j) {
        double sum = 0.0;
        for (int i = j + 1; i < nsing; ++i) sum += COL(r, j)[i] * wa[i];
        wa[j] = (wa[j] - sum) / sdiag[j];
    }
    for (int j = 0; j < n; ++j) x[ipvt[j]] = wa[j];
}

static void lmpar(int n, double *r, int lda, const int *ipvt, const double *diag, const double *qtb,
                  double delta, double *par, double *x, double *sdiag) {
    double wa1[LM_MAXN], wa2[LM_MAXN];
    int nsing = n;
    for (int j = 0; j < n; ++j) {
        wa1[j] = qtb[j];
        if (COL(r, j)[j] == 0.0 && nsing == n) nsing = j;
        if (nsing < n) wa1[j] = 0.0;
    }
    for (int j = nsing - 1; j >= 0; --j) {
        wa1[j] /= COL(r, j)[j];
        const double temp = wa1[j];
        for (int i = 0; i < j; ++i) wa1[i] -= COL(r, j)[i] * temp;
    }
    for (int j = 0; j < n; ++j) x[ipvt[j]] = wa1[j];
    int iter = 0;
    for (int j = 0; j < n; ++j) wa2[j] = diag[j] * x[j];
    double dxnorm = enorm(n, wa2);
    double fp = dxnorm - delta;
    if (fp <= 0.1 * delta) {
        *par = 0.0;
        return;
    }
    double parl = 0.0;
    if (nsing >= n) {
        for (int j = 0; j < n; ++j) {
            const int l = ipvt[j];
            wa1[j] = diag[l] * (wa2[l] / dxnorm);
        }
        for (int j = 0; j < n; ++j) {
            double sum = 0.0;
            for (int i = 0; i < j; ++i) sum += COL(r, j)[i] * wa1[i];
            wa1[j] = (wa1[j] - sum) / COL(r, j)[j];
        }
        const double temp = enorm(n, wa1);
        parl = ((fp / delta) / temp) / temp;
    }
    for (int j = 0; j < n; ++j) {
        double sum = 0.0;
        for (int i = 0; i <= j; ++i) sum += COL(r, j)[i] * qtb[i];
        wa1[j] = sum / diag[ipvt[j]];
    }
    const double gnorm = enorm(n, wa1);
    double paru = gnorm / delta;
    if (paru == 0.0) paru = DWARF / (delta < 0.1 ? delta : 0.1);
    if (*par < parl) *par = parl;
    if (*par > paru) *par = paru;
    if (*par == 0.0) *par = gnorm / dxnorm;
    for (;;) {
        ++iter;
        if (*par == 0.0) *par = DWARF > 0.001 * paru ? DWARF : 0.001 * paru;
        const double temp = sqrt(*par);
        for (int j = 0; j < n; ++j) wa1[j] = temp * diag[j];
        qrsolv(n, r, lda, ipvt, wa1, qtb, x, sdiag);
        for (int j = 0; j < n; ++j) wa2[j] = diag[j] * x[j];
        dxnorm = enorm(n, wa2);
        const double fp_old = fp;
        fp = dxnorm - delta;
        if (fabs(fp) <= 0.1 * delta || (parl == 0.0 && fp <= fp_old && fp_old < 0.0) || iter == 10) break;
        for (int j = 0; j < n; ++j) {
            const int l = ipvt[j];
            wa1[j] = diag[l] * (wa2[l] / dxnorm);
        }
        for (int j = 0; j < n; ++j) {
            wa1[j] /= sdiag[j];
            const double t = wa1[j];
            for (int i = j + 1; i < n; ++i) wa1[i] -= COL(r, j)[i] * t;
        }
        const double t = enorm(n, wa1);
        const double parc = ((fp / delta) / t) / t;
        if (fp > 0.0 && parl < *par) parl = *par;
        if (fp < 0.0 && paru > *par) paru = *par;
        *par = parl > *par + parc ? parl : *par + parc;
    }
    if (iter == 0) *par = 0.0;
}

/* lmdif with scipy's arguments (mode 2, diag = ones, factor 100,
 * epsfcn = EPS).  Returns MINPACK's info; *nfev_out the evaluations. */
int orc_lmdif(lm_fcn fcn, const void *ctx, int m, int n, double *x, double ftol, double xtol, double gtol,
              int maxfev, int *nfev_out) {
    double diag[LM_MAXN], qtf[LM_MAXN], wa1[LM_MAXN], wa2[LM_MAXN], wa3[LM_MAXN];
    int ipvt[LM_MAXN];
    const int lda = m;
    double *buf = (double *)malloc(sizeof(double) * (size_t)m * (n + 3));
    double *fvec = buf, *wa4 = buf + m, *wf = buf + 2 * (size_t)m, *fjac = buf + 3 * (size_t)m;
    const double factor = 100.0;
    int info = 0, nfev = 0;
    for (int j = 0; j < n; ++j) diag[j] = 1.0;
    fcn(x, fvec, ctx);
    nfev = 1;
    double fnorm = enorm(m, fvec);
    double par = 0.0, delta = 0.0, xnorm = 0.0;
    int iter = 1;
    const double eps = sqrt(EPSMCH);  /* fdjac2: sqrt(max(epsfcn, epsmch)) */
    for (;;) {
        /* fdjac2: forward differences */
        for (int j = 0; j < n; ++j) {
            const double temp = x[j];
            double h = eps * fabs(temp);
            if (h == 0.0) h = eps;
            x[j] = temp + h;
            fcn(x, wf, ctx);
            x[j] = temp;
            for (int i = 0; i < m; ++i) COL(fjac, j)[i] = (wf[i] - fvec[i]) / h;
        }
        nfev += n;
        qrfac(m, n, fjac, lda, ipvt, wa1, wa2);
        if (iter == 1) {
            for (int j = 0; j < n; ++j) wa3[j] = diag[j] * x[j];
            xnorm = enorm(n, wa3);
            delta = factor * xnorm;
            if (delta == 0.0) delta = factor;
        }
        for (int i = 0; i < m; ++i) wa4[i] = fvec[i];
        for (int j = 0; j < n; ++j) {
            if (COL(fjac, j)[j] != 0.0) {
                double sum = 0.0;
                for (int i = j; i < m; ++i) sum += COL(fjac, j)[i] * wa4[i];
                const double temp = -sum / COL(fjac, j)[j];
                for (int i = j; i < m; ++i) wa4[i] += COL(fjac, j)[i] * temp;
            }
            COL(fjac, j)[j] = wa1[j];
            qtf[j] = wa4[j];
        }
        double gnorm = 0.0;
        if (fnorm != 0.0) {
            for (int j = 0; j < n; ++j) {
                const int l = ipvt[j];
                if (wa2[l] != 0.0) {
                    double sum = 0.0;
                    for (int i = 0; i <= j; ++i) sum += COL(fjac, j)[i] * (qtf[i] / fnorm);
                    const double g = fabs(sum / wa2[l]);
                    if (g > gnorm) gnorm = g;
                }
            }
        }
        if (gnorm <= gtol) info = 4;
        if (info != 0) break;
        /* inner loop */
        double ratio;
        do {
            lmpar(n, fjac, lda, ipvt, diag, qtf, delta, &par, wa1, wa2);
            for (int j = 0; j < n; ++j) {
                wa1[j] = -wa1[j];
                wa2[j] = x[j] + wa1[j];
                wa3[j] = diag[j] * wa1[j];
            }
            const double pnorm = enorm(n, wa3);
            if (iter == 1 && pnorm < delta) delta = pnorm;
            fcn(wa2, wa4, ctx);
            nfev += 1;
            const double fnorm1 = enorm(m, wa4);
            double actred = -1.0;
            if (0.1 * fnorm1 < fnorm) {
                const double t = fnorm1 / fnorm;
                actred = 1.0 - t * t;
            }
            for (int j = 0; j < n; ++j) {
                wa3[j] = 0.0;
                const double temp = wa1[ipvt[j]];
                for (int i = 0; i <= j; ++i) wa3[i] += COL(fjac, j)[i] * temp;
            }
            const double temp1 = enorm(n, wa3) / fnorm;
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
                for (int j = 0; j < n; ++j) {
                    x[j] = wa2[j];
                    wa2[j] = diag[j] * x[j];
                }
                for (int i = 0; i < m; ++i) fvec[i] = wa4[i];
                xnorm = enorm(n, wa2);
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
    if (nfev_out) *nfev_out = nfev;
    free(buf);
    return info;
}

/* ------------------------------------------------ non-linear triangulation */
typedef struct {
    const double *P1, *P2;
    double u1, v1, u2, v2;
} nltri_ctx;

/* NonLinearTriangulation.py:5-50 Loss: reprojection error, with the
 * |z| < 1e-8 fallback that makes the residual of that view zero */
static void nltri_loss(const double *X, double *f, const void *vctx) {
    const nltri_ctx *c = (const nltri_ctx *)vctx;
    const double *Ps[2] = {c->P1, c->P2};
    const double obs[4] = {c->u1, c->v1, c->u2, c->v2};
    for (int v = 0; v < 2; ++v) {
        const double *P = Ps[v];
        /* P @ [X, 1]: numpy's 3x4 @ 4 mat-vec sums the even and odd terms
         * pairwise, (p0 x0 + p2 x2) + (p1 x1 + p3 * 1) (measured, no FMA) */
        double h[3];
        for (int r = 0; r < 3; ++r)
            h[r] = (P[4 * r] * X[0] + P[4 * r + 2] * X[2]) + (P[4 * r + 1] * X[1] + P[4 * r + 3]);
        double px, py;
        if (fabs(h[2]) < 1e-8) {
            px = obs[2 * v];
            py = obs[2 * v + 1];
        } else {
            px = h[0] / h[2];
            py = h[1] / h[2];
        }
        f[2 * v] = obs[2 * v] - px;
        f[2 * v + 1] = obs[2 * v + 1] - py;
    }
}

/* NonLinearTriangulation.py:53-121: per point, least_squares(method='lm',
 * max_nfev=50) from x0 = X0[i]; any exception (x0 not finite -> the bounds
 * check fails; residuals at x0 not finite -> ValueError) keeps X0[i].
 * info_out[i] = MINPACK info, or -1 for the exception path. */
void orc_nltri(const double *P1, const double *P2, const double *x1, const double *x2, const double *X0,
               int64_t n, int32_t max_nfev, double *X, int32_t *info_out) {
    for (int64_t i = 0; i < n; ++i) {
        nltri_ctx c = {P1, P2, x1[2 * i], x1[2 * i + 1], x2[2 * i], x2[2 * i + 1]};
        double x[3] = {X0[3 * i], X0[3 * i + 1], X0[3 * i + 2]};
        int info = -1;
        /* scipy in_bounds(x0, -inf, inf): a NaN fails the comparison */
        int ok = !(isnan(x[0]) || isnan(x[1]) || isnan(x[2]));
        if (ok) {
            double f0[4];
            nltri_loss(x, f0, &c);
            for (int k = 0; k < 4; ++k)
                if (!isfinite(f0[k])) ok = 0;
        }
        if (ok) {
            int nfev = 0;
            info = orc_lmdif(nltri_loss, &c, 4, 3, x, 1e-8, 1e-8, 1e-8, max_nfev, &nfev);
        } else {
            x[0] = X0[3 * i];
            x[1] = X0[3 * i + 1];
            x[2] = X0[3 * i + 2];
        }
        memcpy(X + 3 * i, x, 3 * sizeof(double));
        if (info_out) info_out[i] = info;
    }
}
