/* TEST INFRASTRUCTURE -- the "CPU-strong" baseline of SURVEY §8(d): the
 * same Schur-complement LM as orc_ba_lm (sfm_oracle.c; reference residual
 * BundleAdjustment.py:43-110, observations point-major as :164-169), written
 * for throughput on the host's cores with OpenMP:
 *   - linearisation, elimination, back substitution and the trial cost are
 *     parallel over points (observations of a point stay on one thread);
 *   - W = Jc^T Jp and Y = W V^-1 are formed once per observation (parallel
 *     over points); the reduced camera system is then accumulated by camera
 *     ROW: a thread owns a block row (camera c1, dynamic schedule) and walks
 *     c1's observations (camera-major list), adding every pair (c1 <= c2)
 *     of their points into its own row -- no per-thread copies of S, no
 *     reduction, no atomics, a fixed order per row;
 *   - the dense Cholesky is blocked (64-wide panels, parallel panel solve
 *     and trailing update).
 * Only bench.py's cpu_baseline leg and tests/ use it.  Not the reference:
 * the reference path (MINPACK lmdif with a dense forward-difference
 * Jacobian) cannot run at cfg4/cfg5.
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    int32_t max_iterations;
    double function_tolerance;
    double gradient_tolerance;
    double parameter_tolerance;
    double initial_lambda;
} cs_opts;

typedef struct {
    int32_t iterations, accepted, status, threads;
    double cost0, cost;
} cs_report;

void orc_rotvec_to_R(const double *w, double *R);
void orc_R_to_rotvec(const double *R, double *w);

static double clampd(double x) { return x < 1e-6 ? 1e-6 : (x > 1e32 ? 1e32 : x); }

/* residual and Jacobians of one observation (left-perturbed rotation) */
static void lin_obs(const double *Rc, const double *t, const double *X, const double *K, const double *ob,
                    double *e, double *Jc, double *Jp) {
    double p[3], u[3];
    for (int i = 0; i < 3; ++i) p[i] = Rc[3 * i] * X[0] + Rc[3 * i + 1] * X[1] + Rc[3 * i + 2] * X[2];
    const double x0 = p[0] + t[0], x1 = p[1] + t[1], x2 = p[2] + t[2];
    for (int i = 0; i < 3; ++i) u[i] = K[3 * i] * x0 + K[3 * i + 1] * x1 + K[3 * i + 2] * x2;
    const double iw = 1.0 / (u[2] + 1e-8), pu = u[0] * iw, pv = u[1] * iw;
    e[0] = ob[0] - pu;
    e[1] = ob[1] - pv;
    if (!Jc) return;
    double A[6];
    for (int c = 0; c < 3; ++c) {
        A[c] = -(iw * K[c] - pu * iw * K[6 + c]);
        A[3 + c] = -(iw * K[3 + c] - pv * iw * K[6 + c]);
    }
    for (int a = 0; a < 2; ++a) {
        const double *Aa = A + 3 * a;
        double *J = Jc + 6 * a;
        J[0] = Aa[1] * (-p[2]) + Aa[2] * p[1];
        J[1] = Aa[0] * p[2] + Aa[2] * (-p[0]);
        J[2] = Aa[0] * (-p[1]) + Aa[1] * p[0];
        J[3] = Aa[0]; J[4] = Aa[1]; J[5] = Aa[2];
        for (int c = 0; c < 3; ++c) Jp[3 * a + c] = Aa[0] * Rc[c] + Aa[1] * Rc[3 + c] + Aa[2] * Rc[6 + c];
    }
}

static void inv3_sym(const double *M, double *I) {
    double a = M[0], b = M[1], c = M[2], d = M[4], e = M[5], f = M[8];
    double A = d * f - e * e, B = c * e - b * f, C = b * e - c * d;
    double id = 1.0 / (a * A + b * B + c * C);
    I[0] = A * id; I[1] = B * id; I[2] = C * id;
    I[3] = B * id; I[4] = (a * f - c * c) * id; I[5] = (b * c - a * e) * id;
    I[6] = C * id; I[7] = (b * c - a * e) * id; I[8] = (a * d - b * b) * id;
}

/* dense lower Cholesky of the full symmetric S (n x n, row-major; the lower
 * triangle is read and overwritten by L) + the two triangular solves; blocked
 * right-looking with NB-wide panels: the diagonal block serially, the panel
 * rows and the trailing update in parallel over rows */
#define CS_NB 64
static int chol_solve_par(double *S, int n, double *b) {
    int bad = 0;
    for (int k0 = 0; k0 < n && !bad; k0 += CS_NB) {
        const int k1 = k0 + CS_NB < n ? k0 + CS_NB : n;
        for (int j = k0; j < k1; ++j) { /* diagonal block, unblocked (its columns k0..j-1 updated) */
            double *Sj = S + (size_t)j * n;
            double d = Sj[j];
            for (int k = k0; k < j; ++k) d -= Sj[k] * Sj[k];
            if (!(d > 0)) { bad = 1; break; }
            d = sqrt(d);
            Sj[j] = d;
            for (int i = j + 1; i < k1; ++i) {
                double *Si = S + (size_t)i * n;
                double v = Si[j];
                for (int k = k0; k < j; ++k) v -= Si[k] * Sj[k];
                Si[j] = v / d;
            }
        }
        if (bad) break;
#pragma omp parallel for schedule(static)
        for (int i = k1; i < n; ++i) { /* panel rows: L_ik = S_ik L_kk^-T */
            double *Si = S + (size_t)i * n;
            for (int j = k0; j < k1; ++j) {
                const double *Sj = S + (size_t)j * n;
                double v = Si[j];
                for (int k = k0; k < j; ++k) v -= Si[k] * Sj[k];
                Si[j] = v / Sj[j];
            }
        }
#pragma omp parallel for schedule(dynamic, 8)
        for (int i = k1; i < n; ++i) { /* trailing update of row i: S_ij -= L_i. L_j. (j <= i) */
            double *Si = S + (size_t)i * n;
            for (int j = k1; j <= i; ++j) {
                const double *Sj = S + (size_t)j * n;
                double v = 0;
                for (int k = k0; k < k1; ++k) v += Si[k] * Sj[k];
                Si[j] -= v;
            }
        }
    }
    if (bad) return -1;
    for (int i = 0; i < n; ++i) {
        double v = b[i];
        for (int k = 0; k < i; ++k) v -= S[(size_t)i * n + k] * b[k];
        b[i] = v / S[(size_t)i * n + i];
    }
    for (int i = n - 1; i >= 0; --i) {
        double v = b[i];
        for (int k = i + 1; k < n; ++k) v -= S[(size_t)k * n + i] * b[k];
        b[i] = v / S[(size_t)i * n + i];
    }
    return 0;
}

int cs_ba_lm(int32_t nc, int64_t np_, int64_t no, const int32_t *cam, const int32_t *pt, const double *obs,
             const double *K, double *cams, double *pts, const cs_opts *opt, cs_report *rep) {
    const int ns = 6 * nc;
    const int nth = omp_get_max_threads();
    for (int64_t o = 1; o < no; ++o)
        if (pt[o] < pt[o - 1]) return -3;
    int64_t *pstart = calloc(np_ + 1, sizeof(int64_t));
    for (int64_t o = 0; o < no; ++o) pstart[pt[o] + 1]++;
    for (int64_t p = 0; p < np_; ++p) pstart[p + 1] += pstart[p];
    double *R = malloc(sizeof(double) * 9 * nc), *t = malloc(sizeof(double) * 3 * nc);
    double *Rn = malloc(sizeof(double) * 9 * nc), *tn = malloc(sizeof(double) * 3 * nc);
    double *J = malloc(sizeof(double) * 20 * (no ? no : 1)), *W = malloc(sizeof(double) * 18 * (no ? no : 1));
    double *Y = malloc(sizeof(double) * 18 * (no ? no : 1));
    double *V = malloc(sizeof(double) * 9 * (np_ ? np_ : 1)), *gp = malloc(sizeof(double) * 3 * (np_ ? np_ : 1));
    double *Vi = malloc(sizeof(double) * 9 * (np_ ? np_ : 1)), *dp = malloc(sizeof(double) * 3 * (np_ ? np_ : 1));
    double *Xn = malloc(sizeof(double) * 3 * (np_ ? np_ : 1));
    double *U = malloc(sizeof(double) * 36 * nc), *gc = malloc(sizeof(double) * ns);
    double *S = malloc(sizeof(double) * (size_t)ns * ns), *b = malloc(sizeof(double) * ns);
    double *Vg = malloc(sizeof(double) * 3 * (np_ ? np_ : 1));
    double *Ut = malloc(sizeof(double) * (size_t)nth * (36 * nc + ns));
    /* camera-major observation list (point order within a camera) */
    int64_t *cstart = calloc(nc + 1, sizeof(int64_t)), *cm = malloc(sizeof(int64_t) * (no ? no : 1));
    for (int64_t o = 0; o < no; ++o) cstart[cam[o] + 1]++;
    for (int c = 0; c < nc; ++c) cstart[c + 1] += cstart[c];
    {
        int64_t *fill = malloc(sizeof(int64_t) * (nc ? nc : 1));
        for (int c = 0; c < nc; ++c) fill[c] = cstart[c];
        for (int64_t o = 0; o < no; ++o) cm[fill[cam[o]]++] = o;
        free(fill);
    }
    for (int c = 0; c < nc; ++c) {
        orc_rotvec_to_R(cams + 6 * c, R + 9 * c);
        memcpy(t + 3 * c, cams + 6 * c + 3, 3 * sizeof(double));
    }
    double lambda = opt->initial_lambda, nu = 2.0, cost = 0, cost0 = -1;
    int need_lin = 1, status = 4, accepted = 0, it;
    for (it = 0; it < opt->max_iterations; ++it) {
        if (need_lin) {
            double csum = 0;
            memset(Ut, 0, sizeof(double) * (size_t)nth * (36 * nc + ns));
#pragma omp parallel reduction(+ : csum)
            {
                double *Uc_t = Ut + (size_t)omp_get_thread_num() * (36 * nc + ns), *gc_t = Uc_t + 36 * nc;
#pragma omp for schedule(dynamic, 256)
                for (int64_t p = 0; p < np_; ++p) {
                    double *Vp = V + 9 * p, *g = gp + 3 * p;
                    memset(Vp, 0, 9 * sizeof(double));
                    memset(g, 0, 3 * sizeof(double));
                    for (int64_t o = pstart[p]; o < pstart[p + 1]; ++o) {
                        const int c = cam[o];
                        double *e = J + 20 * o, *Jc = e + 2, *Jp = e + 14;
                        lin_obs(R + 9 * c, t + 3 * c, pts + 3 * p, K, obs + 2 * o, e, Jc, Jp);
                        csum += 0.5 * (e[0] * e[0] + e[1] * e[1]);
                        double *Uc = Uc_t + 36 * c;
                        for (int i = 0; i < 6; ++i) {
                            for (int j = i; j < 6; ++j) Uc[6 * i + j] += Jc[i] * Jc[j] + Jc[6 + i] * Jc[6 + j];
                            gc_t[6 * c + i] += Jc[i] * e[0] + Jc[6 + i] * e[1];
                        }
                        for (int i = 0; i < 3; ++i) {
                            for (int j = 0; j < 3; ++j) Vp[3 * i + j] += Jp[i] * Jp[j] + Jp[3 + i] * Jp[3 + j];
                            g[i] += Jp[i] * e[0] + Jp[3 + i] * e[1];
                        }
                        double *w = W + 18 * o;
                        for (int i = 0; i < 6; ++i)
                            for (int j = 0; j < 3; ++j) w[3 * i + j] = Jc[i] * Jp[j] + Jc[6 + i] * Jp[3 + j];
                    }
                }
            }
            memset(U, 0, sizeof(double) * 36 * nc);
            memset(gc, 0, sizeof(double) * ns);
            for (int th = 0; th < nth; ++th) {
                const double *u = Ut + (size_t)th * (36 * nc + ns);
                for (int k = 0; k < 36 * nc; ++k) U[k] += u[k];
                for (int k = 0; k < ns; ++k) gc[k] += u[36 * nc + k];
            }
            for (int c = 0; c < nc; ++c)
                for (int i = 0; i < 6; ++i)
                    for (int j = 0; j < i; ++j) U[36 * c + 6 * i + j] = U[36 * c + 6 * j + i];
            cost = csum;
            if (cost0 < 0) cost0 = cost;
            double gmax = 0;
            for (int i = 0; i < ns; ++i) if (fabs(gc[i]) > gmax) gmax = fabs(gc[i]);
            for (int64_t i = 0; i < 3 * np_; ++i) if (fabs(gp[i]) > gmax) gmax = fabs(gp[i]);
            if (gmax < opt->gradient_tolerance) { status = 2; break; }
            need_lin = 0;
        }
        /* elimination, pass 1 (parallel over points): V^-1, V^-1 g, Y = W V^-1 */
#pragma omp parallel for schedule(dynamic, 256)
        for (int64_t p = 0; p < np_; ++p) {
            double Vd[9];
            memcpy(Vd, V + 9 * p, sizeof Vd);
            for (int i = 0; i < 3; ++i) Vd[4 * i] += lambda * clampd(V[9 * p + 4 * i]);
            double *Vinv = Vi + 9 * p;
            inv3_sym(Vd, Vinv);
            const double *g = gp + 3 * p;
            for (int i = 0; i < 3; ++i) Vg[3 * p + i] = Vinv[3 * i] * g[0] + Vinv[3 * i + 1] * g[1] + Vinv[3 * i + 2] * g[2];
            for (int64_t oa = pstart[p]; oa < pstart[p + 1]; ++oa) {
                const double *Wa = W + 18 * oa;
                double *Ya = Y + 18 * oa;
                for (int i = 0; i < 6; ++i)
                    for (int j = 0; j < 3; ++j)
                        Ya[3 * i + j] = Wa[3 * i] * Vinv[j] + Wa[3 * i + 1] * Vinv[3 + j] + Wa[3 * i + 2] * Vinv[6 + j];
            }
        }
        /* pass 2 (parallel over camera block rows): row c1 of the upper
         * camera blocks and b_c1, from c1's observations and their points */
#pragma omp parallel for schedule(dynamic, 1)
        for (int c1 = 0; c1 < nc; ++c1) {
            for (int i = 0; i < 6; ++i) {
                memset(S + (size_t)(6 * c1 + i) * ns + 6 * c1, 0, sizeof(double) * (ns - 6 * c1));
                b[6 * c1 + i] = -gc[6 * c1 + i];
            }
            for (int64_t k = cstart[c1]; k < cstart[c1 + 1]; ++k) {
                const int64_t oa = cm[k], p = pt[oa];
                const double *Wa = W + 18 * oa, *Ya = Y + 18 * oa, *vg = Vg + 3 * p;
                for (int i = 0; i < 6; ++i) b[6 * c1 + i] += Wa[3 * i] * vg[0] + Wa[3 * i + 1] * vg[1] + Wa[3 * i + 2] * vg[2];
                for (int64_t ob = pstart[p]; ob < pstart[p + 1]; ++ob) {
                    const int c2 = cam[ob];
                    if (c2 < c1) continue;  /* the upper block (c1 <= c2) */
                    const double *Wb = W + 18 * ob;
                    double *blk = S + (size_t)(6 * c1) * ns + 6 * c2;
                    for (int i = 0; i < 6; ++i)
                        for (int j = 0; j < 6; ++j)
                            blk[(size_t)i * ns + j] -= Ya[3 * i] * Wb[3 * j] + Ya[3 * i + 1] * Wb[3 * j + 1] + Ya[3 * i + 2] * Wb[3 * j + 2];
                }
            }
            /* + U and the damping on the diagonal block */
            for (int i = 0; i < 6; ++i) {
                for (int j = 0; j < 6; ++j) S[(size_t)(6 * c1 + i) * ns + 6 * c1 + j] += U[36 * c1 + 6 * i + j];
                S[(size_t)(6 * c1 + i) * ns + 6 * c1 + i] += lambda * clampd(U[36 * c1 + 7 * i]);
            }
        }
        /* mirror the upper blocks into the lower triangle (read by the factor) */
#pragma omp parallel for schedule(static)
        for (int r = 0; r < ns; ++r)
            for (int j = 0; j < r; ++j) S[(size_t)r * ns + j] = S[(size_t)j * ns + r];
        double *dc = b;
        const int ok = chol_solve_par(S, ns, b) == 0;
        double model = 0, cost_new = 0, dnorm = 0, xnorm = 0;
        if (ok) {
            double mp = 0, dn = 0, xn = 0, cn = 0;
            for (int c = 0; c < nc; ++c) {
                double dR[9], *Rnc = Rn + 9 * c;
                orc_rotvec_to_R(dc + 6 * c, dR);
                for (int i = 0; i < 3; ++i)
                    for (int j = 0; j < 3; ++j)
                        Rnc[3 * i + j] = dR[3 * i] * R[9 * c + j] + dR[3 * i + 1] * R[9 * c + 3 + j] + dR[3 * i + 2] * R[9 * c + 6 + j];
                for (int i = 0; i < 3; ++i) { tn[3 * c + i] = t[3 * c + i] + dc[6 * c + 3 + i]; xnorm += t[3 * c + i] * t[3 * c + i]; }
                for (int i = 0; i < 6; ++i) {
                    const double d = dc[6 * c + i];
                    model += d * (lambda * clampd(U[36 * c + 7 * i]) * d - gc[6 * c + i]);
                    dnorm += d * d;
                }
            }
#pragma omp parallel for schedule(dynamic, 256) reduction(+ : mp, dn, xn, cn)
            for (int64_t p = 0; p < np_; ++p) {
                double rhs[3] = {-gp[3 * p], -gp[3 * p + 1], -gp[3 * p + 2]};
                for (int64_t o = pstart[p]; o < pstart[p + 1]; ++o) {
                    const double *w = W + 18 * o, *d = dc + 6 * cam[o];
                    for (int j = 0; j < 3; ++j) {
                        double s = 0;
                        for (int i = 0; i < 6; ++i) s += w[3 * i + j] * d[i];
                        rhs[j] -= s;
                    }
                }
                const double *Vinv = Vi + 9 * p;
                for (int i = 0; i < 3; ++i) {
                    const double d = Vinv[3 * i] * rhs[0] + Vinv[3 * i + 1] * rhs[1] + Vinv[3 * i + 2] * rhs[2];
                    dp[3 * p + i] = d;
                    mp += d * (lambda * clampd(V[9 * p + 4 * i]) * d - gp[3 * p + i]);
                    dn += d * d;
                    xn += pts[3 * p + i] * pts[3 * p + i];
                    Xn[3 * p + i] = pts[3 * p + i] + d;
                }
                for (int64_t o = pstart[p]; o < pstart[p + 1]; ++o) {
                    double e[2];
                    const int c = cam[o];
                    lin_obs(Rn + 9 * c, tn + 3 * c, Xn + 3 * p, K, obs + 2 * o, e, NULL, NULL);
                    cn += 0.5 * (e[0] * e[0] + e[1] * e[1]);
                }
            }
            model = 0.5 * (model + mp);
            dnorm += dn;
            xnorm += xn;
            cost_new = cn;
        }
        const double rho = ok && model > 0 ? (cost - cost_new) / model : -1.0;
        if (ok && rho > 1e-3 && isfinite(cost_new)) {
            const double dcost = cost - cost_new;
            memcpy(R, Rn, sizeof(double) * 9 * nc);
            memcpy(t, tn, sizeof(double) * 3 * nc);
            memcpy(pts, Xn, sizeof(double) * 3 * np_);
            accepted++;
            double f = 2.0 * rho - 1.0;
            f = 1.0 - f * f * f;
            lambda *= f > 1.0 / 3.0 ? f : 1.0 / 3.0;
            nu = 2.0;
            cost = cost_new;
            need_lin = 1;
            if (dcost < opt->function_tolerance * cost) { status = 1; it++; break; }
            if (sqrt(dnorm) < opt->parameter_tolerance * (sqrt(xnorm) + opt->parameter_tolerance)) { status = 3; it++; break; }
        } else {
            lambda *= nu;
            nu *= 2.0;
            if (lambda > 1e32) { status = 5; it++; break; }
        }
    }
    for (int c = 0; c < nc; ++c) {
        orc_R_to_rotvec(R + 9 * c, cams + 6 * c);
        memcpy(cams + 6 * c + 3, t + 3 * c, 3 * sizeof(double));
    }
    if (rep) {
        rep->iterations = it; rep->accepted = accepted; rep->status = status; rep->threads = nth;
        rep->cost0 = cost0; rep->cost = cost;
    }
    free(pstart); free(R); free(t); free(Rn); free(tn); free(J); free(W); free(Y); free(V); free(gp); free(Vi);
    free(dp); free(Xn); free(U); free(gc); free(S); free(b); free(Vg); free(Ut); free(cstart); free(cm);
    return 0;
}

/* ---------------------------------------------------------------------
 * CPU-strong RANSAC (bench.py's cpu leg): orc_ransac's loop with the
 * hypotheses split over the OpenMP threads (each fits its F with orc_f8 and
 * counts with orc_ransac_score), then the reference's strict-'>' winner
 * (GetInliersRANSAC.py:85-88: most inliers, earliest iteration) in
 * iteration order.  Same counts as orc_ransac.
 * --------------------------------------------------------------------- */
int orc_f8(const double *p1, const double *p2, int64_t n, double *F_out);
void orc_ransac_score(const double *x1, const double *x2, int64_t n, const double *F, int64_t H, double thr,
                      int32_t *counts);

int64_t cs_ransac(const double *x1, const double *x2, int64_t n, const int32_t *samples, int64_t H, int k,
                  double thr, int32_t *counts) {
    if (k > 64) return -2;
#pragma omp parallel for schedule(dynamic, 64)
    for (int64_t h = 0; h < H; ++h) {
        double p1[2 * 64], p2[2 * 64], F[9];
        for (int j = 0; j < k; ++j) {
            const int32_t s = samples[h * k + j];
            p1[2 * j] = x1[2 * s]; p1[2 * j + 1] = x1[2 * s + 1];
            p2[2 * j] = x2[2 * s]; p2[2 * j + 1] = x2[2 * s + 1];
        }
        int32_t c = 0;
        if (orc_f8(p1, p2, k, F) == 0) orc_ransac_score(x1, x2, n, F, 1, thr, &c);
        counts[h] = c;
    }
    int64_t best = -1;
    int32_t best_c = 0;
    for (int64_t h = 0; h < H; ++h)
        if (counts[h] > best_c) { best_c = counts[h]; best = h; }
    return best;
}

/* thread count of the OpenMP legs (0: leave OMP_NUM_THREADS' choice) */
void cs_set_threads(int n) {
    if (n > 0) omp_set_num_threads(n);
}
int cs_max_threads(void) { return omp_get_max_threads(); }
