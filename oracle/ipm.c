/*
 * oracle/ipm.c -- Ipopt 3.12.8 restated (TEST INFRASTRUCTURE ONLY, see ora.h).
 *
 * The reference hands its NLP to CppAD::ipopt::solve (mpc_ros/include/cppad/ipopt/
 * solve.hpp:419-589) which runs IpoptApplication::OptimizeTNLP with the options of
 * mpc_planner.cpp:356-368 (print_level 0, sparse reverse derivatives, max_cpu_time
 * 0.5) and Ipopt defaults otherwise.  Ipopt is not vendored and not in the image,
 * so this file restates its published algorithm (Waechter & Biegler 2006, "On the
 * implementation of an interior-point filter line-search algorithm for large-scale
 * nonlinear programming", Algorithm A + Algorithm IC), with the Ipopt 3.12 defaults:
 *
 *   mu_init 0.1, kappa_eps 10, kappa_mu 0.2, theta_mu 1.5, tau_min 0.99,
 *   bound_push = bound_frac = 0.01 (and the slack_* equivalents), bound_mult_init 1,
 *   constr_mult_init_max 1000 (least-squares y0), kappa_sigma 1e10, kappa_d 1e-5,
 *   gamma_theta 1e-5, gamma_phi 1e-8, delta 1, gamma_alpha 0.05, s_theta 1.1,
 *   s_phi 2.3, eta_phi 1e-8, theta_max 1e4*max(1,theta0), theta_min 1e-4*max(1,theta0),
 *   inertia correction delta_w0 1e-4, delta_w_min 1e-20, delta_w_max 1e40,
 *   kappa_w- 1/3, kappa_w+ 8, kappa_w+bar 100, delta_c 1e-8 mu^0.25,
 *   bound_relax_factor 1e-8 (capped by constr_viol_tol 1e-4), honor_original_bounds,
 *   gradient-based NLP scaling (nlp_scaling_max_gradient 100),
 *   termination: scaled E_0 <= tol (s_max 100) and dual_inf_tol 1,
 *   constr_viol_tol 1e-4, compl_inf_tol 1e-4.
 *
 * Not restated (documented in DESIGN.md): second-order corrections, the feasibility
 * restoration phase (a line-search failure returns RESTORATION_FAILURE), the
 * watchdog (off by default in Ipopt), and "acceptable" termination.
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "ora.h"

#define INF_BOUND 1e19

void ora_ipm_default_opts(ora_ipm_opts* o) {
    o->tol = 1e-8;
    o->max_iter = 3000;
    o->bound_relax_factor = 1e-8;
    o->honor_original_bounds = 1;
    o->mu_init = 0.1;
    o->print_level = 0;
}

typedef struct {
    const ora_nlp* nlp;
    int n, m, nw, mI;
    int* ineq_of_row;   /* row -> slack index or -1 */
    double obj_scale;
    double* c_scale;    /* per constraint row */
    double *wl, *wu;    /* relaxed bounds on w = (x, s) */
    char *hasL, *hasU;
    /* work */
    double *gf, *gv, *jac, *hess, *lam_unscaled;
} ipm_ctx;

static double amax(int n, const double* v) {
    double m = 0.0;
    for (int i = 0; i < n; ++i) m = fmax(m, fabs(v[i]));
    return m;
}

/* scaled objective */
static double eval_f(ipm_ctx* c, const double* w) { return c->obj_scale * c->nlp->f(c->nlp->ctx, w); }

static void eval_grad(ipm_ctx* c, const double* w, double* g) {
    c->nlp->grad_f(c->nlp->ctx, w, g);
    for (int i = 0; i < c->n; ++i) g[i] *= c->obj_scale;
    for (int i = c->n; i < c->nw; ++i) g[i] = 0.0;
}

/* scaled constraint residual c(w): eq rows g - gl; ineq rows g - s */
static void eval_c(ipm_ctx* c, const double* w, double* cv) {
    const ora_nlp* p = c->nlp;
    p->g(p->ctx, w, c->gv);
    for (int r = 0; r < c->m; ++r) {
        int s = c->ineq_of_row[r];
        double v = (s < 0) ? c->gv[r] - p->gl[r] : c->gv[r] - w[c->n + s];
        cv[r] = c->c_scale[r] * v;
    }
}

/* scaled Jacobian of c wrt w, dense m x nw row-major */
static void eval_A(ipm_ctx* c, const double* w, double* A) {
    const ora_nlp* p = c->nlp;
    p->jac_g(p->ctx, w, c->jac);
    for (int r = 0; r < c->m; ++r) {
        double* row = A + (size_t)r * c->nw;
        for (int j = 0; j < c->n; ++j) row[j] = c->c_scale[r] * c->jac[(size_t)r * c->n + j];
        for (int j = c->n; j < c->nw; ++j) row[j] = 0.0;
        int s = c->ineq_of_row[r];
        if (s >= 0) row[c->n + s] = -c->c_scale[r];
    }
}

/* scaled Lagrangian Hessian (x block), full n x n */
static void eval_W(ipm_ctx* c, const double* w, const double* y, double* W) {
    for (int r = 0; r < c->m; ++r) c->lam_unscaled[r] = y[r] * c->c_scale[r];
    c->nlp->hess(c->nlp->ctx, w, c->obj_scale, c->lam_unscaled, W);
}

static double barrier_phi(ipm_ctx* c, const double* w, double mu, int* ok) {
    const double kd = 1e-5;
    double phi = eval_f(c, w);
    *ok = 1;
    for (int i = 0; i < c->nw; ++i) {
        if (c->hasL[i]) {
            double d = w[i] - c->wl[i];
            if (!(d > 0)) { *ok = 0; return INFINITY; }
            phi -= mu * log(d);
            if (!c->hasU[i]) phi += kd * mu * d;
        }
        if (c->hasU[i]) {
            double d = c->wu[i] - w[i];
            if (!(d > 0)) { *ok = 0; return INFINITY; }
            phi -= mu * log(d);
            if (!c->hasL[i]) phi += kd * mu * d;
        }
    }
    if (!isfinite(phi)) *ok = 0;
    return phi;
}

static void barrier_grad(ipm_ctx* c, const double* w, double mu, const double* gf, double* gphi) {
    const double kd = 1e-5;
    for (int i = 0; i < c->nw; ++i) {
        double g = gf[i];
        if (c->hasL[i]) {
            g -= mu / (w[i] - c->wl[i]);
            if (!c->hasU[i]) g += kd * mu;
        }
        if (c->hasU[i]) {
            g += mu / (c->wu[i] - w[i]);
            if (!c->hasL[i]) g -= kd * mu;
        }
        gphi[i] = g;
    }
}

static double l1(int n, const double* v) {
    double s = 0.0;
    for (int i = 0; i < n; ++i) s += fabs(v[i]);
    return s;
}

typedef struct { double th, ph; } fpair;

int ora_ipm_solve(const ora_nlp* nlp, const ora_ipm_opts* opts_in, double* x_out, double* zl_out,
                  double* zu_out, double* lambda_out, double* g_out, ora_ipm_result* res) {
    ora_ipm_opts opts;
    if (opts_in) opts = *opts_in; else ora_ipm_default_opts(&opts);
    const int n = nlp->n, m = nlp->m;
    ipm_ctx C;
    memset(&C, 0, sizeof C);
    C.nlp = nlp;
    C.n = n;
    C.m = m;
    C.ineq_of_row = (int*)malloc(sizeof(int) * (m > 0 ? m : 1));
    int mI = 0;
    for (int r = 0; r < m; ++r) {
        if (nlp->gl[r] == nlp->gu[r]) C.ineq_of_row[r] = -1;
        else C.ineq_of_row[r] = mI++;
    }
    C.mI = mI;
    const int nw = n + mI;
    C.nw = nw;
    const int K = nw + m;
    double* mem = (double*)calloc((size_t)(
        20 * nw + 10 * m + (size_t)m * n + (size_t)n * n + (size_t)m * nw + (size_t)K * K + 4 * K + 16), sizeof(double));
    double* p = mem;
#define TAKE(ptr, cnt) do { ptr = p; p += (cnt); } while (0)
    double *w, *wt, *y, *zL, *zU, *dw, *dy, *dzL, *dzU, *gf, *gphi, *cv, *ct, *rd, *A, *W, *KKT, *rhs, *wl0, *wu0;
    TAKE(w, nw); TAKE(wt, nw); TAKE(y, m); TAKE(zL, nw); TAKE(zU, nw); TAKE(dw, nw); TAKE(dy, m);
    TAKE(dzL, nw); TAKE(dzU, nw); TAKE(gf, nw); TAKE(gphi, nw); TAKE(cv, m); TAKE(ct, m); TAKE(rd, nw);
    TAKE(A, (size_t)m * nw); TAKE(W, (size_t)n * n); TAKE(KKT, (size_t)K * K); TAKE(rhs, K);
    TAKE(wl0, nw); TAKE(wu0, nw);
    TAKE(C.wl, nw); TAKE(C.wu, nw); TAKE(C.gv, m); TAKE(C.jac, (size_t)m * n); TAKE(C.lam_unscaled, m);
    TAKE(C.c_scale, m);
#undef TAKE
    int* ipiv = (int*)malloc(sizeof(int) * K);
    C.hasL = (char*)calloc(nw, 1);
    C.hasU = (char*)calloc(nw, 1);
    int nfilter = 0, capfilter = 256;
    fpair* filter = (fpair*)malloc(sizeof(fpair) * capfilter);

    /* ---- bounds on w (original), then relaxation (Ipopt bound_relax_factor) ---- */
    for (int i = 0; i < n; ++i) { wl0[i] = nlp->xl[i]; wu0[i] = nlp->xu[i]; }
    for (int r = 0; r < m; ++r) {
        int s = C.ineq_of_row[r];
        if (s >= 0) { wl0[n + s] = nlp->gl[r]; wu0[n + s] = nlp->gu[r]; }
    }
    for (int i = 0; i < nw; ++i) {
        C.hasL[i] = wl0[i] > -INF_BOUND;
        C.hasU[i] = wu0[i] < INF_BOUND;
        double rl = fmin(1e-4, opts.bound_relax_factor * fmax(1.0, fabs(wl0[i])));
        double ru = fmin(1e-4, opts.bound_relax_factor * fmax(1.0, fabs(wu0[i])));
        C.wl[i] = C.hasL[i] ? wl0[i] - rl : -INFINITY;
        C.wu[i] = C.hasU[i] ? wu0[i] + ru : INFINITY;
    }

    /* ---- starting point: x0 pushed inside (bound_push/bound_frac 0.01) ---- */
    for (int i = 0; i < n; ++i) w[i] = nlp->x0[i];
    /* gradient-based scaling at the user's starting point */
    {
        nlp->grad_f(nlp->ctx, w, gf);
        double gmax = amax(n, gf);
        C.obj_scale = (gmax > 100.0) ? 100.0 / gmax : 1.0;
        nlp->jac_g(nlp->ctx, w, C.jac);
        for (int r = 0; r < m; ++r) {
            double rm = amax(n, C.jac + (size_t)r * n);
            C.c_scale[r] = (rm > 100.0) ? 100.0 / rm : 1.0;
        }
    }
    nlp->g(nlp->ctx, w, C.gv);
    for (int r = 0; r < m; ++r) {
        int s = C.ineq_of_row[r];
        if (s >= 0) w[n + s] = C.gv[r];
    }
    for (int i = 0; i < nw; ++i) {
        const double k1 = 0.01, k2 = 0.01;
        if (C.hasL[i] && C.hasU[i]) {
            double pl = fmin(k1 * fmax(1.0, fabs(C.wl[i])), k2 * (C.wu[i] - C.wl[i]));
            double pu = fmin(k1 * fmax(1.0, fabs(C.wu[i])), k2 * (C.wu[i] - C.wl[i]));
            if (w[i] < C.wl[i] + pl) w[i] = C.wl[i] + pl;
            if (w[i] > C.wu[i] - pu) w[i] = C.wu[i] - pu;
        } else if (C.hasL[i]) {
            double pl = k1 * fmax(1.0, fabs(C.wl[i]));
            if (w[i] < C.wl[i] + pl) w[i] = C.wl[i] + pl;
        } else if (C.hasU[i]) {
            double pu = k1 * fmax(1.0, fabs(C.wu[i]));
            if (w[i] > C.wu[i] - pu) w[i] = C.wu[i] - pu;
        }
    }
    for (int i = 0; i < nw; ++i) {
        zL[i] = C.hasL[i] ? 1.0 : 0.0;
        zU[i] = C.hasU[i] ? 1.0 : 0.0;
    }
    int nbnd = 0;
    for (int i = 0; i < nw; ++i) nbnd += C.hasL[i] + C.hasU[i];

    /* ---- least-squares multiplier estimate (constr_mult_init_max 1000) ---- */
    eval_grad(&C, w, gf);
    eval_A(&C, w, A);
    memset(KKT, 0, sizeof(double) * (size_t)K * K);
    for (int i = 0; i < nw; ++i) KKT[i + (size_t)i * K] = 1.0;
    for (int r = 0; r < m; ++r)
        for (int j = 0; j < nw; ++j) KKT[(nw + r) + (size_t)j * K] = A[(size_t)r * nw + j];
    for (int i = 0; i < nw; ++i) rhs[i] = -(gf[i] - zL[i] + zU[i]);
    for (int r = 0; r < m; ++r) rhs[nw + r] = 0.0;
    {
        int np, nn, nz;
        ora_ldlt_factor(K, KKT, ipiv, 1e-300, &np, &nn, &nz);
        if (nz == 0) {
            ora_ldlt_solve(K, KKT, ipiv, rhs);
            double ym = amax(m, rhs + nw);
            for (int r = 0; r < m; ++r) y[r] = (ym <= 1000.0) ? rhs[nw + r] : 0.0;
        } else {
            for (int r = 0; r < m; ++r) y[r] = 0.0;
        }
    }

    double mu = opts.mu_init;
    const double mu_min = opts.tol / 10.0;
    double tau = fmax(0.99, 1.0 - mu);
    const double kappa_eps = 10.0, kappa_mu = 0.2, theta_mu = 1.5, kappa_sigma = 1e10;
    const double gamma_theta = 1e-5, gamma_phi = 1e-8, delta_sw = 1.0, gamma_alpha = 0.05;
    const double s_theta = 1.1, s_phi = 2.3, eta_phi = 1e-8;
    eval_c(&C, w, cv);
    const double theta0 = l1(m, cv);
    const double theta_max = 1e4 * fmax(1.0, theta0);
    const double theta_min = 1e-4 * fmax(1.0, theta0);
    double delta_w_last = 0.0;
    int status = ORA_MAXITER_EXCEEDED;
    int iter = 0;
    double final_err = INFINITY;

    for (iter = 0; iter <= opts.max_iter; ++iter) {
        /* ---- evaluate at current iterate ---- */
        eval_grad(&C, w, gf);
        eval_c(&C, w, cv);
        eval_A(&C, w, A);
        for (int i = 0; i < nw; ++i) rd[i] = gf[i] - zL[i] + zU[i];
        for (int r = 0; r < m; ++r)
            for (int j = 0; j < nw; ++j) rd[j] += A[(size_t)r * nw + j] * y[r];
        double sd = fmax(100.0, (l1(m, y) + l1(nw, zL) + l1(nw, zU)) / (double)(m + nbnd > 0 ? m + nbnd : 1)) / 100.0;
        double sc = fmax(100.0, (l1(nw, zL) + l1(nw, zU)) / (double)(nbnd > 0 ? nbnd : 1)) / 100.0;
        double dual_inf = amax(nw, rd);
        double prim_inf = amax(m, cv);
        double compl0 = 0.0;
        for (int i = 0; i < nw; ++i) {
            if (C.hasL[i]) compl0 = fmax(compl0, fabs((w[i] - C.wl[i]) * zL[i]));
            if (C.hasU[i]) compl0 = fmax(compl0, fabs((C.wu[i] - w[i]) * zU[i]));
        }
        double E0 = fmax(dual_inf / sd, fmax(prim_inf, compl0 / sc));
        /* unscaled checks (Ipopt dual_inf_tol / constr_viol_tol / compl_inf_tol) */
        double dual_unscaled = dual_inf / C.obj_scale;
        double prim_unscaled = 0.0;
        for (int r = 0; r < m; ++r) prim_unscaled = fmax(prim_unscaled, fabs(cv[r] / C.c_scale[r]));
        final_err = fmax(dual_unscaled, fmax(prim_unscaled, compl0));
        if (opts.print_level > 0)
            fprintf(stderr, "iter %3d mu %.2e E0 %.3e dual %.3e prim %.3e compl %.3e f %.10e\n", iter,
                    mu, E0, dual_inf, prim_inf, compl0, eval_f(&C, w) / C.obj_scale);
        /* Ipopt's finiteness test of f and g at an evaluated point (OrigIpoptNLP, Ipopt
         * 3.12.8, not vendored in the reference) -> INVALID_NUMBER_DETECTED: amax()
         * drops a NaN, the l1 norm and f do not */
        if (!isfinite(E0) || !isfinite(l1(m, cv)) || !isfinite(eval_f(&C, w))) {
            status = ORA_INVALID_NUMBER_DETECTED;
            break;
        }
        if (E0 <= opts.tol && dual_unscaled <= 1.0 && prim_unscaled <= 1e-4 && compl0 <= 1e-4) {
            status = ORA_SUCCESS;
            break;
        }
        if (iter == opts.max_iter) { status = ORA_MAXITER_EXCEEDED; break; }

        /* ---- monotone barrier update (A-3), possibly several times ---- */
        for (;;) {
            double complmu = 0.0;
            for (int i = 0; i < nw; ++i) {
                if (C.hasL[i]) complmu = fmax(complmu, fabs((w[i] - C.wl[i]) * zL[i] - mu));
                if (C.hasU[i]) complmu = fmax(complmu, fabs((C.wu[i] - w[i]) * zU[i] - mu));
            }
            double Emu = fmax(dual_inf / sd, fmax(prim_inf, complmu / sc));
            if (Emu > kappa_eps * mu || mu <= mu_min) break;
            double mnew = fmax(mu_min, fmin(kappa_mu * mu, pow(mu, theta_mu)));
            if (mnew >= mu) break;
            mu = mnew;
            tau = fmax(0.99, 1.0 - mu);
            nfilter = 0;
        }

        /* ---- primal-dual system with inertia correction (Algorithm IC) ---- */
        eval_W(&C, w, y, W);
        barrier_grad(&C, w, mu, gf, gphi);
        double delta_w = 0.0, delta_c = 0.0;
        int attempt = 0, ok = 0;
        for (;;) {
            memset(KKT, 0, sizeof(double) * (size_t)K * K);
            for (int j = 0; j < n; ++j)
                for (int i = j; i < n; ++i) KKT[i + (size_t)j * K] = W[(size_t)i * n + j];
            for (int i = 0; i < nw; ++i) {
                double sig = 0.0;
                if (C.hasL[i]) sig += zL[i] / (w[i] - C.wl[i]);
                if (C.hasU[i]) sig += zU[i] / (C.wu[i] - w[i]);
                KKT[i + (size_t)i * K] += sig + delta_w;
            }
            for (int r = 0; r < m; ++r) {
                for (int j = 0; j < nw; ++j) KKT[(nw + r) + (size_t)j * K] = A[(size_t)r * nw + j];
                KKT[(nw + r) + (size_t)(nw + r) * K] = -delta_c;
            }
            int np, nn, nz;
            ora_ldlt_factor(K, KKT, ipiv, 1e-300, &np, &nn, &nz);
            if (np == nw && nn == m && nz == 0) {
                ok = 1;
                if (delta_w > 0) delta_w_last = delta_w;
                break;
            }
            if (nz > 0 && delta_c == 0.0) delta_c = 1e-8 * pow(mu, 0.25);
            if (attempt == 0) {
                delta_w = (delta_w_last == 0.0) ? 1e-4 : fmax(1e-20, delta_w_last / 3.0);
            } else {
                delta_w = (delta_w_last == 0.0) ? 100.0 * delta_w : 8.0 * delta_w;
            }
            ++attempt;
            if (delta_w > 1e40) break;
        }
        if (!ok) { status = ORA_ERROR_IN_STEP_COMPUTATION; break; }
        for (int i = 0; i < nw; ++i) {
            double s = gphi[i];
            for (int r = 0; r < m; ++r) s += A[(size_t)r * nw + i] * y[r];
            rhs[i] = -s;
        }
        for (int r = 0; r < m; ++r) rhs[nw + r] = -cv[r];
        ora_ldlt_solve(K, KKT, ipiv, rhs);
        for (int i = 0; i < nw; ++i) dw[i] = rhs[i];
        for (int r = 0; r < m; ++r) dy[r] = rhs[nw + r];
        for (int i = 0; i < nw; ++i) {
            dzL[i] = C.hasL[i] ? mu / (w[i] - C.wl[i]) - zL[i] - zL[i] / (w[i] - C.wl[i]) * dw[i] : 0.0;
            dzU[i] = C.hasU[i] ? mu / (C.wu[i] - w[i]) - zU[i] + zU[i] / (C.wu[i] - w[i]) * dw[i] : 0.0;
        }

        /* ---- fraction-to-the-boundary ---- */
        double amax_p = 1.0, amax_z = 1.0;
        for (int i = 0; i < nw; ++i) {
            if (C.hasL[i] && dw[i] < 0) amax_p = fmin(amax_p, -tau * (w[i] - C.wl[i]) / dw[i]);
            if (C.hasU[i] && dw[i] > 0) amax_p = fmin(amax_p, tau * (C.wu[i] - w[i]) / dw[i]);
            if (C.hasL[i] && dzL[i] < 0) amax_z = fmin(amax_z, -tau * zL[i] / dzL[i]);
            if (C.hasU[i] && dzU[i] < 0) amax_z = fmin(amax_z, -tau * zU[i] / dzU[i]);
        }

        /* ---- filter line search (A-5) ---- */
        int okphi;
        double phik = barrier_phi(&C, w, mu, &okphi);
        double thetak = l1(m, cv);
        double gd = 0.0;
        for (int i = 0; i < nw; ++i) gd += gphi[i] * dw[i];
        double alpha_min;
        if (gd < 0 && thetak <= theta_min)
            alpha_min = gamma_alpha * fmin(gamma_theta, fmin(-gamma_phi * thetak / gd,
                                                             delta_sw * pow(thetak, s_theta) / pow(-gd, s_phi)));
        else if (gd < 0)
            alpha_min = gamma_alpha * fmin(gamma_theta, -gamma_phi * thetak / gd);
        else
            alpha_min = gamma_alpha * gamma_theta;
        /* tiny step (Ipopt's tiny_step_tol = 10*eps_mach) */
        double rel = 0.0;
        for (int i = 0; i < nw; ++i) rel = fmax(rel, fabs(dw[i]) / (1.0 + fabs(w[i])));
        int tiny = (rel < 10.0 * 2.2e-16);
        double alpha = amax_p;
        int accepted = 0, ftype = 0;
        for (int ls = 0; ls < 60; ++ls) {
            for (int i = 0; i < nw; ++i) wt[i] = w[i] + alpha * dw[i];
            if (tiny) { accepted = 1; ftype = 1; break; }
            if (alpha < alpha_min) break;
            int okt;
            double phit = barrier_phi(&C, wt, mu, &okt);
            eval_c(&C, wt, ct);
            double thetat = l1(m, ct);
            if (okt && isfinite(thetat) && thetat < theta_max) {
                int infilt = 0;
                for (int f = 0; f < nfilter; ++f)
                    if (thetat >= filter[f].th && phit >= filter[f].ph) { infilt = 1; break; }
                if (!infilt) {
                    int sw = (gd < 0) && (alpha * pow(-gd, s_phi) > delta_sw * pow(thetak, s_theta));
                    if (thetak <= theta_min && sw) {
                        if (phit <= phik + eta_phi * alpha * gd) { accepted = 1; ftype = 1; break; }
                    } else if (thetat <= (1.0 - gamma_theta) * thetak || phit <= phik - gamma_phi * thetak) {
                        accepted = 1;
                        ftype = 0;
                        break;
                    }
                }
            }
            alpha *= 0.5;
        }
        if (!accepted) { status = ORA_RESTORATION_FAILURE; break; }
        if (!ftype) {
            if (nfilter == capfilter) {
                capfilter *= 2;
                filter = (fpair*)realloc(filter, sizeof(fpair) * capfilter);
            }
            filter[nfilter].th = (1.0 - gamma_theta) * thetak;
            filter[nfilter].ph = phik - gamma_phi * thetak;
            ++nfilter;
        }
        /* ---- accept ---- */
        for (int i = 0; i < nw; ++i) w[i] = wt[i];
        for (int r = 0; r < m; ++r) y[r] += alpha * dy[r];
        for (int i = 0; i < nw; ++i) {
            if (C.hasL[i]) {
                double z = zL[i] + amax_z * dzL[i];
                double s = w[i] - C.wl[i];
                zL[i] = fmax(fmin(z, kappa_sigma * mu / s), mu / (kappa_sigma * s));
            }
            if (C.hasU[i]) {
                double z = zU[i] + amax_z * dzU[i];
                double s = C.wu[i] - w[i];
                zU[i] = fmax(fmin(z, kappa_sigma * mu / s), mu / (kappa_sigma * s));
            }
        }
    }

    /* ---- outputs (unscaled), honor_original_bounds ---- */
    for (int i = 0; i < n; ++i) {
        double xv = w[i];
        if (opts.honor_original_bounds) {
            if (C.hasL[i] && xv < wl0[i]) xv = wl0[i];
            if (C.hasU[i] && xv > wu0[i]) xv = wu0[i];
        }
        x_out[i] = xv;
        if (zl_out) zl_out[i] = zL[i] / C.obj_scale;
        if (zu_out) zu_out[i] = zU[i] / C.obj_scale;
    }
    if (lambda_out)
        for (int r = 0; r < m; ++r) lambda_out[r] = y[r] * C.c_scale[r] / C.obj_scale;
    if (g_out) nlp->g(nlp->ctx, x_out, g_out);
    if (res) {
        res->status = status;
        res->iters = iter;
        res->obj = nlp->f(nlp->ctx, x_out);
        res->kkt_inf = final_err;
    }
    free(ipiv);
    free(C.hasL);
    free(C.hasU);
    free(C.ineq_of_row);
    free(filter);
    free(mem);
    return status;
}
