/*
 * oracle/ipm.c -- Ipopt 3.12.8 restated (TEST INFRASTRUCTURE ONLY, see ora.h).
 *
 * The reference hands its NLP to CppAD::ipopt::solve (mpc_ros/include/cppad/ipopt/
 * solve.hpp:419-589) which runs IpoptApplication::OptimizeTNLP (:586) with the options
 * of mpc_planner.cpp:356-368 (print_level 0, sparse reverse derivatives, max_cpu_time
 * 0.5) and Ipopt defaults otherwise.  Ipopt is not vendored (pinned only by
 * assets/document/ipopt_install/ipopt_x86_install_tutorial.md:9) and not in the image,
 * so this file restates its published algorithm -- Waechter & Biegler, Math. Prog.
 * 106(1):25-57, 2006 (Algorithm A, Algorithm IC, the filter line search with second-order
 * corrections, the feasibility restoration phase of section 3.3) -- and the Ipopt 3.12
 * sources' handling of it.  The Ipopt file/function each part follows is named at the
 * part (IpIpoptAlg.cpp, IpOptErrorConvCheck.cpp, IpMonotoneMuUpdate.cpp,
 * IpPDPerturbationHandler.cpp, IpBacktrackingLineSearch.cpp, IpFilterLSAcceptor.cpp,
 * IpFilter.cpp, IpRestoMinC_1Nrm.cpp, IpRestoIpoptNLP.cpp, IpRestoConvCheck.cpp,
 * IpRestoIterateInitializer.cpp).  Defaults (3.12):
 *
 *   mu_init 0.1, barrier_tol_factor 10, mu_linear_decrease_factor 0.2,
 *   mu_superlinear_decrease_power 1.5, mu_min = min(tol, compl_inf_tol)/(kappa_eps + 1),
 *   tau_min 0.99, bound_push = bound_frac = 0.01, bound_mult_init_val 1,
 *   constr_mult_init_max 1000 (least-squares y0), kappa_sigma 1e10, kappa_d 1e-5,
 *   gamma_theta 1e-5, gamma_phi 1e-8, delta 1, alpha_min_frac 0.05, s_theta 1.1,
 *   s_phi 2.3, eta_phi 1e-8, theta_max_fact 1e4, theta_min_fact 1e-4, obj_max_inc 5,
 *   max_soc 4, kappa_soc 0.99, watchdog_shortened_iter_trigger 10,
 *   watchdog_trial_iter_max 3, soft_resto_pderror_reduction_factor 0.9999,
 *   max_soft_resto_iters 10, max_filter_resets 5, filter_reset_trigger 5,
 *   tiny_step_tol 10 eps, tiny_step_y_tol 1e-2,
 *   inertia correction delta_w0 1e-4, delta_w_min 1e-20, max_hessian_perturbation 1e20 (the
 *   3.12 option default, IpPDPerturbationHandler.cpp; the paper's delta_w^max is 1e40) -- a
 *   larger perturbation skips the iteration into the restoration phase,
 *   kappa_w- 1/3, kappa_w+ 8, kappa_w+bar 100, delta_c 1e-8 mu^0.25,
 *   bound_relax_factor 1e-8 (capped by constr_viol_tol 1e-4), honor_original_bounds,
 *   gradient-based NLP scaling (nlp_scaling_max_gradient 100),
 *   termination: scaled E_0 <= tol (s_max 100), dual_inf_tol 1, constr_viol_tol 1e-4,
 *   compl_inf_tol 1e-4; acceptable_tol 1e-6 for acceptable_iter 15 iterations
 *   (acceptable_dual_inf_tol 1e10, acceptable_constr_viol_tol 1e-2,
 *   acceptable_compl_inf_tol 1e-2, acceptable_obj_change_tol 1e20);
 *   restoration phase: resto_penalty_parameter 1000, resto_proximity_weight 1,
 *   required_infeasibility_reduction 0.9, constr_mult_reset_threshold 0,
 *   bound_mult_reset_threshold 1000.
 *
 * Ipopt's iterative refinement of the KKT solution (PDFullSpaceSolver: min_refinement_steps,
 * residual_ratio_max 1e-10, at most 10 steps) is restated as ora_ipm_opts.refine_steps (off by
 * default: the dense LDL^T solve here is accurate to rounding, and the refinement changes no
 * fixture row's status or restoration count; see solve_step).
 * Not restated (documented in DESIGN.md): slack moves for
 * slacks below eps*min(1,mu) (AdjustedTrialSlacks: never triggered on the fixtures -- the
 * smallest margin is recorded, ora_ipm_result.min_slack_margin), and a
 * restoration phase inside the restoration phase (a failed line search of the
 * restoration problem returns RESTORATION_FAILURE).  The restoration phase is
 * restated for equality-constrained problems (the MPC NLP has no inequality rows).
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "ora.h"

#define INF_BOUND 1e19
#define EPS_MACH 2.220446049250313e-16

void ora_ipm_default_opts(ora_ipm_opts* o) {
    memset(o, 0, sizeof *o);
    o->tol = 1e-8;
    o->max_iter = 3000;
    o->bound_relax_factor = 1e-8;
    o->honor_original_bounds = 1;
    o->mu_init = 0.1;
    o->print_level = 0;
    o->acceptable_tol = 1e-6;
    o->acceptable_iter = 15;
    o->acceptable_dual_inf_tol = 1e10;
    o->acceptable_constr_viol_tol = 1e-2;
    o->acceptable_compl_inf_tol = 1e-2;
    o->acceptable_obj_change_tol = 1e20;
    o->max_soc = 4;
    o->kappa_soc = 0.99;
    o->watchdog_shortened_iter_trigger = 10;
    o->watchdog_trial_iter_max = 3;
    o->soft_resto_pderror_reduction_factor = 0.9999;
    o->max_soft_resto_iters = 10;
    o->restoration = 1;
    o->obj_max_inc = 5.0;
    o->max_filter_resets = 5;
    o->filter_reset_trigger = 5;
    o->tiny_step_tol = 10.0 * EPS_MACH;
    o->tiny_step_y_tol = 1e-2;
    o->cpu_iter_budget = -1;
    o->dual_inf_tol = 1.0;
    o->constr_viol_tol = 1e-4;
    o->compl_inf_tol = 1e-4;
}

int ora_cpu_iter_budget(double max_cpu_time, int steps) {
    if (!(max_cpu_time > 0) || max_cpu_time >= 999999.0) return -1;  /* Ipopt: no limit at >= 1e6 */
    const double setup = fmax(0.0, 0.1205e-3 * steps - 0.89e-3);     /* 1.52 ms @20, 3.93 ms @40 */
    /* per iteration: CppAD's derivatives (0.225 ms @20, 0.467 ms @40) + Ipopt's own work,
     * calibrated by this oracle's structured-KKT iteration on one EPYC 9575F core (0.103 ms
     * @20, linear in N: 5.14 us per stage; profiles/r3/cpu_iter_cost.json) */
    const double per = fmax(0.0121e-3 * steps - 0.017e-3, 1e-5) + 5.14e-6 * steps;
    const double b = floor((max_cpu_time - setup) / per);
    return b < 0 ? 0 : (b > 1e9 ? 1000000000 : (int)b);
}

/* ------------------------------------------------------------------ problem */
/* The problem in Ipopt's internal form: min f(w) s.t. c(w) = 0, wl <= w <= wu, with f and
 * c already scaled (OrigIpoptNLP + gradient-based scaling, or RestoIpoptNLP on top of it). */
typedef struct iprob iprob;
struct iprob {
    int nw, m;
    void* ctx;
    double (*f)(iprob*, const double* w, double mu);
    void (*grad)(iprob*, const double* w, double mu, double* g);
    void (*cons)(iprob*, const double* w, double* c);
    void (*jac)(iprob*, const double* w, double* A);                                    /* m x nw row-major */
    void (*hess)(iprob*, const double* w, double sigma, double mu, const double* y, double* W); /* nw x nw */
    double *wl, *wu;
    char *hasL, *hasU;
    double obj_scale;  /* for the unscaled termination tests (1 in the restoration problem) */
    double* c_scale;   /* per row (NULL: 1) */
};

/* --- the user's NLP with inequality slacks and gradient-based scaling (OrigIpoptNLP) --- */
typedef struct {
    const ora_nlp* nlp;
    int n, m, mI;
    int* ineq_of_row;
    double obj_scale;
    double* c_scale;
    double *gv, *jac, *lam, *H;
} orig_ctx;

static double orig_f(iprob* P, const double* w, double mu) {
    (void)mu;
    orig_ctx* o = (orig_ctx*)P->ctx;
    return o->obj_scale * o->nlp->f(o->nlp->ctx, w);
}
static void orig_grad(iprob* P, const double* w, double mu, double* g) {
    (void)mu;
    orig_ctx* o = (orig_ctx*)P->ctx;
    o->nlp->grad_f(o->nlp->ctx, w, g);
    for (int i = 0; i < o->n; ++i) g[i] *= o->obj_scale;
    for (int i = o->n; i < P->nw; ++i) g[i] = 0.0;
}
static void orig_cons(iprob* P, const double* w, double* c) {
    orig_ctx* o = (orig_ctx*)P->ctx;
    const ora_nlp* p = o->nlp;
    p->g(p->ctx, w, o->gv);
    for (int r = 0; r < o->m; ++r) {
        int s = o->ineq_of_row[r];
        double v = (s < 0) ? o->gv[r] - p->gl[r] : o->gv[r] - w[o->n + s];
        c[r] = o->c_scale[r] * v;
    }
}
static void orig_jac(iprob* P, const double* w, double* A) {
    orig_ctx* o = (orig_ctx*)P->ctx;
    const ora_nlp* p = o->nlp;
    p->jac_g(p->ctx, w, o->jac);
    for (int r = 0; r < o->m; ++r) {
        double* row = A + (size_t)r * P->nw;
        for (int j = 0; j < o->n; ++j) row[j] = o->c_scale[r] * o->jac[(size_t)r * o->n + j];
        for (int j = o->n; j < P->nw; ++j) row[j] = 0.0;
        int s = o->ineq_of_row[r];
        if (s >= 0) row[o->n + s] = -o->c_scale[r];
    }
}
static void orig_hess(iprob* P, const double* w, double sigma, double mu, const double* y, double* W) {
    (void)mu;
    orig_ctx* o = (orig_ctx*)P->ctx;
    const int n = o->n, nw = P->nw;
    for (int r = 0; r < o->m; ++r) o->lam[r] = y[r] * o->c_scale[r];
    o->nlp->hess(o->nlp->ctx, w, sigma * o->obj_scale, o->lam, o->H);
    memset(W, 0, sizeof(double) * (size_t)nw * nw);
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) W[(size_t)i * nw + j] = o->H[(size_t)i * n + j];
}

/* --- the restoration problem (RestoIpoptNLP, equality rows only) ---
 *   min  rho sum(p + n) + eta(mu)/2 ||D_R (x - x_R)||^2,  eta(mu) = resto_proximity_weight sqrt(mu),
 *   s.t. c(x) - p + n = 0,  x in the (relaxed) bounds of the original,  p, n >= 0,
 *   D_R = diag(1 / max(1, |x_R|)); c is the scaled constraint of the original problem. */
typedef struct {
    iprob* orig;
    int nx, m;
    double rho;
    const double *xR, *DR;
    double *c, *A;
} resto_ctx;

static double resto_f(iprob* P, const double* v, double mu) {
    resto_ctx* r = (resto_ctx*)P->ctx;
    const double eta = sqrt(mu);
    double s = 0.0, q = 0.0;
    for (int i = 0; i < 2 * r->m; ++i) s += v[r->nx + i];
    for (int i = 0; i < r->nx; ++i) {
        double d = r->DR[i] * (v[i] - r->xR[i]);
        q += d * d;
    }
    return r->rho * s + 0.5 * eta * q;
}
static void resto_grad(iprob* P, const double* v, double mu, double* g) {
    resto_ctx* r = (resto_ctx*)P->ctx;
    const double eta = sqrt(mu);
    for (int i = 0; i < r->nx; ++i) g[i] = eta * r->DR[i] * r->DR[i] * (v[i] - r->xR[i]);
    for (int i = 0; i < 2 * r->m; ++i) g[r->nx + i] = r->rho;
}
static void resto_cons(iprob* P, const double* v, double* c) {
    resto_ctx* r = (resto_ctx*)P->ctx;
    r->orig->cons(r->orig, v, c);
    for (int i = 0; i < r->m; ++i) c[i] += -v[r->nx + i] + v[r->nx + r->m + i];
}
static void resto_jac(iprob* P, const double* v, double* A) {
    resto_ctx* r = (resto_ctx*)P->ctx;
    const int nv = P->nw;
    r->orig->jac(r->orig, v, r->A);
    memset(A, 0, sizeof(double) * (size_t)r->m * nv);
    for (int i = 0; i < r->m; ++i) {
        memcpy(A + (size_t)i * nv, r->A + (size_t)i * r->nx, sizeof(double) * r->nx);
        A[(size_t)i * nv + r->nx + i] = -1.0;
        A[(size_t)i * nv + r->nx + r->m + i] = 1.0;
    }
}
static void resto_hess(iprob* P, const double* v, double sigma, double mu, const double* y, double* W) {
    resto_ctx* r = (resto_ctx*)P->ctx;
    const int nv = P->nw, nx = r->nx;
    double* Wx = (double*)malloc(sizeof(double) * (size_t)nx * nx);
    r->orig->hess(r->orig, v, 0.0, mu, y, Wx);  /* constraint curvature only */
    memset(W, 0, sizeof(double) * (size_t)nv * nv);
    const double eta = sqrt(mu);
    for (int i = 0; i < nx; ++i) {
        for (int j = 0; j < nx; ++j) W[(size_t)i * nv + j] = Wx[(size_t)i * nx + j];
        W[(size_t)i * nv + i] += sigma * eta * r->DR[i] * r->DR[i];
    }
    free(Wx);
}

/* ------------------------------------------------------------------ solver */
typedef struct ipm ipm;
struct ipm {
    iprob* P;
    const ora_ipm_opts* o;
    int nw, m, K, nbnd;
    int is_resto;
    ipm* outer;        /* restoration phase: the original problem's solver */
    int* iter;         /* shared iteration counter (the restoration phase counts on) */
    /* iterate, direction (the Newton step), actual step (SOC), trial point */
    double *w, *y, *zL, *zU;
    double *dw, *dy, *dzL, *dzU;
    double *aw, *ay, *azL, *azU;
    double *wt, *yt, *zLt, *zUt;
    double *gf, *cv, *A, *W, *gphi, *rd, *ct, *csoc, *gft, *At, *rdt;
    double *KKT, *rhs;
    double* KKT0;      /* refine_steps > 0: the matrix before its factorisation */
    int* ipiv;
    double mu, tau, dw_last;
    /* statistics of the current iterate */
    double f, theta, phi, E0, dual_inf, prim_inf, compl0, dual_uns, prim_uns, compl_uns, gd;
    double sd, sc;
    /* filter line search acceptor (IpFilterLSAcceptor.cpp) */
    double *fth, *fph;
    int nf, capf;
    double theta_max, theta_min;
    double ref_theta, ref_phi, ref_gd;
    int last_rej_filter, count_filter_rej, n_filter_resets;
    /* watchdog (IpBacktrackingLineSearch.cpp) */
    int in_wd, wd_short, wd_trial_iter;
    double wd_alpha_test, wd_theta, wd_phi, wd_gd, last_mu;
    double *wd_w, *wd_y, *wd_zL, *wd_zU, *wd_dw, *wd_dy, *wd_dzL, *wd_dzU;
    int tiny_last, tiny_flag;
    int in_soft, soft_count;
    /* acceptable-point tracking (IpOptErrorConvCheck.cpp) */
    int acc_counter, last_obj_iter;
    double last_obj, curr_obj;
    int have_acc;
    double *acc_w, *acc_y, *acc_zL, *acc_zU;
    int resto_first;   /* restoration problem: first convergence check */
    ora_ipm_result* diag;
    ora_ipm_result* slk; /* the slack margins (barrier_phi), the restoration problem's too */
    double* mem;
    /* kkt_structured: position of KKT row i in the banded order, envelope of the factor */
    int *kpos, *klast;
};

static double amax(int n, const double* v) {
    double m = 0.0;
    for (int i = 0; i < n; ++i) m = fmax(m, fabs(v[i]));
    return m;
}
static double l1(int n, const double* v) {
    double s = 0.0;
    for (int i = 0; i < n; ++i) s += fabs(v[i]);
    return s;
}
/* IpUtils.cpp Compare_le: lhs - rhs <= 10 eps |BasVal| */
static int compare_le(double lhs, double rhs, double bas) { return lhs - rhs <= 10.0 * EPS_MACH * fabs(bas); }

static void ipm_alloc(ipm* S, iprob* P, const ora_ipm_opts* o) {
    memset(S, 0, sizeof *S);
    S->P = P;
    S->o = o;
    S->nw = P->nw;
    S->m = P->m;
    S->K = P->nw + P->m;
    const size_t nw = P->nw, m = P->m, K = S->K;
    S->mem = (double*)calloc(40 * nw + 20 * m + 2 * m * nw + nw * nw + K * K + 3 * K + 16, sizeof(double));
    double* p = S->mem;
#define TAKE(ptr, cnt) do { S->ptr = p; p += (cnt); } while (0)
    TAKE(w, nw); TAKE(y, m); TAKE(zL, nw); TAKE(zU, nw);
    TAKE(dw, nw); TAKE(dy, m); TAKE(dzL, nw); TAKE(dzU, nw);
    TAKE(aw, nw); TAKE(ay, m); TAKE(azL, nw); TAKE(azU, nw);
    TAKE(wt, nw); TAKE(yt, m); TAKE(zLt, nw); TAKE(zUt, nw);
    TAKE(gf, nw); TAKE(cv, m); TAKE(A, m * nw); TAKE(W, nw * nw); TAKE(gphi, nw); TAKE(rd, nw);
    TAKE(ct, m); TAKE(csoc, m); TAKE(gft, nw); TAKE(At, m * nw); TAKE(rdt, nw);
    TAKE(KKT, K * K); TAKE(rhs, 2 * K);
    TAKE(wd_w, nw); TAKE(wd_y, m); TAKE(wd_zL, nw); TAKE(wd_zU, nw);
    TAKE(wd_dw, nw); TAKE(wd_dy, m); TAKE(wd_dzL, nw); TAKE(wd_dzU, nw);
    TAKE(acc_w, nw); TAKE(acc_y, m); TAKE(acc_zL, nw); TAKE(acc_zU, nw);
#undef TAKE
    S->ipiv = (int*)malloc(sizeof(int) * K);
    if (o->refine_steps > 0) S->KKT0 = (double*)malloc(sizeof(double) * K * K + sizeof(double) * 2 * K);
    S->capf = 64;
    S->fth = (double*)malloc(sizeof(double) * S->capf);
    S->fph = (double*)malloc(sizeof(double) * S->capf);
    for (int i = 0; i < P->nw; ++i) S->nbnd += P->hasL[i] + P->hasU[i];
    S->theta_max = -1.0;
    S->theta_min = -1.0;
    S->last_obj_iter = -1;
    S->curr_obj = -1e50;
    S->last_mu = -1.0;
}
static void ipm_free(ipm* S) {
    free(S->KKT0);
    free(S->kpos);
    free(S->klast);
    free(S->mem);
    free(S->ipiv);
    free(S->fth);
    free(S->fph);
}

/* barrier function phi_mu(w) (IpIpoptCalculatedQuantities.cpp curr_barrier_obj), with
 * the kappa_d damping of one-sided bounds; ok = 0 outside the bounds or not finite */
static double barrier_phi(ipm* S, const double* w, int* ok) {
    iprob* P = S->P;
    const double kd = 1e-5, mu = S->mu;
    double phi = P->f(P, w, mu);
    /* Ipopt moves a slack below eps * min(1, mu) (CalculateSafeSlack) and then relaxes that
     * bound (AcceptTrialPoint, AdjustedTrialSlacks): not restated -- the smallest margin
     * s / (eps min(1, mu)) of every point whose barrier is evaluated is recorded instead,
     * so a test can show the move never triggers (tests/test_oracle.py) */
    const double smin = EPS_MACH * fmin(1.0, mu);
    double rmin = INFINITY;
    *ok = 1;
    for (int i = 0; i < S->nw; ++i) {
        if (P->hasL[i]) {
            double d = w[i] - P->wl[i];
            if (!(d > 0)) { *ok = 0; return INFINITY; }
            phi -= mu * log(d);
            if (!P->hasU[i]) phi += kd * mu * d;
            rmin = fmin(rmin, d / smin);
        }
        if (P->hasU[i]) {
            double d = P->wu[i] - w[i];
            if (!(d > 0)) { *ok = 0; return INFINITY; }
            phi -= mu * log(d);
            if (!P->hasL[i]) phi += kd * mu * d;
            rmin = fmin(rmin, d / smin);
        }
    }
    if (!isfinite(phi)) *ok = 0;
    if (S->slk) {
        if (rmin < S->slk->min_slack_margin) S->slk->min_slack_margin = rmin;
        if (rmin < 1.0) ++S->slk->n_slack_moves;
    }
    return phi;
}
static void barrier_grad(ipm* S, const double* w, const double* gf, double* gphi) {
    iprob* P = S->P;
    const double kd = 1e-5, mu = S->mu;
    for (int i = 0; i < S->nw; ++i) {
        double g = gf[i];
        if (P->hasL[i]) {
            g -= mu / (w[i] - P->wl[i]);
            if (!P->hasU[i]) g += kd * mu;
        }
        if (P->hasU[i]) {
            g += mu / (P->wu[i] - w[i]);
            if (!P->hasL[i]) g -= kd * mu;
        }
        gphi[i] = g;
    }
}

/* gradient of the Lagrangian rd = gf + A^T y - zL + zU */
static void lag_grad(ipm* S, const double* gf, const double* A, const double* y, const double* zL, const double* zU,
                     double* rd) {
    for (int i = 0; i < S->nw; ++i) rd[i] = gf[i] - zL[i] + zU[i];
    for (int r = 0; r < S->m; ++r)
        for (int j = 0; j < S->nw; ++j) rd[j] += A[(size_t)r * S->nw + j] * y[r];
}

/* complementarity max |s z - mu_t| (NORM_MAX) or sum (NORM_1) */
static double compl_norm(ipm* S, const double* w, const double* zL, const double* zU, double mu_t, int one) {
    iprob* P = S->P;
    double c = 0.0;
    for (int i = 0; i < S->nw; ++i) {
        if (P->hasL[i]) {
            double v = fabs((w[i] - P->wl[i]) * zL[i] - mu_t);
            c = one ? c + v : fmax(c, v);
        }
        if (P->hasU[i]) {
            double v = fabs((P->wu[i] - w[i]) * zU[i] - mu_t);
            c = one ? c + v : fmax(c, v);
        }
    }
    return c;
}

/* evaluate the current iterate: gf, c, A, the optimality-error statistics */
static void eval_current(ipm* S) {
    iprob* P = S->P;
    P->grad(P, S->w, S->mu, S->gf);
    P->cons(P, S->w, S->cv);
    P->jac(P, S->w, S->A);
    S->f = P->f(P, S->w, S->mu);
    lag_grad(S, S->gf, S->A, S->y, S->zL, S->zU, S->rd);
    const int m = S->m, nbnd = S->nbnd;
    /* ComputeOptimalityErrorScaling (s_max 100) */
    S->sd = fmax(100.0, (l1(m, S->y) + l1(S->nw, S->zL) + l1(S->nw, S->zU)) / (double)(m + nbnd > 0 ? m + nbnd : 1)) / 100.0;
    S->sc = fmax(100.0, (l1(S->nw, S->zL) + l1(S->nw, S->zU)) / (double)(nbnd > 0 ? nbnd : 1)) / 100.0;
    S->dual_inf = amax(S->nw, S->rd);
    S->prim_inf = amax(m, S->cv);
    S->theta = l1(m, S->cv);
    S->compl0 = compl_norm(S, S->w, S->zL, S->zU, 0.0, 0);
    S->E0 = fmax(S->dual_inf / S->sd, fmax(S->prim_inf, S->compl0 / S->sc));
    /* unscaled_curr_dual_infeasibility / unscaled_curr_nlp_constraint_violation /
     * unscaled_curr_complementarity: objective scaling undone */
    S->dual_uns = S->dual_inf / P->obj_scale;
    double pu = 0.0;
    for (int r = 0; r < m; ++r) pu = fmax(pu, fabs(S->cv[r] / (P->c_scale ? P->c_scale[r] : 1.0)));
    S->prim_uns = pu;
    S->compl_uns = S->compl0 / P->obj_scale;
}

/* OptimalityErrorConvergenceCheck::CurrentIsAcceptable (the objective-change bookkeeping
 * runs once per iteration) */
static int current_is_acceptable(ipm* S) {
    const ora_ipm_opts* o = S->o;
    if (*S->iter != S->last_obj_iter) {
        S->last_obj = S->curr_obj;
        S->curr_obj = S->f;
        S->last_obj_iter = *S->iter;
    }
    return S->E0 <= o->acceptable_tol && S->dual_uns <= o->acceptable_dual_inf_tol &&
           S->prim_uns <= o->acceptable_constr_viol_tol && S->compl_uns <= o->acceptable_compl_inf_tol &&
           fabs(S->last_obj - S->curr_obj) / fmax(1.0, fabs(S->curr_obj)) <= o->acceptable_obj_change_tol;
}

/* --------------------------------------------------------------- the filter */
static void filter_add(ipm* S, double ph, double th) {
    /* Filter::AddEntry: drop the entries the new one dominates, then append */
    int k = 0;
    for (int i = 0; i < S->nf; ++i) {
        int dominated = (ph <= S->fph[i]) && (th <= S->fth[i]);
        if (!dominated) {
            S->fph[k] = S->fph[i];
            S->fth[k] = S->fth[i];
            ++k;
        }
    }
    S->nf = k;
    if (S->nf == S->capf) {
        S->capf *= 2;
        S->fth = (double*)realloc(S->fth, sizeof(double) * S->capf);
        S->fph = (double*)realloc(S->fph, sizeof(double) * S->capf);
    }
    S->fph[S->nf] = ph;
    S->fth[S->nf] = th;
    ++S->nf;
}
static int filter_acceptable(const ipm* S, double ph, double th) {
    for (int i = 0; i < S->nf; ++i)
        if (!(ph < S->fph[i] || th < S->fth[i])) return 0;
    return 1;
}
static void augment_filter(ipm* S) {
    const double gamma_theta = 1e-5, gamma_phi = 1e-8;
    filter_add(S, S->ref_phi - gamma_phi * S->ref_theta, (1.0 - gamma_theta) * S->ref_theta);
}
static int is_ftype(const ipm* S, double alpha_test) {
    const double delta = 1.0, s_theta = 1.1, s_phi = 2.3;
    return S->ref_gd < 0.0 && alpha_test * pow(-S->ref_gd, s_phi) > delta * pow(S->ref_theta, s_theta);
}
static int armijo_holds(const ipm* S, double alpha_test, double phit) {
    const double eta_phi = 1e-8;
    return compare_le(phit - S->ref_phi, eta_phi * alpha_test * S->ref_gd, S->ref_phi);
}
static int acceptable_to_current_iterate(const ipm* S, double phit, double thetat, int from_resto) {
    const double gamma_theta = 1e-5, gamma_phi = 1e-8;
    if (!from_resto && phit > S->ref_phi) {
        double basval = 1.0;
        if (fabs(S->ref_phi) > 10.0) basval = log10(fabs(S->ref_phi));
        if (log10(phit - S->ref_phi) > S->o->obj_max_inc * basval) return 0;
    }
    return compare_le(thetat, (1.0 - gamma_theta) * S->ref_theta, S->ref_theta) ||
           compare_le(phit - S->ref_phi, -gamma_phi * S->ref_theta, S->ref_phi);
}
/* FilterLSAcceptor::CheckAcceptabilityOfTrialPoint */
static int check_acceptability(ipm* S, double alpha_test, double phit, double thetat) {
    if (S->theta_max < 0.0) S->theta_max = 1e4 * fmax(1.0, S->ref_theta);
    if (S->theta_min < 0.0) S->theta_min = 1e-4 * fmax(1.0, S->ref_theta);
    if (S->theta_max > 0 && thetat > S->theta_max) return 0;
    int accept;
    if (alpha_test > 0.0 && is_ftype(S, alpha_test) && S->ref_theta <= S->theta_min)
        accept = armijo_holds(S, alpha_test, phit);
    else
        accept = acceptable_to_current_iterate(S, phit, thetat, 0);
    if (!accept) {
        S->last_rej_filter = 0;
        return 0;
    }
    if (!filter_acceptable(S, phit, thetat)) {
        S->last_rej_filter = 1;
        return 0;
    }
    /* filter reset heuristic */
    if (S->o->max_filter_resets > 0 && S->n_filter_resets < S->o->max_filter_resets) {
        if (S->last_rej_filter) {
            if (++S->count_filter_rej >= S->o->filter_reset_trigger) {
                S->nf = 0;
                S->count_filter_rej = 0;
                ++S->n_filter_resets;
            }
        } else {
            S->count_filter_rej = 0;
        }
    }
    return 1;
}
/* FilterLSAcceptor::CalculateAlphaMin (on the reference point's values) */
static double alpha_min_of(const ipm* S) {
    const double gamma_theta = 1e-5, gamma_phi = 1e-8, delta = 1.0, s_theta = 1.1, s_phi = 2.3;
    const double gBD = S->ref_gd, th = S->ref_theta;
    double a;
    if (gBD < 0) {
        a = fmin(gamma_theta, gamma_phi * th / (-gBD));
        if (th <= S->theta_min) a = fmin(a, delta * pow(th, s_theta) / pow(-gBD, s_phi));
    } else {
        a = gamma_theta;
    }
    return 0.05 * a;
}

/* ------------------------------------------------- the primal-dual system */
/* Build and factor the KKT matrix of the current iterate with inertia correction
 * (PDPerturbationHandler, Algorithm IC).  Returns 1 on success. */
static int factor_kkt(ipm* S) {
    iprob* P = S->P;
    const int nw = S->nw, m = S->m, K = S->K;
    P->hess(P, S->w, 1.0, S->mu, S->y, S->W);
    double delta_w = 0.0, delta_c = 0.0;
    int attempt = 0;
    for (;;) {
        memset(S->KKT, 0, sizeof(double) * (size_t)K * K);
        if (S->kpos) {  /* kkt_structured: the same matrix in the banded order, envelope factor */
            const int* q = S->kpos;
#define KL(i, j) S->KKT[(q[i] > q[j] ? q[i] : q[j]) + (size_t)(q[i] > q[j] ? q[j] : q[i]) * K]
            for (int j = 0; j < nw; ++j)
                for (int i = j; i < nw; ++i)
                    if (S->W[(size_t)i * nw + j] != 0.0) KL(i, j) = S->W[(size_t)i * nw + j];
            for (int i = 0; i < nw; ++i) {
                double sig = 0.0;
                if (P->hasL[i]) sig += S->zL[i] / (S->w[i] - P->wl[i]);
                if (P->hasU[i]) sig += S->zU[i] / (P->wu[i] - S->w[i]);
                KL(i, i) += sig + delta_w;
            }
            for (int r = 0; r < m; ++r) {
                for (int j = 0; j < nw; ++j)
                    if (S->A[(size_t)r * nw + j] != 0.0) KL(nw + r, j) = S->A[(size_t)r * nw + j];
                KL(nw + r, nw + r) = -delta_c;
            }
#undef KL
            int np, nn, nz;
            ora_ldlt_factor_env(K, S->KKT, S->ipiv, 1e-300, &np, &nn, &nz, S->klast);
            if (np == nw && nn == m && nz == 0) {
                if (delta_w > 0) S->dw_last = delta_w;
                return 1;
            }
            if (nz > 0 && delta_c == 0.0) delta_c = 1e-8 * pow(S->mu, 0.25);
            if (attempt == 0)
                delta_w = (S->dw_last == 0.0) ? 1e-4 : fmax(1e-20, S->dw_last / 3.0);
            else
                delta_w = (S->dw_last == 0.0) ? 100.0 * delta_w : 8.0 * delta_w;
            ++attempt;
            if (delta_w > 1e20) return 0;
            continue;
        }
        for (int j = 0; j < nw; ++j)
            for (int i = j; i < nw; ++i) S->KKT[i + (size_t)j * K] = S->W[(size_t)i * nw + j];
        for (int i = 0; i < nw; ++i) {
            double sig = 0.0;
            if (P->hasL[i]) sig += S->zL[i] / (S->w[i] - P->wl[i]);
            if (P->hasU[i]) sig += S->zU[i] / (P->wu[i] - S->w[i]);
            S->KKT[i + (size_t)i * K] += sig + delta_w;
        }
        for (int r = 0; r < m; ++r) {
            for (int j = 0; j < nw; ++j) S->KKT[(nw + r) + (size_t)j * K] = S->A[(size_t)r * nw + j];
            S->KKT[(nw + r) + (size_t)(nw + r) * K] = -delta_c;
        }
        int np, nn, nz;
        if (S->KKT0) memcpy(S->KKT0, S->KKT, sizeof(double) * (size_t)K * K);
        ora_ldlt_factor(K, S->KKT, S->ipiv, 1e-300, &np, &nn, &nz);
        if (np == nw && nn == m && nz == 0) {
            if (delta_w > 0) S->dw_last = delta_w;
            return 1;
        }
        if (nz > 0 && delta_c == 0.0) delta_c = 1e-8 * pow(S->mu, 0.25);
        if (attempt == 0)
            delta_w = (S->dw_last == 0.0) ? 1e-4 : fmax(1e-20, S->dw_last / 3.0);
        else
            delta_w = (S->dw_last == 0.0) ? 100.0 * delta_w : 8.0 * delta_w;
        ++attempt;
        if (delta_w > 1e20) return 0;
    }
}
/* Solve the factored system for the step with constraint right-hand side -crhs; the
 * stationarity rows carry the barrier gradient (Ipopt's grad_lag_with_damping plus the
 * relaxed complementarity, eliminated).  z steps from the complementarity rows. */
static void solve_step(ipm* S, const double* crhs, double* dw, double* dy, double* dzL, double* dzU) {
    iprob* P = S->P;
    const int nw = S->nw, m = S->m;
    for (int i = 0; i < nw; ++i) {
        double s = S->gphi[i];
        for (int r = 0; r < m; ++r) s += S->A[(size_t)r * nw + i] * S->y[r];
        S->rhs[i] = -s;
    }
    for (int r = 0; r < m; ++r) S->rhs[nw + r] = -crhs[r];
    if (S->kpos) {
        double* b = S->rhs + S->K;  /* (a second K-vector after rhs) */
        for (int i = 0; i < S->K; ++i) b[S->kpos[i]] = S->rhs[i];
        ora_ldlt_solve_env(S->K, S->KKT, S->ipiv, S->klast, b);
        for (int i = 0; i < S->K; ++i) S->rhs[i] = b[S->kpos[i]];
    } else if (S->KKT0) {
        /* PDFullSpaceSolver::Solve's iterative refinement: residual r = b - K x of the
         * unfactored matrix (lower triangle, symmetric), correction K c = r, x += c; at least
         * refine_steps steps, more while |r| / (|x| + |b|) > 1e-10, at most 10 */
        const int K = S->K;
        double* b = S->KKT0 + (size_t)K * K;
        double* r = b + K;
        memcpy(b, S->rhs, sizeof(double) * K);
        ora_ldlt_solve(K, S->KKT, S->ipiv, S->rhs);
        for (int step = 0; step < 10; ++step) {
            for (int i = 0; i < K; ++i) r[i] = b[i];
            for (int j = 0; j < K; ++j) {
                const double xj = S->rhs[j];
                r[j] -= S->KKT0[j + (size_t)j * K] * xj;
                for (int i = j + 1; i < K; ++i) {
                    const double a = S->KKT0[i + (size_t)j * K];
                    if (a != 0.0) {
                        r[i] -= a * xj;
                        r[j] -= a * S->rhs[i];
                    }
                }
            }
            const double ratio = amax(K, r) / (amax(K, S->rhs) + amax(K, b));
            if (step >= S->o->refine_steps && !(ratio > 1e-10)) break;
            ora_ldlt_solve(K, S->KKT, S->ipiv, r);
            for (int i = 0; i < K; ++i) S->rhs[i] += r[i];
        }
    } else {
        ora_ldlt_solve(S->K, S->KKT, S->ipiv, S->rhs);
    }
    for (int i = 0; i < nw; ++i) dw[i] = S->rhs[i];
    for (int r = 0; r < m; ++r) dy[r] = S->rhs[nw + r];
    for (int i = 0; i < nw; ++i) {
        dzL[i] = P->hasL[i] ? S->mu / (S->w[i] - P->wl[i]) - S->zL[i] - S->zL[i] / (S->w[i] - P->wl[i]) * dw[i] : 0.0;
        dzU[i] = P->hasU[i] ? S->mu / (P->wu[i] - S->w[i]) - S->zU[i] + S->zU[i] / (P->wu[i] - S->w[i]) * dw[i] : 0.0;
    }
}
static double primal_frac(const ipm* S, const double* w, const double* dw) {
    iprob* P = S->P;
    double a = 1.0;
    for (int i = 0; i < S->nw; ++i) {
        if (P->hasL[i] && dw[i] < 0) a = fmin(a, -S->tau * (w[i] - P->wl[i]) / dw[i]);
        if (P->hasU[i] && dw[i] > 0) a = fmin(a, S->tau * (P->wu[i] - w[i]) / dw[i]);
    }
    return a;
}
static double dual_frac(const ipm* S, const double* zL, const double* zU, const double* dzL, const double* dzU) {
    iprob* P = S->P;
    double a = 1.0;
    for (int i = 0; i < S->nw; ++i) {
        if (P->hasL[i] && dzL[i] < 0) a = fmin(a, -S->tau * zL[i] / dzL[i]);
        if (P->hasU[i] && dzU[i] < 0) a = fmin(a, -S->tau * zU[i] / dzU[i]);
    }
    return a;
}

/* trial primal point w + alpha d: phi, theta (c at the trial point in S->ct); ok = 0 on an
 * evaluation error (outside the bounds, non-finite) */
static int eval_trial(ipm* S, double alpha, const double* d, double* phit, double* thetat) {
    for (int i = 0; i < S->nw; ++i) S->wt[i] = S->w[i] + alpha * d[i];
    int ok;
    *phit = barrier_phi(S, S->wt, &ok);
    S->P->cons(S->P, S->wt, S->ct);
    *thetat = l1(S->m, S->ct);
    return ok && isfinite(*thetat);
}
/* PerformDualStep: z with alpha_dual, y with the primal step length (alpha_for_y primal) */
static void dual_step(ipm* S, double alpha_p, double alpha_d, const double* dy, const double* dzL,
                      const double* dzU) {
    for (int r = 0; r < S->m; ++r) S->yt[r] = S->y[r] + alpha_p * dy[r];
    for (int i = 0; i < S->nw; ++i) {
        S->zLt[i] = S->zL[i] + alpha_d * dzL[i];
        S->zUt[i] = S->zU[i] + alpha_d * dzU[i];
    }
}
static void copy_dir(ipm* S, double* w, double* y, double* zL, double* zU, const double* w2, const double* y2,
                     const double* zL2, const double* zU2) {
    memcpy(w, w2, sizeof(double) * S->nw);
    memcpy(y, y2, sizeof(double) * S->m);
    memcpy(zL, zL2, sizeof(double) * S->nw);
    memcpy(zU, zU2, sizeof(double) * S->nw);
}

/* FilterLSAcceptor::TrySecondOrderCorrection */
static int try_soc(ipm* S, double alpha_test, double* alpha, double theta_trial) {
    const ora_ipm_opts* o = S->o;
    if (o->max_soc <= 0) return 0;
    int count = 0, accept = 0;
    double theta_old = 0.0, alpha_soc = *alpha;
    memcpy(S->csoc, S->cv, sizeof(double) * S->m);
    double* sw = (double*)malloc(sizeof(double) * (2 * S->nw + S->nw + S->m));
    double *dzl = sw, *dzu = sw + S->nw, *dws = sw + 2 * S->nw, *dys = dws + S->nw;
    while (count < o->max_soc && !accept && (count == 0 || theta_trial <= o->kappa_soc * theta_old)) {
        theta_old = theta_trial;
        for (int r = 0; r < S->m; ++r) S->csoc[r] = S->ct[r] + alpha_soc * S->csoc[r];
        solve_step(S, S->csoc, dws, dys, dzl, dzu);
        alpha_soc = primal_frac(S, S->w, dws);
        double phit, thetat;
        int ok = eval_trial(S, alpha_soc, dws, &phit, &thetat);
        accept = ok && check_acceptability(S, alpha_test, phit, thetat);
        if (accept) {
            *alpha = alpha_soc;
            copy_dir(S, S->aw, S->ay, S->azL, S->azU, dws, dys, dzl, dzu);
            if (S->diag) ++S->diag->n_soc;
        } else {
            ++count;
            theta_trial = thetat;
        }
    }
    free(sw);
    return accept;
}

/* BacktrackingLineSearch::DoBacktrackingLineSearch on the actual step (aw, ...). */
static int backtracking(ipm* S, int skip_first, double* alpha_out, int* n_steps, int* eval_error) {
    *eval_error = 0;
    const double alpha_max = primal_frac(S, S->w, S->aw);
    const double alpha_min = S->in_wd ? alpha_max : alpha_min_of(S);
    double alpha = alpha_max;
    double alpha_test = S->in_wd ? S->wd_alpha_test : alpha;
    if (skip_first) alpha *= 0.5;
    int accept = 0;
    *n_steps = 0;
    while (alpha > alpha_min || *n_steps == 0) {
        double phit, thetat;
        int ok = eval_trial(S, alpha, S->aw, &phit, &thetat);
        if (!S->in_wd) alpha_test = alpha;
        if (ok) {
            accept = check_acceptability(S, alpha_test, phit, thetat);
        } else {
            accept = 0;
            *eval_error = 1;
        }
        if (accept) {
            /* UpdateForNextIteration: augment unless an f-type step with Armijo */
            if (!is_ftype(S, alpha_test) || !armijo_holds(S, alpha_test, phit)) augment_filter(S);
            break;
        }
        if (S->in_wd) break;
        if (!*eval_error && alpha == alpha_max && S->theta <= thetat) {
            accept = try_soc(S, alpha_test, &alpha, thetat);
            if (accept) {
                /* the SOC trial point is in wt; its filter bookkeeping as above */
                double phis;
                int oks;
                phis = barrier_phi(S, S->wt, &oks);
                if (!is_ftype(S, alpha_test) || !armijo_holds(S, alpha_test, phis)) augment_filter(S);
                break;
            }
        }
        alpha *= 0.5;
        ++*n_steps;
    }
    *alpha_out = alpha;
    return accept;
}

static void start_watchdog(ipm* S) {
    S->in_wd = 1;
    copy_dir(S, S->wd_w, S->wd_y, S->wd_zL, S->wd_zU, S->w, S->y, S->zL, S->zU);
    copy_dir(S, S->wd_dw, S->wd_dy, S->wd_dzL, S->wd_dzU, S->dw, S->dy, S->dzL, S->dzU);
    S->wd_trial_iter = 0;
    S->wd_alpha_test = primal_frac(S, S->w, S->dw);
    S->wd_theta = S->ref_theta;
    S->wd_phi = S->ref_phi;
    S->wd_gd = S->ref_gd;
    if (S->diag) ++S->diag->n_watchdog;
}
static void stop_watchdog(ipm* S) {
    S->in_wd = 0;
    copy_dir(S, S->w, S->y, S->zL, S->zU, S->wd_w, S->wd_y, S->wd_zL, S->wd_zU);
    copy_dir(S, S->aw, S->ay, S->azL, S->azU, S->wd_dw, S->wd_dy, S->wd_dzL, S->wd_dzU);
    S->ref_theta = S->wd_theta;
    S->ref_phi = S->wd_phi;
    S->ref_gd = S->wd_gd;
    S->wd_short = 0;
    /* the current iterate is the restored one */
    eval_current(S);
    int ok;
    S->phi = barrier_phi(S, S->w, &ok);
}

/* primal-dual system error of (w, y, zL, zU) for the soft restoration phase
 * (curr_primal_dual_system_error: 1-norms of the dual infeasibility, the constraint
 * violation and the mu-complementarity, averaged over all their entries) */
static double pd_error(ipm* S, const double* w, const double* y, const double* zL, const double* zU, int trial) {
    iprob* P = S->P;
    double *g = trial ? S->gft : S->gf, *A = trial ? S->At : S->A, *rd = trial ? S->rdt : S->rd;
    double *c = trial ? S->ct : S->cv;
    if (trial) {
        P->grad(P, w, S->mu, g);
        P->jac(P, w, A);
        P->cons(P, w, c);
    }
    lag_grad(S, g, A, y, zL, zU, rd);
    const double du = l1(S->nw, rd), pr = l1(S->m, c), cm = compl_norm(S, w, zL, zU, S->mu, 1);
    return (du + pr + cm) / (double)(S->nw + S->m + S->nbnd);
}
/* BacktrackingLineSearch::TrySoftRestoStep */
static int try_soft_resto(ipm* S, int* satisfies_orig) {
    *satisfies_orig = 0;
    const double ap = primal_frac(S, S->w, S->aw);
    const double ad = dual_frac(S, S->zL, S->zU, S->azL, S->azU);
    const double a = fmin(ap, ad);
    double phit, thetat;
    int ok = eval_trial(S, a, S->aw, &phit, &thetat);
    dual_step(S, a, a, S->ay, S->azL, S->azU);
    if (!ok) return 0;
    if (check_acceptability(S, 0.0, phit, thetat)) {
        *satisfies_orig = 1;
        if (S->diag) ++S->diag->n_soft_resto;
        return 1;
    }
    const double et = pd_error(S, S->wt, S->yt, S->zLt, S->zUt, 1);
    const double ec = pd_error(S, S->w, S->y, S->zL, S->zU, 0);
    if (et <= S->o->soft_resto_pderror_reduction_factor * ec) {
        if (S->diag) ++S->diag->n_soft_resto;
        return 1;
    }
    return 0;
}

static int ipm_iterate(ipm* S);

/* MinC_1NrmRestorationPhase::PerformRestoration.  On success the trial point (wt, yt,
 * zLt, zUt) holds the point to continue from and 0 is returned; otherwise a status. */
static int perform_restoration(ipm* S) {
    iprob* P = S->P;
    const int nx = S->nw, m = S->m, nv = nx + 2 * m;
    if (S->diag) ++S->diag->n_resto;
    resto_ctx rc;
    rc.orig = P;
    rc.nx = nx;
    rc.m = m;
    rc.rho = 1000.0;
    double* buf = (double*)calloc((size_t)2 * nx + m + (size_t)m * nx + 2 * nv + 2 * nv, sizeof(double));
    double *xR = buf, *DR = xR + nx;
    rc.c = DR + nx;
    rc.A = rc.c + m;
    double *vl = rc.A + (size_t)m * nx, *vu = vl + nv;
    char* hb = (char*)calloc(2 * nv, 1);
    for (int i = 0; i < nx; ++i) {
        xR[i] = S->w[i];
        DR[i] = 1.0 / fmax(1.0, fabs(S->w[i]));
    }
    rc.xR = xR;
    rc.DR = DR;
    iprob R;
    memset(&R, 0, sizeof R);
    R.nw = nv;
    R.m = m;
    R.ctx = &rc;
    R.f = resto_f;
    R.grad = resto_grad;
    R.cons = resto_cons;
    R.jac = resto_jac;
    R.hess = resto_hess;
    R.wl = vl;
    R.wu = vu;
    R.hasL = hb;
    R.hasU = hb + nv;
    R.obj_scale = 1.0;
    R.c_scale = NULL;
    for (int i = 0; i < nx; ++i) {
        vl[i] = P->wl[i];
        vu[i] = P->wu[i];
        R.hasL[i] = P->hasL[i];
        R.hasU[i] = P->hasU[i];
    }
    for (int i = nx; i < nv; ++i) {
        vl[i] = 0.0;
        vu[i] = INFINITY;
        R.hasL[i] = 1;
        R.hasU[i] = 0;
    }
    ipm Rs;
    ipm_alloc(&Rs, &R, S->o);
    Rs.is_resto = 1;
    Rs.outer = S;
    Rs.iter = S->iter;
    Rs.diag = NULL;
    Rs.slk = S->slk;
    Rs.resto_first = 1;
    /* RestoIterateInitializer: mu_R = max(mu, ||c||_inf), p and n the minimisers of the
     * l1 penalty with barrier for fixed x, x bound multipliers min(rho, z), p/n
     * multipliers mu_R / p, mu_R / n, y = 0 */
    const double muR = fmax(S->mu, amax(m, S->cv));
    Rs.mu = muR;
    Rs.tau = fmax(0.99, 1.0 - muR);
    for (int i = 0; i < nx; ++i) {
        Rs.w[i] = S->w[i];
        Rs.zL[i] = P->hasL[i] ? fmin(rc.rho, S->zL[i]) : 0.0;
        Rs.zU[i] = P->hasU[i] ? fmin(rc.rho, S->zU[i]) : 0.0;
    }
    for (int r = 0; r < m; ++r) {
        const double c = S->cv[r];
        const double a = muR / (2.0 * rc.rho) - 0.5 * c, b = c * muR / (2.0 * rc.rho);
        const double nn = a + sqrt(a * a + b), pp = c + nn;
        Rs.w[nx + r] = pp;
        Rs.w[nx + m + r] = nn;
        Rs.zL[nx + r] = muR / pp;
        Rs.zL[nx + m + r] = muR / nn;
        Rs.y[r] = 0.0;
    }
    const int it0 = *S->iter;
    int st = ipm_iterate(&Rs);
    if (S->diag) S->diag->resto_iters += *S->iter - it0;
    if (st == 0) {
        /* back to the original problem: x from the restoration phase, y = 0
         * (constr_mult_reset_threshold 0), bound multipliers by a Newton step of the
         * complementarity with the whole restoration step as the primal step
         * (ComputeBoundMultiplierStep), reset to 1 above bound_mult_reset_threshold */
        for (int i = 0; i < nx; ++i) S->wt[i] = Rs.w[i];
        for (int r = 0; r < m; ++r) S->yt[r] = 0.0;
        double* dz = (double*)malloc(sizeof(double) * 2 * nx);
        for (int i = 0; i < nx; ++i) {
            double dl = 0.0, du = 0.0;
            if (P->hasL[i]) {
                const double sc = S->w[i] - P->wl[i], st_ = S->wt[i] - P->wl[i];
                dl = (S->mu + S->zL[i] * (sc - st_)) / sc - S->zL[i];
            }
            if (P->hasU[i]) {
                const double sc = P->wu[i] - S->w[i], st_ = P->wu[i] - S->wt[i];
                du = (S->mu + S->zU[i] * (sc - st_)) / sc - S->zU[i];
            }
            dz[i] = dl;
            dz[nx + i] = du;
        }
        const double ad = dual_frac(S, S->zL, S->zU, dz, dz + nx);
        double zmax = 0.0;
        for (int i = 0; i < nx; ++i) {
            S->zLt[i] = S->zL[i] + ad * dz[i];
            S->zUt[i] = S->zU[i] + ad * dz[nx + i];
            zmax = fmax(zmax, fmax(fabs(S->zLt[i]), fabs(S->zUt[i])));
        }
        if (zmax > 1000.0)
            for (int i = 0; i < nx; ++i) {
                S->zLt[i] = P->hasL[i] ? 1.0 : 0.0;
                S->zUt[i] = P->hasU[i] ? 1.0 : 0.0;
            }
        free(dz);
    }
    ipm_free(&Rs);
    free(buf);
    free(hb);
    return st;
}

/* BacktrackingLineSearch::FindAcceptableTrialPoint.  Returns 0 with the accepted trial
 * point in (wt, yt, zLt, zUt), or a termination status. */
static int find_trial_point(ipm* S, int goto_resto) {
    const ora_ipm_opts* o = S->o;
    if (S->mu != S->last_mu) {
        S->in_wd = 0;
        S->wd_short = 0;
        S->last_mu = S->mu;
    }
    if (!S->is_resto && o->acceptable_iter > 0 && current_is_acceptable(S)) {
        copy_dir(S, S->acc_w, S->acc_y, S->acc_zL, S->acc_zU, S->w, S->y, S->zL, S->zU);
        S->have_acc = 1;
    }
    copy_dir(S, S->aw, S->ay, S->azL, S->azU, S->dw, S->dy, S->dzL, S->dzU);
    if (!goto_resto) {
        /* InitThisLineSearch */
        if (S->in_wd) {
            S->ref_theta = S->wd_theta;
            S->ref_phi = S->wd_phi;
            S->ref_gd = S->wd_gd;
        } else {
            S->ref_theta = S->theta;
            S->ref_phi = S->phi;
            S->ref_gd = S->gd;
        }
    }
    int accept = 0, n_steps = 0, soft_or_resto = 0;
    double alpha = 0.0;
    /* DetectTinyStep */
    int tiny = 0;
    if (!goto_resto && o->tiny_step_tol > 0) {
        double rel = 0.0;
        for (int i = 0; i < S->nw; ++i) rel = fmax(rel, fabs(S->dw[i]) / (1.0 + fabs(S->w[i])));
        tiny = rel <= o->tiny_step_tol && (S->m == 0 || amax(S->m, S->dy) <= o->tiny_step_y_tol);
    }
    if (S->in_wd && (goto_resto || tiny)) {
        stop_watchdog(S);
        goto_resto = 0;
        tiny = 0;
    }
    if (o->watchdog_shortened_iter_trigger > 0 && !S->in_wd && !goto_resto && !tiny && !S->in_soft &&
        S->wd_short >= o->watchdog_shortened_iter_trigger)
        start_watchdog(S);
    if (tiny) {
        alpha = primal_frac(S, S->w, S->dw);
        double phit, thetat;
        eval_trial(S, alpha, S->dw, &phit, &thetat);
        if (S->tiny_last) S->tiny_flag = 1;
        S->tiny_last = 1;
        accept = 1;
    } else {
        S->tiny_last = 0;
    }
    if (!goto_resto && !tiny) {
        if (S->in_soft) {
            if (++S->soft_count > o->max_soft_resto_iters) {
                accept = 0;
            } else {
                int sat;
                accept = try_soft_resto(S, &sat);
                if (accept && sat) {
                    S->in_soft = 0;
                    S->soft_count = 0;
                }
            }
            soft_or_resto = accept;
        } else {
            int done = 0, skip_first = 0, eval_error;
            while (!done) {
                accept = backtracking(S, skip_first, &alpha, &n_steps, &eval_error);
                if (S->in_wd) {
                    if (accept) {
                        S->in_wd = 0;
                        done = 1;
                    } else {
                        ++S->wd_trial_iter;
                        if (eval_error || S->wd_trial_iter > o->watchdog_trial_iter_max) {
                            stop_watchdog(S);
                            skip_first = 1;
                        } else {
                            done = 1;
                            accept = 1;
                        }
                    }
                } else {
                    done = 1;
                }
            }
        }
    }
    if (!accept) {
        if (!S->in_soft && o->soft_resto_pderror_reduction_factor > 0.0 && !goto_resto) {
            augment_filter(S); /* PrepareRestoPhaseStart */
            int sat;
            if (try_soft_resto(S, &sat)) {
                S->in_soft = !sat;
                accept = 1;
                soft_or_resto = 1;
            }
        }
        if (!accept) {
            if (!S->in_soft) augment_filter(S);
            if (S->is_resto || S->m == 0) return ORA_RESTORATION_FAILURE;
            /* almost feasible: restore the stored acceptable point, if any */
            if (S->theta <= 1e-2 * o->tol) {
                if (S->have_acc) {
                    copy_dir(S, S->w, S->y, S->zL, S->zU, S->acc_w, S->acc_y, S->acc_zL, S->acc_zU);
                    return ORA_STOP_AT_ACCEPTABLE_POINT;
                }
                return ORA_RESTORATION_FAILURE;
            }
            /* (restoration = 0: stop where the restoration phase would start -- the
             * device's no_restoration option) */
            if (!o->restoration) return ORA_RESTORATION_FAILURE;
            if (((orig_ctx*)S->P->ctx)->mI > 0) return ORA_RESTORATION_FAILURE;
            S->in_soft = 0;
            S->soft_count = 0;
            S->wd_short = 0;
            int st = perform_restoration(S);
            if (st) return st;
            return 0; /* trial point set by the restoration phase (no dual step here) */
        }
    }
    if (!soft_or_resto) {
        /* dual step of the accepted primal step and the watchdog counter */
        const double ad = dual_frac(S, S->zL, S->zU, S->azL, S->azU);
        dual_step(S, alpha, ad, S->ay, S->azL, S->azU);
        if (n_steps == 0)
            S->wd_short = 0;
        else
            ++S->wd_short;
    }
    return 0;
}

/* IpoptAlgorithm::AcceptTrialPoint: bound multipliers kept within kappa_sigma of mu / s */
static void accept_trial(ipm* S) {
    iprob* P = S->P;
    const double ks = 1e10, mu = S->mu;
    memcpy(S->w, S->wt, sizeof(double) * S->nw);
    memcpy(S->y, S->yt, sizeof(double) * S->m);
    for (int i = 0; i < S->nw; ++i) {
        if (P->hasL[i]) {
            const double s = S->w[i] - P->wl[i];
            S->zL[i] = fmax(fmin(S->zLt[i], ks * mu / s), mu / (ks * s));
        } else {
            S->zL[i] = 0.0;
        }
        if (P->hasU[i]) {
            const double s = P->wu[i] - S->w[i];
            S->zU[i] = fmax(fmin(S->zUt[i], ks * mu / s), mu / (ks * s));
        } else {
            S->zU[i] = 0.0;
        }
    }
}

/* convergence check of the restoration problem (RestoConvergenceCheck +
 * RestoFilterConvergenceCheck::TestOrigProgress).  Returns -1 to continue, 0 when the
 * original problem can take over, or a status. */
static int resto_convergence(ipm* S) {
    ipm* O = S->outer;
    const ora_ipm_opts* o = S->o;
    int status = -1;
    if (S->resto_first) {
        S->resto_first = 0;
    } else {
        int ok;
        const double bt = barrier_phi(O, S->w, &ok);
        O->P->cons(O->P, S->w, O->ct);
        const double tt = l1(O->m, O->ct);
        if (ok && isfinite(tt) && tt <= 0.9 * O->theta && filter_acceptable(O, bt, tt) &&
            acceptable_to_current_iterate(O, bt, tt, 1))
            status = 0;
    }
    if (status < 0) {
        /* the restoration problem's own optimality */
        if (S->E0 <= o->tol && S->dual_uns <= o->dual_inf_tol && S->prim_uns <= o->constr_viol_tol &&
            S->compl_uns <= o->compl_inf_tol) {
            O->P->cons(O->P, S->w, O->ct);
            return amax(O->m, O->ct) <= 1e2 * o->tol ? ORA_FEASIBLE_POINT_FOUND : ORA_LOCAL_INFEASIBILITY;
        }
        if (*S->iter >= o->max_iter) return ORA_MAXITER_EXCEEDED;
        if (o->cpu_iter_budget >= 0 && *S->iter > o->cpu_iter_budget) return ORA_UNKNOWN;
    }
    return status;
}

/* The main loop (IpoptAlgorithm::Optimize).  Returns a status, or (restoration problem) 0
 * when the original problem can take over. */
static int ipm_iterate(ipm* S) {
    const ora_ipm_opts* o = S->o;
    const double kappa_eps = 10.0, kappa_mu = 0.2, theta_mu = 1.5;
    const double mu_min = fmin(o->tol, o->compl_inf_tol) / (kappa_eps + 1.0);
    for (;;) {
        eval_current(S);
        {
            int okp;
            S->phi = barrier_phi(S, S->w, &okp);
        }
        if (o->print_level > 0)
            fprintf(stderr, "%s%3d mu %.2e E0 %.3e dual %.3e prim %.3e compl %.3e th %.3e f %.10e nf %d\n",
                    S->is_resto ? "r" : "", *S->iter, S->mu, S->E0, S->dual_inf, S->prim_inf, S->compl0, S->theta,
                    S->f, S->nf);
        /* Ipopt's finiteness test of f and g at an evaluated point (OrigIpoptNLP) ->
         * INVALID_NUMBER_DETECTED: amax() drops a NaN, the l1 norm and f do not */
        if (!isfinite(S->E0) || !isfinite(S->theta) || !isfinite(S->f)) return ORA_INVALID_NUMBER_DETECTED;
        /* ---- convergence (OptimalityErrorConvergenceCheck::CheckConvergence) ---- */
        if (S->is_resto) {
            int st = resto_convergence(S);
            if (st >= 0) return st;
        } else {
            if (S->E0 <= o->tol && S->dual_uns <= o->dual_inf_tol && S->prim_uns <= o->constr_viol_tol &&
                S->compl_uns <= o->compl_inf_tol)
                return ORA_SUCCESS;
            if (o->acceptable_iter > 0 && current_is_acceptable(S)) {
                if (++S->acc_counter >= o->acceptable_iter) return ORA_STOP_AT_ACCEPTABLE_POINT;
            } else {
                S->acc_counter = 0;
            }
            if (*S->iter >= o->max_iter) return ORA_MAXITER_EXCEEDED;
            if (o->cpu_iter_budget >= 0 && *S->iter > o->cpu_iter_budget) return ORA_UNKNOWN;
        }
        /* ---- monotone barrier update (MonotoneMuUpdate::UpdateBarrierParameter) ---- */
        {
            int tiny_flag = S->tiny_flag;
            S->tiny_flag = 0;
            int done = 0;
            double complmu = compl_norm(S, S->w, S->zL, S->zU, S->mu, 0);
            double Emu = fmax(S->dual_inf / S->sd, fmax(S->prim_inf, complmu / S->sc));
            while ((Emu <= kappa_eps * S->mu || tiny_flag) && !done) {
                double mnew = fmax(fmin(kappa_mu * S->mu, pow(S->mu, theta_mu)), mu_min);
                int changed = mnew != S->mu;
                if (!changed && tiny_flag) return ORA_STOP_AT_TINY_STEP;
                S->mu = mnew;
                S->tau = fmax(0.99, 1.0 - mnew);
                if (!changed) {
                    done = 1;
                } else {
                    if (S->is_resto) eval_current(S); /* the restoration objective depends on mu */
                    complmu = compl_norm(S, S->w, S->zL, S->zU, S->mu, 0);
                    Emu = fmax(S->dual_inf / S->sd, fmax(S->prim_inf, complmu / S->sc));
                    done = Emu > kappa_eps * S->mu;
                }
                if (done && changed) {
                    /* BacktrackingLineSearch::Reset */
                    S->in_soft = 0;
                    S->in_wd = 0;
                    S->wd_short = 0;
                    S->nf = 0;
                }
                tiny_flag = 0;
            }
        }
        /* the barrier function changed with mu */
        if (S->is_resto) {
            /* the restoration objective depends on mu (eta = sqrt(mu)) */
            eval_current(S);
        }
        {
            int okp;
            S->phi = barrier_phi(S, S->w, &okp);
        }
        /* ---- search direction ---- */
        barrier_grad(S, S->w, S->gf, S->gphi);
        int goto_resto = 0;
        if (factor_kkt(S)) {
            solve_step(S, S->cv, S->dw, S->dy, S->dzL, S->dzU);
        } else {
            if (S->is_resto || !o->restoration) return ORA_ERROR_IN_STEP_COMPUTATION;
            goto_resto = 1; /* fallback: restoration phase */
            memset(S->dw, 0, sizeof(double) * S->nw);
            memset(S->dy, 0, sizeof(double) * S->m);
            memset(S->dzL, 0, sizeof(double) * S->nw);
            memset(S->dzU, 0, sizeof(double) * S->nw);
        }
        S->gd = 0.0;
        for (int i = 0; i < S->nw; ++i) S->gd += S->gphi[i] * S->dw[i];
        /* ---- line search ---- */
        int st = find_trial_point(S, goto_resto);
        if (st) return st;
        accept_trial(S);
        ++*S->iter;
    }
}

int ora_ipm_solve(const ora_nlp* nlp, const ora_ipm_opts* opts_in, double* x_out, double* zl_out, double* zu_out,
                  double* lambda_out, double* g_out, ora_ipm_result* res) {
    ora_ipm_opts opts;
    if (opts_in) opts = *opts_in; else ora_ipm_default_opts(&opts);
    const int n = nlp->n, m = nlp->m;
    orig_ctx oc;
    memset(&oc, 0, sizeof oc);
    oc.nlp = nlp;
    oc.n = n;
    oc.m = m;
    oc.ineq_of_row = (int*)malloc(sizeof(int) * (m > 0 ? m : 1));
    int mI = 0;
    for (int r = 0; r < m; ++r) oc.ineq_of_row[r] = (nlp->gl[r] == nlp->gu[r]) ? -1 : mI++;
    oc.mI = mI;
    const int nw = n + mI;
    double* buf = (double*)calloc((size_t)6 * nw + 3 * m + (size_t)m * n + (size_t)n * n + 8, sizeof(double));
    double *wl0 = buf, *wu0 = wl0 + nw, *wl = wu0 + nw, *wu = wl + nw, *gf0 = wu + nw;
    oc.c_scale = gf0 + nw;
    oc.gv = oc.c_scale + m;
    oc.lam = oc.gv + m;
    oc.jac = oc.lam + m;
    oc.H = oc.jac + (size_t)m * n;
    char* hb = (char*)calloc(2 * (size_t)nw + 2, 1);
    iprob P;
    memset(&P, 0, sizeof P);
    P.nw = nw;
    P.m = m;
    P.ctx = &oc;
    P.f = orig_f;
    P.grad = orig_grad;
    P.cons = orig_cons;
    P.jac = orig_jac;
    P.hess = orig_hess;
    P.wl = wl;
    P.wu = wu;
    P.hasL = hb;
    P.hasU = hb + nw;
    P.c_scale = oc.c_scale;

    /* ---- bounds on w (original), then relaxation (bound_relax_factor) ---- */
    for (int i = 0; i < n; ++i) { wl0[i] = nlp->xl[i]; wu0[i] = nlp->xu[i]; }
    for (int r = 0; r < m; ++r) {
        int s = oc.ineq_of_row[r];
        if (s >= 0) { wl0[n + s] = nlp->gl[r]; wu0[n + s] = nlp->gu[r]; }
    }
    for (int i = 0; i < nw; ++i) {
        P.hasL[i] = wl0[i] > -INF_BOUND;
        P.hasU[i] = wu0[i] < INF_BOUND;
        double rl = fmin(opts.constr_viol_tol, opts.bound_relax_factor * fmax(1.0, fabs(wl0[i])));
        double ru = fmin(opts.constr_viol_tol, opts.bound_relax_factor * fmax(1.0, fabs(wu0[i])));
        wl[i] = P.hasL[i] ? wl0[i] - rl : -INFINITY;
        wu[i] = P.hasU[i] ? wu0[i] + ru : INFINITY;
    }
    /* ---- gradient-based scaling at the user's starting point ---- */
    {
        nlp->grad_f(nlp->ctx, nlp->x0, gf0);
        double gmax = amax(n, gf0);
        oc.obj_scale = (gmax > 100.0) ? 100.0 / gmax : 1.0;
        nlp->jac_g(nlp->ctx, nlp->x0, oc.jac);
        for (int r = 0; r < m; ++r) {
            double rm = amax(n, oc.jac + (size_t)r * n);
            oc.c_scale[r] = (rm > 100.0) ? 100.0 / rm : 1.0;
        }
    }
    P.obj_scale = oc.obj_scale;

    ipm S;
    ipm_alloc(&S, &P, &opts);
    if (opts.kkt_structured && nlp->kkt_order && mI == 0) {
        S.kpos = (int*)malloc(sizeof(int) * (size_t)S.K);
        S.klast = (int*)malloc(sizeof(int) * (size_t)S.K);
        for (int i = 0; i < S.K; ++i) S.kpos[nlp->kkt_order[i]] = i;
    }
    int iter = 0;
    S.iter = &iter;
    ora_ipm_result diag;
    memset(&diag, 0, sizeof diag);
    diag.min_slack_margin = INFINITY;
    S.diag = &diag;
    S.slk = &diag;

    /* ---- starting point: x0 pushed inside (bound_push/bound_frac 0.01) ---- */
    for (int i = 0; i < n; ++i) S.w[i] = nlp->x0[i];
    nlp->g(nlp->ctx, S.w, oc.gv);
    for (int r = 0; r < m; ++r) {
        int s = oc.ineq_of_row[r];
        if (s >= 0) S.w[n + s] = oc.gv[r];
    }
    for (int i = 0; i < nw; ++i) {
        const double k1 = 0.01, k2 = 0.01;
        if (P.hasL[i] && P.hasU[i]) {
            double pl = fmin(k1 * fmax(1.0, fabs(wl[i])), k2 * (wu[i] - wl[i]));
            double pu = fmin(k1 * fmax(1.0, fabs(wu[i])), k2 * (wu[i] - wl[i]));
            if (S.w[i] < wl[i] + pl) S.w[i] = wl[i] + pl;
            if (S.w[i] > wu[i] - pu) S.w[i] = wu[i] - pu;
        } else if (P.hasL[i]) {
            double pl = k1 * fmax(1.0, fabs(wl[i]));
            if (S.w[i] < wl[i] + pl) S.w[i] = wl[i] + pl;
        } else if (P.hasU[i]) {
            double pu = k1 * fmax(1.0, fabs(wu[i]));
            if (S.w[i] > wu[i] - pu) S.w[i] = wu[i] - pu;
        }
    }
    for (int i = 0; i < nw; ++i) {
        S.zL[i] = P.hasL[i] ? 1.0 : 0.0;
        S.zU[i] = P.hasU[i] ? 1.0 : 0.0;
    }
    /* ---- least-squares multiplier estimate (constr_mult_init_max 1000) ---- */
    {
        const int K = S.K;
        P.grad(&P, S.w, 0.0, S.gf);
        P.jac(&P, S.w, S.A);
        memset(S.KKT, 0, sizeof(double) * (size_t)K * K);
        for (int i = 0; i < nw; ++i) S.KKT[i + (size_t)i * K] = 1.0;
        for (int r = 0; r < m; ++r)
            for (int j = 0; j < nw; ++j) S.KKT[(nw + r) + (size_t)j * K] = S.A[(size_t)r * nw + j];
        for (int i = 0; i < nw; ++i) S.rhs[i] = -(S.gf[i] - S.zL[i] + S.zU[i]);
        for (int r = 0; r < m; ++r) S.rhs[nw + r] = 0.0;
        int np, nn, nz;
        ora_ldlt_factor(K, S.KKT, S.ipiv, 1e-300, &np, &nn, &nz);
        if (nz == 0) {
            ora_ldlt_solve(K, S.KKT, S.ipiv, S.rhs);
            double ym = amax(m, S.rhs + nw);
            for (int r = 0; r < m; ++r) S.y[r] = (ym <= 1000.0) ? S.rhs[nw + r] : 0.0;
        }
    }
    S.mu = opts.mu_init;
    S.tau = fmax(0.99, 1.0 - S.mu);

    int status = ipm_iterate(&S);

    /* ---- outputs (unscaled), honor_original_bounds ---- */
    for (int i = 0; i < n; ++i) {
        double xv = S.w[i];
        if (opts.honor_original_bounds) {
            if (P.hasL[i] && xv < wl0[i]) xv = wl0[i];
            if (P.hasU[i] && xv > wu0[i]) xv = wu0[i];
        }
        x_out[i] = xv;
        if (zl_out) zl_out[i] = S.zL[i] / oc.obj_scale;
        if (zu_out) zu_out[i] = S.zU[i] / oc.obj_scale;
    }
    if (lambda_out)
        for (int r = 0; r < m; ++r) lambda_out[r] = S.y[r] * oc.c_scale[r] / oc.obj_scale;
    if (g_out) nlp->g(nlp->ctx, x_out, g_out);
    if (res) {
        *res = diag;
        res->status = status;
        res->iters = iter;
        res->obj = nlp->f(nlp->ctx, x_out);
        res->kkt_inf = fmax(S.dual_uns, fmax(S.prim_uns, S.compl_uns));
    }
    ipm_free(&S);
    free(oc.ineq_of_row);
    free(buf);
    free(hb);
    return status;
}
