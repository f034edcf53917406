/*
 * oracle/nlp_hs071.c -- the reference's only known-answer test (TEST INFRASTRUCTURE ONLY).
 *
 * assets/document/example/CppAD_Ipopt.cpp:61-83 (FG_eval) and :97-112 (start/bounds):
 *   min x1 x4 (x1+x2+x3) + x3   s.t.  x1 x2 x3 x4 >= 25,  sum xi^2 = 40,  1 <= xi <= 5
 * Known answer (:146-150): x* = (1.000000, 4.743000, 3.82115, 1.379408),
 * zl* = (1.087871, 0, 0, 0), zu* = 0 at rel/abs tol 1e-6.  Used to pin the Ipopt
 * restatement in ipm.c on a problem with an inequality, an equality and an active bound.
 */
#include <string.h>
#include "ora.h"

static double hs_f(void* c, const double* x) {
    (void)c;
    return x[0] * x[3] * (x[0] + x[1] + x[2]) + x[2];
}
static void hs_grad(void* c, const double* x, double* g) {
    (void)c;
    g[0] = x[3] * (x[0] + x[1] + x[2]) + x[0] * x[3];
    g[1] = x[0] * x[3];
    g[2] = x[0] * x[3] + 1.0;
    g[3] = x[0] * (x[0] + x[1] + x[2]);
}
static void hs_g(void* c, const double* x, double* g) {
    (void)c;
    g[0] = x[0] * x[1] * x[2] * x[3];
    g[1] = x[0] * x[0] + x[1] * x[1] + x[2] * x[2] + x[3] * x[3];
}
static void hs_jac(void* c, const double* x, double* J) {
    (void)c;
    J[0] = x[1] * x[2] * x[3];
    J[1] = x[0] * x[2] * x[3];
    J[2] = x[0] * x[1] * x[3];
    J[3] = x[0] * x[1] * x[2];
    for (int i = 0; i < 4; ++i) J[4 + i] = 2.0 * x[i];
}
static void hs_hess(void* c, const double* x, double s, const double* l, double* H) {
    (void)c;
    memset(H, 0, sizeof(double) * 16);
#define H_(i, j, v) do { H[(i) * 4 + (j)] += (v); if ((i) != (j)) H[(j) * 4 + (i)] += (v); } while (0)
    H_(0, 0, s * 2.0 * x[3]);
    H_(1, 0, s * x[3]);
    H_(2, 0, s * x[3]);
    H_(3, 0, s * (2.0 * x[0] + x[1] + x[2]));
    H_(3, 1, s * x[0]);
    H_(3, 2, s * x[0]);
    H_(1, 0, l[0] * x[2] * x[3]);
    H_(2, 0, l[0] * x[1] * x[3]);
    H_(3, 0, l[0] * x[1] * x[2]);
    H_(2, 1, l[0] * x[0] * x[3]);
    H_(3, 1, l[0] * x[0] * x[2]);
    H_(3, 2, l[0] * x[0] * x[1]);
    for (int i = 0; i < 4; ++i) H_(i, i, l[1] * 2.0);
#undef H_
}

int ora_hs071_solve(const ora_ipm_opts* opts, double* x4, double* zl4, double* zu4, int* iters) {
    static const double xi[4] = {1.0, 5.0, 5.0, 1.0};
    static const double xl[4] = {1.0, 1.0, 1.0, 1.0}, xu[4] = {5.0, 5.0, 5.0, 5.0};
    static const double gl[2] = {25.0, 40.0}, gu[2] = {1.0e19, 40.0};
    ora_nlp nlp;
    memset(&nlp, 0, sizeof nlp);
    nlp.n = 4;
    nlp.m = 2;
    nlp.ctx = 0;
    nlp.f = hs_f;
    nlp.grad_f = hs_grad;
    nlp.g = hs_g;
    nlp.jac_g = hs_jac;
    nlp.hess = hs_hess;
    nlp.xl = xl;
    nlp.xu = xu;
    nlp.gl = gl;
    nlp.gu = gu;
    nlp.x0 = xi;
    double lam[2], gv[2];
    ora_ipm_result res;
    int st = ora_ipm_solve(&nlp, opts, x4, zl4, zu4, lam, gv, &res);
    if (iters) *iters = res.iters;
    return st;
}
