/*
 * oracle/nlp_mpc.c -- the reference NLP, restated (TEST INFRASTRUCTURE ONLY, see ora.h).
 *
 * Variable layout (mpc_ros/src/mpc_planner.cpp:252-259, MPC::LoadParams):
 *   x[0..N) y[N..2N) theta[2N..3N) v[3N..4N) cte[4N..5N) etheta[5N..6N)
 *   angvel[6N..7N-1) a[7N-1..8N-2)                      nx = 8N-2
 * Constraint layout (mpc_planner.cpp:153-216): row s*N + i for state s in
 *   (x,y,theta,v,cte,etheta) and stage i; i == 0 is the initial-state row
 *   (fg[1 + start]), i >= 1 the dynamics defect of step i-1 (fg[2 + start + i-1]).
 *                                                      ng = 6N
 * Cost (mpc_planner.cpp:122-147):
 *   sum_{i<N}   W_CTE (cte_i-REF_CTE)^2 + W_EPSI (eth_i-REF_ETHETA)^2 + W_V (v_i-REF_V)^2
 *   sum_{i<N-1} W_ANGVEL w_i^2 + W_A a_i^2
 *   sum_{i<N-2} W_DANGVEL (w_{i+1}-w_i)^2 + W_DA (a_{i+1}-a_i)^2
 * Dynamics (mpc_planner.cpp:202-215), f(x) = sum_k c_k x^k (:186-190):
 *   x1 - (x0 + v0 cos(th0) dt)       y1 - (y0 + v0 sin(th0) dt)
 *   th1 - (th0 + w0 dt)              v1 - (v0 + a0 dt)
 *   cte1 - ((f(x0) - y0) + v0 sin(eth0) dt)      eth1 - (eth0 + w0 dt)
 * The dead trj_grad0 = atan(f'(x0)) (:192-198) does not reach fg and is omitted.
 * model 1 (kinematic bicycle, ora.h): w is the steering angle delta and the heading
 * rows are th1 - (th0 + v0 * delta0 / lf * dt), eth1 - (eth0 + v0 * delta0 / lf * dt).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include "ora.h"
#ifdef _OPENMP
#include <omp.h>
#endif

int ora_mpc_nx(int N) { return 6 * N + 2 * (N - 1); }
int ora_mpc_ng(int N) { return 6 * N; }

/* CppAD::pow(AD, int) -> pow_int: repeated multiplication (cppad/utility/pow_int.hpp:115-137) */
static double powi(double x, int k) {
    double r = 1.0;
    for (int i = 0; i < k; ++i) r *= x;
    return r;
}
static double fpoly(const double* c, double x) {
    double f = 0.0;
    for (int k = 0; k < 4; ++k) f += c[k] * powi(x, k);
    return f;
}
static double fpoly_d1(const double* c, double x) { return c[1] + 2.0 * c[2] * x + 3.0 * c[3] * x * x; }
static double fpoly_d2(const double* c, double x) { return 2.0 * c[2] + 6.0 * c[3] * x; }

#define IX(N) 0
#define IY(N) (N)
#define ITH(N) (2 * (N))
#define IV(N) (3 * (N))
#define ICTE(N) (4 * (N))
#define IETH(N) (5 * (N))
#define IW(N) (6 * (N))
#define IA(N) (7 * (N)-1)

void ora_mpc_fg(const ora_mpc_params* p, const double* c, const double* v, double* fg) {
    const int N = p->steps;
    const double dt = p->dt;
    double f = 0.0;
    for (int i = 0; i < N; ++i) {
        double e1 = v[ICTE(N) + i] - p->ref_cte;
        double e2 = v[IETH(N) + i] - p->ref_etheta;
        double e3 = v[IV(N) + i] - p->ref_v;
        f += p->w_cte * e1 * e1;
        f += p->w_etheta * e2 * e2;
        f += p->w_v * e3 * e3;
    }
    for (int i = 0; i < N - 1; ++i) {
        f += p->w_angvel * v[IW(N) + i] * v[IW(N) + i];
        f += p->w_accel * v[IA(N) + i] * v[IA(N) + i];
    }
    for (int i = 0; i < N - 2; ++i) {
        double dw = v[IW(N) + i + 1] - v[IW(N) + i];
        double da = v[IA(N) + i + 1] - v[IA(N) + i];
        f += p->w_angvel_d * dw * dw;
        f += p->w_accel_d * da * da;
    }
    fg[0] = f;
    double* g = fg + 1;
    for (int s = 0; s < 6; ++s) g[s * N] = v[s * N];
    for (int i = 0; i < N - 1; ++i) {
        double x0 = v[IX(N) + i], y0 = v[IY(N) + i], th0 = v[ITH(N) + i], v0 = v[IV(N) + i];
        double eth0 = v[IETH(N) + i];
        double w0 = v[IW(N) + i], a0 = v[IA(N) + i];
        g[0 * N + i + 1] = v[IX(N) + i + 1] - (x0 + v0 * cos(th0) * dt);
        g[1 * N + i + 1] = v[IY(N) + i + 1] - (y0 + v0 * sin(th0) * dt);
        const double turn = p->model == 1 ? v0 * w0 / p->lf * dt : w0 * dt;
        g[2 * N + i + 1] = v[ITH(N) + i + 1] - (th0 + turn);
        g[3 * N + i + 1] = v[IV(N) + i + 1] - (v0 + a0 * dt);
        g[4 * N + i + 1] = v[ICTE(N) + i + 1] - ((fpoly(c, x0) - y0) + v0 * sin(eth0) * dt);
        g[5 * N + i + 1] = v[IETH(N) + i + 1] - (eth0 + turn);
    }
}

void ora_mpc_grad_f(const ora_mpc_params* p, const double* c, const double* v, double* gf) {
    (void)c;
    const int N = p->steps;
    const int nx = ora_mpc_nx(N);
    memset(gf, 0, sizeof(double) * nx);
    for (int i = 0; i < N; ++i) {
        gf[ICTE(N) + i] = 2.0 * p->w_cte * (v[ICTE(N) + i] - p->ref_cte);
        gf[IETH(N) + i] = 2.0 * p->w_etheta * (v[IETH(N) + i] - p->ref_etheta);
        gf[IV(N) + i] = 2.0 * p->w_v * (v[IV(N) + i] - p->ref_v);
    }
    for (int i = 0; i < N - 1; ++i) {
        gf[IW(N) + i] = 2.0 * p->w_angvel * v[IW(N) + i];
        gf[IA(N) + i] = 2.0 * p->w_accel * v[IA(N) + i];
    }
    for (int i = 0; i < N - 2; ++i) {
        double dw = v[IW(N) + i + 1] - v[IW(N) + i];
        double da = v[IA(N) + i + 1] - v[IA(N) + i];
        gf[IW(N) + i + 1] += 2.0 * p->w_angvel_d * dw;
        gf[IW(N) + i] -= 2.0 * p->w_angvel_d * dw;
        gf[IA(N) + i + 1] += 2.0 * p->w_accel_d * da;
        gf[IA(N) + i] -= 2.0 * p->w_accel_d * da;
    }
}

void ora_mpc_jac_g(const ora_mpc_params* p, const double* c, const double* v, double* J) {
    const int N = p->steps;
    const int nx = ora_mpc_nx(N), ng = ora_mpc_ng(N);
    const double dt = p->dt;
    memset(J, 0, sizeof(double) * (size_t)nx * ng);
#define JJ(r, col) J[(size_t)(r) * nx + (col)]
    for (int s = 0; s < 6; ++s) JJ(s * N, s * N) = 1.0;
    for (int i = 0; i < N - 1; ++i) {
        double x0 = v[IX(N) + i], th0 = v[ITH(N) + i], v0 = v[IV(N) + i], eth0 = v[IETH(N) + i];
        int r;
        r = 0 * N + i + 1;
        JJ(r, IX(N) + i + 1) = 1.0;
        JJ(r, IX(N) + i) = -1.0;
        JJ(r, ITH(N) + i) = v0 * sin(th0) * dt;
        JJ(r, IV(N) + i) = -cos(th0) * dt;
        r = 1 * N + i + 1;
        JJ(r, IY(N) + i + 1) = 1.0;
        JJ(r, IY(N) + i) = -1.0;
        JJ(r, ITH(N) + i) = -v0 * cos(th0) * dt;
        JJ(r, IV(N) + i) = -sin(th0) * dt;
        const double w0 = v[IW(N) + i];
        /* d(turn)/d(w), d(turn)/d(v) */
        const double tw = p->model == 1 ? v0 / p->lf * dt : dt;
        const double tv = p->model == 1 ? w0 / p->lf * dt : 0.0;
        r = 2 * N + i + 1;
        JJ(r, ITH(N) + i + 1) = 1.0;
        JJ(r, ITH(N) + i) = -1.0;
        JJ(r, IW(N) + i) = -tw;
        if (p->model == 1) JJ(r, IV(N) + i) = -tv;
        r = 3 * N + i + 1;
        JJ(r, IV(N) + i + 1) = 1.0;
        JJ(r, IV(N) + i) = -1.0;
        JJ(r, IA(N) + i) = -dt;
        r = 4 * N + i + 1;
        JJ(r, ICTE(N) + i + 1) = 1.0;
        JJ(r, IX(N) + i) = -fpoly_d1(c, x0);
        JJ(r, IY(N) + i) = 1.0;
        JJ(r, IV(N) + i) = -sin(eth0) * dt;
        JJ(r, IETH(N) + i) = -v0 * cos(eth0) * dt;
        r = 5 * N + i + 1;
        JJ(r, IETH(N) + i + 1) = 1.0;
        JJ(r, IETH(N) + i) = -1.0;
        JJ(r, IW(N) + i) = -tw;
        if (p->model == 1) JJ(r, IV(N) + i) = -tv;
    }
#undef JJ
}

void ora_mpc_hess(const ora_mpc_params* p, const double* c, const double* v, double sigma,
                  const double* lam, double* H) {
    const int N = p->steps;
    const int nx = ora_mpc_nx(N);
    const double dt = p->dt;
    memset(H, 0, sizeof(double) * (size_t)nx * nx);
#define HH(a, b) H[(size_t)(a) * nx + (b)]
#define HADD(a, b, val) do { double _v = (val); HH(a, b) += _v; if ((a) != (b)) HH(b, a) += _v; } while (0)
    for (int i = 0; i < N; ++i) {
        HADD(ICTE(N) + i, ICTE(N) + i, sigma * 2.0 * p->w_cte);
        HADD(IETH(N) + i, IETH(N) + i, sigma * 2.0 * p->w_etheta);
        HADD(IV(N) + i, IV(N) + i, sigma * 2.0 * p->w_v);
    }
    for (int i = 0; i < N - 1; ++i) {
        HADD(IW(N) + i, IW(N) + i, sigma * 2.0 * p->w_angvel);
        HADD(IA(N) + i, IA(N) + i, sigma * 2.0 * p->w_accel);
    }
    for (int i = 0; i < N - 2; ++i) {
        HADD(IW(N) + i + 1, IW(N) + i + 1, sigma * 2.0 * p->w_angvel_d);
        HADD(IW(N) + i, IW(N) + i, sigma * 2.0 * p->w_angvel_d);
        HADD(IW(N) + i + 1, IW(N) + i, -sigma * 2.0 * p->w_angvel_d);
        HADD(IA(N) + i + 1, IA(N) + i + 1, sigma * 2.0 * p->w_accel_d);
        HADD(IA(N) + i, IA(N) + i, sigma * 2.0 * p->w_accel_d);
        HADD(IA(N) + i + 1, IA(N) + i, -sigma * 2.0 * p->w_accel_d);
    }
    for (int i = 0; i < N - 1; ++i) {
        double x0 = v[IX(N) + i], th0 = v[ITH(N) + i], v0 = v[IV(N) + i], eth0 = v[IETH(N) + i];
        double lx = lam[0 * N + i + 1], ly = lam[1 * N + i + 1], lc = lam[4 * N + i + 1];
        /* x-defect: -v cos(th) dt */
        HADD(ITH(N) + i, ITH(N) + i, lx * v0 * cos(th0) * dt);
        HADD(ITH(N) + i, IV(N) + i, lx * sin(th0) * dt);
        /* y-defect: -v sin(th) dt */
        HADD(ITH(N) + i, ITH(N) + i, ly * v0 * sin(th0) * dt);
        HADD(ITH(N) + i, IV(N) + i, -ly * cos(th0) * dt);
        /* cte-defect: -(f(x) - y) - v sin(eth) dt */
        HADD(IX(N) + i, IX(N) + i, -lc * fpoly_d2(c, x0));
        HADD(IETH(N) + i, IETH(N) + i, lc * v0 * sin(eth0) * dt);
        HADD(IETH(N) + i, IV(N) + i, -lc * cos(eth0) * dt);
        if (p->model == 1) {
            /* heading rows: -(v delta / lf) dt */
            const double lt = lam[2 * N + i + 1], le = lam[5 * N + i + 1];
            HADD(IW(N) + i, IV(N) + i, -(lt + le) / p->lf * dt);
        }
    }
#undef HADD
#undef HH
}

void ora_mpc_bounds(const ora_mpc_params* p, const double* st, double* x0, double* xl, double* xu,
                    double* gl, double* gu) {
    const int N = p->steps;
    const int nx = ora_mpc_nx(N), ng = ora_mpc_ng(N);
    const int angvel_start = IW(N), a_start = IA(N);
    for (int i = 0; i < nx; ++i) x0[i] = 0.0;                         /* :288-292 */
    for (int s = 0; s < 6; ++s) x0[s * N] = st[s];                    /* :295-300 */
    for (int i = 0; i < angvel_start; ++i) { xl[i] = -p->bound; xu[i] = p->bound; }       /* :308-312 */
    for (int i = angvel_start; i < a_start; ++i) { xl[i] = -p->max_angvel; xu[i] = p->max_angvel; }
    for (int i = a_start; i < nx; ++i) { xl[i] = -p->max_throttle; xu[i] = p->max_throttle; }
    for (int i = 0; i < ng; ++i) { gl[i] = 0.0; gu[i] = 0.0; }          /* :330-335 */
    for (int s = 0; s < 6; ++s) { gl[s * N] = st[s]; gu[s * N] = st[s]; } /* :336-347 */
}

typedef struct {
    const ora_mpc_params* p;
    const double* c;
    double* fgbuf;
} mpc_ctx;

static double cb_f(void* ctx, const double* x) {
    mpc_ctx* m = (mpc_ctx*)ctx;
    ora_mpc_fg(m->p, m->c, x, m->fgbuf);
    return m->fgbuf[0];
}
static void cb_grad(void* ctx, const double* x, double* g) {
    mpc_ctx* m = (mpc_ctx*)ctx;
    ora_mpc_grad_f(m->p, m->c, x, g);
}
static void cb_g(void* ctx, const double* x, double* g) {
    mpc_ctx* m = (mpc_ctx*)ctx;
    ora_mpc_fg(m->p, m->c, x, m->fgbuf);
    memcpy(g, m->fgbuf + 1, sizeof(double) * ora_mpc_ng(m->p->steps));
}
static void cb_jac(void* ctx, const double* x, double* J) {
    mpc_ctx* m = (mpc_ctx*)ctx;
    ora_mpc_jac_g(m->p, m->c, x, J);
}
static void cb_hess(void* ctx, const double* x, double sigma, const double* lam, double* H) {
    mpc_ctx* m = (mpc_ctx*)ctx;
    ora_mpc_hess(m->p, m->c, x, sigma, lam, H);
}

int ora_mpc_solve_res(const ora_mpc_params* p, const ora_ipm_opts* opts, const double* st, const double* coeffs,
                      double* u0, double* traj, double* xfull, ora_ipm_result* res) {
    const int N = p->steps;
    const int nx = ora_mpc_nx(N), ng = ora_mpc_ng(N);
    double* buf = (double*)malloc(sizeof(double) * (size_t)(6 * nx + 3 * ng + 1));
    double *x0 = buf, *xl = x0 + nx, *xu = xl + nx, *x = xu + nx, *zl = x + nx, *zu = zl + nx;
    double *gl = zu + nx, *gu = gl + ng, *fg = gu + ng;
    ora_mpc_bounds(p, st, x0, xl, xu, gl, gu);
    mpc_ctx ctx = {p, coeffs, fg};
    ora_nlp nlp;
    nlp.n = nx;
    nlp.m = ng;
    nlp.ctx = &ctx;
    nlp.f = cb_f;
    nlp.grad_f = cb_grad;
    nlp.g = cb_g;
    nlp.jac_g = cb_jac;
    nlp.hess = cb_hess;
    nlp.xl = xl;
    nlp.xu = xu;
    nlp.gl = gl;
    nlp.gu = gu;
    nlp.x0 = x0;
    /* KKT rows in stage order: stage k's state (6), control (2, k < N-1) and its
     * constraint rows (the initial-state rows at k = 0, the defect into stage k else) --
     * a band of ~2.5 stages (ora_ipm_opts.kkt_structured) */
    int* kord = (int*)malloc(sizeof(int) * (size_t)(nx + ng));
    {
        int q = 0;
        for (int k = 0; k < N; ++k) {
            for (int sv = 0; sv < 6; ++sv) kord[q++] = nx + sv * N + k;  /* c rows into stage k */
            for (int sv = 0; sv < 6; ++sv) kord[q++] = sv * N + k;       /* state s_k */
            if (k < N - 1) {
                kord[q++] = IW(N) + k;
                kord[q++] = IA(N) + k;
            }
        }
    }
    nlp.kkt_order = kord;
    double* lam = (double*)malloc(sizeof(double) * (size_t)ng * 2);
    int status = ora_ipm_solve(&nlp, opts, x, zl, zu, lam, lam + ng, res);
    /* outputs, mpc_planner.cpp:388-401 */
    for (int i = 0; i < N; ++i) {
        traj[i] = x[IX(N) + i];
        traj[N + i] = x[IY(N) + i];
        traj[2 * N + i] = x[ITH(N) + i];
    }
    u0[0] = x[IW(N)];
    u0[1] = x[IA(N)];
    if (xfull) memcpy(xfull, x, sizeof(double) * nx);
    free(kord);
    free(lam);
    free(buf);
    return status;
}

int ora_mpc_solve(const ora_mpc_params* p, const ora_ipm_opts* opts, const double* st, const double* coeffs,
                  double* u0, double* traj, double* obj, int* iters, double* kkt_inf, double* xfull) {
    ora_ipm_result res;
    int status = ora_mpc_solve_res(p, opts, st, coeffs, u0, traj, xfull, &res);
    if (obj) *obj = res.obj;
    if (iters) *iters = res.iters;
    if (kkt_inf) *kkt_inf = res.kkt_inf;
    return status;
}

int ora_mpc_solve_batch_diag(const ora_mpc_params* p, const ora_ipm_opts* opts, int64_t B, const double* state,
                             const double* coeffs, double* u0, double* traj, double* obj, int32_t* status,
                             int32_t* iters, int32_t* diag, int nthreads) {
    const int N = p->steps;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1)
#else
    (void)nthreads;
#endif
    for (int64_t b = 0; b < B; ++b) {
        ora_ipm_result res;
        int st = ora_mpc_solve_res(p, opts, state + 6 * b, coeffs + 4 * b, u0 + 2 * b, traj + (size_t)3 * N * b,
                                   NULL, &res);
        if (obj) obj[b] = res.obj;
        if (status) status[b] = st;
        if (iters) iters[b] = res.iters;
        if (diag) {
            int32_t* d = diag + 7 * b;
            d[0] = res.n_soc;
            d[1] = res.n_watchdog;
            d[2] = res.n_soft_resto;
            d[3] = res.n_resto;
            d[4] = res.resto_iters;
            d[5] = res.n_slack_moves;
            d[6] = (int32_t)floor(log10(fmax(fmin(res.min_slack_margin, 1e300), 1e-300)));
        }
    }
    return 0;
}

int ora_mpc_solve_batch(const ora_mpc_params* p, const ora_ipm_opts* opts, int64_t B, const double* state,
                        const double* coeffs, double* u0, double* traj, double* obj, int32_t* status,
                        int32_t* iters, int nthreads) {
    return ora_mpc_solve_batch_diag(p, opts, B, state, coeffs, u0, traj, obj, status, iters, NULL, nthreads);
}

/* Independent first-order certificate for a primal point x of the NLP: the
 * multipliers are recovered by least squares from stationarity, with bound
 * multipliers taken from the sign of the residual at active bounds.  Used by the
 * tests to certify GPU solutions without trusting any solver's multipliers. */
double ora_mpc_kkt_residual(const ora_mpc_params* p, const double* st, const double* c, const double* x,
                            double* out_dual, double* out_primal, double* out_bound) {
    const int N = p->steps;
    const int nx = ora_mpc_nx(N), ng = ora_mpc_ng(N);
    double* fg = (double*)malloc(sizeof(double) * (ng + 1));
    double* gf = (double*)malloc(sizeof(double) * nx);
    double* J = (double*)malloc(sizeof(double) * (size_t)nx * ng);
    double *x0 = (double*)malloc(sizeof(double) * nx * 3), *xl = x0 + nx, *xu = xl + nx;
    double* gl = (double*)malloc(sizeof(double) * ng * 2);
    double* gu = gl + ng;
    ora_mpc_bounds(p, st, x0, xl, xu, gl, gu);
    ora_mpc_fg(p, c, x, fg);
    ora_mpc_grad_f(p, c, x, gf);
    ora_mpc_jac_g(p, c, x, J);
    double prim = 0.0;
    for (int r = 0; r < ng; ++r) prim = fmax(prim, fabs(fg[1 + r] - gl[r]));
    double bnd = 0.0;
    for (int i = 0; i < nx; ++i) bnd = fmax(bnd, fmax(xl[i] - x[i], x[i] - xu[i]));
    /* J is square in the state block: every variable except the controls has exactly one
     * "defining" row (identity entry).  Solve J_S^T lam = -gf_S on the state columns by
     * back substitution over stages (rows of stage i+1 define stage i+1 variables). */
    double* lam = (double*)calloc(ng, sizeof(double));
    /* order: stage N-1 down to 0; state column s*N+i has +1 in row s*N+i. */
    for (int i = N - 1; i >= 0; --i) {
        for (int s = 5; s >= 0; --s) {
            int col = s * N + i;
            double acc = -gf[col];
            for (int r = 0; r < ng; ++r)
                if (r != col) acc -= J[(size_t)r * nx + col] * lam[r];
            lam[col] = acc; /* J[col][col] == 1 */
        }
    }
    double dual = 0.0;
    for (int j = 6 * N; j < nx; ++j) {
        double rj = gf[j];
        for (int r = 0; r < ng; ++r) rj += J[(size_t)r * nx + j] * lam[r];
        /* rj = zl - zu; at an active lower bound rj >= 0 is allowed, at upper rj <= 0 */
        double tolb = 1e-7 * fmax(1.0, fabs(xu[j]));
        if (x[j] <= xl[j] + tolb && rj > 0) rj = 0.0;
        if (x[j] >= xu[j] - tolb && rj < 0) rj = 0.0;
        dual = fmax(dual, fabs(rj));
    }
    if (out_dual) *out_dual = dual;
    if (out_primal) *out_primal = prim;
    if (out_bound) *out_bound = bnd;
    free(fg); free(gf); free(J); free(x0); free(gl); free(lam);
    return fmax(dual, fmax(prim, fmax(bnd, 0.0)));
}
