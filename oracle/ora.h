/*
 * oracle/ora.h -- CPU ORACLE for the MPC::Solve hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in mpc_ros_amd/ (the product) may include,
 * link or call this code.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py use it, and only as the checker.
 *
 * What it restates (fp64, plain C):
 *   - the reference NLP built by FG_eval   (mpc_ros/src/mpc_planner.cpp:102-217)
 *     with MPC::Solve's start point, variable bounds and constraint bounds
 *     (mpc_ros/src/mpc_planner.cpp:265-348) and its outputs (:388-401);
 *   - the solver the reference calls, Ipopt 3.12.8 (pinned by
 *     assets/document/ipopt_install/ipopt_x86_install_tutorial.md:9; not vendored,
 *     absent from the image) restated from its published algorithm
 *     (Waechter & Biegler, Math. Prog. 106(1):25-57, 2006 -- the paper the
 *     reference's own example cites at assets/document/example/CppAD_Ipopt.cpp:124-126):
 *     primal-dual barrier method, monotone mu update, fraction-to-boundary rule,
 *     filter line search, inertia correction with a Bunch-Kaufman LDL^T;
 *   - the caller-side preprocessing Tracking::findBestPath / polyfit / polyeval
 *     (mpc_ros/src/driving_state.cpp:175-300) and the speed post-processing (:262-269).
 *
 * Pinning: HS071 known answer from assets/document/example/CppAD_Ipopt.cpp:146-150;
 * NLP derivative values cross-checked against the reference's vendored CppAD
 * (oracle/ref_probe, built into oracle/_ref/).  See DESIGN.md "Oracle".
 */
#ifndef MPCG_ORACLE_H
#define MPCG_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------- LDL^T --- */
/* Bunch-Kaufman symmetric indefinite factorisation, lower storage, column-major
 * n x n array a (only the lower triangle is read/written).  ipiv as LAPACK dsytf2.
 * Returns inertia in (npos, nneg, nzero).  tiny: |pivot| <= tiny counts as zero. */
int ora_ldlt_factor(int n, double* a, int* ipiv, double tiny, int* npos, int* nneg, int* nzero);
void ora_ldlt_solve(int n, const double* a, const int* ipiv, double* b);
/* The same factorisation and solve restricted to the matrix envelope (last[n]: the last
 * possibly nonzero row of each column, computed by the factorisation): bitwise the
 * dense results for finite data, O(n b^2) for a banded matrix. */
int ora_ldlt_factor_env(int n, double* a, int* ipiv, double tiny, int* npos, int* nneg, int* nzero, int* last);
void ora_ldlt_solve_env(int n, const double* a, const int* ipiv, const int* last, double* b);

/* ------------------------------------------------------------ generic NLP --- */
/* min f(x) s.t. gl <= g(x) <= gu, xl <= x <= xu.  Dense callbacks.
 * |bound| >= 1e19 means "no bound" (Ipopt nlp_lower/upper_bound_inf).
 * Lagrangian convention (Ipopt/CppAD eval_h): sigma * f + sum_i lambda_i g_i. */
typedef struct ora_nlp {
    int n, m;
    void* ctx;
    double (*f)(void* ctx, const double* x);
    void (*grad_f)(void* ctx, const double* x, double* gf);
    void (*g)(void* ctx, const double* x, double* gv);
    void (*jac_g)(void* ctx, const double* x, double* jac);           /* dense m x n, row-major */
    void (*hess)(void* ctx, const double* x, double sigma, const double* lam,
                 double* h);                                          /* dense n x n, full symmetric */
    const double *xl, *xu, *gl, *gu, *x0;
    /* optional (NULL: none): an order of the n + m KKT rows (variables 0..n-1, then
     * constraint rows n..n+m-1) in which the KKT matrix is banded -- used by
     * ora_ipm_opts.kkt_structured */
    const int* kkt_order;
} ora_nlp;

typedef struct ora_ipm_opts {
    double tol;                 /* Ipopt "tol" (default 1e-8) */
    int max_iter;               /* Ipopt "max_iter" (default 3000) */
    double bound_relax_factor;  /* default 1e-8 */
    int honor_original_bounds;  /* default 1 */
    double mu_init;             /* default 0.1 */
    int print_level;            /* 0 = silent */
    /* ---- Ipopt 3.12 defaults restated in round 2 (0 / negative disables a feature) ---- */
    double acceptable_tol;              /* 1e-6 */
    int acceptable_iter;                /* 15 (0: no acceptable termination) */
    double acceptable_dual_inf_tol;     /* 1e10 */
    double acceptable_constr_viol_tol;  /* 1e-2 */
    double acceptable_compl_inf_tol;    /* 1e-2 */
    double acceptable_obj_change_tol;   /* 1e20 */
    int max_soc;                        /* 4 (second-order corrections) */
    double kappa_soc;                   /* 0.99 */
    int watchdog_shortened_iter_trigger;/* 10 (0: no watchdog) */
    int watchdog_trial_iter_max;        /* 3 */
    double soft_resto_pderror_reduction_factor; /* 0.9999 (0: no soft restoration) */
    int max_soft_resto_iters;           /* 10 */
    int restoration;                    /* 1: feasibility restoration phase; 0: RESTORATION_FAILURE */
    double obj_max_inc;                 /* 5 */
    int max_filter_resets;              /* 5 */
    int filter_reset_trigger;           /* 5 */
    double tiny_step_tol;               /* 10 eps */
    double tiny_step_y_tol;             /* 1e-2 */
    /* the reference's "max_cpu_time 0.5" (mpc_planner.cpp:368) as a deterministic iteration
     * budget: CPUTIME_EXCEEDED (-> solve_result unknown, solve_callback.hpp:1165-1167) once
     * iter > cpu_iter_budget; < 0 = no budget (see ora_cpu_iter_budget) */
    int cpu_iter_budget;
    double dual_inf_tol;                /* 1 */
    double constr_viol_tol;             /* 1e-4 */
    double compl_inf_tol;               /* 1e-4 */
    /* 0 (default, the checker): dense Bunch-Kaufman of the KKT matrix in the NLP's own
     * order.  1: the KKT matrix in the NLP's kkt_order (stage order for the MPC NLP),
     * factored within its envelope (ora_ldlt_factor_env) -- the sparse-solver cost of
     * Ipopt + MUMPS on this band, for the CPU baseline; same algorithm, iterates equal
     * to rounding (a different pivot order) */
    int kkt_structured;
    /* Ipopt's iterative refinement of each KKT solve (PDFullSpaceSolver: min_refinement_steps 1,
     * max_refinement_steps 10, residual_ratio_max 1e-10) on the dense path: 0 (default, the
     * pinned fixtures) = none; k > 0 = at least k steps, more while the residual ratio exceeds
     * 1e-10, at most 10 -- restated in round 4 to measure what omitting it changes */
    int refine_steps;
} ora_ipm_opts;

/* Result; status uses CppAD::ipopt::solve_result::status_type numbering
 * (mpc_ros/include/cppad/ipopt/solve_result.hpp:30-46). */
enum {
    ORA_NOT_DEFINED = 0, ORA_SUCCESS = 1, ORA_MAXITER_EXCEEDED = 2, ORA_STOP_AT_TINY_STEP = 3,
    ORA_STOP_AT_ACCEPTABLE_POINT = 4, ORA_LOCAL_INFEASIBILITY = 5, ORA_USER_REQUESTED_STOP = 6,
    ORA_FEASIBLE_POINT_FOUND = 7, ORA_DIVERGING_ITERATES = 8, ORA_RESTORATION_FAILURE = 9,
    ORA_ERROR_IN_STEP_COMPUTATION = 10, ORA_INVALID_NUMBER_DETECTED = 11,
    ORA_TOO_FEW_DEGREES_OF_FREEDOM = 12, ORA_INTERNAL_ERROR = 13, ORA_UNKNOWN = 14
};

typedef struct ora_ipm_result {
    int status;
    int iters;
    double obj;
    double kkt_inf;             /* final unscaled max(dual inf, primal inf, compl) */
    /* diagnostics: second-order corrections accepted, watchdog activations, soft
     * restoration steps, restoration phases entered, restoration-phase iterations */
    int n_soc, n_watchdog, n_soft_resto, n_resto, resto_iters;
    /* the smallest slack of any point whose barrier was evaluated (original and restoration
     * problem) over eps * min(1, mu), and how many points fell below 1: Ipopt would move
     * those slacks (CalculateSafeSlack / AdjustedTrialSlacks, not restated) */
    double min_slack_margin;
    int n_slack_moves;
    /* x[n], zl[n], zu[n], lambda[m], g[m] written to caller buffers */
} ora_ipm_result;

void ora_ipm_default_opts(ora_ipm_opts* o);
/* Iteration budget equivalent to max_cpu_time seconds of the reference's Solve at horizon
 * N: (max_cpu_time - setup(N)) / per_iter(N), with the CppAD taping and per-iteration
 * derivative costs measured in this container (1.52 ms + 0.225 ms/iter at
 * N = 20, 3.93 ms + 0.467 ms/iter at N = 40, linear in N).  Ipopt's own linear algebra
 * is not included (Ipopt is absent), so the budget errs generous. */
int ora_cpu_iter_budget(double max_cpu_time, int steps);
int ora_ipm_solve(const ora_nlp* nlp, const ora_ipm_opts* opts, double* x, double* zl,
                  double* zu, double* lambda, double* gval, ora_ipm_result* res);

/* ------------------------------------------------------------ MPC NLP --- */
/* The 15 keys of MPC::LoadParams / FG_eval::LoadParams (mpc_planner.cpp:73-85, 247-250). */
typedef struct ora_mpc_params {
    int steps;
    double dt, ref_cte, ref_etheta, ref_v;
    double w_cte, w_etheta, w_v, w_angvel, w_accel, w_angvel_d, w_accel_d;
    double max_angvel, max_throttle, bound;
    /* model 0: differential drive (FG_eval).  model 1: kinematic bicycle (no reference
     * implementation in the fork): the control w is the steering angle
     * delta and the heading rows read th1 - (th0 + v0 delta0 / lf dt),
     * eth1 - (eth0 + v0 delta0 / lf dt) (driving_state.cpp:247's commented
     * theta_act = v * steering * dt / Lf). */
    int model;
    double lf;
} ora_mpc_params;

int ora_mpc_nx(int steps);  /* 6N + 2(N-1) */
int ora_mpc_ng(int steps);  /* 6N */
/* FG_eval::operator() (mpc_planner.cpp:102-217): fg[0] = cost, fg[1..ng] = constraints. */
void ora_mpc_fg(const ora_mpc_params* p, const double* coeffs4, const double* vars, double* fg);
/* Analytic derivatives of the same (dense). */
void ora_mpc_grad_f(const ora_mpc_params* p, const double* coeffs4, const double* vars, double* gf);
void ora_mpc_jac_g(const ora_mpc_params* p, const double* coeffs4, const double* vars, double* jac);
void ora_mpc_hess(const ora_mpc_params* p, const double* coeffs4, const double* vars,
                  double sigma, const double* lam, double* h);
/* MPC::Solve bounds/start (mpc_planner.cpp:281-348). */
void ora_mpc_bounds(const ora_mpc_params* p, const double* state6, double* x0, double* xl,
                    double* xu, double* gl, double* gu);

/* Full MPC::Solve restatement for one problem.
 * out: u0[2] = {omega0, a0}; traj[3N] = mpc_x | mpc_y | mpc_theta; xfull[nx] optional.
 * Returns status (solve_result numbering). */
int ora_mpc_solve(const ora_mpc_params* p, const ora_ipm_opts* opts, const double* state6,
                  const double* coeffs4, double* u0, double* traj, double* obj, int* iters,
                  double* kkt_inf, double* xfull);

/* ora_mpc_solve with the solver's diagnostics (ora_ipm_result) */
int ora_mpc_solve_res(const ora_mpc_params* p, const ora_ipm_opts* opts, const double* state6,
                      const double* coeffs4, double* u0, double* traj, double* xfull, ora_ipm_result* res);
/* Batched, with per-problem diagnostics diag[B][5] = n_soc, n_watchdog, n_soft_resto,
 * n_resto, resto_iters (may be NULL). */
int ora_mpc_solve_batch_diag(const ora_mpc_params* p, const ora_ipm_opts* opts, int64_t B,
                             const double* state, const double* coeffs, double* u0, double* traj,
                             double* obj, int32_t* status, int32_t* iters, int32_t* diag, int nthreads);

/* Batched convenience (OpenMP over problems when built with -fopenmp). */
int ora_mpc_solve_batch(const ora_mpc_params* p, const ora_ipm_opts* opts, int64_t B,
                        const double* state, const double* coeffs, double* u0, double* traj,
                        double* obj, int32_t* status, int32_t* iters, int nthreads);

/* KKT residual of the NLP at (x, lambda, zl, zu) -- used to certify candidate solutions
 * independently of how they were computed.  Returns max of the four residual norms. */
double ora_mpc_kkt_residual(const ora_mpc_params* p, const double* state6, const double* coeffs4,
                            const double* x, double* out_dual, double* out_primal,
                            double* out_bound);

/* ------------------------------------------------------------ HS071 --- */
/* assets/document/example/CppAD_Ipopt.cpp:61-83 with start/bounds :97-112. */
int ora_hs071_solve(const ora_ipm_opts* opts, double* x4, double* zl4, double* zu4, int* iters);

/* ------------------------------------------------------ preprocessing --- */
/* Tracking::findBestPath (driving_state.cpp:175-271) for one problem.
 * px,py,yaw: robot pose; v: feedback speed; w, throttle: previous command;
 * dt: control period; plan: M waypoints (x,y interleaved); delay_mode.
 * Out: state6, coeffs4.  Returns 0 ok, -1 for an empty plan. */
int ora_find_best_path(double px, double py, double yaw, double v, double w, double throttle,
                       double dt, int M, const double* plan_xy, int delay_mode, double* state6,
                       double* coeffs4);
/* polyfit (driving_state.cpp:283-300): Householder QR least squares, order <= 8. */
int ora_polyfit(int M, const double* xs, const double* ys, int order, double* coeffs);

#ifdef __cplusplus
}
#endif
#endif
