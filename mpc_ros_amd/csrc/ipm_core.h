// mpc_ros_amd/csrc/ipm_core.h -- parameters, statuses and math kernels shared by the
// wavefront solver (wide_core.h) and its host emulation.
//
// The solver (wide_core.h) is the solve that replaces CppAD::ipopt::solve inside MPC::Solve
// (mpc_ros/src/mpc_planner.cpp:373-375).  It runs Ipopt 3.12.8's algorithm --
// primal-dual barrier method with monotone mu, fraction-to-the-boundary, filter
// line search and inertia correction (Waechter & Biegler 2006; the reference's
// options, mpc_planner.cpp:356-368, leave every algorithmic option at its default) --
// on the reference NLP in its reference variable layout, so that its iterates
// follow the reference solver's path and land in the same local minimum of this
// nonconvex problem.  What differs is the linear algebra: instead of a sparse
// LDL^T (MUMPS) of the (nx+ng)-dim KKT matrix, every Newton system is solved by
// a stage-wise Riccati recursion on its block-tridiagonal structure, and Ipopt's
// inertia test (n positive, m negative eigenvalues) is replaced by the equivalent
// test that every stage's reduced control Hessian is positive definite.
//
// Notation: stage k has state s_k = (x, y, th, v, cte, eth) (k < N) and control
// u_k = (w, a) (k < N-1).  Constraint rows: c_0 = s_0 - state_init and
// c_{k+1} = s_{k+1} - F(s_k, u_k) (FG_eval, mpc_planner.cpp:153-216).  Rate
// penalties couple u_{k-1} and u_k, so the Riccati state is augmented with u_{k-1}
// (8 states, 2 controls).  Multipliers are kept in "row form" yh_r = c_scale_r * y_r
// (Ipopt's scaled multiplier times the row scale), so the Lagrangian Hessian
// sum_r yh_r grad^2 c_r is independent of the scaling.
//
// Everything the oracle (oracle/ipm.c) does, the solver does in the same order with the
// same constants; tests/ compare the two iterate for iterate.  (Round 1 also had a
// one-problem-per-lane solver here; it was removed in round 2 when the solver gained
// Ipopt's second-order corrections, watchdog and soft restoration.)
#ifndef MPCG_IPM_CORE_H
#define MPCG_IPM_CORE_H

#include <math.h>
#include <stdint.h>

#if defined(__HIPCC__)
#define MPCG_HD __host__ __device__ __forceinline__
#define MPCG_NOINLINE __host__ __device__ __attribute__((noinline))
#else
#define MPCG_HD inline
#define MPCG_NOINLINE __attribute__((noinline))
#endif
namespace mpcg {

struct IpmParams {
    int N;
    double dt, ref_cte, ref_eth, ref_v;
    double w_cte, w_eth, w_v, w_w, w_a, w_dw, w_da;
    double max_w, max_a, bound;
    double tol;                 // Ipopt tol (default 1e-8)
    double bound_relax_factor;  // Ipopt default 1e-8
    double mu_init;             // Ipopt default 0.1
    int max_iter;               // Ipopt default 3000
    int filter_cap;             // filter entries kept per problem (non-dominated entries; oldest dropped beyond)
    int model;                  // 0 differential drive (FG_eval), 1 kinematic bicycle
    double lf;                  // model 1: wheelbase [m]
    // Ipopt 3.12 options the reference leaves at their defaults (oracle/ipm.c header)
    double acceptable_tol;              // 1e-6
    int acceptable_iter;                // 15 (0 = off)
    double acceptable_dual_inf_tol;     // 1e10
    double acceptable_constr_viol_tol;  // 1e-2
    double acceptable_compl_inf_tol;    // 1e-2
    double acceptable_obj_change_tol;   // 1e20
    int max_soc;                        // 4 (0 = no second-order corrections)
    double kappa_soc;                   // 0.99
    int watchdog_trigger;               // watchdog_shortened_iter_trigger 10 (0 = off)
    int watchdog_trial_max;             // watchdog_trial_iter_max 3
    double soft_resto_factor;           // soft_resto_pderror_reduction_factor 0.9999 (0 = off)
    int max_soft_resto_iters;           // 10
    double obj_max_inc;                 // 5
    int max_filter_resets;              // 5
    int filter_reset_trigger;           // 5
    double tiny_step_tol;               // 10 eps
    double tiny_step_y_tol;             // 1e-2
    double dual_inf_tol;                // 1
    double constr_viol_tol;             // 1e-4
    double compl_inf_tol;               // 1e-4
    int cpu_iter_budget;                // max_cpu_time as iterations (-1 = none): status UNKNOWN beyond
    int precision;                      // 0: fp64 (Ipopt's); 1: fp32 solver (differential drive)
    int no_resto;                       // 1: RESTORATION_FAILURE where the restoration phase would start
    int park_cap;                       // park-area entries (0: max(256, B / 128); host side only)
};

// The Ipopt 3.12 options the reference leaves at their defaults (mpc_planner.cpp:356-368:
// only print_level, the derivative mode and max_cpu_time are set), as mpcg_api.cpp's
// ipopt_defaults fills them.  A kernel instance for exactly these values compiles them as
// constants (fewer wave-uniform values held through the solve); launch_wide_solve takes
// it only when every field below equals the handle's option.
MPCG_HD void ipopt_default_options(IpmParams& q) {
    q.no_resto = 0;
    q.tol = 1e-8;
    q.bound_relax_factor = 1e-8;
    q.mu_init = 0.1;
    q.max_iter = 3000;
    q.filter_cap = 64;
    q.acceptable_tol = 1e-6;
    q.acceptable_iter = 15;
    q.acceptable_dual_inf_tol = 1e10;
    q.acceptable_constr_viol_tol = 1e-2;
    q.acceptable_compl_inf_tol = 1e-2;
    q.acceptable_obj_change_tol = 1e20;
    q.max_soc = 4;
    q.kappa_soc = 0.99;
    q.watchdog_trigger = 10;
    q.watchdog_trial_max = 3;
    q.soft_resto_factor = 0.9999;
    q.max_soft_resto_iters = 10;
    q.obj_max_inc = 5.0;
    q.max_filter_resets = 5;
    q.filter_reset_trigger = 5;
    q.tiny_step_tol = 10.0 * 2.220446049250313e-16;
    q.tiny_step_y_tol = 1e-2;
    q.dual_inf_tol = 1.0;
    q.constr_viol_tol = 1e-4;
    q.compl_inf_tol = 1e-4;
}
inline bool ipopt_options_are_default(const IpmParams& p) {
    IpmParams q = p;
    ipopt_default_options(q);
    return p.tol == q.tol && p.bound_relax_factor == q.bound_relax_factor && p.mu_init == q.mu_init &&
           p.max_iter == q.max_iter && p.filter_cap == q.filter_cap && p.acceptable_tol == q.acceptable_tol &&
           p.acceptable_iter == q.acceptable_iter && p.acceptable_dual_inf_tol == q.acceptable_dual_inf_tol &&
           p.acceptable_constr_viol_tol == q.acceptable_constr_viol_tol &&
           p.acceptable_compl_inf_tol == q.acceptable_compl_inf_tol &&
           p.acceptable_obj_change_tol == q.acceptable_obj_change_tol && p.max_soc == q.max_soc &&
           p.kappa_soc == q.kappa_soc && p.watchdog_trigger == q.watchdog_trigger &&
           p.watchdog_trial_max == q.watchdog_trial_max && p.soft_resto_factor == q.soft_resto_factor &&
           p.max_soft_resto_iters == q.max_soft_resto_iters && p.obj_max_inc == q.obj_max_inc &&
           p.max_filter_resets == q.max_filter_resets && p.filter_reset_trigger == q.filter_reset_trigger &&
           p.tiny_step_tol == q.tiny_step_tol && p.tiny_step_y_tol == q.tiny_step_y_tol &&
           p.dual_inf_tol == q.dual_inf_tol && p.constr_viol_tol == q.constr_viol_tol &&
           p.compl_inf_tol == q.compl_inf_tol && p.no_resto == q.no_resto;
}

// Status numbering of CppAD::ipopt::solve_result::status_type
// (mpc_ros/include/cppad/ipopt/solve_result.hpp:30-46).
enum : int32_t {
    IPM_SUCCESS = 1,
    IPM_MAXITER = 2,
    IPM_TINY_STEP = 3,
    IPM_ACCEPTABLE = 4,
    IPM_LOCAL_INFEASIBILITY = 5,  // the restoration phase converged to a point that is not feasible
    IPM_FEASIBLE_POINT = 7,       // the restoration phase converged to a feasible point (FEASIBLE_POINT_FOUND)
    IPM_RESTORATION_FAILURE = 9,
    IPM_ERROR_IN_STEP = 10,
    IPM_INVALID_NUMBER = 11,
    IPM_UNKNOWN = 14,  // CPUTIME_EXCEEDED maps here (solve_callback.hpp:1165-1167)
};

template <typename T>
struct IpmProblem {
    T init[6];  // x, y, theta, v, cte, etheta (MPC::Solve state argument)
    T c[4];     // reference polynomial coefficients
};


// sin and cos of one angle.  |a| < 2^19 pi/2 (every angle a bounded trajectory can
// reach): Cody-Waite reduction by pi/2 with a three-part constant and FMA, then the
// fdlibm minimax kernels on [-pi/4, pi/4] (degree 13 / 14) and quadrant selection --
// ~35 instructions, within 1-2 ulp of the correctly rounded values.  Larger
// arguments take the library routine.
// A double constant materialised at its use (two scalar moves) rather than hoisted
// and kept live across the solver's loops, where it would be spilled to scratch.
MPCG_HD double kc(double v) {
#if defined(__HIP_DEVICE_COMPILE__)
    __asm__ volatile("" : "+s"(v));
#endif
    return v;
}

MPCG_HD void sincos_small(double a, double* s, double* c) {
    const double inv_pio2 = kc(6.36619772367581382433e-01);
    const double p1 = kc(1.57079632679489655800e+00), p2 = kc(6.12323399573676603587e-17),
                 p3 = kc(-1.49738490485916983e-33);
    const double n = rint(a * inv_pio2);
    double r = __builtin_fma(-n, p1, a);
    r = __builtin_fma(-n, p2, r);
    r = __builtin_fma(-n, p3, r);
    const double z = r * r;
    const double S1 = kc(-1.66666666666666324348e-01), S2 = kc(8.33333333332248946124e-03),
                 S3 = kc(-1.98412698298579493134e-04), S4 = kc(2.75573137070700676789e-06),
                 S5 = kc(-2.50507602534068634195e-08), S6 = kc(1.58969099521155010221e-10);
    const double C1 = kc(4.16666666666666019037e-02), C2 = kc(-1.38888888888741095749e-03),
                 C3 = kc(2.48015872894767294178e-05), C4 = kc(-2.75573143513906633035e-07),
                 C5 = kc(2.08757232129817482790e-09), C6 = kc(-1.13596475577881948265e-11);
    const double ps = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
    const double sr = __builtin_fma(r * z, __builtin_fma(z, ps, S1), r);
    const double pc = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
    const double hz = 0.5 * z;
    const double w = 1.0 - hz;
    const double cr = w + (((1.0 - w) - hz) + z * pc);
    const int q = (int)((long long)n & 3);
    const double sv = (q & 1) ? cr : sr;
    const double cv = (q & 1) ? sr : cr;
    *s = (q & 2) ? -sv : sv;
    *c = ((q + 1) & 2) ? -cv : cv;
}

#if defined(__HIPCC__)
static __host__ __device__ __attribute__((noinline))
#else
static inline
#endif
void sincos_large(double a, double* s, double* c) {
#if defined(__HIP_DEVICE_COMPILE__)
    sincos(a, s, c);
#else
    *s = sin(a);
    *c = cos(a);
#endif
}

MPCG_HD void sc_t(double a, double* s, double* c) {
    if (__builtin_expect(fabs(a) < 823549.6, 1))
        sincos_small(a, s, c);
    else
        sincos_large(a, s, c);  // out of line: never reached by a bounded trajectory
}
// fp32 solver: the same kernel in double, rounded once
MPCG_HD void sc_t(float a, float* s, float* c) {
    double sd, cd;
    sc_t((double)a, &sd, &cd);
    *s = (float)sd;
    *c = (float)cd;
}

// x^y for finite x > 0 as exp(y log x): fdlibm's log kernel (Lg1..Lg7 on s = f / (2 + f))
// and a degree-13 Taylor exp after Cody-Waite reduction by ln 2 -- ~60 instructions
// against ~250 for the library pow, within ~|y log x| ulp of it.  For the filter line
// search's switching-condition powers (-gd)^s_phi and theta^s_theta, thresholds that
// a few ulp do not move.
MPCG_HD double pow_pos(double x, double y) {
    int e;
    double m = frexp(x, &e);  // x = m 2^e, m in [0.5, 1)
    if (m < 0.70710678118654752440) {
        m = m + m;
        e -= 1;
    }
    const double f = m - 1.0;
    const double s = f / (2.0 + f);
    const double z = s * s, w = z * z;
    const double Lg1 = kc(6.666666666666735130e-01), Lg2 = kc(3.999999999940941908e-01),
                 Lg3 = kc(2.857142874366239149e-01), Lg4 = kc(2.222219843214978396e-01),
                 Lg5 = kc(1.818357216161805012e-01), Lg6 = kc(1.531383769920937332e-01),
                 Lg7 = kc(1.479819860511658591e-01);
    const double t1 = w * (Lg2 + w * (Lg4 + w * Lg6)), t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
    const double R = t2 + t1, hfsq = 0.5 * f * f;
    const double ln2_hi = kc(6.93147180369123816490e-01), ln2_lo = kc(1.90821492927058770002e-10);
    const double de = (double)e;
    const double lg = de * ln2_hi - ((hfsq - (s * (hfsq + R) + de * ln2_lo)) - f);
    const double a = y * lg;
    const double n = rint(a * kc(1.44269504088896338700e+00));
    double r = __builtin_fma(-n, ln2_hi, a);
    r = __builtin_fma(-n, ln2_lo, r);
    double p = kc(1.6059043836821614599e-10);  // 1/13!
    p = __builtin_fma(p, r, kc(2.0876756987868098979e-09));
    p = __builtin_fma(p, r, kc(2.5052108385441718775e-08));
    p = __builtin_fma(p, r, kc(2.7557319223985890653e-07));
    p = __builtin_fma(p, r, kc(2.7557319223985892510e-06));
    p = __builtin_fma(p, r, kc(2.4801587301587301566e-05));
    p = __builtin_fma(p, r, kc(1.9841269841269841253e-04));
    p = __builtin_fma(p, r, kc(1.3888888888888889419e-03));
    p = __builtin_fma(p, r, kc(8.3333333333333332177e-03));
    p = __builtin_fma(p, r, kc(4.1666666666666664354e-02));
    p = __builtin_fma(p, r, kc(1.6666666666666665741e-01));
    p = __builtin_fma(p, r, 0.5);
    p = __builtin_fma(p, r, 1.0);
    p = __builtin_fma(p, r, 1.0);
    return ldexp(p, (int)n);
}

// max / min with C fmax / fmin (IEEE maxNum) semantics, as the oracle: one v_max_f64 /
// v_min_f64 on the device (a compare and two selects otherwise)
template <typename T>
MPCG_HD T tmax(T a, T b) { return fmax(a, b); }
template <typename T>
MPCG_HD T tmin(T a, T b) { return fmin(a, b); }

// Reciprocal: on the device v_rcp_f64 refined by two Newton steps (5 instructions,
// within an ulp of 1/x) instead of the ~10-instruction correctly rounded division;
// every slack of every variable needs one per sweep.
MPCG_HD double rcp(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
    double r = __builtin_amdgcn_rcp(x);
    double e = __builtin_fma(-x, r, 1.0);
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-x, r, 1.0);
    return __builtin_fma(r, e, r);
#else
    return 1.0 / x;
#endif
}
MPCG_HD float rcp(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
    float r = __builtin_amdgcn_rcpf(x);
    return __builtin_fmaf(r, __builtin_fmaf(-x, r, 1.0f), r);
#else
    return 1.0f / x;
#endif
}

// Linearisation of the dynamics of one stage at (s, u).
template <typename T>
struct Lin {
    T st, ct, se, ce;  // sin/cos theta, sin/cos etheta
    T f, f1, f2;       // f(x), f'(x), f''(x)
    MPCG_HD void eval(const T* c, const T* s) {
        sc_t(s[2], &st, &ct);
        sc_t(s[5], &se, &ce);
        const T x = s[0];
        // f(x) = sum_k c_k x^k with CppAD::pow(x,k) = repeated products (pow_int.hpp:115-137)
        f = c[0] + c[1] * x + c[2] * (x * x) + c[3] * (x * x * x);
        f1 = c[1] + (T)2 * c[2] * x + (T)3 * c[3] * x * x;
        f2 = (T)2 * c[2] + (T)6 * c[3] * x;
    }
    // F(s, u)   (mpc_planner.cpp:202-215)
    MPCG_HD void next(const T* s, const T* u, T dt, T* out) const {
        out[0] = s[0] + s[3] * ct * dt;
        out[1] = s[1] + s[3] * st * dt;
        out[2] = s[2] + u[0] * dt;
        out[3] = s[3] + u[1] * dt;
        out[4] = (f - s[1]) + s[3] * se * dt;
        out[5] = s[5] + u[0] * dt;
    }
    // non-trivial entries of A = dF/ds (dF_c/dy = -1 and the unit diagonal are implicit)
    MPCG_HD void jac(const T* s, T dt, T* a) const {
        a[0] = -s[3] * st * dt;  // dx+/dth
        a[1] = ct * dt;          // dx+/dv
        a[2] = s[3] * ct * dt;   // dy+/dth
        a[3] = st * dt;          // dy+/dv
        a[4] = f1;               // dc+/dx
        a[5] = se * dt;          // dc+/dv
        a[6] = s[3] * ce * dt;   // dc+/deth
    }
};

// y = A^T lam (6x6 dynamics Jacobian)
template <typename T>
MPCG_HD void AT_mul(const T* a, const T* lam, T* y) {
    y[0] = lam[0] + a[4] * lam[4];
    y[1] = lam[1] - lam[4];
    y[2] = a[0] * lam[0] + a[2] * lam[1] + lam[2];
    y[3] = a[1] * lam[0] + a[3] * lam[1] + lam[3] + a[5] * lam[4];
    y[4] = 0;
    y[5] = a[6] * lam[4] + lam[5];
}
// y = A x
template <typename T>
MPCG_HD void A_mul(const T* a, const T* x, T* y) {
    y[0] = x[0] + a[0] * x[2] + a[1] * x[3];
    y[1] = x[1] + a[2] * x[2] + a[3] * x[3];
    y[2] = x[2];
    y[3] = x[3];
    y[4] = a[4] * x[0] - x[1] + a[5] * x[3] + a[6] * x[5];
    y[5] = x[5];
}



}  // namespace mpcg
#endif
