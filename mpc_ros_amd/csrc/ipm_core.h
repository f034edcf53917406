// mpc_ros_amd/csrc/ipm_core.h -- per-problem structured interior-point solver (one problem per lane).
//
// This is the solve that replaces CppAD::ipopt::solve inside MPC::Solve
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
// Everything the oracle (oracle/ipm.c) does, this does in the same order with the
// same constants; tests/ compare the two iterate for iterate.
#ifndef MPCG_IPM_CORE_H
#define MPCG_IPM_CORE_H

#include <math.h>
#include <stdint.h>

#if defined(__HIPCC__)
#define MPCG_HD __host__ __device__ __forceinline__
#else
#define MPCG_HD inline
#endif
// MPCG_NOINLINE_PASSES keeps the four sweeps of an iteration as separate device
// functions (no spills, but the call overhead measured slower: 606K vs 794K solves/s),
// so the default inlines them.
#if defined(__HIPCC__) && defined(MPCG_NOINLINE_PASSES)
#define MPCG_PASS __host__ __device__ __attribute__((noinline))
#elif defined(__HIPCC__)
#define MPCG_PASS MPCG_HD
#else
#define MPCG_PASS inline
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
    int filter_cap;             // filter entries kept per problem
    int model;                  // 0 differential drive (FG_eval), 1 kinematic bicycle (wide solver only)
    double lf;                  // model 1: wheelbase [m]
};

// Status numbering of CppAD::ipopt::solve_result::status_type
// (mpc_ros/include/cppad/ipopt/solve_result.hpp:30-46).
enum : int32_t {
    IPM_SUCCESS = 1,
    IPM_MAXITER = 2,
    IPM_RESTORATION_FAILURE = 9,
    IPM_ERROR_IN_STEP = 10,
    IPM_INVALID_NUMBER = 11,
};

// Workspace layout of one problem, in elements (doubles).  Everything is stage-major:
// stage k's primal block is [x y th v cte eth | w a] (8 elements), likewise its bound
// multipliers, step, multipliers (6 rows + 2 pad) and Riccati record (80).  The device
// accessor stores element pairs (2j, 2j+1) of one problem contiguously and pairs of
// consecutive problems next to each other, so a lane moves 16 B per instruction and
// a wavefront 1 KB of contiguous memory.
struct IpmLayout {
    int N;
    static constexpr int RS = 80;  // Riccati record: K[16] kff[2] P[36] p[8] A[7]+pad d[6] (+pad)
    static constexpr int RK = 0, RKFF = 16, RP = 18, Rp = 54, RA = 62, RD = 70;
    MPCG_HD int W(int k, int j) const { return 8 * k + j; }
    MPCG_HD int ZL(int k, int j) const { return 8 * N + 8 * k + j; }
    MPCG_HD int ZU(int k, int j) const { return 16 * N + 8 * k + j; }
    MPCG_HD int DW(int k, int j) const { return 24 * N + 8 * k + j; }
    MPCG_HD int Y(int k, int j) const { return 32 * N + 8 * k + j; }
    MPCG_HD int YP(int k, int j) const { return 40 * N + 8 * k + j; }
    MPCG_HD int REC(int k, int j) const { return 48 * N + RS * k + j; }
    MPCG_HD int FI(int j) const { return 128 * N + j; }
    // per-problem scalar state between the phase kernels (SC_* below), after the filter
    int cap;
    MPCG_HD int SC(int j) const { return 128 * N + 2 * cap + 2 + j; }
    MPCG_HD int total(int cap_) const { return 128 * N + 2 * cap_ + 2 + 32; }
};

// Scalar state of one problem, stored in its workspace between phase kernels.
enum : int {
    SC_SF = 0,          // objective scale
    SC_RA = 1,          // 6 row scales of the dynamics rows into stage 1
    SC_RB = 7,          // 6 row scales of the dynamics rows into stages >= 2
    SC_MU = 13, SC_TAU = 14, SC_THMAX = 15, SC_THMIN = 16, SC_DWLAST = 17,
    SC_ACCA = 18, SC_ACCZ = 19,                       // accepted step, applied by the next stats sweep
    SC_AMAXP = 20, SC_AMAXZ = 21, SC_GD = 22, SC_REL = 23,  // direction statistics
    SC_FVAL = 24, SC_LOGSUM = 25, SC_THETA = 26,      // objective, barrier log-sum, violation at the iterate
    SC_ITER = 27, SC_NFILTER = 28, SC_STATUS = 29,    // status 0 = still iterating
    SC_KKT = 30, SC_LSOK = 31,
};

template <typename T>
struct IpmProblem {
    T init[6];  // x, y, theta, v, cte, etheta (MPC::Solve state argument)
    T c[4];     // reference polynomial coefficients
};

struct IpmResult {
    int32_t status;
    int32_t iters;
    double obj;
    double kkt_inf;
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

template <typename T>
MPCG_HD void sc_t(T a, T* s, T* c) {
    if (__builtin_expect(fabs(a) < 823549.6, 1))
        sincos_small(a, s, c);
    else
        sincos_large(a, s, c);  // out of line: never reached by a bounded trajectory
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

// Sum of logs accumulated as mantissa * 2^exponent: one log per pass.
template <typename T>
struct LogAcc {
    T m;
    int e;
    MPCG_HD void init() { m = 1; e = 0; }
    MPCG_HD void mul(T v) {
        int ex;
        m = frexp(m * v, &ex);
        e += ex;
    }
    MPCG_HD T value() const { return log(m) + (T)e * (T)0.69314718055994530942; }
};

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

MPCG_HD constexpr int pidx(int i, int j) { return i >= j ? i * (i + 1) / 2 + j : j * (j + 1) / 2 + i; }


// One stage's iterate as loaded from the workspace.
template <typename T>
struct StageIt {
    T w[8], dw[8], zl[8], zu[8], y[6], yp[6];
};

template <typename T, class WS>
struct IpmSolver {
    // held by value: a reference member would force the kernel-argument structs into
    // private (scratch) memory and turn every workspace access into a flat access
    const IpmParams P;
    const IpmProblem<T> pr;
    WS ws;
    IpmLayout L;
    int N;
    T dt;
    T sl, su, wl, wu, al, au;        // relaxed bounds: states, angvel, accel
    T sl0, su0, wl0, wu0, al0, au0;  // original bounds
    T sf;                            // objective scale
    // row scales of the dynamics rows into stage 1 (a*) and into stages >= 2 (b*), as scalars:
    // an array member selected by stage would become a dynamic address and keep the
    // whole solver object out of registers
    T ra0, ra1, ra2, ra3, ra4, ra5, rb0, rb1, rb2, rb3, rb4, rb5;
    T mu, tau;
    // statistics of the current iterate
    T fval, logsum, theta, prim_inf, prim_uns, dual_inf, compl0, pmin, pmax, l1y, l1z;
    int nfilter;

    MPCG_HD IpmSolver(const IpmParams& P_, const IpmProblem<T>& pr_, const WS& ws_)
        : P(P_), pr(pr_), ws(ws_), L{P_.N, P_.filter_cap}, N(P_.N), dt((T)P_.dt) {}

    // -------------------------------------------------------- memory helpers
    MPCG_HD void ld8(int e, T* v) const {
#pragma unroll
        for (int j = 0; j < 8; j += 2) ws.ld2(e + j, v[j], v[j + 1]);
    }
    MPCG_HD void ld6(int e, T* v) const {
#pragma unroll
        for (int j = 0; j < 6; j += 2) ws.ld2(e + j, v[j], v[j + 1]);
    }
    MPCG_HD void st8(int e, const T* v) const {
#pragma unroll
        for (int j = 0; j < 8; j += 2) ws.st2(e + j, v[j], v[j + 1]);
    }
    MPCG_HD void st6(int e, const T* v) const {
#pragma unroll
        for (int j = 0; j < 6; j += 2) ws.st2(e + j, v[j], v[j + 1]);
    }
    MPCG_HD void load_stage(int k, StageIt<T>& S, bool with_dir) const {
        ld8(L.W(k, 0), S.w);
        ld8(L.ZL(k, 0), S.zl);
        ld8(L.ZU(k, 0), S.zu);
        ld6(L.Y(k, 0), S.y);
        if (with_dir) {
            ld8(L.DW(k, 0), S.dw);
            ld6(L.YP(k, 0), S.yp);
        }
    }

    MPCG_HD T rowscale(int s, int k) const {
        T a, b;
        switch (s) {
            case 0: a = ra0; b = rb0; break;
            case 1: a = ra1; b = rb1; break;
            case 2: a = ra2; b = rb2; break;
            case 3: a = ra3; b = rb3; break;
            case 4: a = ra4; b = rb4; break;
            default: a = ra5; b = rb5; break;
        }
        return k == 0 ? (T)1 : (k == 1 ? a : b);
    }
    MPCG_HD T vlo(int j) const { return j < 6 ? sl : (j == 6 ? wl : al); }
    MPCG_HD T vhi(int j) const { return j < 6 ? su : (j == 6 ? wu : au); }

    // objective pieces (unscaled) -- FG_eval cost, mpc_planner.cpp:122-147
    MPCG_HD T cost_state(const T* s) const {
        const T e1 = s[4] - (T)P.ref_cte, e2 = s[5] - (T)P.ref_eth, e3 = s[3] - (T)P.ref_v;
        return (T)P.w_cte * e1 * e1 + (T)P.w_eth * e2 * e2 + (T)P.w_v * e3 * e3;
    }
    MPCG_HD void grad_state(const T* s, T* g) const {
        g[0] = 0; g[1] = 0; g[2] = 0;
        g[3] = (T)(2.0 * P.w_v) * (s[3] - (T)P.ref_v);
        g[4] = (T)(2.0 * P.w_cte) * (s[4] - (T)P.ref_cte);
        g[5] = (T)(2.0 * P.w_eth) * (s[5] - (T)P.ref_eth);
    }
    MPCG_HD T hess_state(int j) const {
        return j == 3 ? (T)(2.0 * P.w_v) : (j == 4 ? (T)(2.0 * P.w_cte) : (j == 5 ? (T)(2.0 * P.w_eth) : (T)0));
    }
    // gradient w.r.t. u_k given u_{k-1} (used if k>=1) and u_{k+1} (used if k<=N-3)
    MPCG_HD void grad_ctrl(int k, const T* um, const T* u, const T* up, T* g) const {
        g[0] = (T)(2.0 * P.w_w) * u[0];
        g[1] = (T)(2.0 * P.w_a) * u[1];
        if (k >= 1) {
            g[0] += (T)(2.0 * P.w_dw) * (u[0] - um[0]);
            g[1] += (T)(2.0 * P.w_da) * (u[1] - um[1]);
        }
        if (k <= N - 3) {
            g[0] -= (T)(2.0 * P.w_dw) * (up[0] - u[0]);
            g[1] -= (T)(2.0 * P.w_da) * (up[1] - u[1]);
        }
    }
    MPCG_HD T hess_ctrl(int k, int j) const {
        const double wd = j == 0 ? P.w_dw : P.w_da;
        const double w = j == 0 ? P.w_w : P.w_a;
        return (T)(2.0 * w + 2.0 * wd * ((k >= 1 ? 1 : 0) + (k <= N - 3 ? 1 : 0)));
    }
    MPCG_HD T cost_ctrl(int k, const T* u, const T* up) const {
        T f = (T)P.w_w * u[0] * u[0] + (T)P.w_a * u[1] * u[1];
        if (k <= N - 3)
            f += (T)P.w_dw * (up[0] - u[0]) * (up[0] - u[0]) + (T)P.w_da * (up[1] - u[1]) * (up[1] - u[1]);
        return f;
    }

    // ------------------------------------------------------------------ setup
    // Bounds of MPC::Solve (mpc_planner.cpp:303-325) relaxed as Ipopt does;
    // gradient-based scaling at the user's starting point; starting point pushed
    // inside the box; bound multipliers 1; least-squares equality multipliers.
    MPCG_HD void rowscales_at(const T* s, T* rs) const {
        Lin<T> ln;
        ln.eval(pr.c, s);
        T m[6];
        m[0] = tmax((T)1, tmax((T)fabs(s[3] * ln.st * dt), (T)fabs(ln.ct * dt)));
        m[1] = tmax((T)1, tmax((T)fabs(s[3] * ln.ct * dt), (T)fabs(ln.st * dt)));
        m[2] = tmax((T)1, dt);
        m[3] = tmax((T)1, dt);
        m[4] = tmax(tmax((T)1, (T)fabs(ln.f1)), tmax((T)fabs(ln.se * dt), (T)fabs(s[3] * ln.ce * dt)));
        m[5] = tmax((T)1, dt);
#pragma unroll
        for (int j = 0; j < 6; ++j) rs[j] = m[j] > (T)100 ? (T)100 / m[j] : (T)1;
    }

    MPCG_HD void setup() {
        const T rl = (T)fmin(1e-4, P.bound_relax_factor * fmax(1.0, P.bound));
        sl0 = (T)-P.bound; su0 = (T)P.bound; sl = sl0 - rl; su = su0 + rl;
        const T rw = (T)fmin(1e-4, P.bound_relax_factor * fmax(1.0, P.max_w));
        wl0 = (T)-P.max_w; wu0 = (T)P.max_w; wl = wl0 - rw; wu = wu0 + rw;
        const T ra = (T)fmin(1e-4, P.bound_relax_factor * fmax(1.0, P.max_a));
        al0 = (T)-P.max_a; au0 = (T)P.max_a; al = al0 - ra; au = au0 + ra;
        // objective scale from grad f at the user start (zeros except s_0)
        T g[6];
        grad_state(pr.init, g);
        T gm = tmax((T)fabs(g[3]), tmax((T)fabs(g[4]), (T)fabs(g[5])));
        if (N >= 2) {
            const T z[6] = {0, 0, 0, 0, 0, 0};
            grad_state(z, g);
            gm = tmax(gm, tmax((T)fabs(g[3]), tmax((T)fabs(g[4]), (T)fabs(g[5]))));
        }
        sf = gm > (T)100 ? (T)100 / gm : (T)1;
        T r[6];
        rowscales_at(pr.init, r);
        ra0 = r[0]; ra1 = r[1]; ra2 = r[2]; ra3 = r[3]; ra4 = r[4]; ra5 = r[5];
        const T z6[6] = {0, 0, 0, 0, 0, 0};
        rowscales_at(z6, r);
        rb0 = r[0]; rb1 = r[1]; rb2 = r[2]; rb3 = r[3]; rb4 = r[4]; rb5 = r[5];
    }

    MPCG_HD T push(T v, T lo, T hi) const {
        const T pl = tmin((T)0.01 * tmax((T)1, (T)fabs(lo)), (T)0.01 * (hi - lo));
        const T pu = tmin((T)0.01 * tmax((T)1, (T)fabs(hi)), (T)0.01 * (hi - lo));
        if (v < lo + pl) v = lo + pl;
        if (v > hi - pu) v = hi - pu;
        return v;
    }

    MPCG_HD void init_point() {
        const T one[8] = {1, 1, 1, 1, 1, 1, 1, 1};
        for (int k = 0; k < N; ++k) {
            T w[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) w[j] = push((j < 6 && k == 0) ? pr.init[j] : (T)0, vlo(j), vhi(j));
            st8(L.W(k, 0), w);
            st8(L.ZL(k, 0), one);
            st8(L.ZU(k, 0), one);
        }
    }

    // ------------------------------------------------ accept + statistics
    // One forward sweep.  If `acc`, first applies the previous line-search step to
    // stage k (primal w += alpha dw, z step with the fraction-to-boundary alpha_z
    // and the kappa_sigma safeguard, y += alpha (y+ - y)), then accumulates the
    // statistics of the new iterate: objective, barrier log-sum, constraint
    // violation (l1 and max), dual infeasibility, complementarity extrema and norms.
    // Stage k+1 is loaded one step ahead so its loads overlap stage k's work.
    MPCG_HD void accept_one(T w, T dwv, T zl, T zu, T lo, T hi, T alpha, T amax_z, T* wn, T* zln, T* zun) const {
        const T ksig = (T)1e10, iksig = (T)1e-10;
        const T rdl = rcp(w - lo), rdu = rcp(hi - w);
        const T dzl = mu * rdl - zl - zl * rdl * dwv;
        const T dzu = mu * rdu - zu + zu * rdu * dwv;
        *wn = w + alpha * dwv;
        const T rs2 = rcp(*wn - lo), ru2 = rcp(hi - *wn);
        const T a = zl + amax_z * dzl, b = zu + amax_z * dzu;
        *zln = tmax(tmin(a, ksig * mu * rs2), mu * rs2 * iksig);
        *zun = tmax(tmin(b, ksig * mu * ru2), mu * ru2 * iksig);
    }

    MPCG_PASS void stats(bool acc, T alpha, T amax_z) {
        fval = 0; theta = 0; prim_inf = 0; prim_uns = 0; dual_inf = 0; compl0 = 0;
        pmin = (T)INFINITY; pmax = -(T)INFINITY; l1y = 0; l1z = 0;
        LogAcc<T> la;
        la.init();
        StageIt<T> cur, nxt;
        load_stage(0, cur, acc);
        T Fprev[6] = {0, 0, 0, 0, 0, 0};
        T um[2] = {0, 0};
        for (int k = 0; k < N; ++k) {
            const bool last = (k == N - 1);
            if (!last) load_stage(k + 1, nxt, acc);  // prefetch, ahead of this stage's stores
            // new iterate of stage k
            T w[8], zl[8], zu[8], y[6];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                if (acc && !(last && j >= 6)) {
                    accept_one(cur.w[j], cur.dw[j], cur.zl[j], cur.zu[j], vlo(j), vhi(j), alpha, amax_z, &w[j], &zl[j],
                               &zu[j]);
                } else {
                    w[j] = cur.w[j]; zl[j] = cur.zl[j]; zu[j] = cur.zu[j];
                }
            }
#pragma unroll
            for (int j = 0; j < 6; ++j) y[j] = acc ? cur.y[j] + alpha * (cur.yp[j] - cur.y[j]) : cur.y[j];
            if (acc) {
                st8(L.W(k, 0), w);
                st8(L.ZL(k, 0), zl);
                st8(L.ZU(k, 0), zu);
                st6(L.Y(k, 0), y);
            }
            // new u_{k+1} and y_{k+1} (same formulas as at step k+1)
            T up[2] = {0, 0}, yn[6] = {0, 0, 0, 0, 0, 0};
            if (!last) {
                up[0] = acc ? nxt.w[6] + alpha * nxt.dw[6] : nxt.w[6];
                up[1] = acc ? nxt.w[7] + alpha * nxt.dw[7] : nxt.w[7];
#pragma unroll
                for (int j = 0; j < 6; ++j) yn[j] = acc ? nxt.y[j] + alpha * (nxt.yp[j] - nxt.y[j]) : nxt.y[j];
            }
            // residual rows (., k)
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                const T c = k == 0 ? w[j] - pr.init[j] : w[j] - Fprev[j];
                const T rsc = rowscale(j, k);
                const T cs = rsc * c;
                theta += fabs(cs);
                prim_inf = tmax(prim_inf, (T)fabs(cs));
                prim_uns = tmax(prim_uns, (T)fabs(c));
                l1y += fabs(y[j]) * rcp(rsc);
            }
            fval += cost_state(w);
            T g[6], at[6] = {0, 0, 0, 0, 0, 0};
            grad_state(w, g);
            if (!last) {
                Lin<T> ln;
                ln.eval(pr.c, w);
                T a[7];
                ln.jac(w, dt, a);
                ln.next(w, w + 6, dt, Fprev);
                AT_mul(a, yn, at);
            }
            T gu[2] = {0, 0};
            if (!last) {
                grad_ctrl(k, um, w + 6, up, gu);
                fval += cost_ctrl(k, w + 6, up);
            }
            const T btw = dt * (yn[2] + yn[5]), bta = dt * yn[3];
            const int nv = last ? 6 : 8;
            T slackprod = 1;  // product of the stage's 16 slacks, inside double range for any iterate
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                if (j < nv) {
                    const T gj = j < 6 ? sf * g[j] + y[j] - at[j] : sf * gu[j - 6] - (j == 6 ? btw : bta);
                    const T rd = gj - zl[j] + zu[j];
                    dual_inf = tmax(dual_inf, (T)fabs(rd));
                    const T dl = w[j] - vlo(j), du = vhi(j) - w[j];
                    slackprod *= dl * du;
                    const T p1 = dl * zl[j], p2 = du * zu[j];
                    compl0 = tmax(compl0, tmax((T)fabs(p1), (T)fabs(p2)));
                    pmin = tmin(pmin, tmin(p1, p2));
                    pmax = tmax(pmax, tmax(p1, p2));
                    l1z += fabs(zl[j]) + fabs(zu[j]);
                }
            }
            la.mul(slackprod);
            um[0] = w[6]; um[1] = w[7];
            cur = nxt;
        }
        logsum = la.value();
    }

    // ------------------------------------------------------- Riccati backward
    // mode 0: Newton system of the barrier problem (Hessian of the Lagrangian + Sigma + delta_w I)
    // mode 1: least-squares multiplier system (identity Hessian, zero constraint residual)
    // Returns false when a stage's reduced control Hessian is not positive definite.
    MPCG_PASS bool riccati(int mode, T delta_w) {
        T Pm[36], pv[8];
        // prefetched stage data: W[k], ZL[k], ZU[k] and Y[k+1]
        T cw[8], czl[8], czu[8], cy[6];
        T nw_[8], nzl[8], nzu[8], ny[6];
        ld8(L.W(N - 1, 0), cw);
        ld8(L.ZL(N - 1, 0), czl);
        ld8(L.ZU(N - 1, 0), czu);
        if (N >= 2) {
            ld8(L.W(N - 2, 0), nw_);
            ld8(L.ZL(N - 2, 0), nzl);
            ld8(L.ZU(N - 2, 0), nzu);
            ld6(L.Y(N - 1, 0), ny);
        }
        // terminal stage
        {
            T g[6];
            grad_state(cw, g);
#pragma unroll
            for (int i = 0; i < 36; ++i) Pm[i] = 0;
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                if (mode == 0) {
                    const T rdl = rcp(cw[j] - sl), rdu = rcp(su - cw[j]);
                    Pm[pidx(j, j)] = sf * hess_state(j) + czl[j] * rdl + czu[j] * rdu + delta_w;
                    pv[j] = sf * g[j] - mu * rdl + mu * rdu;
                } else {
                    Pm[pidx(j, j)] = 1;
                    pv[j] = sf * g[j] - czl[j] + czu[j];
                }
            }
            pv[6] = 0; pv[7] = 0;
#pragma unroll
            for (int i = 0; i < 36; i += 2) ws.st2(L.REC(N - 1, IpmLayout::RP + i), Pm[i], Pm[i + 1]);
#pragma unroll
            for (int i = 0; i < 8; i += 2) ws.st2(L.REC(N - 1, IpmLayout::Rp + i), pv[i], pv[i + 1]);
        }
        T snext[6];
#pragma unroll
        for (int j = 0; j < 6; ++j) snext[j] = cw[j];
        T unext[2] = {0, 0};
        for (int k = N - 2; k >= 0; --k) {
            // rotate the prefetch buffers: stage k becomes current
#pragma unroll
            for (int j = 0; j < 8; ++j) { cw[j] = nw_[j]; czl[j] = nzl[j]; czu[j] = nzu[j]; }
#pragma unroll
            for (int j = 0; j < 6; ++j) cy[j] = ny[j];
            if (k >= 1) {  // prefetch stage k-1 before this stage's stores
                ld8(L.W(k - 1, 0), nw_);
                ld8(L.ZL(k - 1, 0), nzl);
                ld8(L.ZU(k - 1, 0), nzu);
                ld6(L.Y(k, 0), ny);
            }
            const T* s = cw;
            const T u[2] = {cw[6], cw[7]};
            const T um[2] = {k >= 1 ? nw_[6] : (T)0, k >= 1 ? nw_[7] : (T)0};
            Lin<T> ln;
            ln.eval(pr.c, s);
            T a[7];
            ln.jac(s, dt, a);
            T Fk[6];
            ln.next(s, u, dt, Fk);
            T d[6];
#pragma unroll
            for (int j = 0; j < 6; ++j) d[j] = (mode == 0) ? Fk[j] - snext[j] : (T)0;
            // stage Hessian Q (6x6, packed), R diag, coupling C, gradients q, r
            T Q[21];
#pragma unroll
            for (int i = 0; i < 21; ++i) Q[i] = 0;
            T q[6], r[2], R0, R1, C0 = 0, C1 = 0;
            T g[6];
            grad_state(s, g);
            T gu[2];
            grad_ctrl(k, um, u, unext, gu);
            if (mode == 0) {
#pragma unroll
                for (int j = 0; j < 6; ++j) {
                    const T rdl = rcp(s[j] - sl), rdu = rcp(su - s[j]);
                    Q[pidx(j, j)] = sf * hess_state(j) + czl[j] * rdl + czu[j] * rdu + delta_w;
                    q[j] = sf * g[j] - mu * rdl + mu * rdu;
                }
                // constraint curvature, weighted by the row-form multipliers of rows k+1
                const T v = s[3];
                Q[pidx(2, 2)] += cy[0] * v * ln.ct * dt + cy[1] * v * ln.st * dt;
                Q[pidx(3, 2)] += cy[0] * ln.st * dt - cy[1] * ln.ct * dt;
                Q[pidx(0, 0)] += -cy[4] * ln.f2;
                Q[pidx(5, 5)] += cy[4] * v * ln.se * dt;
                Q[pidx(5, 3)] += -cy[4] * ln.ce * dt;
                T Rr[2];
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const T rdl = rcp(u[j] - vlo(6 + j)), rdu = rcp(vhi(6 + j) - u[j]);
                    Rr[j] = sf * hess_ctrl(k, j) + czl[6 + j] * rdl + czu[6 + j] * rdu + delta_w;
                    r[j] = sf * gu[j] - mu * rdl + mu * rdu;
                }
                R0 = Rr[0]; R1 = Rr[1];
                if (k >= 1) {
                    C0 = -sf * (T)(2.0 * P.w_dw);
                    C1 = -sf * (T)(2.0 * P.w_da);
                }
            } else {
#pragma unroll
                for (int j = 0; j < 6; ++j) {
                    Q[pidx(j, j)] = 1;
                    q[j] = sf * g[j] - czl[j] + czu[j];
                }
                R0 = 1; R1 = 1;
#pragma unroll
                for (int j = 0; j < 2; ++j) r[j] = sf * gu[j] - czl[6 + j] + czu[6 + j];
            }
            // PA = P' A_hat : nonzero columns 0,1,2,3,5 (rows 0..7); PB = P' B_hat; h = P' d_hat + p'
            T PA[8][5], PB[8][2], h[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const T p0 = Pm[pidx(i, 0)], p1 = Pm[pidx(i, 1)], p2 = Pm[pidx(i, 2)];
                const T p3 = Pm[pidx(i, 3)], p4 = Pm[pidx(i, 4)], p5 = Pm[pidx(i, 5)];
                PA[i][0] = p0 + a[4] * p4;
                PA[i][1] = p1 - p4;
                PA[i][2] = a[0] * p0 + a[2] * p1 + p2;
                PA[i][3] = a[1] * p0 + a[3] * p1 + p3 + a[5] * p4;
                PA[i][4] = a[6] * p4 + p5;  // column 5 (eth)
                // B_hat: w -> dt e2 + dt e5 + e6 ; a -> dt e3 + e7
                PB[i][0] = dt * (p2 + p5) + Pm[pidx(i, 6)];
                PB[i][1] = dt * p3 + Pm[pidx(i, 7)];
                h[i] = pv[i] + p0 * d[0] + p1 * d[1] + p2 * d[2] + p3 * d[3] + p4 * d[4] + p5 * d[5];
            }
            const T Rt00 = R0 + dt * (PB[2][0] + PB[5][0]) + PB[6][0];
            const T Rt01 = dt * (PB[2][1] + PB[5][1]) + PB[6][1];
            const T Rt11 = R1 + dt * PB[3][1] + PB[7][1];
            const T det = Rt00 * Rt11 - Rt01 * Rt01;
            if (!(Rt00 > 0) || !(det > (T)1e-14 * Rt00 * Rt11)) return false;
            // S_tilde (2 x 8): columns 0,1,2,3,5 from B^T P A ; 6,7 the rate coupling ; 4 zero
            T St[2][8];
#pragma unroll
            for (int c = 0; c < 5; ++c) {
                const int col = c < 4 ? c : 5;
                St[0][col] = dt * (PA[2][c] + PA[5][c]) + PA[6][c];
                St[1][col] = dt * PA[3][c] + PA[7][c];
            }
            St[0][4] = 0; St[1][4] = 0;
            St[0][6] = C0; St[0][7] = 0;
            St[1][6] = 0;  St[1][7] = C1;
            const T rt0 = r[0] + dt * (h[2] + h[5]) + h[6];
            const T rt1 = r[1] + dt * h[3] + h[7];
            const T rdet = rcp(det);
            const T i00 = Rt11 * rdet, i01 = -Rt01 * rdet, i11 = Rt00 * rdet;
            T K[2][8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                K[0][j] = -(i00 * St[0][j] + i01 * St[1][j]);
                K[1][j] = -(i01 * St[0][j] + i11 * St[1][j]);
            }
            const T kf0 = -(i00 * rt0 + i01 * rt1);
            const T kf1 = -(i01 * rt0 + i11 * rt1);
            // P_new = Q_hat + A^T (P A) + St^T K, entry by entry into the (now dead) P registers
#pragma unroll
            for (int i = 0; i < 8; ++i) {
#pragma unroll
                for (int j = 0; j <= i; ++j) {
                    T atpa = 0;
                    if (j < 4 || j == 5) {
                        const int c = j < 4 ? j : 4;
                        switch (i) {
                            case 0: atpa = PA[0][c] + a[4] * PA[4][c]; break;
                            case 1: atpa = PA[1][c] - PA[4][c]; break;
                            case 2: atpa = a[0] * PA[0][c] + a[2] * PA[1][c] + PA[2][c]; break;
                            case 3: atpa = a[1] * PA[0][c] + a[3] * PA[1][c] + PA[3][c] + a[5] * PA[4][c]; break;
                            case 5: atpa = a[6] * PA[4][c] + PA[5][c]; break;
                            default: atpa = 0;
                        }
                    }
                    const T qv = (i < 6 && j < 6) ? Q[pidx(i, j)] : (T)0;
                    Pm[pidx(i, j)] = qv + atpa + St[0][i] * K[0][j] + St[1][i] * K[1][j];
                }
            }
            T At_h[6];
            AT_mul(a, h, At_h);
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const T base = (i < 6) ? q[i] + At_h[i] : (T)0;
                pv[i] = base + St[0][i] * kf0 + St[1][i] * kf1;
            }
            // record of stage k (pair stores)
#pragma unroll
            for (int j = 0; j < 8; j += 2) {
                ws.st2(L.REC(k, IpmLayout::RK + j), K[0][j], K[0][j + 1]);
                ws.st2(L.REC(k, IpmLayout::RK + 8 + j), K[1][j], K[1][j + 1]);
            }
            ws.st2(L.REC(k, IpmLayout::RKFF), kf0, kf1);
#pragma unroll
            for (int i = 0; i < 36; i += 2) ws.st2(L.REC(k, IpmLayout::RP + i), Pm[i], Pm[i + 1]);
#pragma unroll
            for (int i = 0; i < 8; i += 2) ws.st2(L.REC(k, IpmLayout::Rp + i), pv[i], pv[i + 1]);
            ws.st2(L.REC(k, IpmLayout::RA + 0), a[0], a[1]);
            ws.st2(L.REC(k, IpmLayout::RA + 2), a[2], a[3]);
            ws.st2(L.REC(k, IpmLayout::RA + 4), a[4], a[5]);
            ws.st2(L.REC(k, IpmLayout::RA + 6), a[6], (T)0);
#pragma unroll
            for (int i = 0; i < 6; i += 2) ws.st2(L.REC(k, IpmLayout::RD + i), d[i], d[i + 1]);
#pragma unroll
            for (int j = 0; j < 6; ++j) snext[j] = cw[j];
            unext[0] = u[0]; unext[1] = u[1];
        }
        return true;
    }

    // -------------------------------------------------------- forward pass
    // Step (DW) and new multipliers (YP) from the Riccati records; also the
    // fraction-to-the-boundary step sizes, grad(phi)^T dw and the tiny-step measure.
    struct Fwd {
        T amax_p, amax_z, gd, rel;
    };

    // branchless: every candidate ratio is computed with one reciprocal and selected
    MPCG_HD void dir_var(T w, T zl, T zu, T lo, T hi, T gphi, T dwv, Fwd& F) const {
        const T dl = w - lo, du = hi - w;
        const T rdl = rcp(dl), rdu = rcp(du), rdw = rcp(dwv);
        const T inf = (T)INFINITY;
        F.amax_p = tmin(F.amax_p, dwv < 0 ? -tau * dl * rdw : (dwv > 0 ? tau * du * rdw : inf));
        const T dzl = mu * rdl - zl - zl * rdl * dwv;
        const T dzu = mu * rdu - zu + zu * rdu * dwv;
        F.amax_z = tmin(F.amax_z, dzl < 0 ? -tau * zl * rcp(dzl) : inf);
        F.amax_z = tmin(F.amax_z, dzu < 0 ? -tau * zu * rcp(dzu) : inf);
        F.gd += gphi * dwv;
        F.rel = tmax(F.rel, (T)fabs(dwv) * rcp((T)1 + (T)fabs(w)));
    }

    MPCG_PASS Fwd forward(int mode) {
        Fwd F{(T)1, (T)1, (T)0, (T)0};
        T ds[8];
        T cw[8], czl[8], czu[8], nw_[8], nzl[8], nzu[8];
        ld8(L.W(0, 0), cw);
        if (mode == 0) {
            ld8(L.ZL(0, 0), czl);
            ld8(L.ZU(0, 0), czu);
        }
#pragma unroll
        for (int j = 0; j < 6; ++j) ds[j] = (mode == 0) ? -(cw[j] - pr.init[j]) : (T)0;
        ds[6] = 0; ds[7] = 0;
        T um[2] = {0, 0};
        for (int k = 0; k < N; ++k) {
            const bool last = (k == N - 1);
            T Pm[36], pv[8];
#pragma unroll
            for (int i = 0; i < 36; i += 2) ws.ld2(L.REC(k, IpmLayout::RP + i), Pm[i], Pm[i + 1]);
#pragma unroll
            for (int i = 0; i < 8; i += 2) ws.ld2(L.REC(k, IpmLayout::Rp + i), pv[i], pv[i + 1]);
            T K[16], kf[2], a[8], d[6];
            if (!last) {
#pragma unroll
                for (int i = 0; i < 16; i += 2) ws.ld2(L.REC(k, IpmLayout::RK + i), K[i], K[i + 1]);
                ws.ld2(L.REC(k, IpmLayout::RKFF), kf[0], kf[1]);
#pragma unroll
                for (int i = 0; i < 8; i += 2) ws.ld2(L.REC(k, IpmLayout::RA + i), a[i], a[i + 1]);
#pragma unroll
                for (int i = 0; i < 6; i += 2) ws.ld2(L.REC(k, IpmLayout::RD + i), d[i], d[i + 1]);
                ld8(L.W(k + 1, 0), nw_);  // prefetch next stage
                if (mode == 0) {
                    ld8(L.ZL(k + 1, 0), nzl);
                    ld8(L.ZU(k + 1, 0), nzu);
                }
            }
            // multipliers of rows (., k): yh+ = -(P ds + p)[0:6]
            T yp[6];
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                T acc = pv[j];
#pragma unroll
                for (int m = 0; m < 8; ++m) acc += Pm[pidx(j, m)] * ds[m];
                yp[j] = -acc;
            }
            st6(L.YP(k, 0), yp);
            T dk[8];
#pragma unroll
            for (int j = 0; j < 6; ++j) dk[j] = ds[j];
            dk[6] = 0; dk[7] = 0;
            if (!last) {
                T du0 = kf[0], du1 = kf[1];
#pragma unroll
                for (int m = 0; m < 8; ++m) {
                    du0 += K[m] * ds[m];
                    du1 += K[8 + m] * ds[m];
                }
                dk[6] = du0; dk[7] = du1;
            }
            st8(L.DW(k, 0), dk);
            if (mode == 0) {
                T g[6];
                grad_state(cw, g);
                T gu[2] = {0, 0};
                if (!last) {
                    const T up[2] = {nw_[6], nw_[7]};
                    grad_ctrl(k, um, cw + 6, up, gu);
                }
                const int nv = last ? 6 : 8;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    if (j < nv) {
                        const T gj = j < 6 ? sf * g[j] : sf * gu[j - 6];
                        const T gphi = gj - mu * rcp(cw[j] - vlo(j)) + mu * rcp(vhi(j) - cw[j]);
                        dir_var(cw[j], czl[j], czu[j], vlo(j), vhi(j), gphi, dk[j], F);
                    }
                }
            }
            if (last) break;
            T nx6[6];
            A_mul(a, ds, nx6);
            nx6[2] += dt * dk[6];
            nx6[3] += dt * dk[7];
            nx6[5] += dt * dk[6];
#pragma unroll
            for (int j = 0; j < 6; ++j) ds[j] = nx6[j] + d[j];
            ds[6] = dk[6];
            ds[7] = dk[7];
            um[0] = cw[6]; um[1] = cw[7];
#pragma unroll
            for (int j = 0; j < 8; ++j) { cw[j] = nw_[j]; czl[j] = nzl[j]; czu[j] = nzu[j]; }
        }
        return F;
    }

    // ------------------------------------------------------------ trial point
    // phi_mu and theta at w + alpha dw; returns false if outside the relaxed box.
    MPCG_PASS bool trial(T alpha, T* phi, T* th) const {
        LogAcc<T> la;
        la.init();
        T f = 0, thv = 0;
        T Fprev[6] = {0, 0, 0, 0, 0, 0};
        bool ok = true;
        T cw[8], cd[8], nw_[8], nd[8];
        ld8(L.W(0, 0), cw);
        ld8(L.DW(0, 0), cd);
        for (int k = 0; k < N; ++k) {
            const bool last = (k == N - 1);
            if (!last) {
                ld8(L.W(k + 1, 0), nw_);
                ld8(L.DW(k + 1, 0), nd);
            }
            T w[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) w[j] = cw[j] + alpha * cd[j];
            const int nv = last ? 6 : 8;
            T slackprod = 1;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                if (j < nv) {
                    const T dl = w[j] - vlo(j), du = vhi(j) - w[j];
                    ok = ok && (dl > 0) && (du > 0);
                    slackprod *= dl * du;
                }
            }
            la.mul(slackprod);
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                const T c = k == 0 ? w[j] - pr.init[j] : w[j] - Fprev[j];
                thv += fabs(rowscale(j, k) * c);
            }
            f += cost_state(w);
            if (last) break;
            T up[2];
            up[0] = nw_[6] + alpha * nd[6];
            up[1] = nw_[7] + alpha * nd[7];
            f += cost_ctrl(k, w + 6, up);
            Lin<T> ln;
            ln.eval(pr.c, w);
            ln.next(w, w + 6, dt, Fprev);
#pragma unroll
            for (int j = 0; j < 8; ++j) { cw[j] = nw_[j]; cd[j] = nd[j]; }
        }
        *phi = sf * f - mu * la.value();
        *th = thv;
        return ok && isfinite((double)*phi);
    }

    // ------------------------------------------------------------ phases
    // The IPM is run as a sequence of phases, each a separate kernel on the device
    // (mpcg_kernels.hip) so that each gets its own register allocation; between
    // phases a problem's scalar state lives in its workspace (SC_*).
    //   init0 -> newton(1) -> direction(1) -> init1 -> { begin -> newton(0) ->
    //   direction(0) -> linesearch }* -> outputs
    // The same sequence run in a loop on one problem is exactly solve() below.
    MPCG_HD T sc(int j) const { return ws.ld(L.SC(j)); }
    MPCG_HD void set_sc(int j, T v) const { ws.st(L.SC(j), v); }
    MPCG_HD int status() const { return (int)sc(SC_STATUS); }
    MPCG_HD void load_scales() {
        sf = sc(SC_SF);
        ra0 = sc(SC_RA + 0); ra1 = sc(SC_RA + 1); ra2 = sc(SC_RA + 2);
        ra3 = sc(SC_RA + 3); ra4 = sc(SC_RA + 4); ra5 = sc(SC_RA + 5);
        rb0 = sc(SC_RB + 0); rb1 = sc(SC_RB + 1); rb2 = sc(SC_RB + 2);
        rb3 = sc(SC_RB + 3); rb4 = sc(SC_RB + 4); rb5 = sc(SC_RB + 5);
    }
    MPCG_HD void bounds_only() {
        const T rl = (T)fmin(1e-4, P.bound_relax_factor * fmax(1.0, P.bound));
        sl0 = (T)-P.bound; su0 = (T)P.bound; sl = sl0 - rl; su = su0 + rl;
        const T rw = (T)fmin(1e-4, P.bound_relax_factor * fmax(1.0, P.max_w));
        wl0 = (T)-P.max_w; wu0 = (T)P.max_w; wl = wl0 - rw; wu = wu0 + rw;
        const T ra = (T)fmin(1e-4, P.bound_relax_factor * fmax(1.0, P.max_a));
        al0 = (T)-P.max_a; au0 = (T)P.max_a; al = al0 - ra; au = au0 + ra;
    }
    // common prologue of every phase after init0
    MPCG_HD void restore() {
        bounds_only();
        load_scales();
        mu = sc(SC_MU);
        tau = sc(SC_TAU);
    }

    // init0: bounds, scaling, starting point, bound multipliers.
    MPCG_HD void phase_init0() {
        setup();
        init_point();
        set_sc(SC_SF, sf);
        set_sc(SC_RA + 0, ra0); set_sc(SC_RA + 1, ra1); set_sc(SC_RA + 2, ra2);
        set_sc(SC_RA + 3, ra3); set_sc(SC_RA + 4, ra4); set_sc(SC_RA + 5, ra5);
        set_sc(SC_RB + 0, rb0); set_sc(SC_RB + 1, rb1); set_sc(SC_RB + 2, rb2);
        set_sc(SC_RB + 3, rb3); set_sc(SC_RB + 4, rb4); set_sc(SC_RB + 5, rb5);
        set_sc(SC_MU, (T)P.mu_init);
        set_sc(SC_TAU, tmax((T)0.99, (T)1 - (T)P.mu_init));
        set_sc(SC_STATUS, 0);
    }

    // init1: least-squares multipliers (constr_mult_init_max 1000) from the mode-1
    // Newton/direction phases, then the statistics of the starting point.
    MPCG_HD void phase_init1() {
        restore();
        const bool ok = sc(SC_LSOK) != 0;
        T ymax = 0;
        if (ok) {
            for (int k = 0; k < N; ++k) {
                T yp[6];
                ld6(L.YP(k, 0), yp);
#pragma unroll
                for (int j = 0; j < 6; ++j) ymax = tmax(ymax, (T)fabs(yp[j] * rcp(rowscale(j, k))));
            }
        }
        const bool use = ok && ymax <= (T)1000;
        for (int k = 0; k < N; ++k) {
            T yp[6];
            ld6(L.YP(k, 0), yp);
#pragma unroll
            for (int j = 0; j < 6; ++j) yp[j] = use ? yp[j] : (T)0;
            st6(L.Y(k, 0), yp);
        }
        stats(false, (T)0, (T)0);
        set_sc(SC_THMAX, (T)1e4 * tmax((T)1, theta));
        set_sc(SC_THMIN, (T)1e-4 * tmax((T)1, theta));
        set_sc(SC_DWLAST, 0);
        set_sc(SC_ACCA, 0);
        set_sc(SC_ACCZ, 0);
        set_sc(SC_ITER, 0);
        set_sc(SC_NFILTER, 0);
        set_sc(SC_KKT, 0);
    }

    // begin: apply the accepted step of the previous iteration, statistics,
    // termination tests, monotone barrier update.  Returns the new status
    // (0 = keep iterating).
    MPCG_HD int phase_begin() {
        restore();
        const int iter = (int)sc(SC_ITER);
        stats(iter > 0, sc(SC_ACCA), sc(SC_ACCZ));
        const int nbnd = 2 * (8 * N - 2);
        const int ng = 6 * N;
        const T sd = tmax((T)100, (l1y + l1z) / (T)(ng + nbnd)) / (T)100;
        const T scc = tmax((T)100, l1z / (T)nbnd) / (T)100;
        const T E0 = tmax(dual_inf / sd, tmax(prim_inf, compl0 / scc));
        const T dual_uns = dual_inf / sf;
        set_sc(SC_KKT, tmax(dual_uns, tmax(prim_uns, compl0)));
        int st = 0;
        // Ipopt's invalid-number test on f and g at the iterate (the max-norms above
        // drop a NaN; the sums do not)
        if (!isfinite((double)E0) || !isfinite((double)theta) || !isfinite((double)fval))
            st = IPM_INVALID_NUMBER;
        else if (E0 <= (T)P.tol && dual_uns <= (T)1 && prim_uns <= (T)1e-4 && compl0 <= (T)1e-4)
            st = IPM_SUCCESS;
        else if (iter == P.max_iter)
            st = IPM_MAXITER;
        if (st) {
            set_sc(SC_STATUS, st);
            return st;
        }
        const T kappa_eps = 10, kappa_mu = (T)0.2, theta_mu = (T)1.5;
        const T mu_min = (T)(P.tol / 10.0);
        int nf = (int)sc(SC_NFILTER);
        for (;;) {
            const T complmu = tmax(pmax - mu, mu - pmin);
            const T Emu = tmax(dual_inf / sd, tmax(prim_inf, complmu / scc));
            if (Emu > kappa_eps * mu || mu <= mu_min) break;
            const T mnew = tmax(mu_min, tmin(kappa_mu * mu, (T)pow((double)mu, (double)theta_mu)));
            if (mnew >= mu) break;
            mu = mnew;
            tau = tmax((T)0.99, (T)1 - mu);
            nf = 0;
        }
        set_sc(SC_MU, mu);
        set_sc(SC_TAU, tau);
        set_sc(SC_NFILTER, (T)nf);
        set_sc(SC_FVAL, fval);
        set_sc(SC_LOGSUM, logsum);
        set_sc(SC_THETA, theta);
        return 0;
    }

    // newton: mode 0 = Newton step of the barrier problem with Ipopt's inertia
    // correction (delta_w schedule); mode 1 = least-squares multiplier system.
    MPCG_HD int phase_newton(int mode) {
        restore();
        if (mode == 1) {
            set_sc(SC_LSOK, riccati(1, (T)0) ? (T)1 : (T)0);
            return 0;
        }
        T delta_w_last = sc(SC_DWLAST);
        T delta_w = 0;
        int attempt = 0;
        bool ok = false;
        for (;;) {
            if (riccati(0, delta_w)) {
                ok = true;
                if (delta_w > 0) delta_w_last = delta_w;
                break;
            }
            if (attempt == 0)
                delta_w = (delta_w_last == 0) ? (T)1e-4 : tmax((T)1e-20, delta_w_last / (T)3);
            else
                delta_w = (delta_w_last == 0) ? (T)100 * delta_w : (T)8 * delta_w;
            ++attempt;
            if (delta_w > (T)1e40) break;
        }
        set_sc(SC_DWLAST, delta_w_last);
        if (!ok) {
            set_sc(SC_STATUS, IPM_ERROR_IN_STEP);
            return IPM_ERROR_IN_STEP;
        }
        return 0;
    }

    // direction: step, new multipliers, fraction-to-the-boundary statistics.
    MPCG_HD void phase_direction(int mode) {
        restore();
        const Fwd F = forward(mode);
        if (mode == 0) {
            set_sc(SC_AMAXP, F.amax_p);
            set_sc(SC_AMAXZ, F.amax_z);
            set_sc(SC_GD, F.gd);
            set_sc(SC_REL, F.rel);
        }
    }

    // linesearch: Ipopt's filter line search; records the accepted step for the
    // next begin phase.  Returns the new status (0 = keep iterating).
    MPCG_HD int phase_linesearch() {
        restore();
        const T gamma_theta = (T)1e-5, gamma_phi = (T)1e-8, delta_sw = 1, gamma_alpha = (T)0.05;
        const T s_theta = (T)1.1, s_phi = (T)2.3, eta_phi = (T)1e-8;
        const T theta_max = sc(SC_THMAX), theta_min = sc(SC_THMIN);
        const T phik = sf * sc(SC_FVAL) - mu * sc(SC_LOGSUM);
        const T thetak = sc(SC_THETA);
        const T gd = sc(SC_GD);
        int nf = (int)sc(SC_NFILTER);
        const int cap = P.filter_cap;
        T alpha_min;
        if (gd < 0 && thetak <= theta_min)
            alpha_min = gamma_alpha * tmin(gamma_theta, tmin(-gamma_phi * thetak / gd,
                                                             delta_sw * (T)pow((double)thetak, (double)s_theta) /
                                                                 (T)pow((double)-gd, (double)s_phi)));
        else if (gd < 0)
            alpha_min = gamma_alpha * tmin(gamma_theta, -gamma_phi * thetak / gd);
        else
            alpha_min = gamma_alpha * gamma_theta;
        const bool tiny = sc(SC_REL) < (T)(10.0 * 2.2e-16);
        T alpha = sc(SC_AMAXP);
        bool accepted = false, ftype = false;
        for (int ls = 0; ls < 60; ++ls) {
            if (tiny) { accepted = true; ftype = true; break; }
            if (alpha < alpha_min) break;
            T phit, thetat;
            const bool okt = trial(alpha, &phit, &thetat);
            if (okt && thetat < theta_max) {
                bool infilt = false;
                for (int f = 0; f < nf; ++f) {
                    const T fth = ws.ld(L.FI(2 * f)), fph = ws.ld(L.FI(2 * f + 1));
                    if (thetat >= fth && phit >= fph) { infilt = true; break; }
                }
                if (!infilt) {
                    // (the powers are evaluated only where the switching condition is read)
                    const bool sw = (thetak <= theta_min) && (gd < 0) &&
                                    (alpha * (T)pow((double)-gd, (double)s_phi) >
                                     delta_sw * (T)pow((double)thetak, (double)s_theta));
                    if (sw) {
                        if (phit <= phik + eta_phi * alpha * gd) { accepted = true; ftype = true; break; }
                    } else if (thetat <= ((T)1 - gamma_theta) * thetak || phit <= phik - gamma_phi * thetak) {
                        accepted = true;
                        ftype = false;
                        break;
                    }
                }
            }
            alpha *= (T)0.5;
        }
        if (!accepted) {
            set_sc(SC_STATUS, IPM_RESTORATION_FAILURE);
            return IPM_RESTORATION_FAILURE;
        }
        if (!ftype) {
            int slot = nf;
            if (nf == cap) {  // full: drop the oldest entry
                for (int f = 1; f < cap; ++f) {
                    ws.st(L.FI(2 * (f - 1)), ws.ld(L.FI(2 * f)));
                    ws.st(L.FI(2 * (f - 1) + 1), ws.ld(L.FI(2 * f + 1)));
                }
                slot = cap - 1;
            } else {
                ++nf;
            }
            ws.st(L.FI(2 * slot), ((T)1 - gamma_theta) * thetak);
            ws.st(L.FI(2 * slot + 1), phik - gamma_phi * thetak);
        }
        set_sc(SC_NFILTER, (T)nf);
        set_sc(SC_ACCA, alpha);  // applied by the next begin phase
        set_sc(SC_ACCZ, sc(SC_AMAXZ));
        set_sc(SC_ITER, sc(SC_ITER) + 1);
        return 0;
    }

    // The whole solve of one problem: the phases in sequence.  Between phases the
    // state is re-read from the workspace; the compiler barrier stops the compiler
    // from forwarding values across phases, so each phase is register-allocated on
    // its own (fused, their live ranges exceed the 512-register file).
    MPCG_HD static void phase_fence() {
#if defined(__HIP_DEVICE_COMPILE__)
        asm volatile("" ::: "memory");
#endif
    }
    MPCG_HD IpmResult solve() {
        phase_init0();
        phase_fence();
        phase_newton(1);
        phase_fence();
        phase_direction(1);
        phase_fence();
        phase_init1();
        for (;;) {
            phase_fence();
            if (phase_begin()) break;
            phase_fence();
            if (phase_newton(0)) break;
            phase_fence();
            phase_direction(0);
            phase_fence();
            if (phase_linesearch()) break;
        }
        phase_fence();
        restore();
        return result();
    }

    MPCG_HD IpmResult result() const {
        IpmResult r;
        r.status = (int32_t)sc(SC_STATUS);
        r.iters = (int32_t)sc(SC_ITER);
        r.obj = 0.0;
        r.kkt_inf = (double)sc(SC_KKT);
        return r;
    }

    // Final point with honor_original_bounds projection; objective at that point.
    MPCG_HD T x_state(int j, int k) const { return tmin(tmax((T)ws.ld(L.W(k, j)), sl0), su0); }
    MPCG_HD T x_ctrl(int j, int k) const {
        const T v = ws.ld(L.W(k, 6 + j));
        return j == 0 ? tmin(tmax(v, wl0), wu0) : tmin(tmax(v, al0), au0);
    }
    MPCG_HD T objective_out() const {
        T f = 0;
        for (int k = 0; k < N; ++k) {
            T s[6];
#pragma unroll
            for (int j = 0; j < 6; ++j) s[j] = x_state(j, k);
            f += cost_state(s);
        }
        for (int k = 0; k < N - 1; ++k) {
            const T u[2] = {x_ctrl(0, k), x_ctrl(1, k)};
            T up[2] = {0, 0};
            if (k <= N - 3) { up[0] = x_ctrl(0, k + 1); up[1] = x_ctrl(1, k + 1); }
            f += cost_ctrl(k, u, up);
        }
        return f;
    }
};

}  // namespace mpcg
#endif
