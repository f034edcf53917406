// mpc_ros_amd/csrc/ddp_core.h -- per-problem NMPC solver core (one problem per lane).
//
// Replaces the CppAD/Ipopt solve of MPC::Solve (mpc_ros/src/mpc_planner.cpp:265-402)
// for ONE problem; the HIP kernel in mpcg_kernels.hip runs it on every lane of a
// wavefront for a batch of independent robots.
//
// Problem (the NLP of FG_eval, mpc_planner.cpp:102-217) in reduced form.  On every
// dynamically feasible trajectory eth_i - theta_i is constant (both integrate w dt,
// :210/:215) and cte_{i+1} = f(x_i) - y_i + v_i sin(eth_i) dt (:213) is an output
// of stage i, so the NLP is equivalent to an optimal-control problem over
//     s = (x, y, theta, v, w_prev, a_prev),   u = (w, a),
//     s+ = (x + v cos(th) dt, y + v sin(th) dt, th + w dt, v + a dt, w, a),
// stage cost  l_k = W_CTE r_k^2 + W_EPSI (th+ce-REF_ETHETA)^2 + W_V (v-REF_V)^2
//                 + W_ANGVEL w^2 + W_A a^2 + [k>=1](W_DANGVEL (w-w_prev)^2 + W_DA (a-a_prev)^2)
//             r_k = f(x) - y + v sin(th+ce) dt - REF_CTE,  ce = eth_0 - th_0,
// terminal    W_EPSI (th+ce-REF_ETHETA)^2 + W_V (v-REF_V)^2,
// box constraints on u (MPC::Solve :315-325).  The state boxes (+-BOUND, :308-312)
// are checked at the solution and reported through the status.
//
// Method: control-limited differential dynamic programming with exact second-order
// dynamics terms (Newton-equivalent, quadratically convergent), box-QP feedforward
// per stage (exact 2-variable active-set solve), Levenberg-Marquardt regularisation
// and Armijo backtracking on the true objective.  Its fixed points are exactly the
// KKT points of the reference NLP (DESIGN.md "Solver").  Bounds are relaxed by
// Ipopt's bound_relax_factor (1e-8) during the solve and the reported controls are
// projected back (honor_original_bounds), as Ipopt does.
#ifndef MPCG_DDP_CORE_H
#define MPCG_DDP_CORE_H

#include <math.h>
#include <stdint.h>

#if defined(__HIPCC__)
#define MPCG_HD __host__ __device__ __forceinline__
#else
#define MPCG_HD inline
#endif

namespace mpcg {

// Solver constants (values the kernel and the host agree on).
struct SolverParams {
    int N;
    double dt, ref_cte, ref_eth, ref_v;
    double w_cte, w_eth, w_v, w_w, w_a, w_dw, w_da;
    double max_w, max_a, bound;
    double relax;        // Ipopt bound_relax_factor
    double tol;          // feedforward step tolerance (control units)
    int max_iter;
    int max_ls;          // line-search halvings before raising the regularisation
};

// Status numbering of CppAD::ipopt::solve_result::status_type
// (mpc_ros/include/cppad/ipopt/solve_result.hpp:30-46).
enum : int32_t {
    ST_SUCCESS = 1,
    ST_MAXITER = 2,
    ST_ERROR_IN_STEP = 10,
    ST_INVALID_NUMBER = 11,
    ST_UNKNOWN = 14,  // state box +-BOUND active: outside the reduced formulation
};

// Workspace layout per problem (element index e; the kernel maps e -> ws[e*B + p]).
//   traj buffer b (b = 0,1): X[k],Y[k],TH[k],V[k] k<N ; W[k],A[k] k<N-1
//   gains: K[k][2][6], kff[k][2]  k<N-1
struct Layout {
    int N;
    MPCG_HD int traj_sz() const { return 6 * N - 2; }
    MPCG_HD int X(int b, int k) const { return b * traj_sz() + k; }
    MPCG_HD int Y(int b, int k) const { return b * traj_sz() + N + k; }
    MPCG_HD int TH(int b, int k) const { return b * traj_sz() + 2 * N + k; }
    MPCG_HD int V(int b, int k) const { return b * traj_sz() + 3 * N + k; }
    MPCG_HD int W(int b, int k) const { return b * traj_sz() + 4 * N + k; }
    MPCG_HD int A(int b, int k) const { return b * traj_sz() + 5 * N - 1 + k; }
    MPCG_HD int G(int k, int j) const { return 2 * traj_sz() + 14 * k + j; }  // j<12: K row-major, 12,13: kff
    MPCG_HD int total() const { return 2 * traj_sz() + 14 * (N - 1); }
};

template <typename T>
MPCG_HD T clampv(T v, T lo, T hi) { return v < lo ? lo : (v > hi ? hi : v); }

// Accessor: element e of this problem's workspace lives at base[e * stride].
template <typename T>
struct Ws {
    T* base;
    int64_t stride;
    MPCG_HD T& operator[](int e) const { return base[(int64_t)e * stride]; }
};

template <typename T>
struct Problem {
    T x0, y0, th0, v0, cte0, eth0;
    T c0, c1, c2, c3;
    T ce, sce, cce;  // eth_0 - th_0 and its sine/cosine
};

template <typename T>
MPCG_HD void sincos_t(T a, T* s, T* c) {
#if defined(__HIP_DEVICE_COMPILE__)
    sincos(a, s, c);
#else
    *s = sin(a);
    *c = cos(a);
#endif
}

// Stage cost of a rollout step (used by the forward pass); returns cost, writes next state.
template <typename T>
MPCG_HD T stage_cost(const SolverParams& P, const Problem<T>& pr, int k, T x, T y, T th, T v, T wp, T ap, T w,
                     T a, T st, T ct) {
    const T dt = (T)P.dt;
    const T S = st * pr.cce + ct * pr.sce;  // sin(th + ce)
    const T f = pr.c0 + x * (pr.c1 + x * (pr.c2 + x * pr.c3));
    const T r = f - y + v * S * dt - (T)P.ref_cte;
    const T e = th + pr.ce - (T)P.ref_eth;
    const T dv = v - (T)P.ref_v;
    T l = (T)P.w_cte * r * r + (T)P.w_eth * e * e + (T)P.w_v * dv * dv + (T)P.w_w * w * w + (T)P.w_a * a * a;
    if (k >= 1) l += (T)P.w_dw * (w - wp) * (w - wp) + (T)P.w_da * (a - ap) * (a - ap);
    return l;
}

template <typename T>
MPCG_HD T terminal_cost(const SolverParams& P, const Problem<T>& pr, T th, T v) {
    const T e = th + pr.ce - (T)P.ref_eth;
    const T dv = v - (T)P.ref_v;
    return (T)P.w_eth * e * e + (T)P.w_v * dv * dv;
}

// Exact solution of min 0.5 d'Hd + g'd, lo <= d <= hi for 2 variables (H SPD).
// free0/free1: whether each coordinate ends strictly inside its box.
template <typename T>
MPCG_HD void box_qp2(T h00, T h01, T h11, T g0, T g1, T lo0, T hi0, T lo1, T hi1, T* d0, T* d1, bool* free0,
                     bool* free1) {
    const T det = h00 * h11 - h01 * h01;
    T u0 = (h01 * g1 - h11 * g0) / det;
    T u1 = (h01 * g0 - h00 * g1) / det;
    if (u0 >= lo0 && u0 <= hi0 && u1 >= lo1 && u1 <= hi1) {
        *d0 = u0; *d1 = u1; *free0 = true; *free1 = true;
        return;
    }
    // Candidates on the four edges (the minimiser lies on one of them); each is the
    // exact 1-D minimiser along that edge, clamped to it.
    T best = (T)INFINITY, bd0 = 0, bd1 = 0;
    bool bf0 = false, bf1 = false;
    T q;
    // d0 fixed at a bound, d1 free on its edge
    for (int s = 0; s < 2; ++s) {
        const T a0 = s ? hi0 : lo0;
        T raw = -(g1 + h01 * a0) / h11;
        T a1 = clampv(raw, lo1, hi1);
        q = (T)0.5 * (h00 * a0 * a0 + 2 * h01 * a0 * a1 + h11 * a1 * a1) + g0 * a0 + g1 * a1;
        if (q < best) { best = q; bd0 = a0; bd1 = a1; bf0 = false; bf1 = (a1 > lo1 && a1 < hi1); }
    }
    for (int s = 0; s < 2; ++s) {
        const T a1 = s ? hi1 : lo1;
        T raw = -(g0 + h01 * a1) / h00;
        T a0 = clampv(raw, lo0, hi0);
        q = (T)0.5 * (h00 * a0 * a0 + 2 * h01 * a0 * a1 + h11 * a1 * a1) + g0 * a0 + g1 * a1;
        if (q < best) { best = q; bd0 = a0; bd1 = a1; bf1 = false; bf0 = (a0 > lo0 && a0 < hi0); }
    }
    *d0 = bd0; *d1 = bd1; *free0 = bf0; *free1 = bf1;
}

// Symmetric 6x6 stored as packed lower triangle (21 entries): idx(i,j), i>=j.
MPCG_HD int sidx(int i, int j) { return i >= j ? i * (i + 1) / 2 + j : j * (j + 1) / 2 + i; }

template <typename T>
struct Tol;
template <>
struct Tol<double> {
    static constexpr double noise = 1e-12;  // relative cost noise floor
};
template <>
struct Tol<float> {
    static constexpr float noise = 2e-6f;
};

// Initial rollout with all controls zero (Ipopt's start has every control at 0,
// mpc_planner.cpp:288-292).  Writes buffer b, returns the objective.
template <typename T, class WS>
MPCG_HD T init_rollout(const SolverParams& P, const Problem<T>& pr, const Layout& L, WS& ws, int b) {
    const int N = P.N;
    const T dt = (T)P.dt;
    T x = pr.x0, y = pr.y0, th = pr.th0, v = pr.v0;
    const T ec = pr.cte0 - (T)P.ref_cte;
    T J = (T)P.w_cte * ec * ec;
    for (int k = 0; k < N - 1; ++k) {
        ws[L.X(b, k)] = x; ws[L.Y(b, k)] = y; ws[L.TH(b, k)] = th; ws[L.V(b, k)] = v;
        ws[L.W(b, k)] = (T)0; ws[L.A(b, k)] = (T)0;
        T st, ct;
        sincos_t(th, &st, &ct);
        J += stage_cost(P, pr, k, x, y, th, v, (T)0, (T)0, (T)0, (T)0, st, ct);
        x = x + v * ct * dt;
        y = y + v * st * dt;
    }
    ws[L.X(b, N - 1)] = x; ws[L.Y(b, N - 1)] = y; ws[L.TH(b, N - 1)] = th; ws[L.V(b, N - 1)] = v;
    J += terminal_cost(P, pr, th, v);
    return J;
}

// Forward pass: rollout of u = clamp(u_nom + alpha kff + K (s - s_nom)) from buffer
// `cur` into buffer `nxt`.  Returns the objective of the new trajectory.
template <typename T, class WS>
MPCG_HD T forward(const SolverParams& P, const Problem<T>& pr, const Layout& L, WS& ws, int cur, int nxt, T alpha,
                  T lbw, T ubw, T lba, T uba) {
    const int N = P.N;
    const T dt = (T)P.dt;
    T x = pr.x0, y = pr.y0, th = pr.th0, v = pr.v0, wp = 0, ap = 0;
    T wpn = 0, apn = 0;
    const T ec = pr.cte0 - (T)P.ref_cte;
    T J = (T)P.w_cte * ec * ec;
    for (int k = 0; k < N - 1; ++k) {
        const T xn = ws[L.X(cur, k)], yn = ws[L.Y(cur, k)], thn = ws[L.TH(cur, k)], vn = ws[L.V(cur, k)];
        const T wn = ws[L.W(cur, k)], an = ws[L.A(cur, k)];
        const T d0 = x - xn, d1 = y - yn, d2 = th - thn, d3 = v - vn, d4 = wp - wpn, d5 = ap - apn;
        T g[14];
#pragma unroll
        for (int j = 0; j < 14; ++j) g[j] = ws[L.G(k, j)];
        T w = wn + alpha * g[12] + g[0] * d0 + g[1] * d1 + g[2] * d2 + g[3] * d3 + g[4] * d4 + g[5] * d5;
        T a = an + alpha * g[13] + g[6] * d0 + g[7] * d1 + g[8] * d2 + g[9] * d3 + g[10] * d4 + g[11] * d5;
        w = clampv(w, lbw, ubw);
        a = clampv(a, lba, uba);
        ws[L.X(nxt, k)] = x; ws[L.Y(nxt, k)] = y; ws[L.TH(nxt, k)] = th; ws[L.V(nxt, k)] = v;
        ws[L.W(nxt, k)] = w; ws[L.A(nxt, k)] = a;
        T st, ct;
        sincos_t(th, &st, &ct);
        J += stage_cost(P, pr, k, x, y, th, v, wp, ap, w, a, st, ct);
        x = x + v * ct * dt;
        y = y + v * st * dt;
        th = th + w * dt;
        v = v + a * dt;
        wp = w; ap = a; wpn = wn; apn = an;
    }
    ws[L.X(nxt, N - 1)] = x; ws[L.Y(nxt, N - 1)] = y; ws[L.TH(nxt, N - 1)] = th; ws[L.V(nxt, N - 1)] = v;
    J += terminal_cost(P, pr, th, v);
    return J;
}

// Backward pass over the nominal trajectory in buffer `cur`: stage-wise quadratic
// model with exact Hessians (incl. the dynamics curvature weighted by the costate),
// box-QP feedforward, feedback gains on the free controls, value update.
// Returns false when a regularised control Hessian is not positive definite.
template <typename T, class WS>
MPCG_HD bool backward(const SolverParams& P, const Problem<T>& pr, const Layout& L, WS& ws, int cur, T rho,
                      T lbw, T ubw, T lba, T uba, T* dV1, T* dV2, T* kmax) {
    const int N = P.N;
    const T dt = (T)P.dt;
    const T Wc2 = (T)(2.0 * P.w_cte), We2 = (T)(2.0 * P.w_eth), Wv2 = (T)(2.0 * P.w_v);
    const T Ww2 = (T)(2.0 * P.w_w), Wa2 = (T)(2.0 * P.w_a);
    T Vs[6], Vss[21];
    {
        const T th = ws[L.TH(cur, N - 1)], v = ws[L.V(cur, N - 1)];
#pragma unroll
        for (int i = 0; i < 21; ++i) Vss[i] = 0;
        Vs[0] = 0; Vs[1] = 0; Vs[4] = 0; Vs[5] = 0;
        Vs[2] = We2 * (th + pr.ce - (T)P.ref_eth);
        Vs[3] = Wv2 * (v - (T)P.ref_v);
        Vss[sidx(2, 2)] = We2;
        Vss[sidx(3, 3)] = Wv2;
    }
    T s1 = 0, s2 = 0, km = 0;
    for (int k = N - 2; k >= 0; --k) {
        const T x = ws[L.X(cur, k)], y = ws[L.Y(cur, k)], th = ws[L.TH(cur, k)], v = ws[L.V(cur, k)];
        const T w = ws[L.W(cur, k)], a = ws[L.A(cur, k)];
        const bool rate = (k >= 1);
        const T wp = rate ? ws[L.W(cur, k - 1)] : (T)0;
        const T ap = rate ? ws[L.A(cur, k - 1)] : (T)0;
        const T Wdw2 = rate ? (T)(2.0 * P.w_dw) : (T)0;
        const T Wda2 = rate ? (T)(2.0 * P.w_da) : (T)0;
        T st, ct;
        sincos_t(th, &st, &ct);
        const T S = st * pr.cce + ct * pr.sce;  // sin(th + ce)
        const T Cc = ct * pr.cce - st * pr.sce; // cos(th + ce)
        const T f = pr.c0 + x * (pr.c1 + x * (pr.c2 + x * pr.c3));
        const T f1 = pr.c1 + x * ((T)2 * pr.c2 + (T)3 * pr.c3 * x);
        const T f2 = (T)2 * pr.c2 + (T)6 * pr.c3 * x;
        const T r = f - y + v * S * dt - (T)P.ref_cte;
        // residual gradient over (x, y, th, v) and its curvature
        const T gr0 = f1, gr1 = (T)-1, gr2 = v * Cc * dt, gr3 = S * dt;
        const T cr = Wc2 * r;
        // dynamics Jacobian entries and costate-weighted curvature
        const T a1 = -v * st * dt, b1 = ct * dt, a2 = v * ct * dt, b2 = st * dt;
        const T p0 = Vs[0], p1 = Vs[1];
        const T hthth = p0 * (-v * ct * dt) + p1 * (-v * st * dt);
        const T hthv = p0 * (-st * dt) + p1 * (ct * dt);
        // Q_s
        T Qs[6];
        Qs[0] = cr * gr0 + p0;
        Qs[1] = cr * gr1 + p1;
        Qs[2] = cr * gr2 + We2 * (th + pr.ce - (T)P.ref_eth) + a1 * p0 + a2 * p1 + Vs[2];
        Qs[3] = cr * gr3 + Wv2 * (v - (T)P.ref_v) + b1 * p0 + b2 * p1 + Vs[3];
        Qs[4] = -Wdw2 * (w - wp);
        Qs[5] = -Wda2 * (a - ap);
        T Qu0 = Ww2 * w + Wdw2 * (w - wp) + dt * Vs[2] + Vs[4];
        T Qu1 = Wa2 * a + Wda2 * (a - ap) + dt * Vs[3] + Vs[5];
        // M = V'' F_s (columns 0..3), rows 0..5
        T M[6][4];
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            const T P0 = Vss[sidx(i, 0)], P1 = Vss[sidx(i, 1)], P2 = Vss[sidx(i, 2)], P3 = Vss[sidx(i, 3)];
            M[i][0] = P0;
            M[i][1] = P1;
            M[i][2] = a1 * P0 + a2 * P1 + P2;
            M[i][3] = b1 * P0 + b2 * P1 + P3;
        }
        T Qss[21];
#pragma unroll
        for (int i = 0; i < 21; ++i) Qss[i] = 0;
        // F_s^T V'' F_s on the (x,y,th,v) block
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const T G0 = M[0][j], G1 = M[1][j];
            const T G2 = a1 * M[0][j] + a2 * M[1][j] + M[2][j];
            const T G3 = b1 * M[0][j] + b2 * M[1][j] + M[3][j];
            if (0 >= j) Qss[sidx(0, j)] += G0;
            if (1 >= j) Qss[sidx(1, j)] += G1;
            if (2 >= j) Qss[sidx(2, j)] += G2;
            Qss[sidx(3, j)] += G3;
        }
        // cost curvature: 2 W_CTE (gr gr^T + r Hr), heading / speed weights
        Qss[sidx(0, 0)] += Wc2 * gr0 * gr0 + cr * f2;
        Qss[sidx(1, 0)] += Wc2 * gr1 * gr0;
        Qss[sidx(1, 1)] += Wc2 * gr1 * gr1;
        Qss[sidx(2, 0)] += Wc2 * gr2 * gr0;
        Qss[sidx(2, 1)] += Wc2 * gr2 * gr1;
        Qss[sidx(2, 2)] += Wc2 * gr2 * gr2 + cr * (-v * S * dt) + We2 + hthth;
        Qss[sidx(3, 0)] += Wc2 * gr3 * gr0;
        Qss[sidx(3, 1)] += Wc2 * gr3 * gr1;
        Qss[sidx(3, 2)] += Wc2 * gr3 * gr2 + cr * (Cc * dt) + hthv;
        Qss[sidx(3, 3)] += Wc2 * gr3 * gr3 + Wv2;
        Qss[sidx(4, 4)] += Wdw2;
        Qss[sidx(5, 5)] += Wda2;
        // Q_us (2 x 6)
        T Qus[2][6];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            Qus[0][j] = dt * M[2][j] + M[4][j];
            Qus[1][j] = dt * M[3][j] + M[5][j];
        }
        Qus[0][4] = -Wdw2; Qus[0][5] = 0;
        Qus[1][4] = 0;     Qus[1][5] = -Wda2;
        // Q_uu
        const T Fw2 = dt * Vss[sidx(2, 2)] + Vss[sidx(4, 2)], Fw4 = dt * Vss[sidx(2, 4)] + Vss[sidx(4, 4)];
        const T Fa2 = dt * Vss[sidx(3, 2)] + Vss[sidx(5, 2)], Fa4 = dt * Vss[sidx(3, 4)] + Vss[sidx(5, 4)];
        const T Fa3 = dt * Vss[sidx(3, 3)] + Vss[sidx(5, 3)], Fa5 = dt * Vss[sidx(3, 5)] + Vss[sidx(5, 5)];
        const T Quu00 = Ww2 + Wdw2 + dt * Fw2 + Fw4;
        const T Quu01 = dt * Fa2 + Fa4;
        const T Quu11 = Wa2 + Wda2 + dt * Fa3 + Fa5;
        // regularised Hessian must be SPD
        const T h00 = Quu00 + rho, h01 = Quu01, h11 = Quu11 + rho;
        const T det = h00 * h11 - h01 * h01;
        if (!(h00 > 0) || !(det > (T)1e-12 * h00 * h11)) return false;
        T d0, d1;
        bool f0, fr1;
        box_qp2(h00, h01, h11, Qu0, Qu1, lbw - w, ubw - w, lba - a, uba - a, &d0, &d1, &f0, &fr1);
        T K[2][6];
        if (f0 && fr1) {
            const T i00 = h11 / det, i01 = -h01 / det, i11 = h00 / det;
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                K[0][j] = -(i00 * Qus[0][j] + i01 * Qus[1][j]);
                K[1][j] = -(i01 * Qus[0][j] + i11 * Qus[1][j]);
            }
        } else {
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                K[0][j] = f0 ? -Qus[0][j] / h00 : (T)0;
                K[1][j] = fr1 ? -Qus[1][j] / h11 : (T)0;
            }
        }
#pragma unroll
        for (int j = 0; j < 6; ++j) { ws[L.G(k, j)] = K[0][j]; ws[L.G(k, 6 + j)] = K[1][j]; }
        ws[L.G(k, 12)] = d0;
        ws[L.G(k, 13)] = d1;
        km = fmax(km, fmax(fabs(d0), fabs(d1)));
        s1 += d0 * Qu0 + d1 * Qu1;
        s2 += (T)0.5 * (d0 * (Quu00 * d0 + Quu01 * d1) + d1 * (Quu01 * d0 + Quu11 * d1));
        // value update (unregularised Q_uu, Tassa et al. 2012 eq. 11)
        const T Qk0 = Quu00 * d0 + Quu01 * d1, Qk1 = Quu01 * d0 + Quu11 * d1;
        T QuuK[2][6];
#pragma unroll
        for (int j = 0; j < 6; ++j) {
            QuuK[0][j] = Quu00 * K[0][j] + Quu01 * K[1][j] + Qus[0][j];
            QuuK[1][j] = Quu01 * K[0][j] + Quu11 * K[1][j] + Qus[1][j];
        }
#pragma unroll
        for (int j = 0; j < 6; ++j)
            Vs[j] = Qs[j] + K[0][j] * (Qk0 + Qu0) + K[1][j] * (Qk1 + Qu1) + Qus[0][j] * d0 + Qus[1][j] * d1;
#pragma unroll
        for (int i = 0; i < 6; ++i) {
#pragma unroll
            for (int j = 0; j <= i; ++j)
                Vss[sidx(i, j)] = Qss[sidx(i, j)] + K[0][i] * QuuK[0][j] + K[1][i] * QuuK[1][j] +
                                  Qus[0][i] * K[0][j] + Qus[1][i] * K[1][j];
        }
    }
    *dV1 = s1;
    *dV2 = s2;
    *kmax = km;
    return true;
}

struct SolveOut {
    int32_t status, iters;
};

// Full solve of one problem.  Results: buffer index holding the solution (cur),
// objective, status, iteration count.
template <typename T, class WS>
MPCG_HD SolveOut solve_one(const SolverParams& P, const Problem<T>& pr, WS& ws, int* cur_out, T* obj) {
    const Layout L{P.N};
    const T lbw = (T)(-P.max_w - fmin(1e-4, P.relax * fmax(1.0, P.max_w)));
    const T ubw = (T)(P.max_w + fmin(1e-4, P.relax * fmax(1.0, P.max_w)));
    const T lba = (T)(-P.max_a - fmin(1e-4, P.relax * fmax(1.0, P.max_a)));
    const T uba = (T)(P.max_a + fmin(1e-4, P.relax * fmax(1.0, P.max_a)));
    const T rho_min = (T)(1e-6 * (2.0 * fmax(P.w_w, P.w_a) + 1.0));
    int cur = 0;
    T J = init_rollout(P, pr, L, ws, cur);
    T rho = 0;
    SolveOut out{ST_MAXITER, 0};
    int it = 0;
    for (; it < P.max_iter; ++it) {
        if (!(J == J) || !isfinite((double)J)) { out.status = ST_INVALID_NUMBER; break; }
        T dV1, dV2, kmax;
        if (!backward(P, pr, L, ws, cur, rho, lbw, ubw, lba, uba, &dV1, &dV2, &kmax)) {
            rho = (rho < rho_min) ? rho_min : (T)8 * rho;
            if (rho > (T)1e12) { out.status = ST_ERROR_IN_STEP; break; }
            continue;
        }
        const T noise = Tol<T>::noise * ((T)1 + fabs(J));
        const int nxt = 1 - cur;
        if (kmax <= (T)P.tol) {
            // converged: the Newton step is below tolerance; take it and stop
            const T Jn = forward(P, pr, L, ws, cur, nxt, (T)1, lbw, ubw, lba, uba);
            if (Jn <= J + noise) { cur = nxt; J = Jn; }
            out.status = ST_SUCCESS;
            ++it;
            break;
        }
        T alpha = 1;
        bool accepted = false;
        T Jn = J;
        for (int ls = 0; ls < P.max_ls; ++ls) {
            Jn = forward(P, pr, L, ws, cur, nxt, alpha, lbw, ubw, lba, uba);
            const T expected = -(alpha * dV1 + alpha * alpha * dV2);
            if (Jn == Jn && (Jn <= J - (T)1e-4 * expected || (expected <= noise && Jn <= J + noise))) {
                accepted = true;
                break;
            }
            alpha *= (T)0.5;
        }
        if (accepted) {
            cur = nxt;
            J = Jn;
            rho = (rho <= rho_min) ? (T)0 : rho * (T)0.25;
        } else {
            rho = (rho < rho_min) ? rho_min : (T)8 * rho;
            if (rho > (T)1e12) { out.status = ST_ERROR_IN_STEP; break; }
        }
    }
    out.iters = it;
    *cur_out = cur;
    *obj = J;
    return out;
}

}  // namespace mpcg
#endif
