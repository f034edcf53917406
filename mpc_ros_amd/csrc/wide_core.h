// mpc_ros_amd/csrc/wide_core.h -- the same interior-point solve, one problem per wavefront.
//
// ipm_core.h runs one problem per lane: a wavefront carries 64 problems and takes as
// long as the slowest of them, and a lone wavefront issues every FP64 instruction of
// its iteration itself (~1M cycles per iteration).  The iteration counts of this NLP
// are heavy-tailed (infinity set: mean 14, p99 35, max >130), so at one problem per
// lane the batch time is set by a handful of slow problems.  This solver spreads one
// problem over the 64 lanes of a wavefront instead:
//
//   * stage-parallel sweeps (accept, statistics, trial points, multipliers, step
//     statistics): lane k owns stage k (N <= 64); sums/extrema by xor-butterflies;
//     the dynamics value F(s_k, u_k) moves to lane k+1 by one lane shift;
//   * the Riccati recursion: lane (i, j) = (t >> 3, t & 7) owns entry (i, j) of the
//     8x8 cost-to-go matrix; per stage one dense 8x8 product M = P' [A | B | d]
//     (entry per lane), the 2x8 projection B^T M by 16 lanes, and the update
//     P = Q + A^T M + S^T K (entry per lane); the stage data that does not depend on
//     P (linearisation, barrier Hessian, gradients) is computed for all stages in
//     parallel before the sweep;
//   * the forward recursion of the step (8-vector) runs replicated in every lane.
//
// The problem state (iterate, multipliers, step, Riccati records, filter) lives in
// the wavefront's LDS for the whole solve.  Per-problem scalars (mu, tau, filter
// size, ...) are wave-uniform; every control decision is taken on butterfly-reduced
// values, which are bitwise identical in all lanes.
//
// Numerically this is ipm_core.h's algorithm with the same constants and formulas;
// only the order of some sums differs (tree instead of sequential), i.e. results
// agree with the one-problem-per-lane solver and with the oracle to rounding.
//
// The wavefront context WV supplies the lane index, the LDS base, the cross-lane
// primitives and mark(phase) (a no-op except in the phase-timing build tools/wide_prof.hip): the device implementation is in mpcg_wide.hip, a host emulation with
// 64 threads in tests/native/wide_host_check.cpp.
#ifndef MPCG_WIDE_CORE_H
#define MPCG_WIDE_CORE_H

#include "ipm_core.h"

namespace mpcg {

// LDS layout of one problem (doubles).
//
// Stage-major arrays are read and written by stage-parallel lanes (lane k = stage k)
// with 16-byte accesses.  Their strides are 2 mod 4 doubles (10 for the 8-entry
// records, 6 for the 6-entry multipliers, 18 for the gain record, 38 / 42 for the stage
// table) so that the 16 lanes of a ds_read_b128 group and the 8 lanes of a
// ds_write_b128 group hit distinct LDS banks; at a 64-byte stride they conflict 4-way.
struct WideLayout {
    int N, cap, SS;  // SS: stage table stride (38; 42 with the bicycle's turn terms)
    // KL: the gain records' stride in LDS -- KS, or 0 for the bicycle and every N > 32, whose
    // gain records live in the problem's workspace (SP_KRG): more problems per CU (bicycle
    // N = 25: 8 instead of 6; fp32 N = 40: 11 instead of 9; fp64 N = 64: 3 instead of 2)
    int KL;
    // (kl >= 0: the caller knows KL at compile time -- the diff-drive split solver, N <= 32 --
    // and the layout's offsets fold to constants)
    MPCG_HD WideLayout(int N_, int cap_, int model, int kl = -1)
        : N(N_), cap(cap_), SS(model == 1 ? 42 : 38), KL(kl >= 0 ? kl : (model == 1 || N_ > 32 ? 0 : KS)) {}
    static constexpr int WS = 10, YS = 6, KS = 18;
    // the iterate record of stage k: w (8), z_L (8), z_U (8), the step dw (8), 2 pad (one record
    // instead of four 10-double arrays: 6 doubles per stage less)
    static constexpr int RS = 34, RZL = 8, RZU = 16, RDW = 24;
    // stage table entries
    static constexpr int SA = 0;    // a[7]: non-trivial entries of A_k (Lin::jac)
    static constexpr int SDT = 7;   // dt
    static constexpr int SD = 8;    // d[6]: F(s_k, u_k) - s_{k+1} (Newton mode)
    static constexpr int SQD = 14;  // diag of the stage Hessian (6 states, 2 controls = R)
    static constexpr int SQV = 22;  // gradient q (6) and r (2)
    static constexpr int SCV = 30;  // curvature of the constraints: Q00 Q22 Q32 Q55 Q53
    static constexpr int SZERO = 35, SONE = 36, SMONE = 37;  // constants 0, 1, -1
    // (the feed-forward gains kff[2] are the last two doubles of the gain record: KR(k) + KF)
    static constexpr int KF = 16;
    // bicycle only: model terms of the heading rows (th, eth): d(turn)/d(w) (B_hat
    // column w: v/lf dt; dt for the differential drive), d(turn)/d(v) (A_hat column v:
    // w/lf dt; 0), and the (v, w) curvature of the Lagrangian (-(y_th + y_eth)/lf dt; 0)
    static constexpr int STW = 38, STV = 39, SHVD = 40;
    MPCG_HD int W(int k) const { return RS * k; }
    MPCG_HD int ZL(int k) const { return RS * k + RZL; }
    MPCG_HD int ZU(int k) const { return RS * k + RZU; }
    MPCG_HD int DW(int k) const { return RS * k + RDW; }
    MPCG_HD int Y(int k) const { return RS * N + YS * k; }
    MPCG_HD int YP(int k) const { return (RS + YS) * N + YS * k; }
    MPCG_HD int KR(int k) const { return (RS + 2 * YS) * N + KS * k; }  // K[0][0..7] K[1][0..7] kff[2]
    MPCG_HD int ST(int k) const { return (RS + 2 * YS + KL) * N + SS * k; }
    // scratch of the Riccati sweep: G^T of the stage, then M^T (M[r][c] at MS c + r) in
    // the same 8 columns, MS = 10 doubles apart (16-byte column reads of different
    // columns fall in different LDS banks); then P row-major
    static constexpr int MS = 10;
    MPCG_HD int SCR() const { return (RS + 2 * YS + KL + SS) * N; }
    MPCG_HD int PSC() const { return SCR() + 8 * MS; }
    MPCG_HD int RSC() const { return SCR() + 8 * MS + 64; }  // row scales: ra[6] rb[6] 1.0 (+pad)
    MPCG_HD int ZB() const { return RSC() + 16; }            // 8 zeros (an absent column)
    MPCG_HD int FI() const { return RSC() + 24; }
    MPCG_HD int C0() const { return FI() + 2 * cap; }  // -c of the initial-state rows (6) + pad
    MPCG_HD int CTL() const { return C0() + 8; }       // 16 wave-uniform solver scalars (WideSolver::CtlRef)
    // the problem data: initial state (6), polynomial coefficients (4, 16-byte aligned), pad
    MPCG_HD int PRB() const { return CTL() + 16; }
    MPCG_HD int PRC() const { return PRB() + 6; }
    MPCG_HD int total() const { return PRB() + 12; }
    // Per-wavefront HBM workspace (elements of T) of the rare paths, one per resident
    // wavefront (mpcg_wide.hip claims a slot per problem).  The watchdog's stored iterate
    // and direction (LDS [W(0), YP(N)) = 46N of a 52N region), the last acceptable iterate
    // (w: 8N of 10N), the Newton direction kept while second-order corrections are tried (DW,
    // YP: 14N of 16N), the iterate kept while a soft-restoration step is evaluated (w, z_L,
    // z_U, y: 30N of 36N).
    MPCG_HD int SP_WD() const { return 0; }
    MPCG_HD int SP_ACC() const { return 52 * N; }
    MPCG_HD int SP_SOC() const { return 62 * N; }
    MPCG_HD int SP_SOFT() const { return 78 * N; }
    // The filter beyond its cap LDS entries: FX more in the workspace (Ipopt's filter is
    // unbounded; the infinity set reaches 71 entries at N = 40), the original problem's at
    // SP_FLT, the restoration problem's at SP_FLTR
    static constexpr int FX = 448;
    MPCG_HD int SP_FLT() const { return 114 * N; }
    // the gain records when KL = 0: written by the Riccati sweep, read by the step recursion of
    // the same Newton system
    MPCG_HD int SP_KRG() const { return 114 * N + 2 * FX; }
    MPCG_HD int spill() const { return SP_KRG() + (KL == 0 ? KS * N : 0); }
    // The feasibility-restoration phase (WideSolver<..., RESTO = true>, entered from the
    // original problem's line search): the original problem's LDS image while the
    // restoration problem uses the LDS (total()), the restoration problem's per-stage
    // records of the penalty variables p, n of the rows into stage k (XS), and their copies
    // for the watchdog / second-order corrections / soft restoration (XSP).  The
    // restoration problem's own LDS-part copies reuse SP_WD, SP_SOC and SP_SOFT (the
    // original's SP_ACC is kept).
    static constexpr int XP = 0, XN = 6, XZP = 12, XZN = 18, XDP = 24, XDN = 30;  // p, n, z_p, z_n, dp, dn
    static constexpr int XCR = 36;  // constraint right-hand side of the rows (scaled): c(x) - p + n, or a SOC's
    static constexpr int XDS = 42;  // sqrt of the rows' diagonal D (unscaled rows) in the reduced system
    static constexpr int XM = 48;    // soft rows: ds_k = M z + m (M 6x6 row-major on the states) ...
    static constexpr int XMN = 84;   // ... their slack e = ds_k - z = N z + m, N = M - I (6x6) ...
    static constexpr int XMV = 120;  // ... m
    static constexpr int XE = 126;   // e of the last step (row form)
    // iterative refinement of the step (WideSolver::refine_resto): the full system's residual in
    // the stage's x rows (8) and the rows' p, n, c rows (6 each) ...
    static constexpr int XRX = 132, XRP = 140, XRN = 146, XRC = 152;
    // ... and the step it refines: dx (8), dp, dn, y+ (6 each), the rows' right-hand side XCR (6)
    static constexpr int XSX = 158, XSP = 166, XSN = 172, XSY = 178, XSC = 184;
    static constexpr int XS = 190;
    static constexpr int XW = 72;   // spill copies: watchdog p n zp zn dp dn (0..35), SOC dp dn (36..47), soft p n zp zn (48..71)
    MPCG_HD int SP_DUMP() const { return spill(); }
    MPCG_HD int SP_EXT() const { return spill() + total(); }
    MPCG_HD int SP_XSP() const { return SP_EXT() + XS * N; }
    MPCG_HD int SP_FLTR() const { return SP_XSP() + XW * N; }
    MPCG_HD int slot() const { return SP_FLTR() + 2 * FX; }
};

// The original problem's values the restoration phase needs (passed by value into its
// out-of-line function) and its result.
template <class T>
struct RestoIn {
    T mu, tau, theta, prim_inf, ref_phi, ref_theta, sf;
    int nf, iter;
};
struct RestoOut {
    int status;  // 0: the restoration phase found a point the original problem accepts
    int iter;
    int fover;  // its filter's dropped entries (diagnostic)
};
// The restoration phase of the problem whose wavefront state is in LDS and whose workspace
// slot is ws (defined after WideSolver; out of line).
template <class WV, int MODEL, class T, int NB>
MPCG_NOINLINE RestoOut resto_phase(const IpmParams& P, IpmProblem<T> pr, WV wv, T* ws, RestoIn<T> in);

// MODEL: 0 differential drive (FG_eval), 1 kinematic bicycle -- a template parameter
// so that the differential-drive kernel carries none of the bicycle's terms.
// SPLIT (N <= 32): the step and multiplier recursions run in both half-waves (lane t and
// t + 32 hold stage t & 31), and the step statistics take the stage's variables 0..3 in
// the lower and 4..7 in the upper half-wave: half the per-variable work per lane.
// TT: the arithmetic type -- double (Ipopt's), or float (the fp32 solver of BASELINE
// configs[2]: every lane value, LDS array and uniform scalar in fp32; the caller states a
// tolerance a float iterate can meet).
// NB: stage blocks -- 1 for N <= 64 (lane t owns stage t), 2 for 64 < N <= 128 (lane t owns
// stages t and 64 + t: the stage-parallel sweeps loop over the blocks, the dynamics of
// stage 63 reach stage 64 by a lane read, the systolic recursions run block by block).
// RESTO: the instance that solves Ipopt's feasibility-restoration problem (RestoIpoptNLP,
// oracle/ipm.c perform_restoration) from the original problem's iterate:
//   min rho sum(p + n) + eta(mu)/2 ||D_R (x - x_R)||^2,  eta = sqrt(mu), D_R = diag(1/max(1,|x_R|))
//   s.t. c(x) - p + n = 0 (c: the original's scaled rows), x in the original's bounds, p, n >= 0.
// Its Newton system eliminates p and n (Ipopt's AugRestoSystemSolver): the dynamics rows
// become soft, J dx - D y+ = -c_hat with a positive diagonal D, and the Riccati recursion
// absorbs each row block by the update P~ = P - P D^1/2 S^-1 D^1/2 P, S = I + D^1/2 P D^1/2
// (the inertia test adds: every S positive definite).  Unsplit sweeps only (SPLIT = false),
// block loops for any N <= 128.  A separate instantiation, called out of line from the
// original problem's line search (resto_phase below): the main kernel's register
// allocation does not see it.
template <class WV, int MODEL = 0, bool SPLIT = false, class TT = double, int NB = 1, bool RESTO = false>
struct WideSolver {
    static_assert(NB == 1 || !SPLIT, "the half-wave split is for N <= 32");
    static_assert(!RESTO || !SPLIT, "the restoration problem runs the unsplit sweeps");
    typedef TT T;
    static constexpr double EPS = sizeof(TT) == 4 ? 1.1920928955078125e-07 : 2.220446049250313e-16;
    const IpmParams P;
    const IpmProblem<T> pr;
    WV wv;
    WideLayout L;
    int N, t;
    T dt;
    T sl, su, wl, wu, al, au, sl0, su0, wl0, wu0, al0, au0;
    T sf;
    T mu, tau;
    // statistics of the current iterate
    T fval, logsum, theta, prim_inf, prim_uns, dual_inf, compl0, pmin, pmax, l1y, l1z;
    // line-search / iteration state
    T theta_min, dw_last, acc_alpha, acc_z, delta_w_used;
    int iter, nf, status;
    bool acc_pending;  // a step (acc_alpha, acc_z) waits to be applied by the next statistics sweep
    // filter line-search acceptor (Ipopt FilterLSAcceptor): reference point, switching-
    // condition powers (-gd)^s_phi and theta^s_theta of the reference, reset heuristic
    T ref_theta, ref_phi, ref_gd, ref_pgd, ref_pth, ref_inc;
    int last_rej_filter, count_filter_rej, n_filter_resets;
    // watchdog, tiny steps, soft restoration, acceptable points (BacktrackingLineSearch,
    // OptimalityErrorConvergenceCheck)
    int in_wd, wd_short, wd_trial_iter, tiny_last, tiny_flag, in_soft, soft_count, acc_counter, have_acc;

    T* spill;  // this problem's HBM spill area (WideLayout::spill() elements)
    int n_fover = 0;  // filter entries dropped beyond cap + FX (diagnostic; Ipopt drops none)
    int nf_peak = 0;  // the most filter entries held at once (diagnostic)
    int n_resto = 0;  // restoration phases entered (diagnostic)
    // Rarely used wave-uniform solver state lives in the problem's LDS control block
    // (registers are the scarcer resource: every scalar held across the iteration loop
    // competes with the sweeps).  x() = v stores (lane 0), x() reads (uniform).
    struct CtlRef {
        const WideSolver* s;
        int i;
        MPCG_HD operator T() const { return s->wv.uni_d(s->ld(s->L.CTL() + i)); }
        MPCG_HD CtlRef& operator=(T v) {
            s->wv.sync();
            if (s->wv.lane() == 0) s->st(s->L.CTL() + i, v);
            s->wv.sync();
            return *this;
        }
        MPCG_HD CtlRef& operator=(const CtlRef& o) { return *this = (T)o; }  // (the value, not the binding)
    };
    MPCG_HD CtlRef wd_alpha_test() const { return CtlRef{this, 0}; }
    MPCG_HD CtlRef wd_theta() const { return CtlRef{this, 1}; }
    MPCG_HD CtlRef wd_phi() const { return CtlRef{this, 2}; }
    MPCG_HD CtlRef wd_gd() const { return CtlRef{this, 3}; }
    MPCG_HD CtlRef wd_amax_z() const { return CtlRef{this, 4}; }
    MPCG_HD CtlRef soc_alpha() const { return CtlRef{this, 5}; }
    MPCG_HD CtlRef soc_amax_z() const { return CtlRef{this, 6}; }
    MPCG_HD CtlRef soc_theta_old() const { return CtlRef{this, 7}; }
    MPCG_HD CtlRef soc_theta_trial() const { return CtlRef{this, 8}; }
    MPCG_HD CtlRef soft_ec() const { return CtlRef{this, 9}; }
    MPCG_HD CtlRef soft_a() const { return CtlRef{this, 10}; }
    MPCG_HD CtlRef last_obj() const { return CtlRef{this, 11}; }
    MPCG_HD CtlRef curr_obj() const { return CtlRef{this, 12}; }
    MPCG_HD CtlRef kkt() const { return CtlRef{this, 13}; }
    MPCG_HD CtlRef theta_max() const { return CtlRef{this, 14}; }
    MPCG_HD CtlRef last_mu() const { return CtlRef{this, 15}; }

    // SPLIT: the sine/cosine pair of the last trial point (the lane's heading theta or
    // etheta), which the next statistics sweep reuses when that trial point was
    // accepted (the accepted iterate is bitwise the trial point: both are w + alpha dw)
    T c_sa = 0, c_ca = 0;
    int c_ok = 0;
    static constexpr int model = MODEL;
    T lf;  // model 1: wheelbase

    // ---- the restoration problem (RESTO instance only; oracle/ipm.c perform_restoration)
    static constexpr double RHO = 1000.0;  // resto_penalty_parameter
    static constexpr double KD = 1e-5;     // kappa_d: the barrier's damping of one-sided bounds (p, n >= 0)
    enum : int { RESTO_DONE = 100 };       // the original problem accepts the restoration iterate
    enum : int { NEED_RESTO = 101 };       // the original problem enters the restoration phase
    T* ext = nullptr;                      // HBM records of the rows into each stage (WideLayout::XS)
    T* xsp = nullptr;                      // HBM copies of the records (WideLayout::XW)
    T* dumpO = nullptr;                    // the original problem's LDS image: x_R = its iterate, its filter
    T o_mu = 0, o_tau = 0, o_theta = 0, o_ref_phi = 0, o_ref_theta = 0, o_sf = 1;
    int o_nf = 0;
    bool resto_first = false;
    // statistics of the restoration iterate: sum(p + n), ||D_R (x - x_R)||^2, and the original
    // problem's barrier function, violation and max violation at x
    T r_spn = 0, r_qx = 0, r_phiO = 0, r_thO = 0, r_pinfO = 0;
    // a correction solve of the iterative refinement: the right-hand side is the residual in
    // the records (XRX, XRP, XRN; XCR holds -r_c), not the barrier gradient (refine_resto)
    bool rf_pass = false;
    // the monotone barrier update's loop state across a re-evaluation (k_rmu)
    T mu_Emu = 0;
    int mu_tf = 0;
    bool mu_done = false;

    MPCG_HD WideSolver(const IpmParams& P_, const IpmProblem<T>& pr_, const WV& wv_, T* spill_)
        : P(P_), pr(pr_), wv(wv_), L(P_.N, P_.filter_cap, MODEL, MODEL == 0 && SPLIT ? WideLayout::KS : -1), N(P_.N), t(wv_.t), dt((T)P_.dt), lf((T)P_.lf),
          spill(spill_) {}

    // ------------------------------------------------------ the model
    // F(s, u): FG_eval's dynamics (Lin::next); for the bicycle the heading rows turn by
    // v w / lf dt instead of w dt (oracle/nlp_mpc.c, same operation order).
    MPCG_HD void next_m(const Lin<T>& ln, const T* s, const T* u, T* out) const {
        ln.next(s, u, dt, out);
        if (model == 1) {
            const T turn = s[3] * u[0] / lf * dt;
            out[2] = s[2] + turn;
            out[5] = s[5] + turn;
        }
    }
    // d(turn)/d(w) and d(turn)/d(v)
    MPCG_HD void turn_d(const T* s, const T* u, T* tw, T* tv) const {
        if (model == 1) {
            *tw = s[3] / lf * dt;
            *tv = u[0] / lf * dt;
        } else {
            *tw = dt;
            *tv = 0;
        }
    }

    // ------------------------------------------------------------ LDS helpers
    MPCG_HD T ld(int i) const { return wv.template Sp<T>()[i]; }
    // the problem data, stored in LDS by setup(): held in registers across the solve it
    // was spilled around the sweeps that read it
    struct C4 {
        T c[4];
    };
    MPCG_HD C4 pcoef() const {
        C4 r;
        wv.ld2(L.PRC(), r.c[0], r.c[1]);
        wv.ld2(L.PRC() + 2, r.c[2], r.c[3]);
        return r;
    }
    MPCG_HD T pinit(int j) const { return ld(L.PRB() + j); }
    MPCG_HD void st(int i, T v) const { wv.template Sp<T>()[i] = v; }
    template <int n>
    MPCG_HD void ldn(int i, T* v) const {
#pragma unroll
        for (int j = 0; j < n; ++j) v[j] = wv.template Sp<T>()[i + j];
    }

    // ------------------------------------------------------ wave reductions
    // Six pairwise steps over symmetric lane pairs (WV::rpart): every lane ends with
    // the same bits.  Several reductions run interleaved step by step.
    enum { RSUM = 0, RMAX = 1, RMIN = 2 };
    template <int s, int n>
    MPCG_HD void rstep(T* v, const int* op) {
        T o[n];
        if constexpr (s == 5) {
            // across the half-waves: {v, o} = {own, partner} in some order (a commutative op
            // leaves both lanes of the pair with the same bits)
#pragma unroll
            for (int q = 0; q < n; ++q) wv.xor32_pair(v[q], v[q], o[q]);
        } else {
#pragma unroll
            for (int q = 0; q < n; ++q) o[q] = wv.template rpart<s>(v[q]);
        }
#pragma unroll
        for (int q = 0; q < n; ++q)
            v[q] = op[q] == RSUM ? v[q] + o[q] : (op[q] == RMAX ? tmax(v[q], o[q]) : tmin(v[q], o[q]));
    }
    // Contributions come from lanes < N only (FULL: from both half-waves): for N <= 32
    // five steps complete the reduction in lanes 0..31 and lane 0's value is made
    // wave-uniform (scalar).
    template <int n, bool FULL = false>
    MPCG_HD void reduce(T* v, const int* op) {
        rstep<0, n>(v, op);
        rstep<1, n>(v, op);
        rstep<2, n>(v, op);
        rstep<3, n>(v, op);
        rstep<4, n>(v, op);
        if (FULL || N > 32) rstep<5, n>(v, op);
#pragma unroll
        for (int q = 0; q < n; ++q) v[q] = wv.uni_d(v[q]);
    }
    MPCG_HD T rsum(T v) {
        const int op[1] = {RSUM};
        reduce<1>(&v, op);
        return v;
    }
    MPCG_HD T rmax(T v) {
        const int op[1] = {RMAX};
        reduce<1>(&v, op);
        return v;
    }
    // 16-byte LDS load of two consecutive doubles (i even)
    MPCG_HD void ld2(int i, T& a, T& b) const { wv.ld2(i, a, b); }
    template <int n>
    MPCG_HD void ldv(int i, T* v) const {
#pragma unroll
        for (int j = 0; j < n; j += 2) wv.ld2(i + j, v[j], v[j + 1]);
    }

    // ------------------------------------------------------ model helpers
    // row scale of dynamics row s into stage k (1 for the initial-state rows), from LDS
    MPCG_HD T rowscale(int s, int k) const { return ld(L.RSC() + (k == 0 ? 12 : (k == 1 ? s : 6 + s))); }
    MPCG_HD T vlo(int j) const { return j < 6 ? sl : (j == 6 ? wl : al); }
    MPCG_HD T vhi(int j) const { return j < 6 ? su : (j == 6 ? wu : au); }
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

    // ------------------------------------------------------------ setup
    // Same as IpmSolver::setup (ipm_core.h), uniform in every lane.
    MPCG_HD void rowscales_at(const T* s, T* rs) const {
        Lin<T> ln;
        ln.eval(pr.c, s);
        T m[6];
        m[0] = tmax((T)1, tmax((T)fabs(s[3] * ln.st * dt), (T)fabs(ln.ct * dt)));
        m[1] = tmax((T)1, tmax((T)fabs(s[3] * ln.ct * dt), (T)fabs(ln.st * dt)));
        // heading rows: the turn's derivatives at the start point (controls there are 0)
        T tw, tv;
        const T u0[2] = {0, 0};
        turn_d(s, u0, &tw, &tv);
        m[2] = tmax((T)1, tmax((T)fabs(tw), (T)fabs(tv)));
        m[3] = tmax((T)1, dt);
        m[4] = tmax(tmax((T)1, (T)fabs(ln.f1)), tmax((T)fabs(ln.se * dt), (T)fabs(s[3] * ln.ce * dt)));
        m[5] = m[2];
#pragma unroll
        for (int j = 0; j < 6; ++j) rs[j] = m[j] > (T)100 ? (T)100 / m[j] : (T)1;
    }
    MPCG_HD void bounds_only() {
        const T rl = (T)fmin(P.constr_viol_tol, P.bound_relax_factor * fmax(1.0, P.bound));
        // (uniform values made scalar: the register allocator keeps them in SGPRs rather
        // than spilling vector copies to scratch)
        sl0 = wv.uni_d((T)-P.bound); su0 = wv.uni_d((T)P.bound); sl = wv.uni_d(sl0 - rl); su = wv.uni_d(su0 + rl);
        const T rw = (T)fmin(P.constr_viol_tol, P.bound_relax_factor * fmax(1.0, P.max_w));
        wl0 = wv.uni_d((T)-P.max_w); wu0 = wv.uni_d((T)P.max_w); wl = wv.uni_d(wl0 - rw); wu = wv.uni_d(wu0 + rw);
        const T rA = (T)fmin(P.constr_viol_tol, P.bound_relax_factor * fmax(1.0, P.max_a));
        al0 = wv.uni_d((T)-P.max_a); au0 = wv.uni_d((T)P.max_a); al = wv.uni_d(al0 - rA); au = wv.uni_d(au0 + rA);
    }
    MPCG_HD void setup() {
        bounds_only();
        T g[6];
        grad_state(pr.init, g);
        T gm = tmax((T)fabs(g[3]), tmax((T)fabs(g[4]), (T)fabs(g[5])));
        if (N >= 2) {
            const T z[6] = {0, 0, 0, 0, 0, 0};
            grad_state(z, g);
            gm = tmax(gm, tmax((T)fabs(g[3]), tmax((T)fabs(g[4]), (T)fabs(g[5]))));
        }
        sf = wv.uni_d(gm > (T)100 ? (T)100 / gm : (T)1);
        T ra[6], rb[6];
        rowscales_at(pr.init, ra);
        const T z6[6] = {0, 0, 0, 0, 0, 0};
        rowscales_at(z6, rb);
        if (t == 0) {
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                st(L.RSC() + j, ra[j]);
                st(L.RSC() + 6 + j, rb[j]);
            }
            st(L.RSC() + 12, 1);
#pragma unroll
            for (int j = 0; j < 6; ++j) st(L.PRB() + j, pr.init[j]);
#pragma unroll
            for (int j = 0; j < 4; ++j) st(L.PRC() + j, pr.c[j]);
        }
        if (t < 8) st(L.ZB() + t, 0);
    }
    MPCG_HD T push(T v, T lo, T hi) const {
        const T pl = tmin((T)0.01 * tmax((T)1, (T)fabs(lo)), (T)0.01 * (hi - lo));
        const T pu = tmin((T)0.01 * tmax((T)1, (T)fabs(hi)), (T)0.01 * (hi - lo));
        if (v < lo + pl) v = lo + pl;
        if (v > hi - pu) v = hi - pu;
        return v;
    }
    MPCG_HD void init_point() {
        for (int b = 0; b < NB; ++b) {
            const int k = t + 64 * b;
            if (k >= N) continue;
            // constant entries of the stage table (dt, 0, 1, -1: gather targets of the
            // Riccati's per-lane offsets), written once
            const int sb = L.ST(k);
            st(sb + WideLayout::SDT, dt);
            st(sb + WideLayout::SZERO, 0);
            st(sb + WideLayout::SONE, 1);
            st(sb + WideLayout::SMONE, -1);
            for (int j = 0; j < 8; ++j) {
                st(L.W(k) + j, push((j < 6 && k == 0) ? pr.init[j] : (T)0, vlo(j), vhi(j)));
                st(L.ZL(k) + j, 1);
                st(L.ZU(k) + j, 1);
                if (j < 6) {
                    st(L.Y(k) + j, 0);
                    st(L.YP(k) + j, 0);
                }
                st(L.DW(k) + j, 0);
            }
        }
    }

    // ------------------------------------------------ accept + statistics
    MPCG_HD void accept_one(T w, T dwv, T zl, T zu, T lo, T hi, T alpha, T amax_z, T* wn, T* zln, T* zun,
                            bool clamp = true) const {
        const T rdl = rcp(w - lo), rdu = rcp(hi - w);
        const T dzl = mu * rdl - zl - zl * rdl * dwv;
        const T dzu = mu * rdu - zu + zu * rdu * dwv;
        *wn = w + alpha * dwv;
        const T a = zl + amax_z * dzl, b = zu + amax_z * dzu;
        if (clamp) {
            clamp_z(*wn, a, b, lo, hi, zln, zun);
        } else {
            *zln = a;
            *zun = b;
        }
    }
    // IpoptAlgorithm::AcceptTrialPoint: bound multipliers within kappa_sigma of mu / s
    MPCG_HD void clamp_z(T w, T a, T b, T lo, T hi, T* zln, T* zun) const {
        const T ksig = (T)1e10, iksig = (T)1e-10;
        const T rs2 = rcp(w - lo), ru2 = rcp(hi - w);
        *zln = tmax(tmin(a, ksig * mu * rs2), mu * rs2 * iksig);
        *zun = tmax(tmin(b, ksig * mu * ru2), mu * ru2 * iksig);
    }

    // Accept the step (w, z_L, z_U with the step lengths, y towards y+): element-parallel
    // over the 8N entries of the stage-major arrays, 64 per round.
    MPCG_HD void accept_all(int t, bool acc, T alpha, T amax_z, bool clamp = true) {
        wv.sync();
        if (acc) {
            // element-parallel: element e = 8k + j of the stage-major arrays, 64 per round
            // (bounds selected among locals: a select between member addresses would
            // force the solver object into scratch)
            const T bl[3] = {sl, wl, al}, bh[3] = {su, wu, au};
            for (int e = t; e < 8 * N; e += 64) {
                const int k = e >> 3, j = e & 7;
                const T lo = j < 6 ? bl[0] : (j == 6 ? bl[1] : bl[2]);
                const T hi = j < 6 ? bh[0] : (j == 6 ? bh[1] : bh[2]);
                if (!(k == N - 1 && j >= 6)) {
                    T wn, zln, zun;
                    accept_one(ld(L.W(k) + j), ld(L.DW(k) + j), ld(L.ZL(k) + j), ld(L.ZU(k) + j), lo, hi,
                               alpha, amax_z, &wn, &zln, &zun, clamp);
                    st(L.W(k) + j, wn);
                    st(L.ZL(k) + j, zln);
                    st(L.ZU(k) + j, zun);
                }
                if (j < 6) {
                    const T y = ld(L.Y(k) + j), yp = ld(L.YP(k) + j);
                    st(L.Y(k) + j, y + alpha * (yp - y));
                }
            }
            if constexpr (RESTO) accept_rows(t, alpha, amax_z, clamp);
        }
        wv.sync();
    }
    // (RESTO) the rows' p, n and their bound multipliers: lane t owns the rows into stages t
    // (and 64 + t) -- their HBM records are read and written by that lane only
    MPCG_HD void accept_rows(int t, T alpha, T amax_z, bool clamp) {
        for (int b = 0; b < NB; ++b) {
            const int k = t + 64 * b;
            if (k >= N) continue;
            T* x = xrec(k);
#pragma unroll
            for (int j = 0; j < 6; ++j) {
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int ov = h ? WideLayout::XN : WideLayout::XP, oz = h ? WideLayout::XZN : WideLayout::XZP;
                    const int od = h ? WideLayout::XDN : WideLayout::XDP;
                    const T v = x[ov + j], z = x[oz + j], dv = x[od + j];
                    const T dz = mu / v - z - z / v * dv;
                    const T vn = v + alpha * dv;
                    T zn = z + amax_z * dz;
                    if (clamp) zn = tmax(tmin(zn, (T)1e10 * mu / vn), mu / ((T)1e10 * vn));
                    x[ov + j] = vn;
                    x[oz + j] = zn;
                }
            }
        }
    }

    // Statistics of the iterate (SPLIT): lane k of the lower half-wave takes stage k's
    // variables 0..3, dynamics rows 0..3 and the heading theta, lane 32 + k the variables
    // 4..7, rows 4, 5 and the heading error; the one Jacobian entry the lower half needs
    // from the upper (d cte+ / d v = sin(etheta) dt) crosses by v_permlane32_swap.  Same
    // per-quantity formulas as the unsplit sweep (stats()); the stage-table entries are
    // written by the half-wave that computes them.
    MPCG_HD void stats_split(bool acc, T alpha, T amax_z) {
        const int t = wv.lane();
        accept_all(t, acc, alpha, amax_z);
        const bool reuse = acc && c_ok;  // (uniform)
        c_ok = 0;
        const int k = t & 31;
        const bool hi = t >= 32, act = k < N, last = k == N - 1;
        const int j0 = hi ? 4 : 0, nr = hi ? 2 : 4;
        T f = 0, th = 0, pinf = 0, puns = 0, dinf = 0, mn = (T)INFINITY, mx = -(T)INFINITY, ly = 0, lz = 0,
          lg = 0;
        T Fa[4] = {0, 0, 0, 0}, A[4] = {0, 0, 0, 0};
        T w[8], zl[4], zu[4], yq[4], yn[6] = {0, 0, 0, 0, 0, 0}, up[2] = {0, 0}, um[2] = {0, 0};
        T twk = dt, tvk = 0, f1 = 0;
        if (act) {
            ldn<8>(L.W(k), w);
            ldv<4>(L.ZL(k) + j0, zl);
            ldv<4>(L.ZU(k) + j0, zu);
            ldv<4>(L.Y(k) + j0, yq);  // (upper half: y4, y5 and two unused entries)
            const int sb = L.ST(k);
            T cv[3] = {0, 0, 0};
            if (!last) {
                ldn<6>(L.Y(k + 1), yn);
                up[0] = ld(L.W(k + 1) + 6);
                up[1] = ld(L.W(k + 1) + 7);
                T sa, ca;
                if (reuse) {
                    sa = c_sa;
                    ca = c_ca;
                } else {
                    sc_t(hi ? w[5] : w[2], &sa, &ca);
                }
                const T x = w[0], v = w[3];
                const C4 pcoef_ = pcoef();
                const T fx = pcoef_.c[0] + pcoef_.c[1] * x + pcoef_.c[2] * (x * x) + pcoef_.c[3] * (x * x * x);
                f1 = pcoef_.c[1] + (T)2 * pcoef_.c[2] * x + (T)3 * pcoef_.c[3] * x * x;
                const T f2 = (T)2 * pcoef_.c[2] + (T)6 * pcoef_.c[3] * x;
                // Lin::jac: lower a0..a3 (x, y rows), upper a4..a6 (cte row)
                A[0] = hi ? f1 : -w[3] * sa * dt;
                A[1] = hi ? sa * dt : ca * dt;
                A[2] = w[3] * ca * dt;
                A[3] = sa * dt;
                // next_m: lower rows 0..3, upper rows 4, 5
                T turn = w[6] * dt;
                if (model == 1) turn = w[3] * w[6] / lf * dt;
                Fa[0] = (hi ? fx - w[1] : w[0]) + w[3] * (hi ? sa : ca) * dt;
                Fa[1] = hi ? (model == 1 ? w[5] + turn : w[5] + w[6] * dt) : w[1] + w[3] * sa * dt;
                Fa[2] = model == 1 ? w[2] + turn : w[2] + w[6] * dt;
                Fa[3] = w[3] + w[7] * dt;
                turn_d(w, w + 6, &twk, &tvk);
                // constraint curvature: lower Q22 Q32, upper Q00 Q55 Q53
                cv[0] = hi ? -yn[4] * f2 : yn[0] * v * ca * dt + yn[1] * v * sa * dt;
                cv[1] = hi ? yn[4] * v * sa * dt : yn[0] * sa * dt - yn[1] * ca * dt;
                cv[2] = -yn[4] * ca * dt;
                T wn[4];
                ldv<4>(L.W(k + 1) + j0, wn);
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    if (q < nr) st(sb + WideLayout::SD + j0 + q, Fa[q] - wn[q]);
            }
            const int na = hi ? 3 : 4;
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (q < na) st(sb + WideLayout::SA + j0 + q, A[q]);
            if (hi) {
                st(sb + WideLayout::SCV + 0, cv[0]);
                st(sb + WideLayout::SCV + 3, cv[1]);
                st(sb + WideLayout::SCV + 4, cv[2]);
            } else {
                st(sb + WideLayout::SCV + 1, cv[0]);
                st(sb + WideLayout::SCV + 2, cv[1]);
            }
            if constexpr (MODEL == 1) {
                if (!hi) {
                    st(sb + WideLayout::STW, twk);
                    st(sb + WideLayout::STV, tvk);
                    st(sb + WideLayout::SHVD, last ? (T)0 : -(yn[2] + yn[5]) / lf * dt);
                }
            }
            if (k >= 1) {
                um[0] = ld(L.W(k - 1) + 6);
                um[1] = ld(L.W(k - 1) + 7);
            }
        }
        // d cte+ / d v of the upper half-wave for the lower half's (A^T yn)[3]
        T a5own, a5;
        wv.xor32_pair(A[1], a5own, a5);
        T Fprev[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) Fprev[q] = wv.up1(Fa[q]);
        if (act) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if (q < nr) {
                    const int j = j0 + q;
                    const T wj = hi ? w[4 + q] : w[q];
                    const T c = k == 0 ? wj - pinit(hi ? 4 + q : q) : wj - Fprev[q];
                    if (k == 0) st(L.C0() + j, -c);  // initial-state rows of the Newton system
                    const T rsc = rowscale(j, k);
                    const T cs = rsc * c;
                    th += fabs(cs);
                    pinf = tmax(pinf, (T)fabs(cs));
                    puns = tmax(puns, (T)fabs(c));
                    ly += fabs(yq[q]) * rcp(rsc);
                }
            }
            const T e1 = w[4] - (T)P.ref_cte, e2 = w[5] - (T)P.ref_eth, e3 = w[3] - (T)P.ref_v;
            T fu = (T)P.w_cte * e1 * e1 + (T)P.w_eth * e2 * e2;
            // gradient of the Lagrangian's constraint part, A^T yn (AT_mul) and B^T yn
            T at[4] = {0, 0, 0, 0}, gu[2] = {0, 0};
            if (!last) {
                if (hi) {
                    at[1] = A[2] * yn[4] + yn[5];  // (A^T yn)[5] = a6 yn4 + yn5
                } else {
                    at[0] = yn[0] + f1 * yn[4];
                    at[1] = yn[1] - yn[4];
                    at[2] = A[0] * yn[0] + A[2] * yn[1] + yn[2];
                    at[3] = A[1] * yn[0] + A[3] * yn[1] + yn[3] + a5 * yn[4];
                    if (model == 1) at[3] += tvk * (yn[2] + yn[5]);
                }
                grad_ctrl(k, um, w + 6, up, gu);
                fu += cost_ctrl(k, w + 6, up);
            }
            f = hi ? fu : (T)P.w_v * e3 * e3;
            const T btw = twk * (yn[2] + yn[5]), bta = dt * yn[3];
            // the objective gradient of this half's variables (scaled): g3 / g4, g5, gu
            const T g3 = (T)(2.0 * P.w_v) * (w[3] - (T)P.ref_v);
            const T g4 = (T)(2.0 * P.w_cte) * (w[4] - (T)P.ref_cte), g5 = (T)(2.0 * P.w_eth) * (w[5] - (T)P.ref_eth);
            const int nv = (last && hi) ? 2 : 4;
            T slackprod = 1;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if (q < nv) {
                    const T wq = hi ? w[4 + q] : w[q];
                    T gj;
                    if (q < 2)
                        gj = hi ? sf * (q == 0 ? g4 : g5) + yq[q] - at[q] : sf * (T)0 + yq[q] - at[q];
                    else
                        gj = hi ? sf * gu[q - 2] - (q == 2 ? btw : bta) : (q == 2 ? sf * (T)0 : sf * g3) + yq[q] - at[q];
                    const T rd = gj - zl[q] + zu[q];
                    dinf = tmax(dinf, (T)fabs(rd));
                    const T lo = q < 2 ? sl : (q == 2 ? (hi ? wl : sl) : (hi ? al : sl));
                    const T hb = q < 2 ? su : (q == 2 ? (hi ? wu : su) : (hi ? au : su));
                    const T dl = wq - lo, du = hb - wq;
                    slackprod *= dl * du;
                    const T p1 = dl * zl[q], p2 = du * zu[q];
                    mn = tmin(mn, tmin(p1, p2));
                    mx = tmax(mx, tmax(p1, p2));
                    lz += fabs(zl[q]) + fabs(zu[q]);
                }
            }
            lg = log(slackprod);
        }
        // (max |z s| = max(max z s, -min z s): one reduction fewer)
        T v[10] = {f, th, pinf, puns, dinf, mn, mx, ly, lz, lg};
        const int op[10] = {RSUM, RSUM, RMAX, RMAX, RMAX, RMIN, RMAX, RSUM, RSUM, RSUM};
        reduce<10, true>(v, op);
        fval = v[0];
        theta = v[1];
        prim_inf = v[2];
        prim_uns = v[3];
        dual_inf = v[4];
        pmin = v[5];
        pmax = v[6];
        compl0 = wv.uni_d(tmax(pmax, -pmin));
        l1y = v[7];
        l1z = v[8];
        logsum = v[9];
        wv.mark(0);
    }

    MPCG_HD void stats(bool acc, T alpha, T amax_z) {
        if constexpr (RESTO) {
            stats_resto(acc, alpha, amax_z);
            return;
        }
        if constexpr (SPLIT) {
            stats_split(acc, alpha, amax_z);
            return;
        }
        if constexpr (NB == 2) {
            stats_blk(acc, alpha, amax_z);
            return;
        }
        const int t = wv.lane();  // (recomputed per phase: nothing lane-dependent is hoisted)
        accept_all(t, acc, alpha, amax_z);
        T f = 0, th = 0, pinf = 0, puns = 0, dinf = 0, c0 = 0, mn = (T)INFINITY, mx = -(T)INFINITY, ly = 0, lz = 0,
          lg = 0;
        T Fk[6] = {0, 0, 0, 0, 0, 0};
        T w[8], zl[8], zu[8], y[6], yn[6] = {0, 0, 0, 0, 0, 0}, up[2] = {0, 0}, um[2] = {0, 0}, a[7];
        T twk = dt, tvk = 0, hvdk = 0;
        const int k = t;
        const bool act = t < N, last = k == N - 1;
        if (act) {
            ldn<8>(L.W(k), w);
            ldn<8>(L.ZL(k), zl);
            ldn<8>(L.ZU(k), zu);
            ldn<6>(L.Y(k), y);
            // linearisation at the iterate, kept in the stage table for the Newton
            // system of this iteration (precompute): A_k, F(s_k, u_k) and the constraint
            // curvature weighted by the new multipliers of rows k+1
            T cvk[5] = {0, 0, 0, 0, 0};
            twk = dt;
            tvk = 0;
            hvdk = 0;
            if (!last) {
                ldn<6>(L.Y(k + 1), yn);
                up[0] = ld(L.W(k + 1) + 6);
                up[1] = ld(L.W(k + 1) + 7);
                Lin<T> ln;
                ln.eval(pcoef().c, w);
                ln.jac(w, dt, a);
                next_m(ln, w, w + 6, Fk);
                turn_d(w, w + 6, &twk, &tvk);
                if (model == 1) hvdk = -(yn[2] + yn[5]) / lf * dt;
                const T v = w[3];
                cvk[0] = -yn[4] * ln.f2;                                   // Q00
                cvk[1] = yn[0] * v * ln.ct * dt + yn[1] * v * ln.st * dt;  // Q22
                cvk[2] = yn[0] * ln.st * dt - yn[1] * ln.ct * dt;          // Q32
                cvk[3] = yn[4] * v * ln.se * dt;                           // Q55
                cvk[4] = -yn[4] * ln.ce * dt;                              // Q53
            } else {
#pragma unroll
                for (int j = 0; j < 7; ++j) a[j] = 0;
            }
            const int sb = L.ST(k);
#pragma unroll
            for (int j = 0; j < 7; ++j) st(sb + WideLayout::SA + j, a[j]);
            if (!last) {
                T wn[6];
                ldn<6>(L.W(k + 1), wn);
#pragma unroll
                for (int j = 0; j < 6; ++j) st(sb + WideLayout::SD + j, Fk[j] - wn[j]);
            }
#pragma unroll
            for (int j = 0; j < 5; ++j) st(sb + WideLayout::SCV + j, cvk[j]);
            if constexpr (MODEL == 1) {
                st(sb + WideLayout::STW, twk);
                st(sb + WideLayout::STV, tvk);
                st(sb + WideLayout::SHVD, hvdk);
            }
            if (k >= 1) {
                um[0] = ld(L.W(k - 1) + 6);
                um[1] = ld(L.W(k - 1) + 7);
            }
        }
        T Fprev[6];
#pragma unroll
        for (int j = 0; j < 6; ++j) Fprev[j] = wv.up1(Fk[j]);
        if (act) {
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                const T c = k == 0 ? w[j] - pinit(j) : w[j] - Fprev[j];
                if (k == 0) st(L.C0() + j, -c);  // initial-state rows of the Newton system
                const T rsc = rowscale(j, k);
                const T cs = rsc * c;
                th += fabs(cs);
                pinf = tmax(pinf, (T)fabs(cs));
                puns = tmax(puns, (T)fabs(c));
                ly += fabs(y[j]) * rcp(rsc);
            }
            f = cost_state(w);
            T g[6], at[6] = {0, 0, 0, 0, 0, 0}, gu[2] = {0, 0};
            grad_state(w, g);
            if (!last) {
                AT_mul(a, yn, at);
                if (model == 1) at[3] += tvk * (yn[2] + yn[5]);
                grad_ctrl(k, um, w + 6, up, gu);
                f += cost_ctrl(k, w + 6, up);
            }
            const T btw = twk * (yn[2] + yn[5]), bta = dt * yn[3];
            const int nv = last ? 6 : 8;
            T slackprod = 1;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                if (j < nv) {
                    const T gj = j < 6 ? sf * g[j] + y[j] - at[j] : sf * gu[j - 6] - (j == 6 ? btw : bta);
                    const T rd = gj - zl[j] + zu[j];
                    dinf = tmax(dinf, (T)fabs(rd));
                    const T dl = w[j] - vlo(j), du = vhi(j) - w[j];
                    slackprod *= dl * du;
                    const T p1 = dl * zl[j], p2 = du * zu[j];
                    c0 = tmax(c0, tmax((T)fabs(p1), (T)fabs(p2)));
                    mn = tmin(mn, tmin(p1, p2));
                    mx = tmax(mx, tmax(p1, p2));
                    lz += fabs(zl[j]) + fabs(zu[j]);
                }
            }
            lg = log(slackprod);
        }
        T v[11] = {f, th, pinf, puns, dinf, c0, mn, mx, ly, lz, lg};
        const int op[11] = {RSUM, RSUM, RMAX, RMAX, RMAX, RMAX, RMIN, RMAX, RSUM, RSUM, RSUM};
        reduce<11>(v, op);
        fval = v[0];
        theta = v[1];
        prim_inf = v[2];
        prim_uns = v[3];
        dual_inf = v[4];
        compl0 = v[5];
        pmin = v[6];
        pmax = v[7];
        l1y = v[8];
        l1z = v[9];
        logsum = v[10];
        wv.mark(0);
    }


    // ------------------------------------------------------- two stage blocks (N > 64)
    // The statistics sweep of stats() for lane t's stages t and 64 + t: stage data and
    // F(s_k, u_k) of both blocks first, then the shift of F to stage k + 1 (stage 63 ->
    // 64 by a lane read), then the statistics (the lane's values reloaded from LDS).
    MPCG_HD void stats_blk(bool acc, T alpha, T amax_z) {
        const int t = wv.lane();
        accept_all(t, acc, alpha, amax_z);
        T f = 0, th = 0, pinf = 0, puns = 0, dinf = 0, c0 = 0, mn = (T)INFINITY, mx = -(T)INFINITY, ly = 0, lz = 0,
          lg = 0;
        T Fk[NB][6];
        for (int b = 0; b < NB; ++b) {
            const int k = t + 64 * b;
#pragma unroll
            for (int j = 0; j < 6; ++j) Fk[b][j] = 0;
            if (k < N) {
                const bool last = k == N - 1;
                T w[8], yn[6] = {0, 0, 0, 0, 0, 0}, a[7] = {0, 0, 0, 0, 0, 0, 0}, cvk[5] = {0, 0, 0, 0, 0};
                T twk = dt, tvk = 0, hvdk = 0;
                ldn<8>(L.W(k), w);
                if (!last) {
                    ldn<6>(L.Y(k + 1), yn);
                    Lin<T> ln;
                    ln.eval(pcoef().c, w);
                    ln.jac(w, dt, a);
                    next_m(ln, w, w + 6, Fk[b]);
                    turn_d(w, w + 6, &twk, &tvk);
                    if (model == 1) hvdk = -(yn[2] + yn[5]) / lf * dt;
                    const T v = w[3];
                    cvk[0] = -yn[4] * ln.f2;
                    cvk[1] = yn[0] * v * ln.ct * dt + yn[1] * v * ln.st * dt;
                    cvk[2] = yn[0] * ln.st * dt - yn[1] * ln.ct * dt;
                    cvk[3] = yn[4] * v * ln.se * dt;
                    cvk[4] = -yn[4] * ln.ce * dt;
                }
                const int sb = L.ST(k);
#pragma unroll
                for (int j = 0; j < 7; ++j) st(sb + WideLayout::SA + j, a[j]);
                if (!last) {
                    T wn[6];
                    ldn<6>(L.W(k + 1), wn);
#pragma unroll
                    for (int j = 0; j < 6; ++j) st(sb + WideLayout::SD + j, Fk[b][j] - wn[j]);
                }
#pragma unroll
                for (int j = 0; j < 5; ++j) st(sb + WideLayout::SCV + j, cvk[j]);
                if constexpr (MODEL == 1) {
                    st(sb + WideLayout::STW, twk);
                    st(sb + WideLayout::STV, tvk);
                    st(sb + WideLayout::SHVD, hvdk);
                }
            }
        }
        T Fprev[NB][6];
        shift_blocks(Fk, Fprev);
        wv.sync();
        for (int b = 0; b < NB; ++b) {
            const int k = t + 64 * b;
            if (k >= N) continue;
            const bool last = k == N - 1;
            T w[8], zl[8], zu[8], y[6], yn[6] = {0, 0, 0, 0, 0, 0}, up[2] = {0, 0}, um[2] = {0, 0}, a[8];
            ldn<8>(L.W(k), w);
            ldn<8>(L.ZL(k), zl);
            ldn<8>(L.ZU(k), zu);
            ldn<6>(L.Y(k), y);
            ldn<7>(L.ST(k) + WideLayout::SA, a);
            T twk = dt, tvk = 0;
            if constexpr (MODEL == 1) {
                twk = ld(L.ST(k) + WideLayout::STW);
                tvk = ld(L.ST(k) + WideLayout::STV);
            }
            if (!last) {
                ldn<6>(L.Y(k + 1), yn);
                up[0] = ld(L.W(k + 1) + 6);
                up[1] = ld(L.W(k + 1) + 7);
            }
            if (k >= 1) {
                um[0] = ld(L.W(k - 1) + 6);
                um[1] = ld(L.W(k - 1) + 7);
            }
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                const T c = k == 0 ? w[j] - pinit(j) : w[j] - Fprev[b][j];
                if (k == 0) st(L.C0() + j, -c);
                const T rsc = rowscale(j, k);
                const T cs = rsc * c;
                th += fabs(cs);
                pinf = tmax(pinf, (T)fabs(cs));
                puns = tmax(puns, (T)fabs(c));
                ly += fabs(y[j]) * rcp(rsc);
            }
            f += cost_state(w);
            T g[6], at[6] = {0, 0, 0, 0, 0, 0}, gu[2] = {0, 0};
            grad_state(w, g);
            if (!last) {
                AT_mul(a, yn, at);
                if (model == 1) at[3] += tvk * (yn[2] + yn[5]);
                grad_ctrl(k, um, w + 6, up, gu);
                f += cost_ctrl(k, w + 6, up);
            }
            const T btw = twk * (yn[2] + yn[5]), bta = dt * yn[3];
            const int nv = last ? 6 : 8;
            T slackprod = 1;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                if (j < nv) {
                    const T gj = j < 6 ? sf * g[j] + y[j] - at[j] : sf * gu[j - 6] - (j == 6 ? btw : bta);
                    const T rd = gj - zl[j] + zu[j];
                    dinf = tmax(dinf, (T)fabs(rd));
                    const T dl = w[j] - vlo(j), du = vhi(j) - w[j];
                    slackprod *= dl * du;
                    const T p1 = dl * zl[j], p2 = du * zu[j];
                    c0 = tmax(c0, tmax((T)fabs(p1), (T)fabs(p2)));
                    mn = tmin(mn, tmin(p1, p2));
                    mx = tmax(mx, tmax(p1, p2));
                    lz += fabs(zl[j]) + fabs(zu[j]);
                }
            }
            lg += log(slackprod);
        }
        T v[11] = {f, th, pinf, puns, dinf, c0, mn, mx, ly, lz, lg};
        const int op[11] = {RSUM, RSUM, RMAX, RMAX, RMAX, RMAX, RMIN, RMAX, RSUM, RSUM, RSUM};
        reduce<11, true>(v, op);
        fval = v[0];
        theta = v[1];
        prim_inf = v[2];
        prim_uns = v[3];
        dual_inf = v[4];
        compl0 = v[5];
        pmin = v[6];
        pmax = v[7];
        l1y = v[8];
        l1z = v[9];
        logsum = v[10];
        wv.mark(0);
    }
    // F of stage k to lane k + 1 over both blocks: DPP shift within a block, lane 63 of
    // block b - 1 to lane 0 of block b
    MPCG_HD void shift_blocks(const T (&Fk)[NB][6], T (&Fprev)[NB][6]) const {
        const int t = wv.lane();
        for (int b = 0; b < NB; ++b) {
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                T v = wv.up1(Fk[b][j]);
                if (b > 0) {
                    const T c = wv.lane63(Fk[b - 1][j]);
                    v = t == 0 ? c : v;
                }
                Fprev[b][j] = v;
            }
        }
    }

    // trial() for two stage blocks
    MPCG_HD bool trial_blk(T alpha, T* phi, T* th) {
        const int t = wv.lane();
        T f = 0, thv = 0, lg = 0;
        int bad = 0;
        T Fk[NB][6];
        for (int b = 0; b < NB; ++b) {
            const int k = t + 64 * b;
#pragma unroll
            for (int j = 0; j < 6; ++j) Fk[b][j] = 0;
            if (k >= N) continue;
            const bool last = k == N - 1;
            T cw[8], cd[8], w[8];
            ldn<8>(L.W(k), cw);
            ldn<8>(L.DW(k), cd);
#pragma unroll
            for (int j = 0; j < 8; ++j) w[j] = cw[j] + alpha * cd[j];
            const int nv = last ? 6 : 8;
            T slackprod = 1;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                if (j < nv) {
                    const T dl = w[j] - vlo(j), du = vhi(j) - w[j];
                    bad |= !((dl > 0) && (du > 0));
                    slackprod *= dl * du;
                }
            }
            lg += log(slackprod);
            f += cost_state(w);
            if (!last) {
                T up[2];
                up[0] = ld(L.W(k + 1) + 6) + alpha * ld(L.DW(k + 1) + 6);
                up[1] = ld(L.W(k + 1) + 7) + alpha * ld(L.DW(k + 1) + 7);
                f += cost_ctrl(k, w + 6, up);
                Lin<T> ln;
                ln.eval(pcoef().c, w);
                next_m(ln, w, w + 6, Fk[b]);
            }
        }
        T Fprev[NB][6];
        shift_blocks(Fk, Fprev);
        for (int b = 0; b < NB; ++b) {
            const int k = t + 64 * b;
            if (k >= N) continue;
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                const T wj = ld(L.W(k) + j) + alpha * ld(L.DW(k) + j);
                const T c = k == 0 ? wj - pinit(j) : wj - Fprev[b][j];
                thv += fabs(rowscale(j, k) * c);
            }
        }
        T v[3] = {f, thv, lg};
        const int op[3] = {RSUM, RSUM, RSUM};
        reduce<3, true>(v, op);
        const bool anybad = wv.any(bad != 0);
        wv.mark(6);
        *phi = sf * v[0] - mu * v[2];
        *th = v[1];
        return !anybad && isfinite((double)*phi);
    }

    // ------------------------------------------------------- Riccati backward
    // Stage data that does not depend on the cost-to-go, all stages in parallel.
    // Stage data of the Newton system (SPLIT): the lower half-wave takes the barrier
    // Hessian diagonal and gradient of stage k's variables 0..3, the upper of 4..7 (the
    // controls' R and r); mode 1's linearisation stays with the lower half.  Same
    // per-variable formulas as the unsplit sweep (precompute()).
    MPCG_HD void precompute_split(int mode, T delta_w) {
        const int t = wv.lane();
        const int k = t & 31;
        const bool hi = t >= 32;
        if (k >= N) return;
        const bool last = k == N - 1;
        const int sb = L.ST(k);
        if (mode == 1 && !hi) {
            T w[8];
            ldn<8>(L.W(k), w);
            T a[7] = {0, 0, 0, 0, 0, 0, 0}, tw = dt, tv = 0;
            if (!last) {
                Lin<T> ln;
                ln.eval(pcoef().c, w);
                ln.jac(w, dt, a);
                turn_d(w, w + 6, &tw, &tv);
            }
#pragma unroll
            for (int j = 0; j < 7; ++j) st(sb + WideLayout::SA + j, a[j]);
            if constexpr (MODEL == 1) {
                st(sb + WideLayout::STW, tw);
                st(sb + WideLayout::STV, tv);
                st(sb + WideLayout::SHVD, 0);
            }
#pragma unroll
            for (int j = 0; j < 6; ++j) st(sb + WideLayout::SD + j, 0);
#pragma unroll
            for (int j = 0; j < 5; ++j) st(sb + WideLayout::SCV + j, 0);
        }
        const int j0 = hi ? 4 : 0;
        T w[4], zl[4], zu[4];
        ldv<4>(L.W(k) + j0, w);
        ldv<4>(L.ZL(k) + j0, zl);
        ldv<4>(L.ZU(k) + j0, zu);
        T gu[2] = {0, 0};
        if (!last) {
            T um[2] = {0, 0}, up[2];
            if (k >= 1) {
                um[0] = ld(L.W(k - 1) + 6);
                um[1] = ld(L.W(k - 1) + 7);
            }
            up[0] = ld(L.W(k + 1) + 6);
            up[1] = ld(L.W(k + 1) + 7);
            grad_ctrl(k, um, w + 2, up, gu);  // (upper half: w + 2 = variables 6, 7)
        }
        const T g3 = (T)(2.0 * P.w_v) * (w[3] - (T)P.ref_v);
        const T g4 = (T)(2.0 * P.w_cte) * (w[0] - (T)P.ref_cte), g5 = (T)(2.0 * P.w_eth) * (w[1] - (T)P.ref_eth);
        const int nv = (last && hi) ? 2 : 4;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            T qd = 0, qv = 0;
            if (q < nv) {
                const T gq = hi ? (q == 0 ? g4 : (q == 1 ? g5 : gu[q - 2])) : (q == 3 ? g3 : (T)0);
                const T hq = hi ? (q < 2 ? hess_state(4 + q) : hess_ctrl(k, q - 2)) : hess_state(q);
                const T lo = q < 2 ? sl : (q == 2 ? (hi ? wl : sl) : (hi ? al : sl));
                const T hb = q < 2 ? su : (q == 2 ? (hi ? wu : su) : (hi ? au : su));
                if (mode == 0) {
                    const T rdl = rcp(w[q] - lo), rdu = rcp(hb - w[q]);
                    qd = sf * hq + zl[q] * rdl + zu[q] * rdu + delta_w;
                    qv = sf * gq - mu * rdl + mu * rdu;
                } else {
                    qd = 1;
                    qv = sf * gq - zl[q] + zu[q];
                }
            }
            // (the last stage's controls: R = r = 0)
            st(sb + WideLayout::SQD + j0 + q, qd);
            st(sb + WideLayout::SQV + j0 + q, qv);
        }
    }

    MPCG_HD void precompute(int mode, T delta_w) {
        if constexpr (RESTO) {
            const int t = wv.lane();
            for (int b = 0; b < NB; ++b) precompute_resto(t + 64 * b, delta_w);
            wv.gsync();  // (the rows' D, written to HBM per stage, are read by every lane of the Riccati sweep)
            return;
        }
        if constexpr (SPLIT) {
            precompute_split(mode, delta_w);
            return;
        }
        const int t = wv.lane();  // (recomputed per phase: nothing lane-dependent is hoisted)
        if constexpr (NB == 2) {
            precompute_stage(t, mode, delta_w);
            precompute_stage(t + 64, mode, delta_w);
            return;
        }
        precompute_stage(t, mode, delta_w);
    }
    MPCG_HD void precompute_stage(int k, int mode, T delta_w) {
        if (k >= N) return;
        const bool last = k == N - 1;
        const int sb = L.ST(k);
        T w[8], zl[8], zu[8];
        ldn<8>(L.W(k), w);
        ldn<8>(L.ZL(k), zl);
        ldn<8>(L.ZU(k), zu);
        T g[6];
        grad_state(w, g);
        // mode 0: A_k, d_k = F(s_k, u_k) - s_{k+1} and the constraint curvature at this
        // iterate were stored by the statistics sweep (stats); mode 1 (least squares)
        // computes A_k and has d = 0, no curvature.
        if (mode == 1) {
            T a[7] = {0, 0, 0, 0, 0, 0, 0}, tw = dt, tv = 0;
            if (!last) {
                Lin<T> ln;
                ln.eval(pcoef().c, w);
                ln.jac(w, dt, a);
                turn_d(w, w + 6, &tw, &tv);
            }
#pragma unroll
            for (int j = 0; j < 7; ++j) st(sb + WideLayout::SA + j, a[j]);
            if constexpr (MODEL == 1) {
                st(sb + WideLayout::STW, tw);
                st(sb + WideLayout::STV, tv);
                st(sb + WideLayout::SHVD, 0);
            }
#pragma unroll
            for (int j = 0; j < 6; ++j) st(sb + WideLayout::SD + j, 0);
#pragma unroll
            for (int j = 0; j < 5; ++j) st(sb + WideLayout::SCV + j, 0);
        }
#pragma unroll
        for (int j = 0; j < 6; ++j) {
            T qd, qv;
            if (mode == 0) {
                const T rdl = rcp(w[j] - sl), rdu = rcp(su - w[j]);
                qd = sf * hess_state(j) + zl[j] * rdl + zu[j] * rdu + delta_w;
                qv = sf * g[j] - mu * rdl + mu * rdu;
            } else {
                qd = 1;
                qv = sf * g[j] - zl[j] + zu[j];
            }
            st(sb + WideLayout::SQD + j, qd);
            st(sb + WideLayout::SQV + j, qv);
        }
        T R[2] = {0, 0}, r[2] = {0, 0};
        if (!last) {
            T um[2] = {0, 0}, up[2], gu[2];
            if (k >= 1) {
                um[0] = ld(L.W(k - 1) + 6);
                um[1] = ld(L.W(k - 1) + 7);
            }
            up[0] = ld(L.W(k + 1) + 6);
            up[1] = ld(L.W(k + 1) + 7);
            grad_ctrl(k, um, w + 6, up, gu);
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                if (mode == 0) {
                    const T rdl = rcp(w[6 + j] - vlo(6 + j)), rdu = rcp(vhi(6 + j) - w[6 + j]);
                    R[j] = sf * hess_ctrl(k, j) + zl[6 + j] * rdl + zu[6 + j] * rdu + delta_w;
                    r[j] = sf * gu[j] - mu * rdl + mu * rdu;
                } else {
                    R[j] = 1;
                    r[j] = sf * gu[j] - zl[6 + j] + zu[6 + j];
                }
            }
        }
        st(sb + WideLayout::SQD + 6, R[0]);
        st(sb + WideLayout::SQD + 7, R[1]);
        st(sb + WideLayout::SQV + 6, r[0]);
        st(sb + WideLayout::SQV + 7, r[1]);
    }

    // Stage-table offset of G[m][s], G = [A_hat cols 0,1,2,3,5 | B_hat cols w,a | d]
    // (s < 0: a zero column).  A_hat = dF/ds with rows 6,7 (u_{k-1}) zero.
    MPCG_HD static int goff(int s, int m) {
        typedef WideLayout W_;
        const int Z = W_::SZERO, O = W_::SONE, A = W_::SA, D = W_::SD;
        // (differential drive: d turn / d w = dt, d turn / d v = 0)
        const int TW = MODEL == 1 ? W_::STW : W_::SDT, TV = MODEL == 1 ? W_::STV : W_::SZERO;
        int o = Z;
        o = (s == 0) ? (m == 0 ? O : (m == 4 ? A + 4 : Z)) : o;
        o = (s == 1) ? (m == 1 ? O : (m == 4 ? W_::SMONE : Z)) : o;
        o = (s == 2) ? (m == 0 ? A + 0 : (m == 1 ? A + 2 : (m == 2 ? O : Z))) : o;
        o = (s == 3) ? (m == 0 ? A + 1 : (m == 1 ? A + 3 : (m == 3 ? O : (m == 4 ? A + 5 : ((m == 2 || m == 5) ? TV : Z))))) : o;
        o = (s == 4) ? (m == 4 ? A + 6 : (m == 5 ? O : Z)) : o;
        // B_hat: w -> tw e2 + tw e5 + e6 (tw = d turn / d w) ; a -> dt e3 + e7
        o = (s == 5) ? ((m == 2 || m == 5) ? TW : (m == 6 ? O : Z)) : o;
        o = (s == 6) ? (m == 3 ? W_::SDT : (m == 7 ? O : Z)) : o;
        o = (s == 7) ? (m < 6 ? D + m : Z) : o;
        return o;
    }
    // slot of augmented-state column j among the A_hat columns of G (-1: zero column)
    MPCG_HD static int aslot(int j) { return j < 4 ? j : (j == 5 ? 4 : -1); }

    // Riccati sweep.  Lane (i, j) owns entry (i, j) of the cost-to-go matrix P (and
    // keeps p_i); P lives only in a 64-entry scratch for the row reads of the next
    // stage: the forward pass needs only the gains, and the multipliers come from the
    // adjoint recursion (forward()).
    MPCG_HD bool riccati(int mode, T delta_w) {
        const int t = wv.lane();  // (recomputed per phase: nothing lane-dependent is hoisted)
        wv.sync();
        precompute(mode, delta_w);
        typedef WideLayout W_;
        const int i = t >> 3, j = t & 7;
        const int si = aslot(i), sj = aslot(j);
        constexpr int MS = WideLayout::MS;
        const int sm = L.SCR(), sp = L.PSC();
        // The stage's G is staged densely (transposed) in the M scratch by the previous
        // stage, each lane copying its entry G[j][i] out of the stage table: a lane then
        // reads G column j and A_hat column i (= G column si) with 16-byte loads off one
        // address each.  An absent A_hat column (si, sj < 0) reads the zero block, so
        // its products vanish without masking.
        const bool hj = sj >= 0, hi = si >= 0;
        const int gj = sm + MS * j, mi = hi ? sm + MS * si : L.ZB(), mj = hj ? sm + MS * sj : L.ZB();
        const int gsrc = goff(i, j);
        // the rate-coupling entries of S_tilde: -sf 2 W_DANGVEL / -sf 2 W_DA on the previous
        // control's columns, the same for every stage (the Newton system, mode 0).  Stage 0
        // has no previous control: its coupling entries act only on K_0's columns 6, 7, which
        // multiply a zero step, and on P_0, which is not used.
        // (the restoration problem's Hessian has no objective terms: no rate coupling)
        const T C0 = (mode == 0 && !RESTO) ? -sf * (T)(2.0 * P.w_dw) : (T)0;
        const T C1 = (mode == 0 && !RESTO) ? -sf * (T)(2.0 * P.w_da) : (T)0;
        const T cc0j = j == 6 ? C0 : (T)0, cc1j = j == 7 ? C1 : (T)0;
        const T cc0i = i == 6 ? C0 : (T)0, cc1i = i == 7 ? C1 : (T)0;
        // the gains' store at ga0 + gak * k: lanes 0..15 K[0][j], K[1][j], lanes 16, 17 k;
        // the other lanes store into their own slot of the G staging, which they
        // overwrite right after
        const int ga0 = t < 18 ? L.KR(0) + t : sm + MS * i + j;
        const int gak = t < 18 ? WideLayout::KS : 0;
        T* const gk = spill + L.SP_KRG() + t;  // (KL = 0: the gain records in the workspace)
        const bool khbm = kr_hbm();
        // (v, w) curvature of the Lagrangian: S_tilde(0, 3) (bicycle; zero otherwise)
        const int hvj = j == 3 ? W_::SHVD : W_::SZERO, hvi = i == 3 ? W_::SHVD : W_::SZERO;
        // Q_hat(i, j): diagonal, constraint curvature
        const int q1 = (i == j && i < 6) ? W_::SQD + i : W_::SZERO;
        int q2 = W_::SZERO;
        q2 = (i == 0 && j == 0) ? W_::SCV + 0 : q2;
        q2 = (i == 2 && j == 2) ? W_::SCV + 1 : q2;
        q2 = ((i == 3 && j == 2) || (i == 2 && j == 3)) ? W_::SCV + 2 : q2;
        q2 = (i == 5 && j == 5) ? W_::SCV + 3 : q2;
        q2 = ((i == 5 && j == 3) || (i == 3 && j == 5)) ? W_::SCV + 4 : q2;
        const int qv = i < 6 ? W_::SQV + i : W_::SZERO;
        wv.sync();
        wv.mark(1);
        // terminal stage
        T Pij, pvi;
        {
            const int sb = L.ST(N - 1);
            Pij = ld(sb + q1);
            pvi = ld(sb + qv);
            st(sp + t, Pij);
            if (N >= 2) st(sm + MS * i + j, ld(L.ST(N - 2) + gsrc));
        }
        bool bad = false;  // a stage's reduced Hessian not positive definite
        for (int k = N - 2; k >= 0; --k) {
            // (RESTO) the soft rows into stage k + 1 absorbed into its cost-to-go first
            if constexpr (RESTO) soft_rows(k + 1, Pij, pvi, bad);
            const int sb = L.ST(k);
            // row i of P' (16-byte reads of the scratch the previous stage wrote) and all
            // P-independent stage data, issued together before anything waits on them
            T pr_[8], g[8], c[8] = {0, 0, 0, 0, 0, 0, 0, 0};
            wv.sync();
            ldv<8>(sp + 8 * i, pr_);
            ldv<8>(gj, g);
            // A_hat column i: rows 0..5 (rows 6, 7 are zero; the differential drive's own
            // entry is row i itself, the bicycle's heading-rate terms rows 2 and 5)
            ldv<6>(mi, c);
            const T gnext = ld(L.ST(k > 0 ? k - 1 : 0) + gsrc);  // next stage's G entry
            T qd6, qd7, qv6, qv7;
            ld2(sb + W_::SQD + 6, qd6, qd7);
            ld2(sb + W_::SQV + 6, qv6, qv7);
            const T qh1 = ld(sb + q1), qh2 = ld(sb + q2);
            const T qvi = ld(sb + qv);
            T hv0j = 0, hv0i = 0;
            if constexpr (MODEL == 1) {
                hv0j = ld(sb + hvj);
                hv0i = ld(sb + hvi);
            }
            const T tw = model == 1 ? ld(sb + W_::STW) : dt;
            wv.sched_fence();  // (nothing above consumes a load: no wait here)
            // M = P' G, entry (i, j) per lane; column 7 adds p' (h = P' d + p')
            T m0 = (j == 7) ? pvi : (T)0, m1 = 0;
#pragma unroll
            for (int q = 0; q < 8; q += 2) {
                m0 += pr_[q] * g[q];
                m1 += pr_[q + 1] * g[q + 1];
            }
            wv.sync();  // the previous stage's reads of M are done
            st(sm + MS * j + i, m0 + m1);
            wv.sync();
            // columns of M: sj and 7 (all rows), B_hat rows (2,3,5,6,7) of 5, 6 and si
            T mc[8], m7[8];
            ldv<8>(mj, mc);
            ldv<8>(sm + MS * 7, m7);
            const T m25 = ld(sm + MS * 5 + 2), m55 = ld(sm + MS * 5 + 5), m65 = ld(sm + MS * 5 + 6);
            const T m26 = ld(sm + MS * 6 + 2), m36 = ld(sm + MS * 6 + 3), m56 = ld(sm + MS * 6 + 5),
                    m66 = ld(sm + MS * 6 + 6), m76 = ld(sm + MS * 6 + 7);
            const T mi2 = ld(mi + 2), mi3 = ld(mi + 3), mi5 = ld(mi + 5), mi6 = ld(mi + 6), mi7 = ld(mi + 7);

            // R_tilde = R + B^T P' B, r_tilde = r + B^T h, S_tilde = B^T P' A (+ rate coupling)
            const T Rt00 = qd6 + (tw * (m25 + m55) + m65);
            const T Rt01 = tw * (m26 + m56) + m66;
            const T Rt11 = qd7 + (dt * m36 + m76);
            const T det = Rt00 * Rt11 - Rt01 * Rt01;
            bad = bad || !(Rt00 > 0) || !(det > (T)(sizeof(T) == 4 ? 1e-6 : 1e-14) * Rt00 * Rt11);
            const T rt0 = qv6 + (tw * (m7[2] + m7[5]) + m7[6]);
            const T rt1 = qv7 + (dt * m7[3] + m7[7]);
            const T rdet = rcp(det);
            const T i00 = Rt11 * rdet, i01 = -Rt01 * rdet, i11 = Rt00 * rdet;
            // (an absent column contributes exact zeros; the coupling entries are zero
            // on the A_hat columns)
            T s0j = tw * (mc[2] + mc[5]) + mc[6] + cc0j;
            const T s1j = dt * mc[3] + mc[7] + cc1j;
            T s0i = tw * (mi2 + mi5) + mi6 + cc0i;
            const T s1i = dt * mi3 + mi7 + cc1i;
            if constexpr (MODEL == 1) {
                s0j += hv0j;
                s0i += hv0i;
            }
            const T K0 = -(i00 * s0j + i01 * s1j);
            const T K1 = -(i01 * s0j + i11 * s1j);
            const T kf0 = -(i00 * rt0 + i01 * rt1);
            const T kf1 = -(i01 * rt0 + i11 * rt1);
            // (A_hat^T M)(i, j) and (A_hat^T h)(i)
            T a0 = 0, a1 = 0, h0 = 0, h1 = 0;
#pragma unroll
            for (int q = 0; q < 6; q += 2) {
                a0 += c[q] * mc[q];
                a1 += c[q + 1] * mc[q + 1];
                h0 += c[q] * m7[q];
                h1 += c[q + 1] * m7[q + 1];
            }
            const T qh = qh1 + qh2;
            Pij = qh + (a0 + a1) + s0i * K0 + s1i * K1;
            pvi = qvi + (h0 + h1) + s0i * kf0 + s1i * kf1;
            st(sp + t, Pij);
            wv.sync();  // this stage's reads of M are done
            // gains K (lanes 0..15: K[0][j], K[1][j]) and k (lanes 16, 17) in one store (the
            // other lanes' store lands in the G slot the next store overwrites)
            if (khbm) {
                if (t < 18) gk[WideLayout::KS * k] = i == 0 ? K0 : (i == 1 ? K1 : (j == 0 ? kf0 : kf1));
            } else {
                st(ga0 + gak * k, i == 0 ? K0 : (i == 1 ? K1 : (j == 0 ? kf0 : kf1)));
            }
            st(sm + MS * i + j, gnext);
        }
        if constexpr (RESTO) {
            soft_rows(0, Pij, pvi, bad);  // the initial-state rows (soft as well)
            wv.gsync();                   // (the gains M, m in HBM are read by other lanes in forward())
        }
        // a failed inertia test anywhere (the stages after it computed values the retry overwrites)
        if (wv.uni(bad)) {
            wv.mark(2);
            return false;
        }
        wv.mark(2);
        return true;
    }

    // -------------------------------------------------------- forward pass
    struct Fwd {
        T amax_p, amax_z, gd, rel;
    };
    MPCG_HD void dir_var(T w, T zl, T zu, T lo, T hi, T gphi, T dwv, Fwd& F) const {
        dir_var_r(w, zl, zu, lo, hi, gphi, dwv, rcp(w - lo), rcp(hi - w), F);
    }
    // (with the reciprocal slacks rdl = rcp(w - lo), rdu = rcp(hi - w) given)
    MPCG_HD void dir_var_r(T w, T zl, T zu, T lo, T hi, T gphi, T dwv, T rdl, T rdu, Fwd& F) const {
        const T dl = w - lo, du = hi - w;
        const T rdw = rcp(dwv);
        const T inf = (T)INFINITY;
        F.amax_p = tmin(F.amax_p, dwv < 0 ? -tau * dl * rdw : (dwv > 0 ? tau * du * rdw : inf));
        const T dzl = mu * rdl - zl - zl * rdl * dwv;
        const T dzu = mu * rdu - zu + zu * rdu * dwv;
        F.amax_z = tmin(F.amax_z, dzl < 0 ? -tau * zl * rcp(dzl) : inf);
        F.amax_z = tmin(F.amax_z, dzu < 0 ? -tau * zu * rcp(dzu) : inf);
        F.gd += gphi * dwv;
        F.rel = tmax(F.rel, (T)fabs(dwv) * rcp((T)1 + (T)fabs(w)));
    }

    // Step statistics of stage k (SPLIT): the lower half-wave takes variables 0..3 (x, y,
    // theta, v), the upper 4..7 (cte, etheta, w, a); same per-variable formulas as the
    // unsplit sweep below (gradient of the barrier function, dir_var).
    MPCG_HD void step_stats_split(int k, const T* xk, const T* duk, Fwd& F) const {
        const int t = wv.lane();  // (recomputed per phase: nothing lane-dependent is hoisted)
        const bool hi = t >= 32, last = k == N - 1;
        const int j0 = hi ? 4 : 0;
        T w[4], zl[4], zu[4];
        ldv<4>(L.W(k) + j0, w);
        ldv<4>(L.ZL(k) + j0, zl);
        ldv<4>(L.ZU(k) + j0, zu);
        // gradient of the objective (scaled): g[3] (lower) / g[4], g[5], gu (upper)
        T gu[2] = {0, 0};
        if (!last) {
            T um[2] = {0, 0}, up[2];
            if (k >= 1) {
                um[0] = ld(L.W(k - 1) + 6);
                um[1] = ld(L.W(k - 1) + 7);
            }
            up[0] = ld(L.W(k + 1) + 6);
            up[1] = ld(L.W(k + 1) + 7);
            const T u[2] = {w[2], w[3]};  // (upper half: variables 6, 7)
            grad_ctrl(k, um, u, up, gu);
        }
        const T g4 = (T)(2.0 * P.w_cte) * (w[0] - (T)P.ref_cte), g5 = (T)(2.0 * P.w_eth) * (w[1] - (T)P.ref_eth);
        const T g3 = (T)(2.0 * P.w_v) * (w[3] - (T)P.ref_v);
        const T gq[4] = {hi ? sf * g4 : sf * (T)0, hi ? sf * g5 : sf * (T)0, hi ? sf * gu[0] : sf * (T)0,
                         hi ? sf * gu[1] : sf * g3};
        const T dq[4] = {hi ? xk[4] : xk[0], hi ? xk[5] : xk[1], hi ? duk[0] : xk[2], hi ? duk[1] : xk[3]};
        const T lo2 = hi ? wl : sl, hi2 = hi ? wu : su, lo3 = hi ? al : sl, hi3 = hi ? au : su;
        const int nv = (last && hi) ? 2 : 4;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if (q < nv) {
                const T lo = q < 2 ? sl : (q == 2 ? lo2 : lo3), up_ = q < 2 ? su : (q == 2 ? hi2 : hi3);
                const T rdl = rcp(w[q] - lo), rdu = rcp(up_ - w[q]);
                const T gphi = gq[q] - mu * rdl + mu * rdu;
                dir_var_r(w[q], zl[q], zu[q], lo, up_, gphi, dq[q], rdl, rdu, F);
            }
        }
    }

    // the gain records are in the workspace (WideLayout::KL = 0; never for the diff-drive's
    // split instances, N <= 32)
    MPCG_HD bool kr_hbm() const {
        if constexpr (MODEL == 0 && SPLIT)
            return false;
        else
            return L.KL == 0;
    }
    // stage k's gains K (2 x 8) and k_ff, written by the Riccati sweep: LDS, or the workspace,
    // ordered after the sweep's stores by forward_begin()
    MPCG_HD void ld_gains(int k, T* K, T* kf) const {
        if (kr_hbm()) {
            const T* g = spill + L.SP_KRG() + WideLayout::KS * k;
#pragma unroll
            for (int q = 0; q < 16; ++q) K[q] = g[q];
            kf[0] = g[WideLayout::KF];
            kf[1] = g[WideLayout::KF + 1];
        } else {
            ldv<16>(L.KR(k), K);
            ldv<2>(L.KR(k) + WideLayout::KF, kf);
        }
    }
    MPCG_HD void forward_begin() const {
        wv.sync();
        if (kr_hbm()) wv.gsync();  // (the gain records: written by other lanes)
    }

    MPCG_HD Fwd forward(int mode) {
        if constexpr (RESTO) return forward_resto();
        if constexpr (NB == 2) return forward_blk(mode);
        const int t = wv.lane();  // (recomputed per phase: nothing lane-dependent is hoisted)
        forward_begin();
        // The step recursion ds_{k+1} = A ds_k + B du_k + d, du_k = kff + K ds_k runs
        // systolically: lane k holds stage k's records, every step every lane applies its
        // own stage map to the vector it holds and passes the result one lane up.  Lane 0
        // keeps its input (no lane below it); after step s lanes 0..s+1 hold their correct
        // inputs, and a lane whose input is correct recomputes the same output (bitwise)
        // at every later step, so nothing needs masking.  (SPLIT: the recursion is correct
        // in the lower half-wave; lane 32 takes lane 31's output, so the upper half's
        // values are replaced by the lower half's after the loop.)
        const int ks = SPLIT ? (t & 31) : t;  // the lane's stage
        T K[16], kf[2], a[8], d[6], twl = 0, tvl = 0;
        if (ks < N - 1) {
            ld_gains(ks, K, kf);
            ldv<8>(L.ST(ks) + WideLayout::SA, a);
            ldv<6>(L.ST(ks) + WideLayout::SD, d);
            if constexpr (MODEL == 1)
                ld2(L.ST(ks) + WideLayout::STW, twl, tvl);
            else
                twl = dt;
        } else {  // last stage (and idle lanes): no control, du = 0
#pragma unroll
            for (int q = 0; q < 16; ++q) K[q] = 0;
            kf[0] = 0;
            kf[1] = 0;
#pragma unroll
            for (int q = 0; q < 8; ++q) a[q] = 0;
#pragma unroll
            for (int q = 0; q < 6; ++q) d[q] = 0;
        }
        T x[8];
        {
            // the initial-state rows' right-hand side (-c_0, or a second-order correction's)
            T c0[6];
            ldv<6>(L.C0(), c0);
#pragma unroll
            for (int j = 0; j < 6; ++j) x[j] = (mode == 0 && ks == 0) ? c0[j] : (T)0;
            x[6] = 0;
            x[7] = 0;
        }
        // after the last step every lane k < N holds its own stage's step and, recomputed
        // from it, its control step
        T du0 = 0, du1 = 0;
        for (int s = 0; s < N; ++s) {
            T u0a = kf[0], u0b = 0, u1a = kf[1], u1b = 0;
#pragma unroll
            for (int m = 0; m < 8; m += 2) {
                u0a += K[m] * x[m];
                u0b += K[m + 1] * x[m + 1];
                u1a += K[8 + m] * x[m];
                u1b += K[9 + m] * x[m + 1];
            }
            du0 = u0a + u0b;
            du1 = u1a + u1b;
            T y[8];
            A_mul(a, x, y);
            if constexpr (MODEL == 1) {
                y[2] += tvl * x[3];
                y[5] += tvl * x[3];
            }
            y[2] += twl * du0;
            y[3] += dt * du1;
            y[5] += twl * du0;
#pragma unroll
            for (int j = 0; j < 6; ++j) y[j] += d[j];
            y[6] = du0;
            y[7] = du1;
            wv.up8(x, y);
        }
        if constexpr (SPLIT) {
            // the upper half-wave's step statistics take variables 4, 5 and the control step
            x[4] = wv.lo_half(x[4]);
            x[5] = wv.lo_half(x[5]);
            du0 = wv.lo_half(du0);
            du1 = wv.lo_half(du1);
        }
        const T* xk = x;
        const T duk[2] = {du0, du1};
        if (t < N) {
#pragma unroll
            for (int j = 0; j < 6; j += 2) {
                // 16-byte stores of the step of stage t
                st(L.DW(t) + j, xk[j]);
                st(L.DW(t) + j + 1, xk[j + 1]);
            }
            st(L.DW(t) + 6, duk[0]);
            st(L.DW(t) + 7, duk[1]);
        }
        // Multipliers of the dynamics rows into stage k from stationarity in s_k:
        //   lam_k = Q_k ds_k + q_k + A_k^T lam_{k+1},   yh+_k = -lam_k
        // (rows 0..5 of the Riccati costate P_k ds_k + p_k), a backward systolic pass:
        // lane k holds stage k's Hessian diagonal and curvature, gradient and A_k.  As in
        // the step recursion no lane is masked: lane 63 keeps its input, and every lane
        // k >= N (both of the upper half-wave's lanes when SPLIT) holds zero records, so
        // they hold and pass on zeros and lane N - 1 sees the terminal lam_N = 0.
        wv.mark(3);
        T lam[6], base[6] = {0, 0, 0, 0, 0, 0}, ak[8], tva = 0;
        {
            if (t < N) {
                T qd[8], qv[8], cv[6], hvd = 0;
                const int sb = L.ST(t);
                ldv<8>(sb + WideLayout::SQD, qd);
                ldv<8>(sb + WideLayout::SQV, qv);
                ldv<6>(sb + WideLayout::SCV, cv);  // cv[0..4] = Q00 Q22 Q32 Q55 Q53
                ldv<8>(sb + WideLayout::SA, ak);
                if constexpr (MODEL == 1) {
                    tva = ld(sb + WideLayout::STV);
                    hvd = ld(sb + WideLayout::SHVD);
                }
                const T* x = xk;
                base[0] = (qd[0] + cv[0]) * x[0] + qv[0];
                base[1] = qd[1] * x[1] + qv[1];
                base[2] = (qd[2] + cv[1]) * x[2] + cv[2] * x[3] + qv[2];
                base[3] = qd[3] * x[3] + cv[2] * x[2] + cv[4] * x[5] + qv[3];
                base[4] = qd[4] * x[4] + qv[4];
                base[5] = (qd[5] + cv[3]) * x[5] + cv[4] * x[3] + qv[5];
                if constexpr (MODEL == 1) base[3] += hvd * duk[0];  // (v, w) curvature times the w step
            } else {
#pragma unroll
                for (int q = 0; q < 8; ++q) ak[q] = 0;
            }
        }
#pragma unroll
        for (int q = 0; q < 6; ++q) lam[q] = 0;
        // (the last step's output in lane k is stage k's)
        T o[6];
        for (int s = N - 1; s >= 0; --s) {
            AT_mul(ak, lam, o);
            if constexpr (MODEL == 1) o[3] += tva * (lam[2] + lam[5]);
#pragma unroll
            for (int q = 0; q < 6; ++q) o[q] += base[q];
            wv.dn6(lam, o);
        }
        if (t < N) {
#pragma unroll
            for (int q = 0; q < 6; ++q) st(L.YP(t) + q, -o[q]);
        }
        wv.mark(4);
        Fwd F{(T)1, (T)1, (T)0, (T)0};
        if constexpr (SPLIT) {
            if (mode == 0 && ks < N) step_stats_split(ks, xk, duk, F);
        } else if (t < N) {
            const int k = t;
            const bool last = k == N - 1;
            if (mode == 0) {
                T w[8], zl[8], zu[8], dk[8];
                ldn<8>(L.W(k), w);
                ldn<8>(L.ZL(k), zl);
                ldn<8>(L.ZU(k), zu);
#pragma unroll
                for (int q = 0; q < 6; ++q) dk[q] = xk[q];
                dk[6] = duk[0];
                dk[7] = duk[1];
                T g[6], gu[2] = {0, 0};
                grad_state(w, g);
                if (!last) {
                    T um[2] = {0, 0}, up[2];
                    if (k >= 1) {
                        um[0] = ld(L.W(k - 1) + 6);
                        um[1] = ld(L.W(k - 1) + 7);
                    }
                    up[0] = ld(L.W(k + 1) + 6);
                    up[1] = ld(L.W(k + 1) + 7);
                    grad_ctrl(k, um, w + 6, up, gu);
                }
                const int nv = last ? 6 : 8;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    if (j < nv) {
                        const T gj = j < 6 ? sf * g[j] : sf * gu[j - 6];
                        const T gphi = gj - mu * rcp(w[j] - vlo(j)) + mu * rcp(vhi(j) - w[j]);
                        dir_var(w[j], zl[j], zu[j], vlo(j), vhi(j), gphi, dk[j], F);
                    }
                }
            }
        }
        if (mode == 0) {
            T v[4] = {F.amax_p, F.amax_z, F.gd, F.rel};
            const int op[4] = {RMIN, RMIN, RSUM, RMAX};
            reduce<4, SPLIT>(v, op);
            F.amax_p = v[0];
            F.amax_z = v[1];
            F.gd = v[2];
            F.rel = v[3];
        }
        wv.mark(5);
        return F;
    }


    // forward() for two stage blocks: the step recursion runs over block 0 (64 stages),
    // lane 63's output seeds lane 0 of block 1; the multiplier recursion runs over block 1,
    // its lane 0 output seeds lane 63 of block 0 (the unmasked systolic scheme of forward()
    // in each block).
    MPCG_HD Fwd forward_blk(int mode) {
        const int t = wv.lane();
        forward_begin();
        T xs[NB][6], dus[NB][2], xlast[8];
        for (int b = 0; b < NB; ++b) {
            const int ks = t + 64 * b;
            T K[16], kf[2], a[8], d[6], twl = 0, tvl = 0;
            if (ks < N - 1) {
                ld_gains(ks, K, kf);
                ldv<8>(L.ST(ks) + WideLayout::SA, a);
                ldv<6>(L.ST(ks) + WideLayout::SD, d);
                if constexpr (MODEL == 1)
                    ld2(L.ST(ks) + WideLayout::STW, twl, tvl);
                else
                    twl = dt;
            } else {
#pragma unroll
                for (int q = 0; q < 16; ++q) K[q] = 0;
                kf[0] = 0;
                kf[1] = 0;
#pragma unroll
                for (int q = 0; q < 8; ++q) a[q] = 0;
#pragma unroll
                for (int q = 0; q < 6; ++q) d[q] = 0;
            }
            T x[8];
            if (b == 0) {
                T c0[6];
                ldv<6>(L.C0(), c0);
#pragma unroll
                for (int j = 0; j < 6; ++j) x[j] = (mode == 0 && t == 0) ? c0[j] : (T)0;
                x[6] = 0;
                x[7] = 0;
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) x[j] = t == 0 ? xlast[j] : (T)0;
            }
            const int steps = b == 0 ? (N < 64 ? N : 64) : N - 64;
            T du0 = 0, du1 = 0, y[8];
            for (int s = 0; s < steps; ++s) {
                T u0a = kf[0], u0b = 0, u1a = kf[1], u1b = 0;
#pragma unroll
                for (int m = 0; m < 8; m += 2) {
                    u0a += K[m] * x[m];
                    u0b += K[m + 1] * x[m + 1];
                    u1a += K[8 + m] * x[m];
                    u1b += K[9 + m] * x[m + 1];
                }
                du0 = u0a + u0b;
                du1 = u1a + u1b;
                A_mul(a, x, y);
                if constexpr (MODEL == 1) {
                    y[2] += tvl * x[3];
                    y[5] += tvl * x[3];
                }
                y[2] += twl * du0;
                y[3] += dt * du1;
                y[5] += twl * du0;
#pragma unroll
                for (int j = 0; j < 6; ++j) y[j] += d[j];
                y[6] = du0;
                y[7] = du1;
                wv.up8(x, y);
            }
            if (b == 0 && NB == 2) {
                // lane 63 computed stage 64's input in the last step
#pragma unroll
                for (int j = 0; j < 8; ++j) xlast[j] = wv.lane63(y[j]);
            }
#pragma unroll
            for (int j = 0; j < 6; ++j) xs[b][j] = x[j];
            dus[b][0] = du0;
            dus[b][1] = du1;
            if (ks < N) {
#pragma unroll
                for (int j = 0; j < 6; ++j) st(L.DW(ks) + j, x[j]);
                st(L.DW(ks) + 6, du0);
                st(L.DW(ks) + 7, du1);
            }
        }
        wv.mark(3);
        // multipliers: upper block first
        T lam_in[6] = {0, 0, 0, 0, 0, 0};
        for (int b = NB - 1; b >= 0; --b) {
            const int k = t + 64 * b;
            T base[6] = {0, 0, 0, 0, 0, 0}, ak[8], tva = 0;
            if (k < N) {
                T qd[8], qv[8], cv[6], hvd = 0;
                const int sb = L.ST(k);
                ldv<8>(sb + WideLayout::SQD, qd);
                ldv<8>(sb + WideLayout::SQV, qv);
                ldv<6>(sb + WideLayout::SCV, cv);
                ldv<8>(sb + WideLayout::SA, ak);
                if constexpr (MODEL == 1) {
                    tva = ld(sb + WideLayout::STV);
                    hvd = ld(sb + WideLayout::SHVD);
                }
                const T* x = xs[b];
                base[0] = (qd[0] + cv[0]) * x[0] + qv[0];
                base[1] = qd[1] * x[1] + qv[1];
                base[2] = (qd[2] + cv[1]) * x[2] + cv[2] * x[3] + qv[2];
                base[3] = qd[3] * x[3] + cv[2] * x[2] + cv[4] * x[5] + qv[3];
                base[4] = qd[4] * x[4] + qv[4];
                base[5] = (qd[5] + cv[3]) * x[5] + cv[4] * x[3] + qv[5];
                if constexpr (MODEL == 1) base[3] += hvd * dus[b][0];
            } else {
#pragma unroll
                for (int q = 0; q < 8; ++q) ak[q] = 0;
            }
            T lam[6];
#pragma unroll
            for (int q = 0; q < 6; ++q) lam[q] = (b < NB - 1 && t == 63) ? lam_in[q] : (T)0;
            const int steps = b == NB - 1 ? N - 64 * b : 64;
            T o[6];
            for (int s = steps - 1; s >= 0; --s) {
                AT_mul(ak, lam, o);
                if constexpr (MODEL == 1) o[3] += tva * (lam[2] + lam[5]);
#pragma unroll
                for (int q = 0; q < 6; ++q) o[q] += base[q];
                wv.dn6(lam, o);
            }
            if (k < N) {
#pragma unroll
                for (int q = 0; q < 6; ++q) st(L.YP(k) + q, -o[q]);
            }
            if (b > 0) {
#pragma unroll
                for (int q = 0; q < 6; ++q) lam_in[q] = wv.lane0(o[q]);
            }
        }
        wv.mark(4);
        Fwd F{(T)1, (T)1, (T)0, (T)0};
        if (mode == 0) {
            for (int b = 0; b < NB; ++b) {
                const int k = t + 64 * b;
                if (k < N) step_stats_stage(k, xs[b], dus[b], F);
            }
            T v[4] = {F.amax_p, F.amax_z, F.gd, F.rel};
            const int op[4] = {RMIN, RMIN, RSUM, RMAX};
            reduce<4, true>(v, op);
            F.amax_p = v[0];
            F.amax_z = v[1];
            F.gd = v[2];
            F.rel = v[3];
        }
        wv.mark(5);
        return F;
    }
    // step statistics of stage k (unsplit): fraction to the boundary, grad phi^T dw, relative step
    MPCG_HD void step_stats_stage(int k, const T* xk, const T* duk, Fwd& F) const {
        const bool last = k == N - 1;
        T w[8], zl[8], zu[8], dk[8];
        ldn<8>(L.W(k), w);
        ldn<8>(L.ZL(k), zl);
        ldn<8>(L.ZU(k), zu);
#pragma unroll
        for (int q = 0; q < 6; ++q) dk[q] = xk[q];
        dk[6] = duk[0];
        dk[7] = duk[1];
        T g[6], gu[2] = {0, 0};
        grad_state(w, g);
        if (!last) {
            T um[2] = {0, 0}, up[2];
            if (k >= 1) {
                um[0] = ld(L.W(k - 1) + 6);
                um[1] = ld(L.W(k - 1) + 7);
            }
            up[0] = ld(L.W(k + 1) + 6);
            up[1] = ld(L.W(k + 1) + 7);
            grad_ctrl(k, um, w + 6, up, gu);
        }
        const int nv = last ? 6 : 8;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if (j < nv) {
                const T gj = j < 6 ? sf * g[j] : sf * gu[j - 6];
                const T gphi = gj - mu * rcp(w[j] - vlo(j)) + mu * rcp(vhi(j) - w[j]);
                dir_var(w[j], zl[j], zu[j], vlo(j), vhi(j), gphi, dk[j], F);
            }
        }
    }

    // ------------------------------------------------------------ trial point
    // Trial point (SPLIT): lane k of the lower half-wave takes stage k's variables 0..3,
    // the heading theta and dynamics rows 0..3, lane 32 + k the variables 4..7, the
    // heading error and rows 4, 5: one sine/cosine and half the slacks per lane.  Same
    // per-quantity formulas as the unsplit sweep (trial()).
    MPCG_HD bool trial_split(T alpha, T* phi, T* th) {
        wv.mark(9);
        const int t = wv.lane();
        const int k = t & 31;
        const bool hi = t >= 32, act = k < N, last = k == N - 1;
        T f = 0, thv = 0, lg = 0;
        int bad = 0;
        T Fa[4] = {0, 0, 0, 0};
        T w[8];
        if (act) {
            T cw[8], cd[8];
            ldn<8>(L.W(k), cw);
            ldn<8>(L.DW(k), cd);
#pragma unroll
            for (int j = 0; j < 8; ++j) w[j] = cw[j] + alpha * cd[j];
            const int nv = (last && hi) ? 2 : 4;
            T slackprod = 1;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if (q < nv) {
                    const T wq = hi ? w[4 + q] : w[q];
                    const T lo = q < 2 ? sl : (q == 2 ? (hi ? wl : sl) : (hi ? al : sl));
                    const T up_ = q < 2 ? su : (q == 2 ? (hi ? wu : su) : (hi ? au : su));
                    const T dl = wq - lo, du = up_ - wq;
                    bad |= !((dl > 0) && (du > 0));
                    slackprod *= dl * du;
                }
            }
            lg = log(slackprod);
            // objective: v term (lower), cte / etheta terms and the controls (upper)
            const T e1 = w[4] - (T)P.ref_cte, e2 = w[5] - (T)P.ref_eth, e3 = w[3] - (T)P.ref_v;
            T fu = (T)P.w_cte * e1 * e1 + (T)P.w_eth * e2 * e2;
            if (!last) {
                T up[2];
                up[0] = ld(L.W(k + 1) + 6) + alpha * ld(L.DW(k + 1) + 6);
                up[1] = ld(L.W(k + 1) + 7) + alpha * ld(L.DW(k + 1) + 7);
                fu += cost_ctrl(k, w + 6, up);
            }
            f = hi ? fu : (T)P.w_v * e3 * e3;
            if (!last) {
                // (Lin::eval / Lin::next / next_m, one angle per half-wave)
                T sa, ca;
                sc_t(hi ? w[5] : w[2], &sa, &ca);
                c_sa = sa;
                c_ca = ca;
                const T x = w[0];
                const C4 pcoef_ = pcoef();
                const T fx = pcoef_.c[0] + pcoef_.c[1] * x + pcoef_.c[2] * (x * x) + pcoef_.c[3] * (x * x * x);
                T turn = w[6] * dt;
                if (model == 1) turn = w[3] * w[6] / lf * dt;
                Fa[0] = (hi ? fx - w[1] : w[0]) + w[3] * (hi ? sa : ca) * dt;
                Fa[1] = hi ? (model == 1 ? w[5] + turn : w[5] + w[6] * dt) : w[1] + w[3] * sa * dt;
                Fa[2] = model == 1 ? w[2] + turn : w[2] + w[6] * dt;
                Fa[3] = w[3] + w[7] * dt;
            }
        }
        c_ok = 1;
        T Fprev[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) Fprev[q] = wv.up1(Fa[q]);
        if (act) {
            const int nr = hi ? 2 : 4;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if (q < nr) {
                    const int j = hi ? 4 + q : q;
                    const T wj = hi ? w[4 + q] : w[q];
                    const T c = k == 0 ? wj - pinit(hi ? 4 + q : q) : wj - Fprev[q];
                    thv += fabs(rowscale(j, k) * c);
                }
            }
        }
        T v[3] = {f, thv, lg};
        const int op[3] = {RSUM, RSUM, RSUM};
        reduce<3, true>(v, op);
        f = v[0];
        thv = v[1];
        lg = v[2];
        const bool anybad = wv.any(bad != 0);
        wv.mark(6);
        *phi = sf * f - mu * lg;
        *th = thv;
        return !anybad && isfinite((double)*phi);
    }

    MPCG_HD bool trial(T alpha, T* phi, T* th) {
        if constexpr (RESTO) return trial_resto(alpha, phi, th);
        if constexpr (SPLIT) return trial_split(alpha, phi, th);
        if constexpr (NB == 2) return trial_blk(alpha, phi, th);
        const int t = wv.lane();  // (recomputed per phase: nothing lane-dependent is hoisted)
        T f = 0, thv = 0, lg = 0;
        int bad = 0;
        T Fk[6] = {0, 0, 0, 0, 0, 0};
        T w[8];
        const int k = t;
        const bool act = t < N, last = k == N - 1;
        if (act) {
            T cw[8], cd[8];
            ldn<8>(L.W(k), cw);
            ldn<8>(L.DW(k), cd);
#pragma unroll
            for (int j = 0; j < 8; ++j) w[j] = cw[j] + alpha * cd[j];
            const int nv = last ? 6 : 8;
            T slackprod = 1;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                if (j < nv) {
                    const T dl = w[j] - vlo(j), du = vhi(j) - w[j];
                    bad |= !((dl > 0) && (du > 0));
                    slackprod *= dl * du;
                }
            }
            lg = log(slackprod);
            f = cost_state(w);
            if (!last) {
                T up[2];
                up[0] = ld(L.W(k + 1) + 6) + alpha * ld(L.DW(k + 1) + 6);
                up[1] = ld(L.W(k + 1) + 7) + alpha * ld(L.DW(k + 1) + 7);
                f += cost_ctrl(k, w + 6, up);
                Lin<T> ln;
                ln.eval(pcoef().c, w);
                next_m(ln, w, w + 6, Fk);
            }
        }
        T Fprev[6];
#pragma unroll
        for (int j = 0; j < 6; ++j) Fprev[j] = wv.up1(Fk[j]);
        if (act) {
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                const T c = k == 0 ? w[j] - pinit(j) : w[j] - Fprev[j];
                thv += fabs(rowscale(j, k) * c);
            }
        }
        T v[3] = {f, thv, lg};
        const int op[3] = {RSUM, RSUM, RSUM};
        reduce<3>(v, op);
        f = v[0];
        thv = v[1];
        lg = v[2];
        const bool anybad = wv.any(bad != 0);
        wv.mark(6);
        *phi = sf * f - mu * lg;
        *th = thv;
        return !anybad && isfinite((double)*phi);
    }

    // ------------------------------------------------------------ the restoration problem's sweeps
    // (RESTO instance.)  x = the stage variables in LDS as in the original problem; the rows'
    // p, n, z_p, z_n and steps in HBM records owned by the lane of the stage the rows lead into.
    MPCG_HD T* xrec(int k) const { return ext + (size_t)k * WideLayout::XS; }
    MPCG_HD T xR(int k, int j) const { return dumpO[L.W(k) + j]; }  // the reference point x_R
    MPCG_HD T dR(int k, int j) const { return (T)1 / tmax((T)1, (T)fabs(xR(k, j))); }
    MPCG_HD T eta_mu() const { return (T)sqrt((double)mu); }  // resto_proximity_weight 1 * sqrt(mu)
    // the barrier function of the current iterate (kappa_d damping of p, n)
    MPCG_HD T phi_cur() const {
        if constexpr (RESTO) return wv.uni_d(fval - mu * logsum + (T)KD * mu * r_spn);
        return wv.uni_d(sf * fval - mu * logsum);
    }
    // the original problem's scaled rows into the lane's stages at the stage variables w
    // (c = rsc (s_k - F(s_{k-1}, u_{k-1})), rows 0: s_0 - init)
    MPCG_HD void rows_c(const T (&w)[NB][8], T (&cs)[NB][6]) {
        const int t = wv.lane();
        T Fk[NB][6], Fprev[NB][6];
        for (int b = 0; b < NB; ++b) {
            const int k = t + 64 * b;
#pragma unroll
            for (int j = 0; j < 6; ++j) Fk[b][j] = 0;
            if (k < N - 1) {
                Lin<T> ln;
                ln.eval(pcoef().c, w[b]);
                next_m(ln, w[b], w[b] + 6, Fk[b]);
            }
        }
        shift_blocks(Fk, Fprev);
        for (int b = 0; b < NB; ++b) {
            const int k = t + 64 * b;
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                const T c = k == 0 ? w[b][j] - pinit(j) : w[b][j] - Fprev[b][j];
                cs[b][j] = k < N ? rowscale(j, k) * c : (T)0;
            }
        }
    }
    MPCG_HD void load_w(T (&w)[NB][8], T alpha, bool step) const {
        const int t = wv.lane();
        for (int b = 0; b < NB; ++b) {
            const int k = t + 64 * b;
#pragma unroll
            for (int j = 0; j < 8; ++j) w[b][j] = 0;
            if (k >= N) continue;
            const int nv = k == N - 1 ? 6 : 8;
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (j < nv) w[b][j] = step ? ld(L.W(k) + j) + alpha * ld(L.DW(k) + j) : ld(L.W(k) + j);
        }
    }

    // RestoIterateInitializer: x = the original iterate, its bound multipliers capped at rho,
    // p and n the minimisers of the penalty with barrier mu_R for fixed x, z_p = mu_R / p,
    // z_n = mu_R / n, y = 0
    MPCG_HD void init_rows() {
        const int t = wv.lane();
        wv.sync();
        T w[NB][8], cs[NB][6];
        load_w(w, (T)0, false);
        rows_c(w, cs);
        for (int b = 0; b < NB; ++b) {
            const int k = t + 64 * b;
            if (k >= N) continue;
            const int nv = k == N - 1 ? 6 : 8;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                if (j < nv) {
                    st(L.ZL(k) + j, tmin((T)RHO, ld(L.ZL(k) + j)));
                    st(L.ZU(k) + j, tmin((T)RHO, ld(L.ZU(k) + j)));
                }
            }
            T* x = xrec(k);
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                st(L.Y(k) + j, 0);
                const T c = cs[b][j];
                const T a = mu / ((T)2 * (T)RHO) - (T)0.5 * c, bb = c * mu / ((T)2 * (T)RHO);
                const T nn = a + (T)sqrt((double)(a * a + bb)), pp = c + nn;
                x[WideLayout::XP + j] = pp;
                x[WideLayout::XN + j] = nn;
                x[WideLayout::XZP + j] = mu / pp;
                x[WideLayout::XZN + j] = mu / nn;
                x[WideLayout::XDP + j] = 0;
                x[WideLayout::XDN + j] = 0;
            }
        }
        wv.sync();
    }

    // Statistics of the restoration iterate (eval_current on RestoIpoptNLP), with the stage
    // data of its Newton system (A_k, curvature) and the rows' right-hand side c(x) - p + n.
    MPCG_HD void stats_resto(bool acc, T alpha, T amax_z) {
        const int t = wv.lane();
        accept_all(t, acc, alpha, amax_z);
        const T eta = eta_mu();
        for (int b = 0; b < NB; ++b) {
            const int k = t + 64 * b;
            if (k >= N) continue;
            const bool last = k == N - 1;
            T w[8], yn[6] = {0, 0, 0, 0, 0, 0}, a[7] = {0, 0, 0, 0, 0, 0, 0}, cvk[5] = {0, 0, 0, 0, 0};
            T twk = dt, tvk = 0, hvdk = 0;
            ldn<8>(L.W(k), w);
            if (!last) {
                ldn<6>(L.Y(k + 1), yn);
                Lin<T> ln;
                ln.eval(pcoef().c, w);
                ln.jac(w, dt, a);
                turn_d(w, w + 6, &twk, &tvk);
                if (model == 1) hvdk = -(yn[2] + yn[5]) / lf * dt;
                const T v = w[3];
                cvk[0] = -yn[4] * ln.f2;
                cvk[1] = yn[0] * v * ln.ct * dt + yn[1] * v * ln.st * dt;
                cvk[2] = yn[0] * ln.st * dt - yn[1] * ln.ct * dt;
                cvk[3] = yn[4] * v * ln.se * dt;
                cvk[4] = -yn[4] * ln.ce * dt;
            }
            const int sb = L.ST(k);
#pragma unroll
            for (int j = 0; j < 7; ++j) st(sb + WideLayout::SA + j, a[j]);
#pragma unroll
            for (int j = 0; j < 5; ++j) st(sb + WideLayout::SCV + j, cvk[j]);
            if constexpr (MODEL == 1) {
                st(sb + WideLayout::STW, twk);
                st(sb + WideLayout::STV, tvk);
                st(sb + WideLayout::SHVD, hvdk);
            }
        }
        T wv8[NB][8], cs[NB][6];
        load_w(wv8, (T)0, false);
        rows_c(wv8, cs);
        T fO = 0, th = 0, pinf = 0, dinf = 0, c0 = 0, mn = (T)INFINITY, mx = -(T)INFINITY, ly = 0, lz = 0, lgx = 0,
          lgpn = 0, spn = 0, qx = 0, thO = 0, pinfO = 0;
        for (int b = 0; b < NB; ++b) {
            const int k = t + 64 * b;
            if (k >= N) continue;
            const bool last = k == N - 1;
            T w[8], zl[8], zu[8], y[6], yn[6] = {0, 0, 0, 0, 0, 0}, up[2] = {0, 0}, um[2] = {0, 0}, a[8];
            ldn<8>(L.W(k), w);
            ldn<8>(L.ZL(k), zl);
            ldn<8>(L.ZU(k), zu);
            ldn<6>(L.Y(k), y);
            ldn<7>(L.ST(k) + WideLayout::SA, a);
            T twk = dt, tvk = 0;
            if constexpr (MODEL == 1) {
                twk = ld(L.ST(k) + WideLayout::STW);
                tvk = ld(L.ST(k) + WideLayout::STV);
            }
            if (!last) {
                ldn<6>(L.Y(k + 1), yn);
                up[0] = ld(L.W(k + 1) + 6);
                up[1] = ld(L.W(k + 1) + 7);
            }
            if (k >= 1) {
                um[0] = ld(L.W(k - 1) + 6);
                um[1] = ld(L.W(k - 1) + 7);
            }
            T* x = xrec(k);
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                const T p = x[WideLayout::XP + j], n = x[WideLayout::XN + j];
                const T zp = x[WideLayout::XZP + j], zn = x[WideLayout::XZN + j];
                const T c = cs[b][j], cr = c - p + n;
                x[WideLayout::XCR + j] = cr;
                th += fabs(cr);
                pinf = tmax(pinf, (T)fabs(cr));
                thO += fabs(c);
                pinfO = tmax(pinfO, (T)fabs(c));
                const T ys = y[j] * rcp(rowscale(j, k));
                ly += fabs(ys);
                const T rdp = (T)RHO - ys - zp, rdn = (T)RHO + ys - zn;
                dinf = tmax(dinf, tmax((T)fabs(rdp), (T)fabs(rdn)));
                const T pp = p * zp, qq = n * zn;
                c0 = tmax(c0, tmax((T)fabs(pp), (T)fabs(qq)));
                mn = tmin(mn, tmin(pp, qq));
                mx = tmax(mx, tmax(pp, qq));
                lz += fabs(zp) + fabs(zn);
                lgpn += log(p * n);
                spn += p + n;
            }
            fO += cost_state(w);
            T at[6] = {0, 0, 0, 0, 0, 0};
            if (!last) {
                AT_mul(a, yn, at);
                if (model == 1) at[3] += tvk * (yn[2] + yn[5]);
                fO += cost_ctrl(k, w + 6, up);
            }
            const T btw = twk * (yn[2] + yn[5]), bta = dt * yn[3];
            const int nv = last ? 6 : 8;
            T slackprod = 1;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                if (j < nv) {
                    const T dr = dR(k, j), dxr = w[j] - xR(k, j);
                    const T gq = eta * dr * dr * dxr;
                    qx += (dr * dxr) * (dr * dxr);
                    const T gj = j < 6 ? gq + y[j] - at[j] : gq - (j == 6 ? btw : bta);
                    dinf = tmax(dinf, (T)fabs(gj - zl[j] + zu[j]));
                    const T dl = w[j] - vlo(j), du = vhi(j) - w[j];
                    slackprod *= dl * du;
                    const T p1 = dl * zl[j], p2 = du * zu[j];
                    c0 = tmax(c0, tmax((T)fabs(p1), (T)fabs(p2)));
                    mn = tmin(mn, tmin(p1, p2));
                    mx = tmax(mx, tmax(p1, p2));
                    lz += fabs(zl[j]) + fabs(zu[j]);
                }
            }
            lgx += log(slackprod);
        }
        T v[15] = {fO, th, pinf, dinf, c0, mn, mx, ly, lz, lgx, lgpn, spn, qx, thO, pinfO};
        const int op[15] = {RSUM, RSUM, RMAX, RMAX, RMAX, RMIN, RMAX, RSUM, RSUM, RSUM, RSUM, RSUM, RSUM, RSUM, RMAX};
        reduce<15, true>(v, op);
        r_spn = v[11];
        r_qx = v[12];
        fval = wv.uni_d((T)RHO * r_spn + (T)0.5 * eta * r_qx);
        theta = v[1];
        prim_inf = v[2];
        prim_uns = v[2];
        dual_inf = v[3];
        compl0 = v[4];
        pmin = v[5];
        pmax = v[6];
        l1y = v[7];
        l1z = v[8];
        logsum = wv.uni_d(v[9] + v[10]);
        // barrier_phi of the original problem at x (its mu; no one-sided bounds)
        r_phiO = wv.uni_d(o_sf * v[0] - o_mu * v[9]);
        r_thO = v[13];
        r_pinfO = v[14];
        wv.mark(0);
    }

    // the restoration problem's barrier function and violation at w + alpha dw, (p, n) + alpha (dp, dn)
    MPCG_HD bool trial_resto(T alpha, T* phi, T* th) {
        const int t = wv.lane();
        const T eta = eta_mu();
        T w[NB][8], cs[NB][6];
        load_w(w, alpha, true);
        rows_c(w, cs);
        T qx = 0, thv = 0, lg = 0, spn = 0;
        int bad = 0;
        for (int b = 0; b < NB; ++b) {
            const int k = t + 64 * b;
            if (k >= N) continue;
            const int nv = k == N - 1 ? 6 : 8;
            T slackprod = 1;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                if (j < nv) {
                    const T dl = w[b][j] - vlo(j), du = vhi(j) - w[b][j];
                    bad |= !((dl > 0) && (du > 0));
                    slackprod *= dl * du;
                    const T d = dR(k, j) * (w[b][j] - xR(k, j));
                    qx += d * d;
                }
            }
            lg += log(slackprod);
            const T* x = xrec(k);
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                const T p = x[WideLayout::XP + j] + alpha * x[WideLayout::XDP + j];
                const T n = x[WideLayout::XN + j] + alpha * x[WideLayout::XDN + j];
                bad |= !((p > 0) && (n > 0));
                lg += log(p * n);
                spn += p + n;
                thv += fabs(cs[b][j] - p + n);
            }
        }
        T v[4] = {qx, thv, lg, spn};
        const int op[4] = {RSUM, RSUM, RSUM, RSUM};
        reduce<4, true>(v, op);
        const bool anybad = wv.any(bad != 0);
        *phi = wv.uni_d((T)RHO * v[3] + (T)0.5 * eta * v[0] - mu * v[2] + (T)KD * mu * v[3]);
        *th = v[1];
        return !anybad && isfinite((double)*phi);
    }

    // Stage data of the reduced Newton system: x's barrier Hessian diagonal and gradient
    // (no objective curvature: eta D_R^2 on the diagonal), and the rows' elimination of p, n
    // (AugRestoSystemSolver): D = 1/(Sigma_p + dw) + 1/(Sigma_n + dw),
    // c_hat = c_R + r_p/(Sigma_p + dw) - r_n/(Sigma_n + dw) + D y (scaled rows), in row form
    // D / rsc^2 and c_hat / rsc; -c_hat is the defect of the step recursion (SD, C0).
    MPCG_HD void precompute_resto(int k, T delta_w) {
        if (k >= N) return;
        const bool last = k == N - 1;
        const int sb = L.ST(k);
        const T eta = eta_mu();
        T w[8], zl[8], zu[8];
        ldn<8>(L.W(k), w);
        ldn<8>(L.ZL(k), zl);
        ldn<8>(L.ZU(k), zu);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            T qd = 0, qv = 0;
            if (j < 6 || !last) {
                const T dr = dR(k, j);
                const T rdl = (T)1 / (w[j] - vlo(j)), rdu = (T)1 / (vhi(j) - w[j]);
                qd = eta * dr * dr + zl[j] * rdl + zu[j] * rdu + delta_w;
                qv = eta * dr * dr * (w[j] - xR(k, j)) - mu * rdl + mu * rdu;
            }
            if (rf_pass) qv = (j < 6 || !last) ? -xrec(k)[WideLayout::XRX + j] : (T)0;
            st(sb + WideLayout::SQD + j, qd);
            st(sb + WideLayout::SQV + j, qv);
        }
        T* x = xrec(k);
#pragma unroll
        for (int j = 0; j < 6; ++j) {
            const T rsc = rowscale(j, k);
            const T ys = ld(L.Y(k) + j) * rcp(rsc);
            const T p = x[WideLayout::XP + j], n = x[WideLayout::XN + j];
            const T sp_ = x[WideLayout::XZP + j] / p + delta_w, sn_ = x[WideLayout::XZN + j] / n + delta_w;
            // (c_hat = c + r_p/sp - r_n/sn + D y = c + gphi_p/sp - gphi_n/sn: the y terms
            // cancel exactly, and are left out -- large where a row is active)
            (void)ys;
            T gp = (T)RHO - mu / p + (T)KD * mu, gn = (T)RHO - mu / n + (T)KD * mu;
            if (rf_pass) {
                gp = -x[WideLayout::XRP + j];
                gn = -x[WideLayout::XRN + j];
            }
            const T D = (T)1 / sp_ + (T)1 / sn_;
            const T ch = x[WideLayout::XCR + j] + gp / sp_ - gn / sn_;
            x[WideLayout::XDS + j] = (T)sqrt((double)(D / (rsc * rsc)));
            const T dbar = -ch / rsc;
            if (k == 0)
                st(L.C0() + j, dbar);
            else
                st(L.ST(k - 1) + WideLayout::SD + j, dbar);
        }
    }

    // The rows into stage kk absorbed into its cost-to-go (P, p of the lane's entry (i, j),
    // row-major P in the scratch): S = I + D^1/2 P_ss D^1/2 (LDL^T, every pivot > 0 or the
    // inertia test fails), P~ = P - P D^1/2 S^-1 D^1/2 P, p~ = p - P D^1/2 S^-1 D^1/2 p,
    // and the gains of the step recursion ds = M z + m, M = I - D^1/2 S^-1 D^1/2 P,
    // m = -D^1/2 S^-1 D^1/2 p (z: the state the hard dynamics would give).  Every lane
    // factors S (the same values); lane (i, j) solves for its column j.
    MPCG_HD void soft_rows(int kk, T& Pij, T& pvi, bool& bad) {
        const int t = wv.lane();
        const int i = t >> 3, j = t & 7;
        const int sp = L.PSC();
        T* x = xrec(kk);
        T ds[6], pv[6], Pr[6][8];
#pragma unroll
        for (int a = 0; a < 6; ++a) ds[a] = x[WideLayout::XDS + a];
#pragma unroll
        for (int a = 0; a < 6; ++a) pv[a] = wv.lanev(pvi, 8 * a);
        wv.sync();
#pragma unroll
        for (int a = 0; a < 6; ++a) ldn<8>(sp + 8 * a, Pr[a]);
        T Lm[6][6], d[6];
        bool ok = true;
#pragma unroll
        for (int a = 0; a < 6; ++a) {
            T s = (T)1 + ds[a] * ds[a] * Pr[a][a];
#pragma unroll
            for (int c = 0; c < a; ++c) s -= Lm[a][c] * Lm[a][c] * d[c];
            d[a] = s;
            ok = ok && (s > 0) && isfinite((double)s);
#pragma unroll
            for (int r = a + 1; r < 6; ++r) {
                T q = ds[r] * ds[a] * Pr[r][a];
#pragma unroll
                for (int c = 0; c < a; ++c) q -= Lm[r][c] * Lm[a][c] * d[c];
                Lm[r][a] = q / s;
            }
        }
        bad = bad || !ok;
        // right-hand sides: u = D^1/2 P[:, j], c = e_j / ds_j (j < 6), v = D^1/2 p -- then S^-1 of each
        T u[6], c[6], v[6];
#pragma unroll
        for (int a = 0; a < 6; ++a) {
            T paj = Pr[a][0];
#pragma unroll
            for (int q = 1; q < 8; ++q)
                if (q == j) paj = Pr[a][q];
            u[a] = ds[a] * paj;
            c[a] = a == j ? (T)1 / ds[a] : (T)0;
            v[a] = ds[a] * pv[a];
        }
        lsolve6(Lm, d, u);
        lsolve6(Lm, d, c);
        lsolve6(Lm, d, v);
        // the lane's row i of the results (selects: no dynamic register indexing)
        T ui = 0, ci = 0, vi = 0, dsi = 1;
#pragma unroll
        for (int a = 0; a < 6; ++a) {
            if (a == i) {
                ui = u[a];
                ci = c[a];
                vi = v[a];
                dsi = ds[a];
            }
        }
        // P~ = M^T P = D^-1/2 S^-1 D^1/2 P and p~ = M^T p = D^-1/2 S^-1 D^1/2 p (no cancellation
        // at either end of D); M = (I + D P)^-1 = D^1/2 S^-1 D^-1/2 for the step recursion
        // and N = M - I = -D^1/2 S^-1 D^1/2 P, m = -D^1/2 S^-1 D^1/2 p for the rows' slack.
        // (Rows / columns 6, 7 -- the previous control -- carry no soft row: M is the identity
        // there, and the restoration problem's P has no entries in them.)
        T Pt = Pij, pt = pvi;
        if (i < 6) {
            Pt = ui / dsi;
            pt = vi / dsi;
            if (j < 6) {
                x[WideLayout::XM + 6 * i + j] = dsi * ci;
                x[WideLayout::XMN + 6 * i + j] = -dsi * ui;
            }
            if (j == 0) x[WideLayout::XMV + i] = -dsi * vi;
        }
        wv.sync();  // every lane's reads of P are done
        st(sp + t, Pt);
        Pij = Pt;
        pvi = pt;
    }
    // S^-1 b for S = L D L^T (6 x 6, unit lower L)
    MPCG_HD static void lsolve6(const T (&Lm)[6][6], const T (&d)[6], T (&b)[6]) {
#pragma unroll
        for (int a = 0; a < 6; ++a) {
#pragma unroll
            for (int c = 0; c < a; ++c) b[a] -= Lm[a][c] * b[c];
        }
#pragma unroll
        for (int a = 0; a < 6; ++a) b[a] /= d[a];
#pragma unroll
        for (int a = 5; a >= 0; --a) {
#pragma unroll
            for (int r = a + 1; r < 6; ++r) b[a] -= Lm[r][a] * b[r];
        }
    }

    // The step recursion through the soft rows (ds_k = M_k z_k + m_k, z_k the hard-dynamics
    // image of stage k - 1, z_0 = -c_hat of the initial rows), the multipliers by the adjoint
    // recursion (stationarity in s is unchanged), then the rows' steps
    // dp = (dy - r_p)/(Sigma_p + dw), dn = -(dy + r_n)/(Sigma_n + dw) and the step statistics.
    MPCG_HD Fwd forward_resto() {
        const int t = wv.lane();
        forward_begin();
        T xs[NB][8], dus[NB][2], xlast[8] = {0, 0, 0, 0, 0, 0, 0, 0}, lin[NB][6];
        for (int b = 0; b < NB; ++b) {
            const int ks = t + 64 * b;
            T K[16], kf[2], a[8], d[6], twl = 0, tvl = 0, Mx[36], Nx[36], mv[6];
            if (ks < N - 1) {
                ld_gains(ks, K, kf);
                ldv<8>(L.ST(ks) + WideLayout::SA, a);
                ldv<6>(L.ST(ks) + WideLayout::SD, d);
                if constexpr (MODEL == 1)
                    ld2(L.ST(ks) + WideLayout::STW, twl, tvl);
                else
                    twl = dt;
            } else {
#pragma unroll
                for (int q = 0; q < 16; ++q) K[q] = 0;
                kf[0] = 0;
                kf[1] = 0;
#pragma unroll
                for (int q = 0; q < 8; ++q) a[q] = 0;
#pragma unroll
                for (int q = 0; q < 6; ++q) d[q] = 0;
            }
            if (ks < N) {
                const T* x = xrec(ks);
#pragma unroll
                for (int q = 0; q < 36; ++q) {
                    Mx[q] = x[WideLayout::XM + q];
                    Nx[q] = x[WideLayout::XMN + q];
                }
#pragma unroll
                for (int q = 0; q < 6; ++q) mv[q] = x[WideLayout::XMV + q];
            } else {
#pragma unroll
                for (int q = 0; q < 36; ++q) {
                    Mx[q] = 0;
                    Nx[q] = 0;
                }
#pragma unroll
                for (int q = 0; q < 6; ++q) mv[q] = 0;
            }
            T z[8];
            if (b == 0) {
                T c0[6];
                ldv<6>(L.C0(), c0);
#pragma unroll
                for (int j = 0; j < 6; ++j) z[j] = t == 0 ? c0[j] : (T)0;
                z[6] = 0;
                z[7] = 0;
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) z[j] = t == 0 ? xlast[j] : (T)0;
            }
            const int steps = b == 0 ? (N < 64 ? N : 64) : N - 64;
            T x[8], du0 = 0, du1 = 0, y[8], e[6];
            for (int s = 0; s < steps; ++s) {
#pragma unroll
                for (int r = 0; r < 6; ++r) {
                    T ax = mv[r], ae = mv[r];
#pragma unroll
                    for (int c = 0; c < 6; ++c) {
                        ax += Mx[6 * r + c] * z[c];
                        ae += Nx[6 * r + c] * z[c];
                    }
                    x[r] = ax;
                    e[r] = ae;
                }
                x[6] = z[6];
                x[7] = z[7];
                T u0a = kf[0], u0b = 0, u1a = kf[1], u1b = 0;
#pragma unroll
                for (int m = 0; m < 8; m += 2) {
                    u0a += K[m] * x[m];
                    u0b += K[m + 1] * x[m + 1];
                    u1a += K[8 + m] * x[m];
                    u1b += K[9 + m] * x[m + 1];
                }
                du0 = u0a + u0b;
                du1 = u1a + u1b;
                A_mul(a, x, y);
                if constexpr (MODEL == 1) {
                    y[2] += tvl * x[3];
                    y[5] += tvl * x[3];
                }
                y[2] += twl * du0;
                y[3] += dt * du1;
                y[5] += twl * du0;
#pragma unroll
                for (int j = 0; j < 6; ++j) y[j] += d[j];
                y[6] = du0;
                y[7] = du1;
                wv.up8(z, y);
            }
            if (b == 0 && NB == 2) {
#pragma unroll
                for (int j = 0; j < 8; ++j) xlast[j] = wv.lane63(y[j]);
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) xs[b][j] = x[j];
            dus[b][0] = du0;
            dus[b][1] = du1;
            // A ds + B du of the stage (the next rows' J dx = ds_{k+1} - this)
            {
                T l8[8];
                A_mul(a, x, l8);
                if constexpr (MODEL == 1) {
                    l8[2] += tvl * x[3];
                    l8[5] += tvl * x[3];
                }
                l8[2] += twl * du0;
                l8[3] += dt * du1;
                l8[5] += twl * du0;
#pragma unroll
                for (int j = 0; j < 6; ++j) lin[b][j] = ks < N - 1 ? l8[j] : (T)0;
            }
            if (ks < N) {
#pragma unroll
                for (int j = 0; j < 6; ++j) st(L.DW(ks) + j, x[j]);
                st(L.DW(ks) + 6, du0);
                st(L.DW(ks) + 7, du1);
                T* xr = xrec(ks);
#pragma unroll
                for (int j = 0; j < 6; ++j) xr[WideLayout::XE + j] = e[j];
            }
        }
        wv.mark(3);
        // the rows' multipliers: the adjoint recursion of stationarity in s (as forward_blk),
        // lam_k = Q_k ds_k + q_k + A_k^T lam_{k+1}, y+ = -lam, except on the soft rows
        // (D >= 0.6404 in Ipopt's scaled units, the Bunch-Kaufman 1x1 pivot test on the
        // row's own diagonal) where y+ = D^-1 e (row form) -- the recursion loses digits
        // there where a bound-active state's barrier Hessian is large, e / D does not;
        // on nearly hard rows e / D would divide a slack's rounding by a small D
        T lam_in[6] = {0, 0, 0, 0, 0, 0};
        for (int b = NB - 1; b >= 0; --b) {
            const int k = t + 64 * b;
            T base[6] = {0, 0, 0, 0, 0, 0}, ak[8], tva = 0, yo[6] = {0, 0, 0, 0, 0, 0};
            bool ov[6] = {false, false, false, false, false, false};
            if (k < N) {
                T qd[8], qv[8], cv[6], hvd = 0;
                const int sb = L.ST(k);
                ldv<8>(sb + WideLayout::SQD, qd);
                ldv<8>(sb + WideLayout::SQV, qv);
                ldv<6>(sb + WideLayout::SCV, cv);
                ldv<8>(sb + WideLayout::SA, ak);
                if constexpr (MODEL == 1) {
                    tva = ld(sb + WideLayout::STV);
                    hvd = ld(sb + WideLayout::SHVD);
                }
                const T* x = xs[b];
                base[0] = (qd[0] + cv[0]) * x[0] + qv[0];
                base[1] = qd[1] * x[1] + qv[1];
                base[2] = (qd[2] + cv[1]) * x[2] + cv[2] * x[3] + qv[2];
                base[3] = qd[3] * x[3] + cv[2] * x[2] + cv[4] * x[5] + qv[3];
                base[4] = qd[4] * x[4] + qv[4];
                base[5] = (qd[5] + cv[3]) * x[5] + cv[4] * x[3] + qv[5];
                if constexpr (MODEL == 1) base[3] += hvd * dus[b][0];
                const T* xr = xrec(k);
#pragma unroll
                for (int j = 0; j < 6; ++j) {
                    const T ds = xr[WideLayout::XDS + j], rsc = rowscale(j, k);
                    const T dbar = ds * ds;
                    ov[j] = dbar * rsc * rsc >= (T)0.6404;
                    yo[j] = -xr[WideLayout::XE + j] / dbar;
                }
            } else {
#pragma unroll
                for (int q = 0; q < 8; ++q) ak[q] = 0;
            }
            T lam[6];
#pragma unroll
            for (int q = 0; q < 6; ++q) lam[q] = (b < NB - 1 && t == 63) ? lam_in[q] : (T)0;
            const int steps = b == NB - 1 ? N - 64 * b : 64;
            T o[6];
            for (int s = steps - 1; s >= 0; --s) {
                AT_mul(ak, lam, o);
                if constexpr (MODEL == 1) o[3] += tva * (lam[2] + lam[5]);
#pragma unroll
                for (int q = 0; q < 6; ++q) o[q] = ov[q] ? yo[q] : o[q] + base[q];
                wv.dn6(lam, o);
            }
            if (k < N) {
#pragma unroll
                for (int q = 0; q < 6; ++q) st(L.YP(k) + q, -o[q]);
            }
            if (b > 0) {
#pragma unroll
                for (int q = 0; q < 6; ++q) lam_in[q] = wv.lane0(o[q]);
            }
        }
        wv.mark(4);
        wv.sync();
        T linp[NB][6];
        shift_blocks(lin, linp);
        for (int b = 0; b < NB; ++b) {
            const int k = t + 64 * b;
            if (k >= N) continue;
            T* x = xrec(k);
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                const T irs = rcp(rowscale(j, k));
                const T p = x[WideLayout::XP + j], n = x[WideLayout::XN + j];
                const T zp = x[WideLayout::XZP + j], zn = x[WideLayout::XZN + j];
                const T sp_ = zp / p + sv_delta, sn_ = zn / n + sv_delta;
                T gpp = (T)RHO - mu / p + (T)KD * mu, gpn = (T)RHO - mu / n + (T)KD * mu;
                if (rf_pass) {
                    gpp = -x[WideLayout::XRP + j];
                    gpn = -x[WideLayout::XRN + j];
                }
                // the rows' steps: a variable whose Sigma dominates its unit coupling to the
                // constraint row (the Bunch-Kaufman 1x1 pivot test, alpha = 0.6404) from its
                // own row (dp = (y+ - gphi_p)/sp, dn = -(y+ + gphi_n)/sn), else from the
                // constraint row dp - dn = J dx + c with J dx from the primal step -- never y+'s
                // rounding divided by a small Sigma
                const T ysn = ld(L.YP(k) + j) * irs;
                const T q = rowscale(j, k) * (xs[b][j] - (k == 0 ? (T)0 : linp[b][j])) + x[WideLayout::XCR + j];
                const T bk = (T)0.6404;
                T dp, dn;
                if (sp_ >= sn_) {
                    dp = (ysn - gpp) / sp_;
                    dn = sn_ >= bk ? -(ysn + gpn) / sn_ : dp - q;
                } else {
                    dn = -(ysn + gpn) / sn_;
                    dp = sp_ >= bk ? (ysn - gpp) / sp_ : dn + q;
                }
                x[WideLayout::XDP + j] = dp;
                x[WideLayout::XDN + j] = dn;
            }
        }
        wv.mark(5);
        return Fwd{(T)1, (T)1, (T)0, (T)0};  // (the statistics: step_stats_resto, after the refinement)
    }

    // The step statistics of the restoration step in DW, XDP, XDN (fraction to the boundary,
    // grad phi^T d, the relative step), after its iterative refinement; the barrier gradient of
    // x as precompute_resto computes it.
    MPCG_HD Fwd step_stats_resto() {
        const int t = wv.lane();
        wv.sync();
        const T eta = eta_mu();
        Fwd F{(T)1, (T)1, (T)0, (T)0};
        for (int b = 0; b < NB; ++b) {
            const int k = t + 64 * b;
            if (k >= N) continue;
            const bool last = k == N - 1;
            T w[8], zl[8], zu[8], dk[8];
            ldn<8>(L.W(k), w);
            ldn<8>(L.ZL(k), zl);
            ldn<8>(L.ZU(k), zu);
            ldn<8>(L.DW(k), dk);
            const int nv = last ? 6 : 8;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                if (j < nv) {
                    const T dr = dR(k, j);
                    const T rdl = (T)1 / (w[j] - vlo(j)), rdu = (T)1 / (vhi(j) - w[j]);
                    const T gq = eta * dr * dr * (w[j] - xR(k, j)) - mu * rdl + mu * rdu;
                    dir_var(w[j], zl[j], zu[j], vlo(j), vhi(j), gq, dk[j], F);
                }
            }
            const T* x = xrec(k);
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                const T p = x[WideLayout::XP + j], n = x[WideLayout::XN + j];
                const T zp = x[WideLayout::XZP + j], zn = x[WideLayout::XZN + j];
                const T gpp = (T)RHO - mu / p + (T)KD * mu, gpn = (T)RHO - mu / n + (T)KD * mu;
                const T dp = x[WideLayout::XDP + j], dn = x[WideLayout::XDN + j];
                dir_one(p, zp, gpp, dp, F);
                dir_one(n, zn, gpn, dn, F);
            }
        }
        T v[4] = {F.amax_p, F.amax_z, F.gd, F.rel};
        const int op[4] = {RMIN, RMIN, RSUM, RMAX};
        reduce<4, true>(v, op);
        F.amax_p = v[0];
        F.amax_z = v[1];
        F.gd = v[2];
        F.rel = v[3];
        return F;
    }

    // The residual of the full restoration system (z eliminated) at the step in DW, XDP, XDN and
    // y+ in YP -- the x rows (H dx + J^T y+ = -grad phi_x), the p rows (Sigma_p dp - dy =
    // -(grad phi_p - y)), the n rows (Sigma_n dn + dy = -(grad phi_n + y)) and the scaled
    // constraint rows (J dx - dp + dn = -XCR) -- into the records (XRX, XRP, XRN, XRC), and
    // Ipopt's residual ratio |r| / (min(|sol|, 1e6 |rhs|) + |rhs|) (max-norms;
    // PDFullSpaceSolver::ComputeResidualRatio).
    MPCG_HD T resid_resto() {
        const int t = wv.lane();
        wv.sync();
        const T eta = eta_mu(), dlt = sv_delta;
        T lin[NB][6], linp[NB][6];
        for (int b = 0; b < NB; ++b) {
            const int k = t + 64 * b;
#pragma unroll
            for (int j = 0; j < 6; ++j) lin[b][j] = 0;
            if (k < N - 1) {
                T a[8], dx[8], twl = dt, tvl = 0;
                ldv<8>(L.ST(k) + WideLayout::SA, a);
                ldn<8>(L.DW(k), dx);
                if constexpr (MODEL == 1) ld2(L.ST(k) + WideLayout::STW, twl, tvl);
                T l8[8];
                A_mul(a, dx, l8);
                if constexpr (MODEL == 1) {
                    l8[2] += tvl * dx[3];
                    l8[5] += tvl * dx[3];
                }
                l8[2] += twl * dx[6];
                l8[3] += dt * dx[7];
                l8[5] += twl * dx[6];
#pragma unroll
                for (int j = 0; j < 6; ++j) lin[b][j] = l8[j];
            }
        }
        shift_blocks(lin, linp);
        T rn = 0, sn = 0, bn = 0;
        for (int b = 0; b < NB; ++b) {
            const int k = t + 64 * b;
            if (k >= N) continue;
            const bool last = k == N - 1;
            T w[8], dx[8], qd[8], a[8], cv[6], yp[6], y[6], ypn[6] = {0, 0, 0, 0, 0, 0}, yn[6] = {0, 0, 0, 0, 0, 0};
            ldn<8>(L.W(k), w);
            ldn<8>(L.DW(k), dx);
            const int sb = L.ST(k);
            ldv<8>(sb + WideLayout::SQD, qd);
            ldv<8>(sb + WideLayout::SA, a);
            ldv<6>(sb + WideLayout::SCV, cv);
            ldn<6>(L.YP(k), yp);
            ldn<6>(L.Y(k), y);
            if (!last) {
                ldn<6>(L.YP(k + 1), ypn);
                ldn<6>(L.Y(k + 1), yn);
            }
            T twk = dt, tvk = 0, hvd = 0;
            if constexpr (MODEL == 1) {
                twk = ld(sb + WideLayout::STW);
                tvk = ld(sb + WideLayout::STV);
                hvd = ld(sb + WideLayout::SHVD);
            }
            T at[6] = {0, 0, 0, 0, 0, 0}, aty[6] = {0, 0, 0, 0, 0, 0};
            if (!last) {
                AT_mul(a, ypn, at);
                AT_mul(a, yn, aty);
                if constexpr (MODEL == 1) {
                    at[3] += tvk * (ypn[2] + ypn[5]);
                    aty[3] += tvk * (yn[2] + yn[5]);
                }
            }
            // H dx: the diagonal (eta D_R^2 + Sigma + delta_w) and the constraints' curvature
            T hx[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) hx[j] = qd[j] * dx[j];
            hx[0] += cv[0] * dx[0];
            hx[2] += cv[1] * dx[2] + cv[2] * dx[3];
            hx[3] += cv[2] * dx[2] + cv[4] * dx[5];
            hx[5] += cv[3] * dx[5] + cv[4] * dx[3];
            if constexpr (MODEL == 1) {
                if (!last) {
                    hx[3] += hvd * dx[6];
                    hx[6] += hvd * dx[3];
                }
            }
            T* x = xrec(k);
            const int nv = last ? 6 : 8;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                T r = 0;
                if (j < nv) {
                    const T dr = dR(k, j);
                    const T rdl = (T)1 / (w[j] - vlo(j)), rdu = (T)1 / (vhi(j) - w[j]);
                    const T gq = eta * dr * dr * (w[j] - xR(k, j)) - mu * rdl + mu * rdu;
                    const T jt = j < 6 ? yp[j] - at[j] : (j == 6 ? -twk * (ypn[2] + ypn[5]) : -dt * ypn[3]);
                    const T jy = j < 6 ? y[j] - aty[j] : (j == 6 ? -twk * (yn[2] + yn[5]) : -dt * yn[3]);
                    r = -(gq + hx[j] + jt);
                    rn = tmax(rn, (T)fabs(r));
                    sn = tmax(sn, (T)fabs(dx[j]));
                    bn = tmax(bn, (T)fabs(gq + jy));
                }
                x[WideLayout::XRX + j] = r;
            }
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                const T rsc = rowscale(j, k), irs = rcp(rsc);
                const T ys = y[j] * irs, ysp = yp[j] * irs;
                const T p = x[WideLayout::XP + j], n = x[WideLayout::XN + j];
                const T sp_ = x[WideLayout::XZP + j] / p + dlt, sn_ = x[WideLayout::XZN + j] / n + dlt;
                const T gpp = (T)RHO - mu / p + (T)KD * mu, gpn = (T)RHO - mu / n + (T)KD * mu;
                const T dp = x[WideLayout::XDP + j], dn = x[WideLayout::XDN + j], cr = x[WideLayout::XCR + j];
                const T rp = -(gpp - ysp) - sp_ * dp;
                const T rq = -(gpn + ysp) - sn_ * dn;
                const T rc = -cr - (rsc * (dx[j] - (k == 0 ? (T)0 : linp[b][j])) - dp + dn);
                x[WideLayout::XRP + j] = rp;
                x[WideLayout::XRN + j] = rq;
                x[WideLayout::XRC + j] = rc;
                rn = tmax(rn, tmax(tmax((T)fabs(rp), (T)fabs(rq)), (T)fabs(rc)));
                sn = tmax(sn, tmax(tmax((T)fabs(dp), (T)fabs(dn)), (T)fabs(ysp - ys)));
                bn = tmax(bn, tmax(tmax((T)fabs(gpp - ys), (T)fabs(gpn + ys)), (T)fabs(cr)));
            }
        }
        T v[3] = {rn, sn, bn};
        const int op[3] = {RMAX, RMAX, RMAX};
        reduce<3, true>(v, op);
        return wv.uni_d(v[0] / (tmin(v[1], (T)1e6 * v[2]) + v[2]));
    }
    // save (to = true) the step in DW, XDP, XDN, YP and the rows' XCR to the records, setting
    // XCR = -r_c for a correction solve; or add the saved step to the correction there and
    // restore XCR
    MPCG_HD void refine_xfer(bool to) {
        const int t = wv.lane();
        wv.sync();
        for (int b = 0; b < NB; ++b) {
            const int k = t + 64 * b;
            if (k >= N) continue;
            T* x = xrec(k);
            const int nv = k == N - 1 ? 6 : 8;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                if (j < nv) {
                    if (to)
                        x[WideLayout::XSX + j] = ld(L.DW(k) + j);
                    else
                        st(L.DW(k) + j, x[WideLayout::XSX + j] + ld(L.DW(k) + j));
                }
            }
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                if (to) {
                    x[WideLayout::XSP + j] = x[WideLayout::XDP + j];
                    x[WideLayout::XSN + j] = x[WideLayout::XDN + j];
                    x[WideLayout::XSY + j] = ld(L.YP(k) + j);
                    x[WideLayout::XSC + j] = x[WideLayout::XCR + j];
                    x[WideLayout::XCR + j] = -x[WideLayout::XRC + j];
                } else {
                    x[WideLayout::XDP + j] = x[WideLayout::XSP + j] + x[WideLayout::XDP + j];
                    x[WideLayout::XDN + j] = x[WideLayout::XSN + j] + x[WideLayout::XDN + j];
                    st(L.YP(k) + j, x[WideLayout::XSY + j] + ld(L.YP(k) + j));
                    x[WideLayout::XCR + j] = x[WideLayout::XSC + j];
                }
            }
        }
        wv.sync();
    }
    // the step before the last correction (the records' XSX, XSP, XSN, XSY)
    MPCG_HD void refine_undo() {
        const int t = wv.lane();
        wv.sync();
        for (int b = 0; b < NB; ++b) {
            const int k = t + 64 * b;
            if (k >= N) continue;
            T* x = xrec(k);
            const int nv = k == N - 1 ? 6 : 8;
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (j < nv) st(L.DW(k) + j, x[WideLayout::XSX + j]);
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                x[WideLayout::XDP + j] = x[WideLayout::XSP + j];
                x[WideLayout::XDN + j] = x[WideLayout::XSN + j];
                st(L.YP(k) + j, x[WideLayout::XSY + j]);
            }
        }
        wv.sync();
    }
    // Ipopt's iterative refinement of the restoration problem's step (PDFullSpaceSolver::Solve
    // with min_refinement_steps 1, max_refinement_steps 10, residual_ratio_max 1e-10,
    // residual_improvement_factor 1): the reduced solve (p, n eliminated, AugRestoSystemSolver)
    // loses digits where a row is nearly hard (Sigma_p, Sigma_n ~ 1e12 near a feasible row at
    // small mu), and the restoration problem's dual infeasibility then stalls; correction solves
    // of the same reduced system with the full system's residual as the right-hand side
    // recover them.  Returns the step statistics of the refined step.
    MPCG_HD Fwd refine_resto() {
        T ratio = resid_resto(), old = ratio;
        for (int it = 1; it <= 10; ++it) {
            refine_xfer(true);
            rf_pass = true;
            const bool ok = wv.uni(riccati(0, sv_delta));
            if (ok) forward_resto();
            rf_pass = false;
            refine_xfer(false);
            if (!ok) break;  // (the same matrix: cannot fail where the first solve did not)
            ratio = resid_resto();
#ifdef MPCG_TRACE
            if (wv.lane() == 0) printf("  refine %d ratio %.3e (first %.3e)\n", it, (double)ratio, (double)old);
#endif
            if (!(ratio > (T)1e-10)) break;
            if (it > 1 && ratio > old) {  // (no improvement: back to the step before this correction)
                refine_undo();
                break;
            }
            old = ratio;
        }
        return step_stats_resto();
    }

    // fraction to the boundary, grad phi^T d and the relative step of a variable with the
    // lower bound 0 only
    MPCG_HD void dir_one(T v, T z, T gphi, T dv, Fwd& F) const {
        const T inf = (T)INFINITY;
        F.amax_p = tmin(F.amax_p, dv < 0 ? -tau * v / dv : inf);
        const T dz = mu / v - z - z / v * dv;
        F.amax_z = tmin(F.amax_z, dz < 0 ? -tau * z / dz : inf);
        F.gd += gphi * dv;
        F.rel = tmax(F.rel, (T)fabs(dv) / ((T)1 + (T)fabs(v)));
    }

    // second-order correction right-hand side: c_soc = c_R(trial) + alpha c_soc (XCR)
    MPCG_HD void soc_rhs_resto(T alpha) {
        const int t = wv.lane();
        wv.sync();
        T w[NB][8], cs[NB][6];
        load_w(w, alpha, true);
        rows_c(w, cs);
        for (int b = 0; b < NB; ++b) {
            const int k = t + 64 * b;
            if (k >= N) continue;
            T* x = xrec(k);
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                const T p = x[WideLayout::XP + j] + alpha * x[WideLayout::XDP + j];
                const T n = x[WideLayout::XN + j] + alpha * x[WideLayout::XDN + j];
                x[WideLayout::XCR + j] = (cs[b][j] - p + n) + alpha * x[WideLayout::XCR + j];
            }
        }
        wv.sync();
    }

    // the restoration problem's primal-dual system error (soft restoration)
    MPCG_HD T pd_error_resto() {
        const int t = wv.lane();
        wv.sync();
        const T eta = eta_mu();
        T w8[NB][8], cs[NB][6];
        load_w(w8, (T)0, false);
        rows_c(w8, cs);
        T du = 0, pr_ = 0, cm = 0;
        for (int b = 0; b < NB; ++b) {
            const int k = t + 64 * b;
            if (k >= N) continue;
            const bool last = k == N - 1;
            T w[8], zl[8], zu[8], y[6], yn[6] = {0, 0, 0, 0, 0, 0}, a[7] = {0, 0, 0, 0, 0, 0, 0};
            T twk = dt, tvk = 0;
            ldn<8>(L.W(k), w);
            ldn<8>(L.ZL(k), zl);
            ldn<8>(L.ZU(k), zu);
            ldn<6>(L.Y(k), y);
            if (!last) {
                ldn<6>(L.Y(k + 1), yn);
                Lin<T> ln;
                ln.eval(pcoef().c, w);
                ln.jac(w, dt, a);
                turn_d(w, w + 6, &twk, &tvk);
            }
            T at[6] = {0, 0, 0, 0, 0, 0};
            if (!last) {
                AT_mul(a, yn, at);
                if (model == 1) at[3] += tvk * (yn[2] + yn[5]);
            }
            const T btw = twk * (yn[2] + yn[5]), bta = dt * yn[3];
            const int nv = last ? 6 : 8;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                if (j < nv) {
                    const T dr = dR(k, j);
                    const T gq = eta * dr * dr * (w[j] - xR(k, j));
                    const T gj = j < 6 ? gq + y[j] - at[j] : gq - (j == 6 ? btw : bta);
                    du += fabs(gj - zl[j] + zu[j]);
                    cm += fabs((w[j] - vlo(j)) * zl[j] - mu) + fabs((vhi(j) - w[j]) * zu[j] - mu);
                }
            }
            const T* x = xrec(k);
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                const T p = x[WideLayout::XP + j], n = x[WideLayout::XN + j];
                const T zp = x[WideLayout::XZP + j], zn = x[WideLayout::XZN + j];
                const T ys = y[j] * rcp(rowscale(j, k));
                pr_ += fabs(cs[b][j] - p + n);
                du += fabs((T)RHO - ys - zp) + fabs((T)RHO + ys - zn);
                cm += fabs(p * zp - mu) + fabs(n * zn - mu);
            }
        }
        T v[3] = {du, pr_, cm};
        const int op[3] = {RSUM, RSUM, RSUM};
        reduce<3, true>(v, op);
        const int nw = (8 * N - 2) + 12 * N, m = 6 * N, nbnd = 2 * (8 * N - 2) + 12 * N;
        return wv.uni_d((v[0] + v[1] + v[2]) / (T)(nw + m + nbnd));
    }

    // copies of the lane-owned HBM records (RESTO; no-op otherwise): stage k's [xoff, xoff + n)
    // to / from its spill copy at soff
    MPCG_HD void xcopy(bool out, int xoff, int soff, int n) {
        if constexpr (RESTO) {
            const int t = wv.lane();
            for (int b = 0; b < NB; ++b) {
                const int k = t + 64 * b;
                if (k >= N) continue;
                T* x = xrec(k);
                T* s = xsp + (size_t)k * WideLayout::XW + soff;
                for (int q = 0; q < n; ++q) {
                    if (out)
                        s[q] = x[xoff + q];
                    else
                        x[xoff + q] = s[q];
                }
            }
        }
    }

    // ------------------------------------------------------------ HBM spill area
    // Copy LDS [lds0, lds0 + n) to / from the problem's spill area at sp0: lane t moves
    // elements t, t + 64, ... both ways, so a lane reads back only what it wrote.
    MPCG_HD void spill_out(int sp0, int lds0, int n) {
        const int t = wv.lane();
        wv.sync();
        for (int e = t; e < n; e += 64) spill[sp0 + e] = ld(lds0 + e);
    }
    MPCG_HD void spill_in(int sp0, int lds0, int n) {
        const int t = wv.lane();
        wv.sync();
        for (int e = t; e < n; e += 64) st(lds0 + e, (T)spill[sp0 + e]);
        wv.sync();
    }
    // the same for the fields [off, off + len) of every stage's iterate record (len N elements
    // at sp0, stage-major)
    template <int off, int len>
    MPCG_HD void rec_out(int sp0) {
        const int t = wv.lane();
        wv.sync();
        for (int e = t; e < len * N; e += 64) spill[sp0 + e] = ld(WideLayout::RS * (e / len) + off + e % len);
    }
    template <int off, int len>
    MPCG_HD void rec_in(int sp0) {
        const int t = wv.lane();
        wv.sync();
        for (int e = t; e < len * N; e += 64) st(WideLayout::RS * (e / len) + off + e % len, (T)spill[sp0 + e]);
        wv.sync();
    }

    // ------------------------------------------------------------ the filter
    // Ipopt's FilterLSAcceptor / Filter (oracle/ipm.c: set_ref .. update_for_next).
    MPCG_HD static bool compare_le(T lhs, T rhs, T bas) {  // IpUtils Compare_le
        return lhs - rhs <= (T)(10.0 * EPS) * (T)fabs(bas);
    }
    // the reference point of a line search; the switching-condition powers once per search
    MPCG_HD void set_ref(T th, T ph, T gd) {
        ref_theta = wv.uni_d(th);
        ref_phi = wv.uni_d(ph);
        ref_gd = wv.uni_d(gd);
        ref_pgd = 0;
        ref_pth = 0;
        // obj_max_inc: a trial barrier value more than 10^(obj_max_inc basval) above the
        // reference is rejected (log10(phi_t - phi_ref) > obj_max_inc basval, evaluated once
        // per search as the threshold)
        // 10^(obj_max_inc log10|phi|) = |phi|^obj_max_inc (|phi| > 10; 10^obj_max_inc else);
        // the default 5 by products
        const T b = tmax((T)fabs(ref_phi), (T)10);
        if (P.obj_max_inc == 5.0) {
            const T b2 = b * b;
            ref_inc = wv.uni_d(b2 * b2 * b);
        } else {
            ref_inc = wv.uni_d((T)pow((double)b, P.obj_max_inc));
        }
        if (wv.uni(gd < 0)) {
            // (-gd)^s_phi in the even lanes and theta^s_theta in the odd ones: one evaluation
            // of the power kernel for both (the wave-uniform operands, one lane each)
            const bool odd = (wv.lane() & 1) != 0;
            const double pw = pow_pos(odd ? (th > 0 ? (double)th : 1.0) : (double)-gd, odd ? 1.1 : 2.3);
            ref_pgd = (T)wv.lane0(pw);
            ref_pth = th > 0 ? (T)wv.lanev(pw, 1) : (T)0;
        }
    }
    MPCG_HD bool is_ftype(T alpha_test) const { return ref_gd < 0 && alpha_test * ref_pgd > ref_pth; }
    MPCG_HD bool armijo_holds(T alpha_test, T phit) const {
        return compare_le(phit - ref_phi, (T)1e-8 * alpha_test * ref_gd, ref_phi);
    }
    MPCG_HD bool acceptable_to_current_iterate(T phit, T thetat) const {
        const T gamma_theta = (T)1e-5, gamma_phi = (T)1e-8;
        if (phit > ref_phi && phit - ref_phi > ref_inc) return false;  // obj_max_inc
        return compare_le(thetat, ((T)1 - gamma_theta) * ref_theta, ref_theta) ||
               compare_le(phit - ref_phi, -gamma_phi * ref_theta, ref_phi);
    }
    // filter entry f (theta, phi): the first filter_cap in LDS, the next WideLayout::FX in
    // the workspace (the restoration problem's own region)
    MPCG_HD int fx_off() const { return RESTO ? L.SP_FLTR() : L.SP_FLT(); }
    MPCG_HD void fget(int f, T& th, T& ph) const {
        if (f < L.cap) {
            th = ld(L.FI() + 2 * f);
            ph = ld(L.FI() + 2 * f + 1);
        } else {
            const T* x = spill + fx_off() + 2 * (f - L.cap);
            th = x[0];
            ph = x[1];
        }
    }
    MPCG_HD void fset(int f, T th, T ph) const {
        if (f < L.cap) {
            st(L.FI() + 2 * f, th);
            st(L.FI() + 2 * f + 1, ph);
        } else {
            T* x = spill + fx_off() + 2 * (f - L.cap);
            x[0] = th;
            x[1] = ph;
        }
    }
    // acceptable to the filter: no entry f with theta >= theta_f and phi >= phi_f (lane f tests entry f)
    MPCG_HD bool filter_ok(T phit, T thetat) {
        const int t = wv.lane();
        bool hit = false;
        for (int f0 = 0; f0 < nf; f0 += 64) {
            const int f = f0 + t;
            T e0 = 0, e1 = 0;
            if (f < nf) fget(f, e0, e1);
            const bool h = f < nf && thetat >= e0 && phit >= e1;
            hit = hit || wv.any(h);
        }
        return !hit;
    }
    // Filter::AddEntry: the entries the new one dominates are dropped (acceptance does not
    // change); the filter holds filter_cap + WideLayout::FX entries, beyond which the oldest
    // is dropped and counted (n_fover)
    MPCG_HD void filter_add(T ph, T th) {
        const int t = wv.lane();
        const int cap = L.cap + WideLayout::FX;
        const bool ext = nf > L.cap;  // (entries in the workspace: cross-lane global-memory order)
        int base = 0;
        for (int f0 = 0; f0 < nf; f0 += 64) {
            const int f = f0 + t;
            T e0 = 0, e1 = 0;
            wv.sync();
            if (f < nf) fget(f, e0, e1);
            const bool keep = f < nf && !(ph <= e1 && th <= e0);
            int cnt;
            const int dst = base + wv.ballot_prefix(keep, &cnt);
            wv.sync();
            if (ext) wv.gsync();
            if (keep) fset(dst, e0, e1);
            base += cnt;
        }
        nf = wv.uni(base);
        int slot = nf;
        if (nf == cap) {  // full: drop the oldest entry
            ++n_fover;
            T e0 = 0, e1 = 0;
            for (int f0 = 0; f0 < cap; f0 += 64) {
                const int f = f0 + t + 1;
                wv.sync();
                wv.gsync();
                if (f < cap) fget(f, e0, e1);
                wv.sync();
                wv.gsync();
                if (f < cap) fset(f - 1, e0, e1);
            }
            slot = cap - 1;
        } else {
            ++nf;
            nf_peak = nf > nf_peak ? nf : nf_peak;
        }
        wv.sync();
        if (t == 0) fset(slot, th, ph);
        wv.sync();
        if (nf > L.cap) wv.gsync();
    }
    MPCG_HD void augment_filter() {
        filter_add(ref_phi - (T)1e-8 * ref_theta, ((T)1 - (T)1e-5) * ref_theta);
    }
    // FilterLSAcceptor::CheckAcceptabilityOfTrialPoint (with the filter reset heuristic)
    MPCG_HD bool check_acceptability(T alpha_test, T phit, T thetat) {
        if (theta_max() < 0) theta_max() = wv.uni_d((T)1e4 * tmax((T)1, ref_theta));
        if (theta_min < 0) theta_min = wv.uni_d((T)1e-4 * tmax((T)1, ref_theta));
        if (wv.uni(thetat > theta_max())) return false;
        bool accept;
        if (alpha_test > 0 && is_ftype(alpha_test) && ref_theta <= theta_min)
            accept = armijo_holds(alpha_test, phit);
        else
            accept = acceptable_to_current_iterate(phit, thetat);
        if (!wv.uni(accept)) {
            last_rej_filter = 0;
            return false;
        }
        if (!filter_ok(phit, thetat)) {
            last_rej_filter = 1;
            return false;
        }
        if (P.max_filter_resets > 0 && n_filter_resets < P.max_filter_resets) {
            if (last_rej_filter) {
                if (++count_filter_rej >= P.filter_reset_trigger) {
                    nf = 0;
                    count_filter_rej = 0;
                    ++n_filter_resets;
                }
            } else {
                count_filter_rej = 0;
            }
        }
        return true;
    }
    // FilterLSAcceptor::UpdateForNextIteration: augment unless an f-type step with Armijo
    MPCG_HD void update_for_next(T alpha_test, T phit) {
        if (wv.uni(!is_ftype(alpha_test) || !armijo_holds(alpha_test, phit))) augment_filter();
    }
    // FilterLSAcceptor::CalculateAlphaMin (reference point values)
    MPCG_HD T alpha_min_of() const {
        const T gamma_theta = (T)1e-5, gamma_phi = (T)1e-8;
        T a;
        if (ref_gd < 0) {
            a = tmin(gamma_theta, gamma_phi * ref_theta * rcp(-ref_gd));
            if (ref_theta <= theta_min) a = tmin(a, ref_pth * rcp(ref_pgd));
        } else {
            a = gamma_theta;
        }
        return (T)0.05 * a;
    }

    // ------------------------------------------------------------ sweeps of the line search
    // Right-hand side of a second-order correction: d_soc = d(trial) + alpha d_soc, i.e.
    // c_soc = c(w + alpha dw) + alpha c_soc on the dynamics rows (stage table SD) and the
    // initial-state rows (C0); the trial point is the last one tried (W + alpha DW).
    MPCG_HD void soc_rhs(T alpha) {
        if constexpr (RESTO) {
            soc_rhs_resto(alpha);
            return;
        }
        const int t = wv.lane();
        wv.sync();
        for (int b = 0; b < NB; ++b) {
        const int k = t + 64 * b;
        T dn[6] = {0, 0, 0, 0, 0, 0}, c0[6] = {0, 0, 0, 0, 0, 0};
        if (k < N) {
            T w[8], cw[8], cd[8];
            ldn<8>(L.W(k), cw);
            ldn<8>(L.DW(k), cd);
#pragma unroll
            for (int j = 0; j < 8; ++j) w[j] = cw[j] + alpha * cd[j];
            if (k < N - 1) {
                T wn[6], cwn[6], cdn[6];
                ldn<6>(L.W(k + 1), cwn);
                ldn<6>(L.DW(k + 1), cdn);
#pragma unroll
                for (int j = 0; j < 6; ++j) wn[j] = cwn[j] + alpha * cdn[j];
                Lin<T> ln;
                ln.eval(pcoef().c, w);
                T F[6];
                next_m(ln, w, w + 6, F);
#pragma unroll
                for (int j = 0; j < 6; ++j) dn[j] = F[j] - wn[j];
            }
#pragma unroll
            for (int j = 0; j < 6; ++j) c0[j] = -(w[j] - pinit(j));
        }
        if (k < N - 1) {
            const int sb = L.ST(k) + WideLayout::SD;
#pragma unroll
            for (int j = 0; j < 6; ++j) st(sb + j, dn[j] + alpha * ld(sb + j));
        }
        if (k == 0) {
#pragma unroll
            for (int j = 0; j < 6; ++j) st(L.C0() + j, c0[j] + alpha * ld(L.C0() + j));
        }
        }
        wv.sync();
    }

    // Primal-dual system error (1-norms of the dual infeasibility, the scaled constraint
    // violation and the mu-complementarity, averaged over their 2(8N-2) + 6N + 8N-2
    // entries) of the iterate in LDS: the soft restoration phase's measure.
    MPCG_HD T pd_error() {
        if constexpr (RESTO) return pd_error_resto();
        const int t = wv.lane();
        wv.sync();
        T du = 0, pr_ = 0, cm = 0;
        T Fk[NB][6];
        for (int b = 0; b < NB; ++b) {
            const int k = t + 64 * b;
#pragma unroll
            for (int j = 0; j < 6; ++j) Fk[b][j] = 0;
            if (k >= N) continue;
            const bool last = k == N - 1;
            T w[8], zl[8], zu[8], y[6], yn[6] = {0, 0, 0, 0, 0, 0}, up[2] = {0, 0}, um[2] = {0, 0},
                a[7] = {0, 0, 0, 0, 0, 0, 0};
            T twk = dt, tvk = 0;
            ldn<8>(L.W(k), w);
            ldn<8>(L.ZL(k), zl);
            ldn<8>(L.ZU(k), zu);
            ldn<6>(L.Y(k), y);
            if (!last) {
                ldn<6>(L.Y(k + 1), yn);
                up[0] = ld(L.W(k + 1) + 6);
                up[1] = ld(L.W(k + 1) + 7);
                Lin<T> ln;
                ln.eval(pcoef().c, w);
                ln.jac(w, dt, a);
                next_m(ln, w, w + 6, Fk[b]);
                turn_d(w, w + 6, &twk, &tvk);
            }
            if (k >= 1) {
                um[0] = ld(L.W(k - 1) + 6);
                um[1] = ld(L.W(k - 1) + 7);
            }
            T g[6], at[6] = {0, 0, 0, 0, 0, 0}, gu[2] = {0, 0};
            grad_state(w, g);
            if (!last) {
                AT_mul(a, yn, at);
                if (model == 1) at[3] += tvk * (yn[2] + yn[5]);
                grad_ctrl(k, um, w + 6, up, gu);
            }
            const T btw = twk * (yn[2] + yn[5]), bta = dt * yn[3];
            const int nv = last ? 6 : 8;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                if (j < nv) {
                    const T gj = j < 6 ? sf * g[j] + y[j] - at[j] : sf * gu[j - 6] - (j == 6 ? btw : bta);
                    du += fabs(gj - zl[j] + zu[j]);
                    cm += fabs((w[j] - vlo(j)) * zl[j] - mu) + fabs((vhi(j) - w[j]) * zu[j] - mu);
                }
            }
        }
        T Fprev[NB][6];
        shift_blocks(Fk, Fprev);
        for (int b = 0; b < NB; ++b) {
            const int k = t + 64 * b;
            if (k >= N) continue;
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                const T wj = ld(L.W(k) + j);
                const T c = k == 0 ? wj - pinit(j) : wj - Fprev[b][j];
                pr_ += fabs(rowscale(j, k) * c);
            }
        }
        T v[3] = {du, pr_, cm};
        const int op[3] = {RSUM, RSUM, RSUM};
        reduce<3, true>(v, op);
        return wv.uni_d((v[0] + v[1] + v[2]) / (T)((8 * N - 2) + 6 * N + 2 * (8 * N - 2)));
    }
    // kappa_sigma correction of every bound multiplier (an immediately accepted step)
    MPCG_HD void clamp_all() {
        const int t = wv.lane();
        wv.sync();
        const T bl[3] = {sl, wl, al}, bh[3] = {su, wu, au};
        for (int e = t; e < 8 * N; e += 64) {
            const int k = e >> 3, j = e & 7;
            if (k == N - 1 && j >= 6) continue;
            const T lo = j < 6 ? bl[0] : (j == 6 ? bl[1] : bl[2]);
            const T hi = j < 6 ? bh[0] : (j == 6 ? bh[1] : bh[2]);
            T zln, zun;
            clamp_z(ld(L.W(k) + j), ld(L.ZL(k) + j), ld(L.ZU(k) + j), lo, hi, &zln, &zun);
            st(L.ZL(k) + j, zln);
            st(L.ZU(k) + j, zun);
        }
        if constexpr (RESTO) {
            for (int b = 0; b < NB; ++b) {
                const int k = t + 64 * b;
                if (k >= N) continue;
                T* x = xrec(k);
#pragma unroll
                for (int j = 0; j < 12; ++j) {  // (p, n then z_p, z_n: XZP = XP + 12)
                    const T v = x[WideLayout::XP + j];
                    x[WideLayout::XZP + j] = tmax(tmin(x[WideLayout::XZP + j], (T)1e10 * mu / v), mu / ((T)1e10 * v));
                }
            }
        }
        wv.sync();
    }
    // max |dy| of the direction (the tiny-step test's multiplier part; Ipopt's scaled multipliers)
    MPCG_HD T dy_max() {
        const int t = wv.lane();
        wv.sync();
        T m = 0;
        for (int b = 0; b < NB; ++b) {
            const int k = t + 64 * b;
            if (k < N) {
#pragma unroll
                for (int j = 0; j < 6; ++j)
                    m = tmax(m, (T)fabs(ld(L.YP(k) + j) - ld(L.Y(k) + j)) * rcp(rowscale(j, k)));
            }
        }
        return rmax(m);
    }


    // ------------------------------------------------------------ the solver as a state machine
    // Every sweep (statistics, Newton system = Riccati + forward pass, trial point,
    // second-order-correction right-hand side, primal-dual error) has exactly one call site
    // in solve(); the control logic between sweeps -- Ipopt's convergence test, barrier
    // update, inertia correction, filter line search with second-order corrections,
    // watchdog and soft restoration -- runs as continuations (K_*) on wave-uniform values.
    // (Inlined at several call sites the sweeps did not fit the register budget.)
    enum Op : int { OP_STATS = 0, OP_SOLVE = 1, OP_TRIAL = 2, OP_PDERR = 3, OP_SOCRHS = 4 };
    enum Ct : int {
        K_LSQ = 0, K_BEGIN, K_NEWTON, K_BT, K_SOCRHS, K_SOC, K_SOC_TRIAL, K_SOFT_TRIAL, K_SOFT_PD0, K_SOFT_PD1,
        K_WD_STATS, K_RMU
    };
    enum : int { LS_CONT = -1 };  // a continuation: the next sweep is set
    int op, ct;
    // operands and results of the sweeps
    bool st_acc, sv_ok, tr_ok;
    int sv_mode;
    T st_alpha, st_z, sv_delta, tr_alpha, tr_test, tr_phi, tr_theta, pd_val;
    bool tr_acc;  // the trial point passed CheckAcceptabilityOfTrialPoint(tr_test)
    Fwd sv_F;
    // line-search state (BacktrackingLineSearch)
    Fwd lsF;  // statistics of the direction in DW / YP
    T ls_alpha, ls_alpha_max, ls_alpha_min, ls_alpha_test, ls_amax_z;
    int ls_n_steps, inertia_attempt, soft_ctx;
    bool ls_eval_error, ls_skip_first, wd_from_tiny;
    int soc_count;
    bool cur_acceptable;

    MPCG_HD int set_op(int o, int c) {
        op = o;
        ct = c;
        return LS_CONT;
    }
    // a trial point, checked by the filter acceptor with step length alpha_test
    MPCG_HD int do_trial(T alpha, T alpha_test, int c) {
        tr_alpha = wv.uni_d(alpha);
        tr_test = wv.uni_d(alpha_test);
        return set_op(OP_TRIAL, c);
    }
    MPCG_HD int do_solve(int mode, T delta, int c) {
        sv_mode = mode;
        sv_delta = wv.uni_d(delta);
        return set_op(OP_SOLVE, c);
    }
    MPCG_HD int do_stats(bool acc, T alpha, T z, int c) {
        st_acc = acc;
        st_alpha = alpha;
        st_z = z;
        return set_op(OP_STATS, c);
    }

    MPCG_HD void init() {
        setup();
        init_point();
        reset_state((T)P.mu_init, 0);
        // least-squares multipliers first (constr_mult_init_max 1000)
        do_solve(1, (T)0, K_LSQ);
    }
    // the solver state at the start of a solve: barrier parameter mu0, iteration count it0
    MPCG_HD void reset_state(T mu0, int it0) {
        mu = wv.uni_d(mu0);
        tau = wv.uni_d(tmax((T)0.99, (T)1 - mu0));
        status = 0;
        theta_max() = -1;
        theta_min = -1;
        dw_last = 0;
        delta_w_used = 0;
        acc_alpha = 0;
        acc_z = 0;
        acc_pending = false;
        iter = it0;
        nf = 0;
        kkt() = 0;
        ref_theta = ref_phi = ref_gd = ref_pgd = ref_pth = 0;
        last_rej_filter = count_filter_rej = n_filter_resets = 0;
        in_wd = wd_short = wd_trial_iter = tiny_last = tiny_flag = in_soft = soft_count = acc_counter = have_acc = 0;
        wd_alpha_test() = wd_theta() = wd_phi() = wd_gd() = wd_amax_z() = 0;
        last_mu() = -1;
        last_obj() = 0;
        curr_obj() = (T)-1e50;
        cur_acceptable = false;
        st_acc = sv_ok = tr_ok = false;
        st_alpha = st_z = tr_alpha = tr_test = tr_phi = tr_theta = pd_val = 0;
        tr_acc = false;
        ls_alpha = ls_alpha_max = ls_alpha_min = ls_alpha_test = ls_amax_z = 0;
        ls_n_steps = inertia_attempt = soft_ctx = 0;
        ls_eval_error = ls_skip_first = wd_from_tiny = false;
        soc_alpha() = soc_amax_z() = soc_theta_old() = soc_theta_trial() = soft_ec() = soft_a() = 0;
        soc_count = 0;
        lsF = Fwd{(T)1, (T)1, (T)0, (T)0};
        sv_F = lsF;
    }

    // The fp32 solver's hand-over to the fp64 solver (BASELINE configs[2], mpcg_params.precision
    // 1): h[0] 1 if the fp32 solve converged (status 1 or 4: the fp64 solver continues from its
    // iterate) else 0 (it is solved again from the start), h[1] mu, h[2] iterations, then the
    // iterate w (8N), z_L (8N), z_U (8N), y (6N) in float (WideLayout's stage-major order).
    static constexpr int HANDOFF_HEAD = 4;
    MPCG_HD static int handoff_elems(int N_) { return HANDOFF_HEAD + 30 * N_; }
    MPCG_HD void handoff_out(float* h) const {
        const int t_ = wv.lane();
        wv.sync();
        if (t_ == 0) {
            h[0] = (status == IPM_SUCCESS || status == IPM_ACCEPTABLE) ? 1.0f : 0.0f;
            h[1] = (float)mu;
            h[2] = (float)iter;
            h[3] = 0.0f;
        }
        float* x = h + HANDOFF_HEAD;
        for (int e = t_; e < 8 * N; e += 64) {
            const int k = e >> 3, j = e & 7;
            x[e] = (float)ld(L.W(k) + j);
            x[8 * N + e] = (float)ld(L.ZL(k) + j);
            x[16 * N + e] = (float)ld(L.ZU(k) + j);
        }
        for (int e = t_; e < 6 * N; e += 64) {
            const int k = e / 6, j = e - 6 * k;
            x[24 * N + e] = (float)ld(L.Y(k) + j);
        }
    }
    // The fp64 solver continued from the fp32 solver's converged iterate (handoff_out): the same
    // setup (scaling and row scales from the problem's initial state), the iterate, multipliers
    // and barrier parameter of the fp32 solve, a fresh filter and line-search state, then the
    // algorithm as from any iterate until Ipopt's fp64 termination test holds.  The iteration
    // count continues the fp32 solve's.
    MPCG_HD void solve_warm(const float* h) {
        init_warm(h);
        run();
    }
    // (the state solve_warm runs from: callers with one run() call site use init_warm / init)
    MPCG_HD void init_warm(const float* h) {
        setup();
        init_point();  // (the stage table's constants; the iterate is overwritten)
        wv.sync();
        const float* x = h + HANDOFF_HEAD;
        for (int e = t; e < 8 * N; e += 64) {
            const int k = e >> 3, j = e & 7;
            if (k == N - 1 && j >= 6) continue;  // (no control at the last stage)
            st(L.W(k) + j, (T)x[e]);
            st(L.ZL(k) + j, (T)x[8 * N + e]);
            st(L.ZU(k) + j, (T)x[16 * N + e]);
        }
        for (int e = t; e < 6 * N; e += 64) {
            const int k = e / 6, j = e - 6 * k;
            st(L.Y(k) + j, (T)x[24 * N + e]);
        }
        wv.sync();
        reset_state((T)h[1], (int)h[2]);
        do_stats(false, (T)0, (T)0, K_BEGIN);
    }

    // K_LSQ: the least-squares multiplier estimate y0, used if |y0| <= 1000
    MPCG_HD int k_lsq() {
        T ymax = 0;
        if (sv_ok) {
            const int t = wv.lane();
            wv.sync();
            T m = 0;
            for (int b = 0; b < NB; ++b) {
                const int k = t + 64 * b;
                if (k < N) {
#pragma unroll
                    for (int j = 0; j < 6; ++j) m = tmax(m, (T)fabs(ld(L.YP(k) + j) * rcp(rowscale(j, k))));
                }
            }
            ymax = rmax(m);
        }
        const bool use = sv_ok && ymax <= (T)1000;
        {
            const int t = wv.lane();
            wv.sync();
            for (int b = 0; b < NB; ++b) {
                const int k = t + 64 * b;
                if (k < N) {
#pragma unroll
                    for (int j = 0; j < 6; ++j) st(L.Y(k) + j, use ? ld(L.YP(k) + j) : (T)0);
                }
            }
        }
        return do_stats(false, (T)0, (T)0, K_BEGIN);
    }

    // K_BEGIN: convergence (OptimalityErrorConvergenceCheck::CheckConvergence) and the
    // monotone barrier update (MonotoneMuUpdate::UpdateBarrierParameter) at the iterate
    // the statistics sweep just evaluated; then the Newton system.
    MPCG_HD int k_begin() {
        if constexpr (RESTO) return k_begin_resto();
        acc_pending = false;
        const int nbnd = 2 * (8 * N - 2);
        const int ng = 6 * N;
        // (quotients by v_rcp_f64 + two Newton steps: 1-2 ulp of the division, a fifth of
        // its instructions; the termination tests are not decided at that resolution)
        const T sd = tmax((T)100, (l1y + l1z) * rcp((T)(ng + nbnd))) * (T)0.01;
        const T scc = tmax((T)100, l1z * rcp((T)nbnd)) * (T)0.01;
        const T isd = rcp(sd), iscc = rcp(scc), isf = rcp(sf);
        const T dsd = dual_inf * isd;
        const T E0 = tmax(dsd, tmax(prim_inf, compl0 * iscc));
        // unscaled_curr_dual_infeasibility / _complementarity: objective scaling undone
        const T dual_uns = dual_inf * isf, compl_uns = compl0 * isf;
        kkt() = wv.uni_d(tmax(dual_uns, tmax(prim_uns, compl_uns)));
        // CurrentIsAcceptable (objective bookkeeping once per iteration)
        last_obj() = curr_obj();
        curr_obj() = wv.uni_d(sf * fval);
        cur_acceptable = wv.uni(E0 <= (T)P.acceptable_tol && dual_uns <= (T)P.acceptable_dual_inf_tol &&
                                prim_uns <= (T)P.acceptable_constr_viol_tol &&
                                compl_uns <= (T)P.acceptable_compl_inf_tol &&
                                fabs(last_obj() - curr_obj()) <=
                                    (T)P.acceptable_obj_change_tol * tmax((T)1, (T)fabs(curr_obj())));
#ifdef MPCG_TRACE
        if (wv.lane() == 0)
            printf("it %d mu %.3e E0 %.3e dual %.3e prim %.3e compl %.3e duns %.3e puns %.3e cuns %.3e th %.3e\n", iter,
                   (double)mu, (double)E0, (double)(dual_inf / sd), (double)prim_inf, (double)(compl0 / scc),
                   (double)dual_uns, (double)prim_uns, (double)compl_uns, (double)theta);
#endif
        int s = 0;
        // Ipopt's invalid-number test on f and g at the iterate (the max-norms above
        // drop a NaN; the sums do not)
        if (!isfinite((double)E0) || !isfinite((double)theta) || !isfinite((double)fval)) {
            s = IPM_INVALID_NUMBER;
        } else if (E0 <= (T)P.tol && dual_uns <= (T)P.dual_inf_tol && prim_uns <= (T)P.constr_viol_tol &&
                   compl_uns <= (T)P.compl_inf_tol) {
            s = IPM_SUCCESS;
        } else {
            if (P.acceptable_iter > 0 && cur_acceptable) {
                if (++acc_counter >= P.acceptable_iter) s = IPM_ACCEPTABLE;
            } else {
                acc_counter = 0;
            }
            if (!s && iter >= P.max_iter) s = IPM_MAXITER;
            if (!s && P.cpu_iter_budget >= 0 && iter > P.cpu_iter_budget) s = IPM_UNKNOWN;
        }
        s = wv.uni(s);
        if (s) return s;
        const T kappa_eps = 10, kappa_mu = (T)0.2, theta_mu = (T)1.5;
        const T mu_min = (T)(fmin(P.tol, P.compl_inf_tol) / 11.0);  // min(tol, compl_inf_tol) / (kappa_eps + 1)
        int tf = tiny_flag;
        tiny_flag = 0;
        bool done = false;
        T complmu = tmax(pmax - mu, mu - pmin);
        T Emu = tmax(dsd, tmax(prim_inf, complmu * iscc));
        while (wv.uni((Emu <= kappa_eps * mu || tf) && !done)) {
            // (mu^1.5 >= 0.2 mu exactly where sqrt(mu) >= 0.2: above 0.0401 the power -- a
            // double-double log and exp, ~250 instructions -- cannot be the minimum, and is
            // skipped; the first update from mu_init 0.1 is such a one)
            const T lin_mu = kappa_mu * mu;
            const T sup_mu = wv.uni(mu > (T)0.0401) ? lin_mu : (T)pow((double)mu, (double)theta_mu);
            const T mnew = wv.uni_d(tmax(tmin(lin_mu, sup_mu), mu_min));
            const bool changed = mnew != mu;
            if (!changed && tf) return IPM_TINY_STEP;
            mu = mnew;
            tau = wv.uni_d(tmax((T)0.99, (T)1 - mu));
            if (!changed) {
                done = true;
            } else {
                complmu = tmax(pmax - mu, mu - pmin);
                Emu = tmax(dsd, tmax(prim_inf, complmu * iscc));
                done = Emu > kappa_eps * mu;
            }
            if (done && changed) {  // BacktrackingLineSearch::Reset
                in_soft = 0;
                in_wd = 0;
                wd_short = 0;
                nf = 0;
            }
            tf = 0;
        }
        wv.mark(8);
        inertia_attempt = 0;
        return do_solve(0, (T)0, K_NEWTON);
    }

    // K_NEWTON: inertia correction (Algorithm IC); once the system is solved, the line search
    MPCG_HD int k_newton() {
        wv.mark(11);
        if (!sv_ok) {
            T delta_w = sv_delta;
            if (inertia_attempt == 0)
                delta_w = (dw_last == 0) ? (T)1e-4 : tmax((T)1e-20, dw_last / (T)3);
            else
                delta_w = (dw_last == 0) ? (T)100 * delta_w : (T)8 * delta_w;
            ++inertia_attempt;
            // max_hessian_perturbation 1e20 (Ipopt 3.12's default): the iteration is skipped
            // into the restoration phase; in the restoration problem it is an error
            if (wv.uni((double)delta_w > 1e20 || !isfinite((double)delta_w))) {
                if constexpr (RESTO) return IPM_ERROR_IN_STEP;
                else return ls_goto_resto();
            }
            return do_solve(0, delta_w, K_NEWTON);
        }
        if (sv_delta > 0) dw_last = sv_delta;
        delta_w_used = sv_delta;
        return ls_begin(sv_F);
    }

    // BacktrackingLineSearch::FindAcceptableTrialPoint, up to the backtracking search
    MPCG_HD int ls_begin(Fwd F) {
        if (mu != last_mu()) {
            in_wd = 0;
            wd_short = 0;
            last_mu() = mu;
        }
        if (!RESTO && P.acceptable_iter > 0 && cur_acceptable) {
            rec_out<0, 8>(L.SP_ACC());
            have_acc = 1;
        }
        const T phik = phi_cur();
        if (in_wd)
            set_ref(wd_theta(), wd_phi(), wd_gd());
        else
            set_ref(theta, phik, F.gd);
        lsF = F;
        wv.mark(12);
        bool tiny = false;
        if (P.tiny_step_tol > 0 && wv.uni(F.rel <= (T)P.tiny_step_tol)) tiny = wv.uni(dy_max() <= (T)P.tiny_step_y_tol);
        if (in_wd && tiny) {
            // the watchdog stops at a tiny step: back to its stored iterate, then the
            // ordinary line search there
            wd_from_tiny = true;
            return stop_watchdog();
        }
        if (P.watchdog_trigger > 0 && !in_wd && !tiny && !in_soft && wd_short >= P.watchdog_trigger)
            start_watchdog(F);
        if (tiny) {
            ls_alpha = F.amax_p;
            ls_amax_z = F.amax_z;
            ls_n_steps = 0;
            c_ok = 0;
            if (tiny_last) tiny_flag = 1;
            tiny_last = 1;
            return ls_finish(true, false);
        }
        tiny_last = 0;
        if (in_soft) {
            if (++soft_count > P.max_soft_resto_iters) return ls_finish(false, false);
            soft_ctx = 0;
            return soft_start();
        }
        ls_skip_first = false;
        return bt_start();
    }

    // BacktrackingLineSearch::DoBacktrackingLineSearch on the direction lsF (DW / YP)
    MPCG_HD int bt_start() {
        ls_alpha_max = lsF.amax_p;
        ls_alpha_min = in_wd ? ls_alpha_max : alpha_min_of();
        ls_alpha = ls_alpha_max;
        ls_amax_z = lsF.amax_z;
        ls_alpha_test = in_wd ? wd_alpha_test() : ls_alpha;
        if (ls_skip_first) ls_alpha *= (T)0.5;
        ls_n_steps = 0;
        ls_eval_error = false;
        return bt_next();
    }
    MPCG_HD int bt_next() {
        // (alpha halves towards alpha_min >= 0; the step bound only ends a zero alpha_min)
        if (wv.uni((ls_alpha > ls_alpha_min || ls_n_steps == 0) && ls_n_steps < 1100)) {
            if (!in_wd) ls_alpha_test = ls_alpha;
            return do_trial(ls_alpha, ls_alpha_test, K_BT);
        }
        return bt_done(false);
    }
    // K_BT: a trial point of the backtracking search was evaluated
    MPCG_HD int k_bt() {
        const bool accept = tr_acc;
        if (!tr_ok) ls_eval_error = true;
        if (accept) {
            update_for_next(ls_alpha_test, tr_phi);
            return bt_done(true);
        }
        if (in_wd) return bt_done(false);
        if (wv.uni(!ls_eval_error && ls_alpha == ls_alpha_max && theta <= tr_theta) && P.max_soc > 0) {
            // FilterLSAcceptor::TrySecondOrderCorrection from the same factorisation; the
            // Newton direction waits in the spill area
            rec_out<WideLayout::RDW, 8>(L.SP_SOC());
            spill_out(L.SP_SOC() + WideLayout::WS * N, L.YP(0), WideLayout::YS * N);
            xcopy(true, WideLayout::XDP, 36, 12);
            soc_count = 0;
            soc_alpha() = ls_alpha;
            soc_theta_old() = 0;
            soc_theta_trial() = tr_theta;
            return soc_next();
        }
        ls_alpha *= (T)0.5;
        ++ls_n_steps;
        return bt_next();
    }
    MPCG_HD int soc_next() {
        if (wv.uni(soc_count < P.max_soc &&
                   (soc_count == 0 || soc_theta_trial() <= (T)P.kappa_soc * soc_theta_old()))) {
            soc_theta_old() = soc_theta_trial();
            return set_op(OP_SOCRHS, K_SOCRHS);
        }
        rec_in<WideLayout::RDW, 8>(L.SP_SOC());
        spill_in(L.SP_SOC() + WideLayout::WS * N, L.YP(0), WideLayout::YS * N);
        xcopy(false, WideLayout::XDP, 36, 12);
        ls_alpha *= (T)0.5;
        ++ls_n_steps;
        return bt_next();
    }
    // K_SOCRHS: c_soc written; solve with the same matrix (same delta_w)
    MPCG_HD int k_socrhs() { return do_solve(0, delta_w_used, K_SOC); }
    // K_SOC: the corrected step is in DW / YP
    MPCG_HD int k_soc() {
        soc_alpha() = wv.uni_d(sv_F.amax_p);
        soc_amax_z() = wv.uni_d(sv_F.amax_z);
        return do_trial(soc_alpha(), ls_alpha_test, K_SOC_TRIAL);
    }
    MPCG_HD int k_soc_trial() {
        const bool accept = tr_acc;
        if (accept) {
            ls_alpha = soc_alpha();
            ls_amax_z = soc_amax_z();
            update_for_next(ls_alpha_test, tr_phi);
            return bt_done(true);
        }
        ++soc_count;
        soc_theta_trial() = tr_theta;
        return soc_next();
    }
    // the watchdog around the backtracking search (FindAcceptableTrialPoint)
    MPCG_HD int bt_done(bool accept) {
        if (in_wd) {
            if (accept) {
                in_wd = 0;
                return ls_finish(true, false);
            }
            ++wd_trial_iter;
            if (ls_eval_error || wd_trial_iter > P.watchdog_trial_max) {
                wd_from_tiny = false;
                return stop_watchdog();
            }
            return ls_finish(true, false);  // the watchdog's unchecked step
        }
        return ls_finish(accept, false);
    }
    MPCG_HD void start_watchdog(const Fwd& F) {
        in_wd = 1;
        spill_out(L.SP_WD(), 0, (WideLayout::RS + 2 * WideLayout::YS) * N);  // W, ZL, ZU, DW records, Y, YP
        xcopy(true, WideLayout::XP, 0, 36);  // (RESTO: p, n, z_p, z_n, dp, dn)
        wd_trial_iter = 0;
        wd_alpha_test() = F.amax_p;
        wd_amax_z() = F.amax_z;
        wd_theta() = ref_theta;
        wd_phi() = ref_phi;
        wd_gd() = ref_gd;
    }
    // back to the watchdog's stored iterate and direction; its statistics next
    MPCG_HD int stop_watchdog() {
        in_wd = 0;
        spill_in(L.SP_WD(), 0, (WideLayout::RS + 2 * WideLayout::YS) * N);
        xcopy(false, WideLayout::XP, 0, 36);
        wd_short = 0;
        c_ok = 0;
        return do_stats(false, (T)0, (T)0, K_WD_STATS);
    }
    MPCG_HD int k_wd_stats() {
        set_ref(wd_theta(), wd_phi(), wd_gd());
        lsF.amax_p = wd_alpha_test();
        lsF.amax_z = wd_amax_z();
        lsF.gd = wd_gd();
        ls_skip_first = !wd_from_tiny;
        return bt_start();
    }

    // BacktrackingLineSearch::TrySoftRestoStep: primal and dual step min(alpha_p, alpha_z),
    // accepted by the original filter or by a reduction of the primal-dual error.
    // soft_ctx 0: an iteration of the soft restoration phase; 1: its first step.
    MPCG_HD int soft_start() {
        soft_a() = wv.uni_d(tmin(lsF.amax_p, lsF.amax_z));
        return do_trial(soft_a(), (T)0, K_SOFT_TRIAL);
    }
    MPCG_HD int k_soft_trial() {
        if (!tr_ok) return soft_done(false, false);
        if (tr_acc) {
            acc_alpha = soft_a();
            acc_z = soft_a();
            acc_pending = true;
            return soft_done(true, true);
        }
        return set_op(OP_PDERR, K_SOFT_PD0);
    }
    MPCG_HD int k_soft_pd0() {
        soft_ec() = pd_val;
        rec_out<0, 24>(L.SP_SOFT());  // W, ZL, ZU
        spill_out(L.SP_SOFT() + 3 * WideLayout::WS * N, L.Y(0), WideLayout::YS * N);
        xcopy(true, WideLayout::XP, 48, 24);  // (RESTO: p, n, z_p, z_n)
        accept_all(wv.lane(), true, soft_a(), soft_a(), false);
        c_ok = 0;
        return set_op(OP_PDERR, K_SOFT_PD1);
    }
    MPCG_HD int k_soft_pd1() {
        if (wv.uni(pd_val <= (T)P.soft_resto_factor * soft_ec())) {
            clamp_all();  // kappa_sigma correction of the accepted multipliers
            return soft_done(true, false);
        }
        rec_in<0, 24>(L.SP_SOFT());
        spill_in(L.SP_SOFT() + 3 * WideLayout::WS * N, L.Y(0), WideLayout::YS * N);
        xcopy(false, WideLayout::XP, 48, 24);
        return soft_done(false, false);
    }
    MPCG_HD int soft_done(bool accept, bool sat) {
        if (soft_ctx == 0) {  // an iteration of the soft restoration phase
            if (accept && sat) {
                in_soft = 0;
                soft_count = 0;
            }
            return accept ? ls_done() : ls_fail();
        }
        if (accept) {  // the first step of the soft restoration phase
            in_soft = !sat;
            return ls_done();
        }
        return ls_fail();
    }

    // the end of FindAcceptableTrialPoint
    MPCG_HD int ls_finish(bool accept, bool soft_or_resto) {
        if (!accept) {
            if (!in_soft && P.soft_resto_factor > 0) {
                augment_filter();  // PrepareRestoPhaseStart
                soft_ctx = 1;
                return soft_start();
            }
            return ls_fail();
        }
        if (!soft_or_resto) {
            acc_alpha = wv.uni_d(ls_alpha);
            acc_z = wv.uni_d(ls_amax_z);
            acc_pending = true;
            if (ls_n_steps == 0)
                wd_short = 0;
            else
                ++wd_short;
        }
        return ls_done();
    }
    // the step is taken (pending or applied): the next iteration
    MPCG_HD int ls_done() {
        wv.mark(7);
        ++iter;
        return do_stats(acc_pending, acc_alpha, acc_z, K_BEGIN);
    }
    MPCG_HD int ls_fail() {
        if (!in_soft) augment_filter();
        if constexpr (RESTO) {
            return IPM_RESTORATION_FAILURE;  // (no restoration phase inside the restoration phase)
        } else {
            // almost feasible: the last acceptable iterate, if any, is the result
            if (wv.uni(theta <= (T)1e-2 * (T)P.tol)) {
                if (have_acc) {
                    rec_in<0, 8>(L.SP_ACC());
                    return IPM_ACCEPTABLE;
                }
                return IPM_RESTORATION_FAILURE;
            }
            if (P.no_resto) return IPM_RESTORATION_FAILURE;  // (mpcg_params no_restoration; oracle restoration = 0)
            in_soft = 0;
            soft_count = 0;
            wd_short = 0;
            return NEED_RESTO;  // (solve() runs the restoration phase outside the state machine's loop)
        }
    }
    // FindAcceptableTrialPoint with the fallback to the restoration phase (the Newton
    // system could not be made to have the right inertia)
    MPCG_HD int ls_goto_resto() {
        if (mu != last_mu()) {
            in_wd = 0;
            wd_short = 0;
            last_mu() = mu;
        }
        if (P.acceptable_iter > 0 && cur_acceptable) {
            rec_out<0, 8>(L.SP_ACC());
            have_acc = 1;
        }
        if (in_wd) {  // the watchdog's stored iterate and direction, searched without skipping
            wd_from_tiny = true;
            return stop_watchdog();
        }
        return ls_fail();
    }
    // MinC_1NrmRestorationPhase::PerformRestoration: the original problem's LDS image goes to
    // the workspace, the restoration problem runs out of line on the same LDS, and on success
    // the image comes back with the new iterate (x of the restoration problem, y = 0, the
    // bound multipliers of its step), which AcceptTrialPoint takes as the next iterate.
    MPCG_HD int restoration() {
        ++n_resto;
        spill_out(L.SP_DUMP(), 0, L.total());
        wv.gsync();
        const RestoIn<T> in{mu, tau, theta, prim_inf, ref_phi, ref_theta, sf, nf, iter};
        const IpmParams Pc = P;
        const RestoOut o = resto_phase<WV, MODEL, T, NB>(Pc, pr, wv, spill, in);
        wv.gsync();
        spill_in(L.SP_DUMP(), 0, L.total());
        iter = wv.uni(o.iter);
        n_fover += wv.uni(o.fover);
        c_ok = 0;
        const int s = wv.uni(o.status);
        if (s) return s;
        clamp_all();
        acc_pending = false;
        ++iter;
        return do_stats(false, (T)0, (T)0, K_BEGIN);
    }

    // ------------------------------------------------------------ the restoration phase's control
    // (RESTO instance: oracle/ipm.c perform_restoration, resto_convergence and the
    // restoration problem's pass through ipm_iterate / find_trial_point.)
    MPCG_HD RestoOut run_resto(const RestoIn<T>& in) {
        dumpO = spill + L.SP_DUMP();
        ext = spill + L.SP_EXT();
        xsp = spill + L.SP_XSP();
        bounds_only();
        sf = wv.uni_d((T)1);  // (RestoIpoptNLP: no objective scaling)
        o_mu = wv.uni_d(in.mu);
        o_tau = wv.uni_d(in.tau);
        o_theta = wv.uni_d(in.theta);
        o_ref_phi = wv.uni_d(in.ref_phi);
        o_ref_theta = wv.uni_d(in.ref_theta);
        o_sf = wv.uni_d(in.sf);
        o_nf = wv.uni(in.nf);
        // mu_R = max(mu, ||c||_inf), tau from it
        mu = wv.uni_d(tmax(in.mu, in.prim_inf));
        tau = wv.uni_d(tmax((T)0.99, (T)1 - mu));
        status = 0;
        theta_max() = -1;
        theta_min = -1;
        dw_last = 0;
        delta_w_used = 0;
        acc_alpha = 0;
        acc_z = 0;
        acc_pending = false;
        iter = wv.uni(in.iter);
        nf = 0;
        kkt() = 0;
        ref_theta = ref_phi = ref_gd = ref_pgd = ref_pth = 0;
        last_rej_filter = count_filter_rej = n_filter_resets = 0;
        in_wd = wd_short = wd_trial_iter = tiny_last = tiny_flag = in_soft = soft_count = acc_counter = have_acc = 0;
        wd_alpha_test() = wd_theta() = wd_phi() = wd_gd() = wd_amax_z() = 0;
        last_mu() = -1;
        last_obj() = 0;
        curr_obj() = (T)-1e50;
        cur_acceptable = false;
        st_acc = sv_ok = tr_ok = false;
        st_alpha = st_z = tr_alpha = tr_test = tr_phi = tr_theta = pd_val = 0;
        tr_acc = false;
        ls_alpha = ls_alpha_max = ls_alpha_min = ls_alpha_test = ls_amax_z = 0;
        ls_n_steps = inertia_attempt = soft_ctx = 0;
        ls_eval_error = ls_skip_first = wd_from_tiny = false;
        soc_alpha() = soc_amax_z() = soc_theta_old() = soc_theta_trial() = soft_ec() = soft_a() = 0;
        soc_count = 0;
        lsF = Fwd{(T)1, (T)1, (T)0, (T)0};
        sv_F = lsF;
        resto_first = true;
        mu_Emu = 0;
        mu_tf = 0;
        mu_done = false;
        init_rows();
        do_stats(false, (T)0, (T)0, K_BEGIN);
        run();
        if (status == RESTO_DONE) {
            resto_finish();
            return RestoOut{0, iter, n_fover};
        }
        return RestoOut{status, iter, n_fover};
    }

    // RestoConvergenceCheck / RestoFilterConvergenceCheck::TestOrigProgress (from the second
    // iterate on), then the restoration problem's own termination; then the monotone update.
    MPCG_HD int k_begin_resto() {
        acc_pending = false;
        const int nbnd = 2 * (8 * N - 2) + 12 * N, ng = 6 * N;
        const T sd = tmax((T)100, (l1y + l1z) / (T)(ng + nbnd)) * (T)0.01;
        const T scc = tmax((T)100, l1z / (T)nbnd) * (T)0.01;
        const T E0 = tmax(dual_inf / sd, tmax(prim_inf, compl0 / scc));
#ifdef MPCG_TRACE
        if (wv.lane() == 0)
            printf("r%3d mu %.3e E0 %.3e dual %.3e prim %.3e compl %.3e th %.3e f %.10e thO %.3e phiO %.10e\n", iter,
                   (double)mu, (double)E0, (double)dual_inf, (double)prim_inf, (double)compl0, (double)theta,
                   (double)fval, (double)r_thO, (double)r_phiO);
#endif
        int s = 0;
        if (!isfinite((double)E0) || !isfinite((double)theta) || !isfinite((double)fval)) {
            s = IPM_INVALID_NUMBER;
        } else {
            if (resto_first)
                resto_first = false;
            else if (orig_progress())
                s = RESTO_DONE;
            if (!s) {
                if (E0 <= (T)P.tol && dual_inf <= (T)P.dual_inf_tol && prim_inf <= (T)P.constr_viol_tol &&
                    compl0 <= (T)P.compl_inf_tol)
                    s = r_pinfO <= (T)1e2 * (T)P.tol ? IPM_FEASIBLE_POINT : IPM_LOCAL_INFEASIBILITY;
                else if (iter >= P.max_iter)
                    s = IPM_MAXITER;
                else if (P.cpu_iter_budget >= 0 && iter > P.cpu_iter_budget)
                    s = IPM_UNKNOWN;
            }
        }
        s = wv.uni(s);
        if (s) return s;
        mu_tf = tiny_flag;
        tiny_flag = 0;
        mu_done = false;
        mu_Emu = wv.uni_d(tmax(dual_inf / sd, tmax(prim_inf, tmax(pmax - mu, mu - pmin) / scc)));
        return mu_loop();
    }
    // the barrier update's loop: each change of mu re-evaluates the restoration problem (its
    // objective depends on mu), continued in k_rmu
    MPCG_HD int mu_loop() {
        const T kappa_eps = 10, kappa_mu = (T)0.2, theta_mu = (T)1.5;
        const T mu_min = (T)(fmin(P.tol, P.compl_inf_tol) / 11.0);
        for (;;) {
            if (!wv.uni((mu_Emu <= kappa_eps * mu || mu_tf) && !mu_done)) break;
            const T mnew = wv.uni_d(tmax(tmin(kappa_mu * mu, (T)pow((double)mu, (double)theta_mu)), mu_min));
            const bool changed = mnew != mu;
            if (!changed && mu_tf) return IPM_TINY_STEP;
            mu = mnew;
            tau = wv.uni_d(tmax((T)0.99, (T)1 - mu));
            if (changed) return do_stats(false, (T)0, (T)0, K_RMU);
            mu_done = true;
            mu_tf = 0;
        }
        inertia_attempt = 0;
        return do_solve(0, (T)0, K_NEWTON);
    }
    MPCG_HD int k_rmu() {
        const int nbnd = 2 * (8 * N - 2) + 12 * N, ng = 6 * N;
        const T sd = tmax((T)100, (l1y + l1z) / (T)(ng + nbnd)) * (T)0.01;
        const T scc = tmax((T)100, l1z / (T)nbnd) * (T)0.01;
        mu_Emu = wv.uni_d(tmax(dual_inf / sd, tmax(prim_inf, tmax(pmax - mu, mu - pmin) / scc)));
        mu_done = wv.uni(mu_Emu > (T)10 * mu);
        if (mu_done) {  // BacktrackingLineSearch::Reset
            in_soft = 0;
            in_wd = 0;
            wd_short = 0;
            nf = 0;
        }
        mu_tf = 0;
        return mu_loop();
    }
    // the original problem accepts the restoration iterate x: its violation reduced below
    // 0.9 of the value at the restoration start, acceptable to its filter and to its last
    // reference point (from the restoration phase: no obj_max_inc test)
    MPCG_HD bool orig_progress() {
        if (!isfinite((double)r_phiO) || !isfinite((double)r_thO)) return false;
        if (!wv.uni(r_thO <= (T)0.9 * o_theta)) return false;
        const int t = wv.lane();
        const int fi = L.FI();
        bool hit = false;
        for (int f0 = 0; f0 < o_nf; f0 += 64) {
            const int f = f0 + t;
            T e0 = 0, e1 = 0;
            if (f < o_nf) {
                const T* x = f < L.cap ? dumpO + fi + 2 * f : spill + L.SP_FLT() + 2 * (f - L.cap);
                e0 = x[0];
                e1 = x[1];
            }
            const bool h = f < o_nf && r_thO >= e0 && r_phiO >= e1;
            hit = hit || wv.any(h);
        }
        if (hit) return false;
        const T gamma_theta = (T)1e-5, gamma_phi = (T)1e-8;
        return wv.uni(compare_le(r_thO, ((T)1 - gamma_theta) * o_ref_theta, o_ref_theta) ||
                      compare_le(r_phiO - o_ref_phi, -gamma_phi * o_ref_theta, o_ref_phi));
    }
    // back to the original problem: x from the restoration phase, y = 0 (constr_mult_reset_
    // threshold 0), the bound multipliers by a Newton step of the complementarity with the
    // whole restoration step as the primal step, cut by the fraction to the boundary
    // (ComputeBoundMultiplierStep), all reset to 1 if one exceeds bound_mult_reset_threshold
    // 1000 -- written into the original problem's LDS image
    MPCG_HD void resto_finish() {
        const int t = wv.lane();
        wv.sync();
        T* dmp = spill + L.SP_DUMP();
        T amin = 1;
        for (int b = 0; b < NB; ++b) {
            const int k = t + 64 * b;
            if (k >= N) continue;
            const int nv = k == N - 1 ? 6 : 8;
            for (int j = 0; j < nv; ++j) {
                const T x = ld(L.W(k) + j), w0 = dmp[L.W(k) + j];
                const T zl = dmp[L.ZL(k) + j], zu = dmp[L.ZU(k) + j];
                const T sc = w0 - vlo(j), sx = x - vlo(j), su = vhi(j) - w0, sxu = vhi(j) - x;
                const T dl = (o_mu + zl * (sc - sx)) / sc - zl, du = (o_mu + zu * (su - sxu)) / su - zu;
                if (dl < 0) amin = tmin(amin, -o_tau * zl / dl);
                if (du < 0) amin = tmin(amin, -o_tau * zu / du);
            }
        }
        const int opm[1] = {RMIN};
        reduce<1, true>(&amin, opm);
        T zmax = 0;
        for (int b = 0; b < NB; ++b) {
            const int k = t + 64 * b;
            if (k >= N) continue;
            const int nv = k == N - 1 ? 6 : 8;
            for (int j = 0; j < nv; ++j) {
                const T x = ld(L.W(k) + j), w0 = dmp[L.W(k) + j];
                const T zl = dmp[L.ZL(k) + j], zu = dmp[L.ZU(k) + j];
                const T sc = w0 - vlo(j), sx = x - vlo(j), su = vhi(j) - w0, sxu = vhi(j) - x;
                const T dl = (o_mu + zl * (sc - sx)) / sc - zl, du = (o_mu + zu * (su - sxu)) / su - zu;
                zmax = tmax(zmax, tmax((T)fabs(zl + amin * dl), (T)fabs(zu + amin * du)));
            }
        }
        const int opx[1] = {RMAX};
        reduce<1, true>(&zmax, opx);
        const bool reset = wv.uni(zmax > (T)1000);
        for (int b = 0; b < NB; ++b) {
            const int k = t + 64 * b;
            if (k >= N) continue;
            const int nv = k == N - 1 ? 6 : 8;
            for (int j = 0; j < nv; ++j) {
                const T x = ld(L.W(k) + j), w0 = dmp[L.W(k) + j];
                const T zl = dmp[L.ZL(k) + j], zu = dmp[L.ZU(k) + j];
                const T sc = w0 - vlo(j), sx = x - vlo(j), su = vhi(j) - w0, sxu = vhi(j) - x;
                const T dl = (o_mu + zl * (sc - sx)) / sc - zl, du = (o_mu + zu * (su - sxu)) / su - zu;
                dmp[L.ZL(k) + j] = reset ? (T)1 : zl + amin * dl;
                dmp[L.ZU(k) + j] = reset ? (T)1 : zu + amin * du;
                dmp[L.W(k) + j] = x;
            }
            for (int j = 0; j < 6; ++j) dmp[L.Y(k) + j] = 0;
        }
    }

    MPCG_HD int step(int c) {
        switch (c) {
            case K_LSQ: return k_lsq();
            case K_BEGIN: return k_begin();
            case K_NEWTON: return k_newton();
            case K_BT: return k_bt();
            case K_SOCRHS: return k_socrhs();
            case K_SOC: return k_soc();
            case K_SOC_TRIAL: return k_soc_trial();
            case K_SOFT_TRIAL: return k_soft_trial();
            case K_SOFT_PD0: return k_soft_pd0();
            case K_SOFT_PD1: return k_soft_pd1();
            case K_RMU: return k_rmu();
            default: return k_wd_stats();
        }
    }

    // The solve up to its end or to the start of a restoration phase (status NEED_RESTO):
    // the kernel that runs the batch contains no call (a call site in the solver's loop costs
    // the whole loop its register allocation); a problem that needs the restoration phase is
    // parked (park()) and continued by a second kernel (unpark(), finish_resto()).
    MPCG_HD void solve() {
        init();
        run();
    }
    // restoration phases and the solve after them, until the solve ends
    MPCG_HD void finish_resto() {
        if constexpr (!RESTO) {
            while (status == NEED_RESTO) {
                const int s = restoration();
                if (s > 0) {
                    status = s;
                    break;
                }
                status = 0;
                run();
            }
        }
    }
    // A parked problem: the solver's persistent scalars (PARK_SCALARS), its LDS image
    // (WideLayout::total()), then a restoration workspace (WideLayout::slot(): the batch
    // kernel's rare-path copies -- of which the acceptable point is kept -- and the restoration
    // phase's records).
    static constexpr int PARK_SCALARS = 32;
    MPCG_HD static int park_elems(const WideLayout& L) { return PARK_SCALARS + L.total() + L.slot(); }
    // (scalar 27: the parked problem's index, written with the scalars and checked by the worker
    // that unparks it -- park_entry_ok: an entry read before it was complete, or one left from
    // another launch, is caught before any of its values is used as an index)
    static constexpr int PARK_TAG = 27;
    MPCG_HD void park(T* dst, int64_t p) {
        const int t = wv.lane();
        wv.sync();
        if (t == 0) {
            const T v[28] = {mu, tau, theta, prim_inf, ref_phi, ref_theta, sf, theta_min, dw_last, delta_w_used,
                             (T)iter, (T)nf, (T)last_rej_filter, (T)count_filter_rej, (T)n_filter_resets,
                             (T)tiny_last, (T)tiny_flag, (T)acc_counter, (T)have_acc, (T)in_wd, (T)wd_short,
                             (T)in_soft, (T)soft_count, (T)wd_trial_iter, (T)n_fover, (T)n_resto, (T)nf_peak,
                             (T)(double)p};
            for (int i = 0; i < 28; ++i) dst[i] = v[i];
        }
        T* img = dst + PARK_SCALARS;
        for (int e = t; e < L.total(); e += 64) img[e] = ld(e);
        T* ws = img + L.total();  // (the acceptable point and the filter's workspace entries)
        for (int e = t; e < WideLayout::WS * N; e += 64) ws[L.SP_ACC() + e] = spill[L.SP_ACC() + e];
        for (int e = t; e < 2 * WideLayout::FX; e += 64) ws[L.SP_FLT() + e] = spill[L.SP_FLT() + e];
    }
    // The entry of problem p as park() wrote it: its tag is p and the scalars unpark() uses as
    // counts or indices are in range (the filter's size indexes the LDS filter and the workspace
    // extension; a tag of a float entry is exact up to 2^24 problems, beyond which only the range
    // checks apply).  Wave-uniform.
    MPCG_HD bool park_entry_ok(const T* src, int64_t p) const {
        const double tag = (double)src[PARK_TAG];
        const bool tag_ok = sizeof(T) == 8 || p < (1 << 24) ? tag == (double)p : tag >= 0;
        const double nf_ = (double)src[11], it = (double)src[10], nr = (double)src[25];
        return wv.uni(tag_ok && nf_ >= 0 && nf_ <= (double)(L.cap + WideLayout::FX) && it >= 0 && nr >= 0 ? 1 : 0) != 0;
    }
    // (the solver constructed with spill = park_entry + PARK_SCALARS + total())
    MPCG_HD void unpark(const T* src) {
        const int t = wv.lane();
        setup();
        wv.sync();
        const T* img = src + PARK_SCALARS;
        for (int e = t; e < L.total(); e += 64) st(e, img[e]);
        wv.sync();
        mu = wv.uni_d(src[0]);
        tau = wv.uni_d(src[1]);
        theta = wv.uni_d(src[2]);
        prim_inf = wv.uni_d(src[3]);
        ref_phi = wv.uni_d(src[4]);
        ref_theta = wv.uni_d(src[5]);
        sf = wv.uni_d(src[6]);
        theta_min = wv.uni_d(src[7]);
        dw_last = wv.uni_d(src[8]);
        delta_w_used = wv.uni_d(src[9]);
        iter = wv.uni((int)src[10]);
        nf = wv.uni((int)src[11]);
        last_rej_filter = wv.uni((int)src[12]);
        count_filter_rej = wv.uni((int)src[13]);
        n_filter_resets = wv.uni((int)src[14]);
        tiny_last = wv.uni((int)src[15]);
        tiny_flag = wv.uni((int)src[16]);
        acc_counter = wv.uni((int)src[17]);
        have_acc = wv.uni((int)src[18]);
        in_wd = wv.uni((int)src[19]);
        wd_short = wv.uni((int)src[20]);
        in_soft = wv.uni((int)src[21]);
        soft_count = wv.uni((int)src[22]);
        wd_trial_iter = wv.uni((int)src[23]);
        n_fover = wv.uni((int)src[24]);
        n_resto = wv.uni((int)src[25]);
        nf_peak = wv.uni((int)src[26]);
        status = NEED_RESTO;
        c_ok = 0;
        acc_pending = false;
        cur_acceptable = false;
    }
    // the state machine from the sweep set by init() / init_resto() to a status
    MPCG_HD void run() {
        for (;;) {
            const int o = wv.uni(op);
            if (o == OP_STATS) {
                stats(st_acc, st_alpha, st_z);
            } else if (o == OP_SOLVE) {
                sv_ok = wv.uni(riccati(sv_mode, sv_delta));
                if (sv_ok) sv_F = forward(sv_mode);
                if constexpr (RESTO) {
                    if (sv_ok) sv_F = refine_resto();
                }
            } else if (o == OP_TRIAL) {
                tr_ok = trial(tr_alpha, &tr_phi, &tr_theta);
                tr_acc = tr_ok && check_acceptability(tr_test, tr_phi, tr_theta);
                wv.mark(10);
            } else if (o == OP_PDERR) {
                pd_val = pd_error();
            } else {
                soc_rhs(soc_alpha());
            }
            const int s = step(wv.uni(ct));
            wv.mark(13);
            if (s > 0) {
                status = s;
                break;
            }
        }
        // iter counts accepted steps
        wv.sync();
    }

    // Final point with honor_original_bounds projection.
    MPCG_HD T x_state(int j, int k) const { return tmin(tmax(ld(L.W(k) + j), sl0), su0); }
    MPCG_HD T x_ctrl(int j, int k) const {
        const T v = ld(L.W(k) + 6 + j);
        return j == 0 ? tmin(tmax(v, wl0), wu0) : tmin(tmax(v, al0), au0);
    }
    MPCG_HD T objective_out() {
        T f = 0;
        for (int b = 0; b < NB; ++b) {
            const int k = t + 64 * b;
            if (k >= N) continue;
            T s[6];
#pragma unroll
            for (int j = 0; j < 6; ++j) s[j] = x_state(j, k);
            f += cost_state(s);
            if (k < N - 1) {
                const T u[2] = {x_ctrl(0, k), x_ctrl(1, k)};
                T up[2] = {0, 0};
                if (k <= N - 3) { up[0] = x_ctrl(0, k + 1); up[1] = x_ctrl(1, k + 1); }
                f += cost_ctrl(k, u, up);
            }
        }
        return rsum(f);
    }
};

template <class WV, int MODEL, class T, int NB>
MPCG_NOINLINE RestoOut resto_phase(const IpmParams& P, IpmProblem<T> pr, WV wv, T* ws, RestoIn<T> in) {
    WideSolver<WV, MODEL, false, T, NB, true> R(P, pr, wv, ws);
    return R.run_resto(in);
}

}  // namespace mpcg
#endif
