// tests/native/wide_host_check.cpp -- TEST HARNESS ONLY.
//
// Runs the one-problem-per-wavefront solver (mpc_ros_amd/csrc/wide_core.h) on the
// host: the 64 lanes of a wavefront are 64 cooperative fibers (ucontext) on one thread,
// LDS is a shared array, a lane exchange is a store / barrier / load / barrier, and the
// wave barrier passes control round-robin to the next lane (lane 0 resumes once lane 63
// has arrived: every lane calls the same barriers, as on the device).  Problems run in
// parallel, one OS thread each (MPCG_HOST_THREADS, default the machine's CPUs).  With
// -DHOST_OS_THREADS the lanes are 64 OS threads and a std::barrier instead (slow under
// oversubscription: a futex round per barrier).  The butterflies run the same pairwise
// operations as the device shuffles.  Never part of the product library.
//
// stdin:  N dt ref_cte ref_eth ref_v w_cte w_eth w_v w_w w_a w_dw w_da max_w max_a bound tol max_iter
//         model lf
//         acceptable_tol acceptable_iter acceptable_dual_inf_tol acceptable_constr_viol_tol
//         acceptable_compl_inf_tol acceptable_obj_change_tol max_soc kappa_soc wd_trigger
//         wd_trial_max soft_factor max_soft_iters obj_max_inc max_filter_resets
//         filter_reset_trigger tiny_step_tol tiny_step_y_tol cpu_iter_budget filter_cap
//         dual_inf_tol constr_viol_tol compl_inf_tol
//         B, then B x (state[6], coeffs[4])
// stdout: per problem: status iters obj u0[2] traj[3N] restoration-phases filter-overflows filter-peak
#include <barrier>
#include <type_traits>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include <ucontext.h>
#ifdef __SANITIZE_ADDRESS__
#include <sanitizer/common_interface_defs.h>
#endif

#include "../../mpc_ros_amd/csrc/wide_core.h"

// 64 lanes as fibers on the calling thread: wait() hands control to the next lane in
// round-robin order, so a lane resumes after every other lane has reached the same barrier
struct Fibers {
    static constexpr size_t kStack = 4u << 20;  // (lazily committed)
    ucontext_t main_ctx, ctx[64];
    std::unique_ptr<char[]> stack[64];
    int ndone = 0;
    void* fn = nullptr;  // the lane body: void(int lane)
    void (*call)(void*, int) = nullptr;
#ifdef __SANITIZE_ADDRESS__
    void* fake = nullptr;
#endif
    void swap_to(ucontext_t* from, int to_lane) {
#ifdef __SANITIZE_ADDRESS__
        __sanitizer_start_switch_fiber(&fake, stack[to_lane].get(), kStack);
#endif
        swapcontext(from, &ctx[to_lane]);
#ifdef __SANITIZE_ADDRESS__
        __sanitizer_finish_switch_fiber(fake, nullptr, nullptr);
#endif
    }
    void wait(int t) { swap_to(&ctx[t], (t + 1) & 63); }
    static void entry(int hi, int lo, int t) {
        Fibers* f = (Fibers*)(((uintptr_t)(unsigned)hi << 32) | (uintptr_t)(unsigned)lo);
#ifdef __SANITIZE_ADDRESS__
        __sanitizer_finish_switch_fiber(f->fake, nullptr, nullptr);
#endif
        f->call(f->fn, t);
        // a finished lane passes on; the last one returns to the caller
        if (++f->ndone == 64) {
#ifdef __SANITIZE_ADDRESS__
            __sanitizer_start_switch_fiber(nullptr, nullptr, 0);
#endif
            setcontext(&f->main_ctx);
        }
        f->swap_to(&f->ctx[t], (t + 1) & 63);
    }
    template <class F>
    void run(F& body) {
        fn = &body;
        call = [](void* b, int t) { (*(F*)b)(t); };
        const uintptr_t me = (uintptr_t)this;
        for (int t = 0; t < 64; ++t) {
            if (!stack[t]) stack[t].reset(new char[kStack]);
            getcontext(&ctx[t]);
            ctx[t].uc_stack.ss_sp = stack[t].get();
            ctx[t].uc_stack.ss_size = kStack;
            ctx[t].uc_link = nullptr;
            makecontext(&ctx[t], (void (*)())entry, 3, (int)(me >> 32), (int)(me & 0xffffffffu), t);
        }
        ndone = 0;
#ifdef __SANITIZE_ADDRESS__
        __sanitizer_start_switch_fiber(&fake, stack[0].get(), kStack);
#endif
        swapcontext(&main_ctx, &ctx[0]);
#ifdef __SANITIZE_ADDRESS__
        __sanitizer_finish_switch_fiber(fake, nullptr, nullptr);
#endif
    }
};

struct HostShared {
#ifdef HOST_OS_THREADS
    std::barrier<> bar{64};
#else
    Fibers* fib = nullptr;
#endif
    double xd[64];
    int xi[64];
    std::vector<double> lds;
};

#ifndef HOST_T
#define HOST_T double  // -DHOST_T=float: the fp32 solver
#endif
typedef HOST_T HT;

struct HostWave {
    HostShared* sh;
    int t;
    double* lds;
    double* S() const { return lds; }
    template <class U>
    U* Sp() const { return reinterpret_cast<U*>(lds); }
#ifdef HOST_OS_THREADS
    void sync() const { sh->bar.arrive_and_wait(); }
#else
    void sync() const { sh->fib->wait(t); }
#endif
    void gsync() const { sync(); }
    template <class U>
    U from(U v, int src) const {
        sh->xd[t] = (double)v;
        sync();
        const U r = (U)sh->xd[src];
        sync();
        return r;
    }
    double xor_(double v, int m) const {
        sh->xd[t] = v;
        sync();
        const double r = sh->xd[t ^ m];
        sync();
        return r;
    }
    template <class U>
    U up1(U v) const {
        sh->xd[t] = (double)v;
        sync();
        const U r = t > 0 ? (U)sh->xd[t - 1] : v;
        sync();
        return r;
    }
    bool any(bool b) const {
        sh->xi[t] = b ? 1 : 0;
        sync();
        int r = 0;
        for (int i = 0; i < 64; ++i) r |= sh->xi[i];
        sync();
        return r != 0;
    }
    int uni(int v) const { return v; }
    int ballot_prefix(bool b, int* total) const {
        sh->xi[t] = b ? 1 : 0;
        sync();
        int c = 0, n = 0;
        for (int i = 0; i < 64; ++i) {
            n += sh->xi[i];
            if (i < t) c += sh->xi[i];
        }
        sync();
        *total = n;
        return c;
    }
    int lane() const { return t; }
    void mark(int) const {}
    void sched_fence() const {}
    template <class U>
    void ld2(int i, U& a, U& b) const {
        if (i & 1) {  // (the device's pair load is a 16-byte (fp32: 8-byte) aligned access)
            std::fprintf(stderr, "ld2 at odd index %d\n", i);
            std::abort();
        }
        a = Sp<U>()[i];
        b = Sp<U>()[i + 1];
    }
    template <class U>
    U dn1(U v) const { return from(v, t < 63 ? t + 1 : t); }
    // device: DPP wave_shr:1 / wave_shl:1 with bound_ctrl off (lane 0 / 63 keeps x)
    template <class U>
    void up8(U* x, const U* y) const {
        for (int q = 0; q < 8; ++q) {
            const U r = from(y[q], t > 0 ? t - 1 : t);
            if (t > 0) x[q] = r;
        }
    }
    template <class U>
    void dn6(U* x, const U* y) const {
        for (int q = 0; q < 6; ++q) {
            const U r = from(y[q], t < 63 ? t + 1 : t);
            if (t < 63) x[q] = r;
        }
    }
    template <class U>
    U lo_half(U v) const { return from(v, t & 31); }
    // device: v_permlane32_swap gives the lower half (own, partner), the upper (partner, own)
    template <class U>
    void xor32_pair(U v, U& a, U& b) const {
        const U o = from(v, t ^ 32);
        a = t < 32 ? v : o;
        b = t < 32 ? o : v;
    }
    template <class U>
    U uni_d(U v) const { return from(v, 0); }
    template <class U>
    U lane63(U v) const { return from(v, 63); }
    template <class U>
    U lane0(U v) const { return from(v, 0); }
    template <class U>
    U lanev(U v, int l) const { return from(v, l); }
    // reduction partners of the device (wave_dev.h): xor 1, xor 2, mirror 8, mirror 16, xor 16, xor 32
    template <int s, class U>
    U rpart(U v) const {
        const int p = s == 0 ? t ^ 1 : s == 1 ? t ^ 2 : s == 2 ? (t & ~7) | (7 - (t & 7))
                    : s == 3 ? (t & ~15) | (15 - (t & 15)) : s == 4 ? t ^ 16 : t ^ 32;
        return from(v, p);
    }
};

int main() {
    mpcg::IpmParams P{};
    if (std::scanf("%d %lf %lf %lf %lf %lf %lf %lf %lf %lf %lf %lf %lf %lf %lf %lf %d", &P.N, &P.dt, &P.ref_cte,
                   &P.ref_eth, &P.ref_v, &P.w_cte, &P.w_eth, &P.w_v, &P.w_w, &P.w_a, &P.w_dw, &P.w_da, &P.max_w,
                   &P.max_a, &P.bound, &P.tol, &P.max_iter) != 17)
        return 1;
    P.bound_relax_factor = 1e-8;
    P.mu_init = 0.1;
    P.filter_cap = 64;
    P.model = 0;
    P.lf = 0.5;
    if (std::scanf("%d %lf", &P.model, &P.lf) != 2) return 1;
    if (std::scanf("%lf %d %lf %lf %lf %lf %d %lf %d %d %lf %d %lf %d %d %lf %lf %d %d", &P.acceptable_tol,
                   &P.acceptable_iter, &P.acceptable_dual_inf_tol, &P.acceptable_constr_viol_tol,
                   &P.acceptable_compl_inf_tol, &P.acceptable_obj_change_tol, &P.max_soc, &P.kappa_soc,
                   &P.watchdog_trigger, &P.watchdog_trial_max, &P.soft_resto_factor, &P.max_soft_resto_iters,
                   &P.obj_max_inc, &P.max_filter_resets, &P.filter_reset_trigger, &P.tiny_step_tol,
                   &P.tiny_step_y_tol, &P.cpu_iter_budget, &P.filter_cap) != 19)
        return 1;
    if (std::scanf("%lf %lf %lf", &P.dual_inf_tol, &P.constr_viol_tol, &P.compl_inf_tol) != 3) return 1;
    long B;
    if (std::scanf("%ld", &B) != 1) return 1;
    const bool two_phase = std::getenv("MPCG_HOST_TWO_PHASE") && std::atoi(std::getenv("MPCG_HOST_TWO_PHASE")) != 0;
    const mpcg::WideLayout L(P.N, P.filter_cap, P.model);
    std::vector<mpcg::IpmProblem<HT>> probs(B);
    for (long b = 0; b < B; ++b) {
        for (HT& v : probs[b].init) { double d; std::scanf("%lf", &d); v = (HT)d; }
        for (HT& v : probs[b].c) { double d; std::scanf("%lf", &d); v = (HT)d; }
    }
    std::vector<std::string> out(B);
    // one problem: its 64 lanes, then its output line
    auto solve_one = [&](long b, void* fibers) {
        const mpcg::IpmProblem<HT> pr = probs[b];
        HostShared sh;
        sh.lds.assign(L.total(), std::nan(""));
        std::vector<HT> spill(L.slot(), (HT)std::nan(""));
        std::vector<HT> park(32 + L.total() + L.slot(), (HT)std::nan(""));
        int status = 0, iters = 0, nresto = 0, nfover = 0, nfpeak = 0;
        double obj = 0, u0 = 0, u1 = 0;
        std::vector<double> traj(3 * P.N);
        // MPCG_HOST_TWO_PHASE=1 (double harness, differential drive, N <= 64): the fp32
        // configuration's two phases (mpcg_wide.hip) -- the fp32 solver with the given options,
        // its hand-over, then the fp64 solver with the reference's options from the fp32 iterate
        // (converged) or from the start (k_warm_wide)
        const bool two = two_phase && P.model == 0 && P.N <= 64;
        mpcg::IpmParams Pd = P;
        if (two) {
            Pd.precision = 0;
            mpcg::ipopt_default_options(Pd);
        }
        std::vector<float> ho(4 + 30 * P.N), spillf(two ? L.slot() : 0);
        auto lane = [&](int t) {
            HostWave wv{&sh, t, sh.lds.data()};
            const float* warm = nullptr;
            if constexpr (std::is_same_v<HT, double>) {
                if (two) {
                    mpcg::IpmParams P32 = P;
                    P32.precision = 1;
                    mpcg::IpmProblem<float> pf;
                    for (int j = 0; j < 6; ++j) pf.init[j] = (float)pr.init[j];
                    for (int j = 0; j < 4; ++j) pf.c[j] = (float)pr.c[j];
                    if (P.N <= 32) {
                        mpcg::WideSolver<HostWave, 0, true, float> S32(P32, pf, wv, spillf.data());
                        S32.solve();
                        S32.handoff_out(ho.data());
                    } else {
                        mpcg::WideSolver<HostWave, 0, false, float> S32(P32, pf, wv, spillf.data());
                        S32.solve();
                        S32.handoff_out(ho.data());
                    }
                    wv.sync();
                    warm = ho.data();
                }
            }
            auto run = [&](auto& S0) {
                typedef std::decay_t<decltype(S0)> Solver;
                if (warm && warm[0] != 0.0f)
                    S0.solve_warm(warm);
                else
                    S0.solve();
                // a restoration phase: parked and continued as the device's second kernel does
                Solver S2(two ? Pd : P, pr, wv, park.data() + Solver::PARK_SCALARS + L.total());
                const bool parked = S0.status == Solver::NEED_RESTO;
                if (parked) {
                    S0.park(park.data(), b);
                    wv.sync();
                    if (!S2.park_entry_ok(park.data(), b)) {
                        std::fprintf(stderr, "park entry check failed (problem %ld): tag %g nf %g iter %g n_resto %g\n", b,
                                     (double)park[27], (double)park[11], (double)park[10], (double)park[25]);
                        std::abort();
                    }
                    S2.unpark(park.data());
                    S2.finish_resto();
                }
                Solver& S = parked ? S2 : S0;
                const double o = S.objective_out();
                if (t == 0) {
                    status = S.status;
                    iters = S.iter;
                    nresto = S.n_resto;
                    nfover = S.n_fover;
                    nfpeak = S.nf_peak;
                    obj = o;
                    u0 = S.x_ctrl(0, 0);
                    u1 = S.x_ctrl(1, 0);
                    for (int s = 0; s < 3; ++s)
                        for (int k = 0; k < P.N; ++k) traj[s * P.N + k] = S.x_state(s, k);
                }
            };
            if (P.model == 1 && P.N > 64) {
                mpcg::WideSolver<HostWave, 1, false, HT, 2> S(P, pr, wv, spill.data());
                run(S);
            } else if (P.model == 0 && P.N > 64) {
                mpcg::WideSolver<HostWave, 0, false, HT, 2> S(P, pr, wv, spill.data());
                run(S);
            } else if (P.model == 1 && P.N <= 32) {
                mpcg::WideSolver<HostWave, 1, true, HT> S(P, pr, wv, spill.data());
                run(S);
            } else if (P.model == 1) {
                mpcg::WideSolver<HostWave, 1, false, HT> S(P, pr, wv, spill.data());
                run(S);
            } else if (P.N <= 32) {
                mpcg::WideSolver<HostWave, 0, true, HT> S(two ? Pd : P, pr, wv, spill.data());
                run(S);
            } else {
                mpcg::WideSolver<HostWave, 0, false, HT> S(two ? Pd : P, pr, wv, spill.data());
                run(S);
            }
        };
#ifdef HOST_OS_THREADS
        (void)fibers;
        std::vector<std::thread> th;
        for (int t = 0; t < 64; ++t) th.emplace_back(lane, t);
        for (auto& x : th) x.join();
#else
        sh.fib = (Fibers*)fibers;
        sh.fib->run(lane);
#endif
        std::string line;
        char buf[64];
        std::snprintf(buf, sizeof buf, "%d %d %.17g %.17g %.17g", status, iters, obj, u0, u1);
        line += buf;
        for (double v : traj) {
            std::snprintf(buf, sizeof buf, " %.17g", v);
            line += buf;
        }
        std::snprintf(buf, sizeof buf, " %d %d %d\n", nresto, nfover, nfpeak);
        line += buf;
        out[b] = line;
    };
    // problems in parallel: one OS thread each, taking the next problem
#ifdef HOST_OS_THREADS
    int nth = 1;  // (64 OS threads per problem already)
#else
    const char* env = std::getenv("MPCG_HOST_THREADS");
    int nth = env ? std::atoi(env) : (int)std::thread::hardware_concurrency();
    nth = nth < 1 ? 1 : nth;
#endif
    if (nth > B) nth = (int)(B > 0 ? B : 1);
    std::atomic<long> next{0};
    auto worker = [&]() {
        auto fib = std::make_unique<Fibers>();
        for (long b; (b = next.fetch_add(1)) < B;) solve_one(b, fib.get());
    };
    std::vector<std::thread> pool;
    for (int i = 1; i < nth; ++i) pool.emplace_back(worker);
    worker();
    for (auto& x : pool) x.join();
    for (long b = 0; b < B; ++b) std::fputs(out[b].c_str(), stdout);
    return 0;
}
