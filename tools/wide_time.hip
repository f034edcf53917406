// tools/wide_time.hip -- time the product wavefront kernel (diagnostic tool for kernel variants).
//
// Compiles mpcg_wide.hip from the include directory given at build time (the product
// sources, or a modified copy of them), solves inputs.bin ([int64 B][B x 6 state]
// [B x 4 coeffs], plugin defaults, N = 20) with the product launch sequence (solve
// order + k_solve_wide), and prints the kernel time (HIP events, 1 warm-up + R timed
// launches), iterations, statuses and the u0 it produced; with a second file it
// reports the largest u0 difference to that file (another variant's output).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I <csrc dir> tools/wide_time.hip -o wt
// (-DWT_OLD_API for sources from before round 3's workspace-size argument)
//   ./wt inputs.bin out_u0.bin [ref_u0.bin]
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <vector>

#include "mpcg_wide.hip"

#define CK(x)                                                              \
    do {                                                                   \
        hipError_t e_ = (x);                                               \
        if (e_ != hipSuccess) {                                            \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));  \
            std::exit(2);                                                  \
        }                                                                  \
    } while (0)

int main(int argc, char** argv) {
    if (argc < 3) return 1;
    FILE* f = std::fopen(argv[1], "rb");
    if (!f) return 1;
    int64_t B;
    if (std::fread(&B, 8, 1, f) != 1) return 1;
    std::vector<double> st(B * 6), cf(B * 4);
    if (std::fread(st.data(), 8, B * 6, f) != (size_t)(B * 6)) return 1;
    if (std::fread(cf.data(), 8, B * 4, f) != (size_t)(B * 4)) return 1;
    std::fclose(f);
    mpcg::IpmParams P{};
    P.N = 20; P.dt = 0.1; P.ref_cte = 0; P.ref_eth = 0; P.ref_v = 1.0;
    P.w_cte = 1000; P.w_eth = 1000; P.w_v = 100; P.w_w = 100; P.w_a = 50; P.w_dw = 0; P.w_da = 10;
    P.max_w = 1.0; P.max_a = 1.0; P.bound = 1000; P.tol = 1e-8; P.bound_relax_factor = 1e-8; P.mu_init = 0.1;
    P.max_iter = 3000; P.filter_cap = 64; P.model = 0; P.lf = 0.5;
    // Ipopt 3.12 defaults and the max_cpu_time budget at N = 20 (mpcg_api.cpp ipopt_defaults, cpu_iter_budget)
    P.acceptable_tol = 1e-6; P.acceptable_iter = 15; P.acceptable_dual_inf_tol = 1e10;
    P.acceptable_constr_viol_tol = 1e-2; P.acceptable_compl_inf_tol = 1e-2; P.acceptable_obj_change_tol = 1e20;
    P.max_soc = 4; P.kappa_soc = 0.99; P.watchdog_trigger = 10; P.watchdog_trial_max = 3;
    P.soft_resto_factor = 0.9999; P.max_soft_resto_iters = 10; P.obj_max_inc = 5; P.max_filter_resets = 5;
    P.filter_reset_trigger = 5; P.tiny_step_tol = 10 * 2.220446049250313e-16; P.tiny_step_y_tol = 1e-2;
    P.dual_inf_tol = 1; P.constr_viol_tol = 1e-4; P.compl_inf_tol = 1e-4; P.cpu_iter_budget = 1520; P.precision = 0;
    double *dst, *dcf, *du0, *dobj;
    int *dit, *dss;
    CK(hipMalloc(&dst, B * 6 * 8));
    CK(hipMalloc(&dcf, B * 4 * 8));
    CK(hipMalloc(&du0, B * 2 * 8));
    CK(hipMalloc(&dobj, B * 8));
    CK(hipMalloc(&dit, B * 4));
    CK(hipMalloc(&dss, B * 4));
    CK(hipMemcpy(dst, st.data(), B * 6 * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dcf, cf.data(), B * 4 * 8, hipMemcpyHostToDevice));
    const size_t sb = mpcg::wide_sched_bytes(B);
    void* dsched;
    CK(hipMalloc(&dsched, sb));
    void* dspill;
    CK(hipMalloc(&dspill, mpcg::wide_spill_bytes(P, B)));
#ifndef WT_OLD_API
    hipStream_t aux;
    hipEvent_t evf, evj;
    CK(hipStreamCreateWithFlags(&aux, hipStreamNonBlocking));
    CK(hipEventCreateWithFlags(&evf, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&evj, hipEventDisableTiming));
#endif
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int R = 5;
    float tot = 0, best = 1e30f;
    for (int r = 0; r <= R; ++r) {
        CK(hipEventRecord(e0));
        int32_t* order = nullptr;
        CK(mpcg::launch_wide_order(B, dcf, dsched, sb, &order, 0));
#ifdef WT_OLD_API
        CK(mpcg::launch_wide_solve(P, B, dst, dcf, du0, nullptr, dss, dobj, dit, order, dspill, 0));
#else
        mpcg::WideStreams ws;
        ws.aux = getenv("WT_SEQ") ? nullptr : aux;
        ws.ev_fork = evf;
        ws.ev_join = evj;
        CK(mpcg::launch_wide_solve(P, B, dst, dcf, du0, nullptr, dss, dobj, dit, nullptr, order, dspill,
                                   mpcg::wide_spill_bytes(P, B), 0, ws));
#endif
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r > 0) {
            tot += ms;
            best = ms < best ? ms : best;
        }
    }
    std::vector<double> u0(B * 2);
    std::vector<int> it(B), ss(B);
    CK(hipMemcpy(u0.data(), du0, B * 16, hipMemcpyDeviceToHost));
    CK(hipMemcpy(it.data(), dit, B * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(ss.data(), dss, B * 4, hipMemcpyDeviceToHost));
    long long isum = 0;
    int imax = 0, nok = 0;
    for (int64_t p = 0; p < B; ++p) {
        isum += it[p];
        imax = it[p] > imax ? it[p] : imax;
        nok += ss[p] == 1;
    }
    std::printf("B=%lld avg %.3f ms best %.3f ms -> %.3f M solves/s; iters mean %.3f max %d; success %d; lds %zu B\n",
                (long long)B, tot / R, best, B / (tot / R) * 1e-3, (double)isum / B, imax, nok,
                mpcg::wide_lds_bytes(P));
    if (getenv("WT_TIMELINE")) {  // (variants whose write_out stores the wall clock in obj)
        std::vector<double> ob(B);
        CK(hipMemcpy(ob.data(), dobj, B * 8, hipMemcpyDeviceToHost));
        std::sort(ob.begin(), ob.end());
        const double t0 = ob[0], span = ob[B - 1] - ob[0];
        std::printf("end-time spread %.3f ms (100 MHz clock);", span * 1e-5);
        for (double q : {0.5, 0.9, 0.99, 0.999, 0.9999})
            std::printf(" %.4g: %.3f", q, (ob[(int64_t)(q * (B - 1))] - t0) * 1e-5);
        std::printf("\n");
    }
    FILE* o = std::fopen(argv[2], "wb");
    if (o) {
        std::fwrite(u0.data(), 8, B * 2, o);
        std::fwrite(it.data(), 4, B, o);
        std::fclose(o);
    }
    if (argc > 3) {
        FILE* rf = std::fopen(argv[3], "rb");
        if (rf) {
            std::vector<double> ru(B * 2);
            std::vector<int> ri(B);
            if (std::fread(ru.data(), 8, B * 2, rf) == (size_t)(B * 2) && std::fread(ri.data(), 4, B, rf) == (size_t)B) {
                double md = 0;
                int nd = 0;
                for (int64_t i = 0; i < B * 2; ++i) md = std::fmax(md, std::fabs(u0[i] - ru[i]));
                for (int64_t p = 0; p < B; ++p) nd += it[p] != ri[p];
                std::printf("vs %s: max |du0| %.3e, iteration counts differ on %d problems\n", argv[3], md, nd);
            }
            std::fclose(rf);
        }
    }
    return 0;
}
