// tools/wide_prof.hip -- phase timing of the one-problem-per-wavefront solver (diagnostic tool).
//
// Builds the wide_core.h solver with a wavefront context whose mark(phase) adds the
// cycles (clock64 = s_memtime) since the previous mark to a per-problem counter, and
// solves the batch in inputs.bin ([int64 B][B x 6 state][B x 4 coeffs], plugin
// defaults, N = 20).  Prints per-phase cycles per solve and per iteration.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I mpc_ros_amd/csrc tools/wide_prof.hip -o wide_prof
//   (or bash tools/build_wp.sh base v1 ...: the product sources or variants/<name>/)
//   ./wide_prof inputs.bin [B_limit]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <vector>

#include "wave_dev.h"
#include "wide_core.h"

namespace mpcg {
constexpr int NPH = 18;
// 9..13: sub-phase stamps of diagnostic variants (variants/stamps)
const char* kPhase[NPH] = {"stats", "ric-pre", "ric-sweep", "fwd-seq", "fwd-adj", "fwd-par", "trial", "ls-rest", "begin-rest",
                           "pre-trial", "accept-chk", "newton-in", "setref", "step-out", "pre-filter", "filter-add", "pre-lsfin", "pre-kbt"};

struct ProfWave : DevWaveBase {
    unsigned long long* acc;
    unsigned int* cnt;  // calls per phase mark
    unsigned long long last;
    __device__ void mark(int id) {
        const unsigned long long now = clock64();
        if (t == 0) {
            acc[id] += now - last;
            cnt[id] += 1;
        }
        last = now;
    }
};

#ifndef WPE
#define WPE 1
#endif
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE))) k_prof(IpmParams P, int64_t B, const double* state, const double* coeffs,
                                             unsigned long long* acc, int* iters, int* status,
                                             unsigned long long* times, unsigned int* cnt, double* spill) {
    const int64_t p = blockIdx.x;
    if (p >= B) return;
    IpmProblem<double> pr;
    for (int j = 0; j < 6; ++j) pr.init[j] = state[p * 6 + j];
    for (int j = 0; j < 4; ++j) pr.c[j] = coeffs[p * 4 + j];
    ProfWave wv;
    wv.t = (int)threadIdx.x;
    wv.acc = acc + p * (NPH + 1);
    wv.cnt = cnt + p * NPH;
    wv.last = (unsigned long long)clock64();
    const unsigned long long t0 = wv.last;
    const unsigned long long r0 = wall_clock64();
    const WideLayout Lw(P.N, P.filter_cap, 0);
    WideSolver<ProfWave, 0, true, double, 1> S(P, pr, wv, spill + p * (int64_t)Lw.spill());  // (N = 20: SPLIT)
    S.solve();
    if (threadIdx.x == 0) {
        times[2 * p] = r0;
        times[2 * p + 1] = wall_clock64();
        acc[p * (NPH + 1) + NPH] = clock64() - t0;
        iters[p] = S.iter;
        status[p] = S.status;
    }
}
}  // namespace mpcg

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));       \
            std::exit(2);                                                       \
        }                                                                       \
    } while (0)

int main(int argc, char** argv) {
    if (argc < 2) return 1;
    FILE* f = std::fopen(argv[1], "rb");
    if (!f) return 1;
    int64_t B;
    if (std::fread(&B, 8, 1, f) != 1) return 1;
    std::vector<double> st(B * 6), cf(B * 4);
    if (std::fread(st.data(), 8, B * 6, f) != (size_t)(B * 6)) return 1;
    if (std::fread(cf.data(), 8, B * 4, f) != (size_t)(B * 4)) return 1;
    std::fclose(f);
    if (argc > 2) B = std::min<int64_t>(B, std::atoll(argv[2]));
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
    double *dst, *dcf;
    unsigned long long* dacc;
    int *dit, *dss;
    const int W = mpcg::NPH + 1;
    CK(hipMalloc(&dst, B * 6 * 8));
    CK(hipMalloc(&dcf, B * 4 * 8));
    CK(hipMalloc(&dacc, B * W * 8));
    CK(hipMalloc(&dit, B * 4));
    CK(hipMalloc(&dss, B * 4));
    unsigned long long* dtm;
    CK(hipMalloc(&dtm, B * 16));
    double* dspill;
    CK(hipMalloc(&dspill, (size_t)mpcg::WideLayout(P.N, P.filter_cap, 0).spill() * 8 * B));
    unsigned int* dcnt;
    CK(hipMalloc(&dcnt, B * mpcg::NPH * 4));
    CK(hipMemset(dcnt, 0, B * mpcg::NPH * 4));
    CK(hipMemcpy(dst, st.data(), B * 6 * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dcf, cf.data(), B * 4 * 8, hipMemcpyHostToDevice));
    CK(hipMemset(dacc, 0, B * W * 8));
    const size_t lds = (size_t)mpcg::WideLayout(P.N, P.filter_cap, P.model).total() * 8;
    CK(hipFuncSetAttribute((const void*)mpcg::k_prof, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(mpcg::k_prof, dim3((unsigned)B), dim3(64), lds, 0, P, B, dst, dcf, dacc, dit, dss, dtm, dcnt, dspill);
    CK(hipGetLastError());
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<unsigned long long> acc(B * W);
    std::vector<int> it(B), ss(B);
    CK(hipMemcpy(acc.data(), dacc, B * W * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(it.data(), dit, B * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(ss.data(), dss, B * 4, hipMemcpyDeviceToHost));
    std::vector<unsigned int> cn(B * mpcg::NPH);
    CK(hipMemcpy(cn.data(), dcnt, B * mpcg::NPH * 4, hipMemcpyDeviceToHost));
    double sum[W] = {0}, iters = 0, calls[W] = {0};
    for (int64_t p = 0; p < B; ++p) {
        for (int j = 0; j < W; ++j) sum[j] += (double)acc[p * W + j];
        for (int j = 0; j < mpcg::NPH; ++j) calls[j] += cn[p * mpcg::NPH + j];
        iters += it[p];
    }
    std::printf("B=%lld kernel %.3f ms  iters/solve %.2f  lds %zu B\n", (long long)B, ms, iters / B, lds);
    for (int j = 0; j < mpcg::NPH; ++j)
        std::printf("  %-10s %10.0f cyc/solve %8.0f cyc/iter  %5.1f%%  %8.0f cyc/call\n", mpcg::kPhase[j], sum[j] / B,
                    sum[j] / iters, 100.0 * sum[j] / sum[mpcg::NPH], calls[j] > 0 ? sum[j] / calls[j] : 0.0);
    std::printf("  %-10s %10.0f cyc/solve %8.0f cyc/iter\n", "total", sum[mpcg::NPH] / B, sum[mpcg::NPH] / iters);
    // dispatch timeline (wall_clock64 ticks, 100 MHz): when problems start and end
    std::vector<unsigned long long> tm(2 * B);
    CK(hipMemcpy(tm.data(), dtm, B * 16, hipMemcpyDeviceToHost));
    unsigned long long tmin = ~0ull, tmax = 0;
    std::vector<double> ends(B);
    for (int64_t p = 0; p < B; ++p) { tmin = std::min(tmin, tm[2 * p]); tmax = std::max(tmax, tm[2 * p + 1]); }
    for (int64_t p = 0; p < B; ++p) ends[p] = (tm[2 * p + 1] - tmin) * 1e-5;  // ms at 100 MHz
    std::vector<double> srt(ends);
    std::sort(srt.begin(), srt.end());
    std::printf("timeline ms: first end %.3f, 50%% %.3f, 90%% %.3f, 99%% %.3f, 99.9%% %.3f, last %.3f\n", srt[0],
                srt[B / 2], srt[(B * 9) / 10], srt[(B * 99) / 100], srt[(B * 999) / 1000], srt[B - 1]);
    int64_t pl = 0;
    for (int64_t p = 0; p < B; ++p) if (ends[p] == srt[B - 1]) pl = p;
    std::printf("last problem %lld: start %.3f ms, iters %d\n", (long long)pl, (tm[2 * pl] - tmin) * 1e-5, it[pl]);
    return 0;
}
