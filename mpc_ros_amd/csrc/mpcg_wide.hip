// mpc_ros_amd/csrc/mpcg_wide.hip -- one problem per wavefront (wide_core.h) on CDNA4.
//
// One workgroup = one wavefront = one problem; the problem's whole state lives in
// the workgroup's LDS (WideLayout: 30 KB at N = 20, i.e. 5 problems resident per
// CU).  Workgroups are dispatched by the hardware as CUs free up, so a slow problem
// occupies one wavefront slot while the rest of the batch streams past it.
#include <hip/hip_runtime.h>

#include "mpcg_internal.h"
#include "wave_dev.h"
#include "wide_core.h"

namespace mpcg {

struct WideArgs {
    IpmParams P;
    int64_t B;
    const double* state;
    const double* coeffs;
    double* u0;
    double* traj;
    int32_t* status;
    double* obj;
    int32_t* iters;
};

// 2 wavefronts per SIMD: 19 KB of LDS per problem allows 8 problems per CU, the register
// budget of 256 per lane lets all of them be resident
template <int MODEL>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) k_solve_wide(WideArgs a) {
    const int64_t p = blockIdx.x;
    if (p >= a.B) return;
    const int t = threadIdx.x;
    IpmProblem<double> pr;
#pragma unroll
    for (int j = 0; j < 6; ++j) pr.init[j] = a.state[p * 6 + j];
#pragma unroll
    for (int j = 0; j < 4; ++j) pr.c[j] = a.coeffs[p * 4 + j];
    DevWave wv;
    wv.t = t;
    WideSolver<DevWave, MODEL> S(a.P, pr, wv);
    S.solve();
    const double o = S.objective_out();
    const int N = a.P.N;
    if (t == 0) {
        a.u0[p * 2 + 0] = S.x_ctrl(0, 0);
        a.u0[p * 2 + 1] = S.x_ctrl(1, 0);
        if (a.status) a.status[p] = S.status;
        if (a.iters) a.iters[p] = S.iter;
        if (a.obj) a.obj[p] = o;
    }
    if (a.traj && t < N) {
        double* tr = a.traj + p * 3 * N;
        tr[t] = S.x_state(0, t);
        tr[N + t] = S.x_state(1, t);
        tr[2 * N + t] = S.x_state(2, t);
    }
}

size_t wide_lds_bytes(const IpmParams& P) { return (size_t)WideLayout{P.N, P.filter_cap}.total() * sizeof(double); }

hipError_t launch_wide_solve(const IpmParams& P, int64_t B, const double* state, const double* coeffs, double* u0,
                             double* traj, int32_t* status, double* obj, int32_t* iters, hipStream_t stream) {
    if (B <= 0) return hipSuccess;
    const size_t lds = wide_lds_bytes(P);
    const void* fn = P.model == 1 ? (const void*)k_solve_wide<1> : (const void*)k_solve_wide<0>;
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    const WideArgs a{P, B, state, coeffs, u0, traj, status, obj, iters};
    if (P.model == 1)
        hipLaunchKernelGGL(k_solve_wide<1>, dim3((unsigned)B), dim3(64), lds, stream, a);
    else
        hipLaunchKernelGGL(k_solve_wide<0>, dim3((unsigned)B), dim3(64), lds, stream, a);
    return hipGetLastError();
}

}  // namespace mpcg
