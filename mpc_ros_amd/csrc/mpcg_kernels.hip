// mpc_ros_amd/csrc/mpcg_kernels.hip -- CDNA4 (gfx950) kernels of the batched NMPC solve.
//
// One problem per lane, 64 problems per wavefront.  Per-problem iterate, Riccati
// records and filter live in a device workspace laid out structure-of-arrays:
// element e of problem p is ws[e * B + p], so every per-stage load or store of a
// wavefront is one fully coalesced 512-byte access.  Every iteration of the
// interior-point method (ipm_core.h) -- evaluation, Riccati backward pass,
// forward pass, filter line search, update -- runs inside one kernel launch with
// no host round trip; lanes that converge early idle under the exec mask until
// the wavefront's slowest problem is done.
#include <hip/hip_runtime.h>

#include "ipm_core.h"
#include "mpcg_internal.h"

namespace mpcg {

// Workspace accessor.  The pointer is typed in the global address space so that
// every access is a global_load/global_store (vmcnt-ordered, pipelinable), never a
// flat access (which orders against LDS too and forces full drains).
template <typename T>
struct DevWs {
    typedef __attribute__((address_space(1))) T gT;
    gT* base;
    int64_t stride;
    __device__ __forceinline__ gT& operator[](int e) const { return base[(int64_t)e * stride]; }
};

__global__ void __launch_bounds__(64, 1)
ipm_solve_kernel(IpmParams P, int64_t B, const double* __restrict__ state, const double* __restrict__ coeffs,
                 double* __restrict__ u0, double* __restrict__ traj, int32_t* __restrict__ status,
                 double* __restrict__ obj, int32_t* __restrict__ iters, double* __restrict__ ws) {
    const int64_t p = (int64_t)blockIdx.x * 64 + threadIdx.x;
    if (p >= B) return;
    IpmProblem<double> pr;
#pragma unroll
    for (int j = 0; j < 6; ++j) pr.init[j] = state[p * 6 + j];
#pragma unroll
    for (int j = 0; j < 4; ++j) pr.c[j] = coeffs[p * 4 + j];
    DevWs<double> w{(DevWs<double>::gT*)(ws + p), B};
    IpmSolver<double, DevWs<double>> S(P, pr, w);
    const IpmResult r = S.solve();
    u0[p * 2 + 0] = S.x_ctrl(0, 0);
    u0[p * 2 + 1] = S.x_ctrl(1, 0);
    if (traj) {
        const int N = P.N;
        double* t = traj + p * 3 * N;
        for (int k = 0; k < N; ++k) {
            t[k] = S.x_state(0, k);
            t[N + k] = S.x_state(1, k);
            t[2 * N + k] = S.x_state(2, k);
        }
    }
    if (status) status[p] = r.status;
    if (iters) iters[p] = r.iters;
    if (obj) obj[p] = S.objective_out();
}

hipError_t launch_ipm_solve(const IpmParams& P, int64_t B, const double* state, const double* coeffs, double* u0,
                            double* traj, int32_t* status, double* obj, int32_t* iters, double* ws,
                            hipStream_t stream) {
    if (B <= 0) return hipSuccess;
    const int64_t blocks = (B + 63) / 64;
    hipLaunchKernelGGL(ipm_solve_kernel, dim3((unsigned)blocks), dim3(64), 0, stream, P, B, state, coeffs, u0, traj,
                       status, obj, iters, ws);
    return hipGetLastError();
}

}  // namespace mpcg
