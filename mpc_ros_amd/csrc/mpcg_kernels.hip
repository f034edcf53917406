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

// Workspace accessor.  The workspace is cut into one tile per wavefront (64
// problems); element e of lane l in a tile lives at
//     tile[2 * ((e >> 1) * 64 + l) + (e & 1)]
// i.e. element pairs (2j, 2j+1) of a problem are adjacent and the pairs of the 64
// lanes follow each other: a wavefront's pair access is one 1 KB contiguous
// global_load/store_dwordx4, and every address is a wave-uniform (scalar) base plus
// one per-lane register.  The pointer is typed in the global address space so that
// no access is ever a flat access.
#if defined(__HIP_DEVICE_COMPILE__)
#define MPCG_GLOBAL __attribute__((address_space(1)))
#else
#define MPCG_GLOBAL
#endif
template <typename T>
struct DevWs {
    typedef MPCG_GLOBAL T gT;
    typedef MPCG_GLOBAL double2 gT2;
    gT* tile;  // wave-uniform: this wavefront's tile
    int lane;  // 0..63
    __device__ __forceinline__ gT* at(int e) const { return tile + (((e >> 1) * 64 + lane) << 1) + (e & 1); }
    __device__ __forceinline__ T ld(int e) const { return *at(e); }
    __device__ __forceinline__ void st(int e, T v) const { *at(e) = v; }
    __device__ __forceinline__ void ld2(int e, T& a, T& b) const {
        const double2 v = *(const gT2*)at(e);
        a = v.x;
        b = v.y;
    }
    __device__ __forceinline__ void st2(int e, T a, T b) const { *(gT2*)at(e) = make_double2(a, b); }
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
    const IpmLayout Lw{P.N};
    const int64_t tile_elems = (int64_t)Lw.total(P.filter_cap) * 64;
    DevWs<double> w{(DevWs<double>::gT*)(ws + (int64_t)blockIdx.x * tile_elems), (int)threadIdx.x};
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
