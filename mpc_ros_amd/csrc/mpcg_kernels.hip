// mpc_ros_amd/csrc/mpcg_kernels.hip -- CDNA4 (gfx950) kernels of the batched NMPC solve.
//
// One problem per lane, 64 problems per wavefront.  The interior-point method of
// ipm_core.h runs as a sequence of phase kernels; every phase sweeps the stages of
// all problems of the batch at once:
//
//   init0 -> newton(LS) -> direction(LS) -> init1 ->
//   { begin -> newton -> direction -> linesearch } x iterations -> outputs
//
// Splitting the iteration into kernels gives each phase its own register
// allocation (a single fused kernel needs more than the 512-register file and
// spills inside the stage loops).  Between phases a problem's state lives in the
// device workspace, one 64-problem tile per wavefront.  Problems that have
// terminated exit each phase at once; a device counter of still-iterating
// problems tells the host driver when to stop launching iterations.
#include <hip/hip_runtime.h>

#include "ipm_core.h"
#include "mpcg_internal.h"

namespace mpcg {

#if defined(__HIP_DEVICE_COMPILE__)
#define MPCG_GLOBAL __attribute__((address_space(1)))
#else
#define MPCG_GLOBAL
#endif

// Workspace accessor.  The workspace is cut into one tile per wavefront (64
// problems); element e of lane l in a tile lives at
//     tile[2 * ((e >> 1) * 64 + l) + (e & 1)]
// i.e. element pairs (2j, 2j+1) of a problem are adjacent and the pairs of the 64
// lanes follow each other: a wavefront's pair access is one 1 KB contiguous
// global_load/store_dwordx4, and every address is a wave-uniform (scalar) base plus
// one per-lane register.  The pointer is typed in the global address space so that
// no access is ever a flat access.
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

typedef IpmSolver<double, DevWs<double>> DevSolver;

struct Args {
    IpmParams P;
    int64_t B;
    const double* state;
    const double* coeffs;
    double* ws;
    int* active;  // problems still iterating
};

__device__ __forceinline__ DevSolver make_solver(const Args& a, int64_t p) {
    IpmProblem<double> pr;
#pragma unroll
    for (int j = 0; j < 6; ++j) pr.init[j] = a.state[p * 6 + j];
#pragma unroll
    for (int j = 0; j < 4; ++j) pr.c[j] = a.coeffs[p * 4 + j];
    const IpmLayout Lw{a.P.N, a.P.filter_cap};
    const int64_t tile_elems = (int64_t)Lw.total(a.P.filter_cap) * 64;
    DevWs<double> w{(DevWs<double>::gT*)(a.ws + (int64_t)blockIdx.x * tile_elems), (int)threadIdx.x};
    return DevSolver(a.P, pr, w);
}

#define PROBLEM_INDEX                                         \
    const int64_t p = (int64_t)blockIdx.x * 64 + threadIdx.x; \
    if (p >= a.B) return;

__global__ void __launch_bounds__(64) k_init0(Args a) {
    PROBLEM_INDEX
    DevSolver S = make_solver(a, p);
    S.phase_init0();
}

__global__ void __launch_bounds__(64) k_init1(Args a) {
    PROBLEM_INDEX
    DevSolver S = make_solver(a, p);
    S.phase_init1();
}

__global__ void __launch_bounds__(64) k_begin(Args a) {
    PROBLEM_INDEX
    DevSolver S = make_solver(a, p);
    if (S.status() != 0) return;
    if (S.phase_begin() != 0) atomicSub(a.active, 1);
}

__global__ void __launch_bounds__(64) k_newton(Args a, int mode) {
    PROBLEM_INDEX
    DevSolver S = make_solver(a, p);
    if (mode == 0 && S.status() != 0) return;
    if (S.phase_newton(mode) != 0) atomicSub(a.active, 1);
}

__global__ void __launch_bounds__(64) k_direction(Args a, int mode) {
    PROBLEM_INDEX
    DevSolver S = make_solver(a, p);
    if (mode == 0 && S.status() != 0) return;
    S.phase_direction(mode);
}

__global__ void __launch_bounds__(64) k_linesearch(Args a) {
    PROBLEM_INDEX
    DevSolver S = make_solver(a, p);
    if (S.status() != 0) return;
    if (S.phase_linesearch() != 0) atomicSub(a.active, 1);
}

__global__ void __launch_bounds__(64) k_outputs(Args a, double* __restrict__ u0, double* __restrict__ traj,
                                                int32_t* __restrict__ status, double* __restrict__ obj,
                                                int32_t* __restrict__ iters) {
    PROBLEM_INDEX
    DevSolver S = make_solver(a, p);
    S.restore();
    const IpmResult r = S.result();
    u0[p * 2 + 0] = S.x_ctrl(0, 0);
    u0[p * 2 + 1] = S.x_ctrl(1, 0);
    if (traj) {
        const int N = a.P.N;
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

__global__ void k_set_active(int* active, int v) { *active = v; }

hipError_t launch_ipm_solve(const IpmParams& P, int64_t B, const double* state, const double* coeffs, double* u0,
                            double* traj, int32_t* status, double* obj, int32_t* iters, double* ws,
                            DriverCtx& ctx, hipStream_t stream) {
    if (B <= 0) return hipSuccess;
    const dim3 grid((unsigned)((B + 63) / 64)), block(64);
    const Args a{P, B, state, coeffs, ws, ctx.d_active};
    hipLaunchKernelGGL(k_set_active, dim3(1), dim3(1), 0, stream, ctx.d_active, (int)B);
    hipLaunchKernelGGL(k_init0, grid, block, 0, stream, a);
    hipLaunchKernelGGL(k_newton, grid, block, 0, stream, a, 1);
    hipLaunchKernelGGL(k_direction, grid, block, 0, stream, a, 1);
    hipLaunchKernelGGL(k_init1, grid, block, 0, stream, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    // Iterations in chunks; after each chunk the active count is copied to pinned
    // host memory.  The host checks chunk c-1's count while chunk c runs, so the
    // GPU never waits for the host; at most two chunks of no-op launches overshoot.
    const int C = ctx.chunk;
    int issued = 0;
    for (int c = 0;; ++c) {
        for (int i = 0; i < C; ++i) {
            hipLaunchKernelGGL(k_begin, grid, block, 0, stream, a);
            hipLaunchKernelGGL(k_newton, grid, block, 0, stream, a, 0);
            hipLaunchKernelGGL(k_direction, grid, block, 0, stream, a, 0);
            hipLaunchKernelGGL(k_linesearch, grid, block, 0, stream, a);
        }
        issued += C;
        e = hipMemcpyAsync(&ctx.h_active[c & 1], ctx.d_active, sizeof(int), hipMemcpyDeviceToHost, stream);
        if (e == hipSuccess) e = hipEventRecord(ctx.ev[c & 1], stream);
        if (e != hipSuccess) return e;
        if (c >= 1) {
            e = hipEventSynchronize(ctx.ev[(c - 1) & 1]);
            if (e != hipSuccess) return e;
            if (ctx.h_active[(c - 1) & 1] == 0) break;
        }
        if (issued > P.max_iter + 1 + C) break;  // every problem has terminated by max_iter
    }
    hipLaunchKernelGGL(k_outputs, grid, block, 0, stream, a, u0, traj, status, obj, iters);
    return hipGetLastError();
}

}  // namespace mpcg
