// tools/diag_stamps.hip -- DIAGNOSTIC BUILD ONLY: per-pass cycle stamps of the solver.
// Reads inputs.bin (int64 B, then B x 10 doubles), writes diag.bin (B x 8 uint64:
// stats, riccati, forward, linesearch, accept, -, iters, status).  The stamp build's
// timings are shares, not the product's run time (stamps add waits).
#define MPCG_DIAG 1
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "ipm_core.h"

using namespace mpcg;
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

__global__ void __launch_bounds__(64, 1) k(IpmParams P, int64_t B, const double* in, double* ws, uint64_t* diag) {
    const int64_t p = (int64_t)blockIdx.x * 64 + threadIdx.x;
    if (p >= B) return;
    IpmProblem<double> pr;
    for (int j = 0; j < 6; ++j) pr.init[j] = in[p * 10 + j];
    for (int j = 0; j < 4; ++j) pr.c[j] = in[p * 10 + 6 + j];
    const IpmLayout Lw{P.N};
    const int64_t tile_elems = (int64_t)Lw.total(P.filter_cap) * 64;
    DevWs<double> w{(DevWs<double>::gT*)(ws + (int64_t)blockIdx.x * tile_elems), (int)threadIdx.x};
    IpmSolver<double, DevWs<double>> S(P, pr, w);
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    IpmResult r = S.solve();
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    for (int j = 0; j < 5; ++j) diag[p * 8 + j] = S.tacc[j];
    diag[p * 8 + 5] = t1 - t0;
    diag[p * 8 + 6] = r.iters;
    diag[p * 8 + 7] = r.status;
}

int main(int argc, char** argv) {
    FILE* f = fopen(argc > 1 ? argv[1] : "inputs.bin", "rb");
    int64_t B;
    if (fread(&B, 8, 1, f) != 1) return 1;
    std::vector<double> in(B * 10);
    if (fread(in.data(), 8, B * 10, f) != (size_t)(B * 10)) return 1;
    fclose(f);
    IpmParams P{20, 0.1, 0, 0, 1.0, 1000, 1000, 100, 100, 50, 0, 10, 1.0, 1.0, 1000, 1e-8, 1e-8, 0.1, 3000, 64};
    IpmLayout L{20};
    double *din, *dws;
    uint64_t* ddiag;
    hipMalloc(&din, B * 80);
    hipMalloc(&dws, (size_t)L.total(64) * 8 * 64 * ((B + 63) / 64));
    hipMalloc(&ddiag, B * 64);
    hipMemcpy(din, in.data(), B * 80, hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k, dim3((B + 63) / 64), dim3(64), 0, 0, P, B, din, dws, ddiag);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    std::vector<uint64_t> diag(B * 8);
    hipMemcpy(diag.data(), ddiag, B * 64, hipMemcpyDeviceToHost);
    FILE* g = fopen(argc > 2 ? argv[2] : "diag.bin", "wb");
    fwrite(diag.data(), 8, B * 8, g);
    fclose(g);
    printf("kernel %.3f ms\n", ms);
    return 0;
}
