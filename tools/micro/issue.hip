// Issue-rate micro-benchmark (diagnostic): cycles per instruction of long streams of
// independent FP64 FMAs, FP64 adds, 32-bit integer ops, DPP moves and ds_read_b128, for
// one wavefront per SIMD (and 2, 4).  32 independent accumulators, 32 ops per loop trip.
#include <hip/hip_runtime.h>
#include <cstdio>

extern __shared__ double lds[];

template <int KIND>
__global__ void __launch_bounds__(64) k(double* out, long long* cyc, int n, double a, double b) {
    double y[32];
#pragma unroll
    for (int r = 0; r < 32; ++r) y[r] = a + (threadIdx.x + r) * 1e-9;
    unsigned u[32];
#pragma unroll
    for (int r = 0; r < 32; ++r) u[r] = threadIdx.x * 7 + r;
    for (int i = threadIdx.x; i < 1024; i += 64) lds[i] = i;
    __syncthreads();
    const long long t0 = clock64();
    for (int i = 0; i < n; ++i) {
        if (KIND == 0) {
#pragma unroll
            for (int r = 0; r < 32; ++r) y[r] = __builtin_fma(y[r], b, a);
        } else if (KIND == 1) {
#pragma unroll
            for (int r = 0; r < 32; ++r) y[r] = y[r] + b;
        } else if (KIND == 2) {
#pragma unroll
            for (int r = 0; r < 32; ++r) u[r] = u[r] + (unsigned)i;
        } else if (KIND == 3) {
#pragma unroll
            for (int r = 0; r < 32; ++r) u[r] = __builtin_amdgcn_mov_dpp(u[r], 0x138, 0xF, 0xF, false);
        } else if (KIND == 4) {  // 32 ds_read_b128 (16 B per lane), independent
            double2 acc[8];
#pragma unroll
            for (int r = 0; r < 8; ++r) acc[r] = double2{0, 0};
#pragma unroll
            for (int r = 0; r < 32; ++r) {
                const double2 v = *(const double2*)&lds[((threadIdx.x * 2 + r * 2 + i) & 511) * 2];
                acc[r & 7].x += v.x;
            }
#pragma unroll
            for (int r = 0; r < 8; ++r) y[r] += acc[r].x;
        } else if (KIND == 5) {  // mixed: 16 FP64 FMA + 16 u32 adds interleaved
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                y[r] = __builtin_fma(y[r], b, a);
                u[r] = u[r] + (unsigned)i;
            }
        }
    }
    const long long t1 = clock64();
    double s = 0;
#pragma unroll
    for (int r = 0; r < 32; ++r) s += y[r] + u[r];
    out[blockIdx.x * 64 + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int KIND>
void run(const char* name, int waves_per_simd) {
    const int n = 4000, blocks = 256 * 4 * waves_per_simd;
    double* out;
    long long* cyc;
    (void)hipMalloc(&out, blocks * 64 * 8);
    (void)hipMalloc(&cyc, blocks * 8);
    hipLaunchKernelGGL(k<KIND>, dim3(blocks), dim3(64), 8192, 0, out, cyc, n, 0.5, 0.999);
    (void)hipDeviceSynchronize();
    long long* h = new long long[blocks];
    (void)hipMemcpy(h, cyc, blocks * 8, hipMemcpyDeviceToHost);
    double s = 0;
    for (int i = 0; i < blocks; ++i) s += h[i];
    s /= blocks;
    printf("%-28s waves/SIMD %d: %.2f cycles per instruction\n", name, waves_per_simd, s / n / 32);
    delete[] h;
    (void)hipFree(out);
    (void)hipFree(cyc);
}

int main() {
    for (int w = 1; w <= 4; w *= 2) {
        run<0>("v_fma_f64", w);
        run<1>("v_add_f64", w);
        run<2>("v_add_u32", w);
        run<3>("v_mov_b32_dpp", w);
        run<4>("ds_read_b128 (+1/4 add)", w);
        run<5>("fma_f64 + add_u32 pairs", w);
    }
    return 0;
}
