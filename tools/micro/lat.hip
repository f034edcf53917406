// Latency micro-benchmarks (diagnostic): dependent chains of FP64 FMA, FP64 FMA with a
// DPP-moved operand, ds_write->ds_read round trips, v_readlane; 1 or 2 waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>

extern __shared__ double lds[];

template <int KIND>
__global__ void __launch_bounds__(64) k(double* out, long long* cyc, int n, double a, double b) {
    double x = a + threadIdx.x * 1e-9;
    const long long t0 = clock64();
    for (int i = 0; i < n; ++i) {
        if (KIND == 0) {  // 8 dependent FMAs
#pragma unroll
            for (int r = 0; r < 8; ++r) x = __builtin_fma(x, b, a);
        } else if (KIND == 1) {  // 8 independent FMA chains (throughput)
            double y[8];
#pragma unroll
            for (int r = 0; r < 8; ++r) y[r] = x + r;
#pragma unroll
            for (int q = 0; q < 8; ++q)
#pragma unroll
                for (int r = 0; r < 8; ++r) y[r] = __builtin_fma(y[r], b, a);
            x = y[0] + y[7];
        } else if (KIND == 2) {  // FMA + DPP shift (wave_shr:1) dependent
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                x = __builtin_fma(x, b, a);
                const int lo = __builtin_amdgcn_mov_dpp(__double2loint(x), 0x138, 0xF, 0xF, false);
                const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(x), 0x138, 0xF, 0xF, false);
                x = __hiloint2double(hi, lo);
            }
        } else if (KIND == 3) {  // FMA + LDS write/read round trip (other lane)
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                x = __builtin_fma(x, b, a);
                lds[threadIdx.x] = x;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                x = lds[(threadIdx.x + 1) & 63];
            }
        } else if (KIND == 4) {  // FMA + v_rcp_f64 + 2 Newton (the Riccati's rcp)
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                double rr = __builtin_amdgcn_rcp(x);
                double e = __builtin_fma(-x, rr, 1.0);
                rr = __builtin_fma(rr, e, rr);
                e = __builtin_fma(-x, rr, 1.0);
                rr = __builtin_fma(rr, e, rr);
                x = __builtin_fma(rr, b, a);
            }
        } else if (KIND == 6) {  // 16 independent FMA chains (issue rate of FP64 FMA)
            double y[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) y[r] = x + r;
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int r = 0; r < 16; ++r) y[r] = __builtin_fma(y[r], b, a);
            double z = 0;
#pragma unroll
            for (int r = 0; r < 16; ++r) z += y[r];
            x = z;
        } else if (KIND == 7) {  // 16 independent 32-bit integer chains (issue rate of v_add_u32 / v_xor)
            unsigned u[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) u[r] = __double2loint(x) + r;
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int r = 0; r < 16; ++r) u[r] = (u[r] * 3u) ^ (unsigned)q;
            unsigned z = 0;
#pragma unroll
            for (int r = 0; r < 16; ++r) z ^= u[r];
            x = __hiloint2double(__double2hiint(x), (int)z);
        } else if (KIND == 5) {  // FMA + readfirstlane (uniform)
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                x = __builtin_fma(x, b, a);
                const int lo = __builtin_amdgcn_readfirstlane(__double2loint(x));
                const int hi = __builtin_amdgcn_readfirstlane(__double2hiint(x));
                x = __hiloint2double(hi, lo);
            }
        }
    }
    const long long t1 = clock64();
    out[blockIdx.x * 64 + threadIdx.x] = x;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int KIND>
void run(const char* name, int waves_per_simd, int ops_per_iter) {
    const int n = 2000, blocks = 256 * 4 * waves_per_simd;
    double* out;
    long long* cyc;
    hipMalloc(&out, blocks * 64 * 8);
    hipMalloc(&cyc, blocks * 8);
    hipLaunchKernelGGL(k<KIND>, dim3(blocks), dim3(64), 1024, 0, out, cyc, n, 0.5, 0.999);
    hipDeviceSynchronize();
    long long* h = new long long[blocks];
    hipMemcpy(h, cyc, blocks * 8, hipMemcpyDeviceToHost);
    double s = 0;
    for (int i = 0; i < blocks; ++i) s += h[i];
    s /= blocks;
    printf("%-34s waves/SIMD %d: %.1f cycles per op (clock64 units)\n", name, waves_per_simd, s / n / ops_per_iter);
    delete[] h;
    hipFree(out);
    hipFree(cyc);
}

int main() {
    for (int w = 1; w <= 4; w *= 2) {
        run<0>("fma f64 dependent", w, 8);
        run<1>("fma f64 8 independent chains", w, 64);
        run<2>("fma + dpp wave_shr (per pair)", w, 8);
        run<3>("fma + lds write/read (per pair)", w, 8);
        run<4>("rcp+2 newton+fma (per 6 ops)", w, 2);
        run<5>("fma + readfirstlane x2 (per pair)", w, 8);
        run<6>("fma f64 16 independent chains", w, 64);
        run<7>("u32 mul+xor 16 chains (per mul+xor)", w, 64);
    }
    return 0;
}
