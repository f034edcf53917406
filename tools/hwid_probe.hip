// tools/hwid_probe.hip -- which hardware wave slots (HW_REG_HW_ID / HW_REG_XCC_ID) the solver's
// workgroups land on (diagnostic): 65,536 one-wavefront workgroups with 19 KB of LDS each.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <set>
#include <vector>
__global__ void __launch_bounds__(64) k(unsigned* o) {
    extern __shared__ double lds[];
    unsigned v, x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(v));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    lds[threadIdx.x] = v;
    __syncthreads();
    for (int i = 0; i < 2000; ++i) __builtin_amdgcn_s_sleep(10);
    if (threadIdx.x == 0) { o[2 * blockIdx.x] = v; o[2 * blockIdx.x + 1] = x + (unsigned)lds[1] * 0; }
}
int main() {
    const int B = 65536;
    unsigned* d;
    hipMalloc(&d, B * 8);
    hipLaunchKernelGGL(k, dim3(B), dim3(64), 18976, 0, d);
    std::vector<unsigned> h(2 * B);
    hipMemcpy(h.data(), d, B * 8, hipMemcpyDeviceToHost);
    std::set<unsigned> se, sh, cu, simd, wave, xcc, key;
    for (int b = 0; b < B; ++b) {
        unsigned v = h[2 * b];
        se.insert((v >> 13) & 7); sh.insert((v >> 12) & 1); cu.insert((v >> 8) & 15); simd.insert((v >> 4) & 3);
        wave.insert(v & 15); xcc.insert(h[2 * b + 1] & 15);
        key.insert(((h[2 * b + 1] & 15) << 16) | (((v >> 13) & 7) << 7) | (((v >> 12) & 1) << 6) | (((v >> 8) & 15) << 2) | ((v >> 4) & 3));
    }
    auto pr = [](const char* n, const std::set<unsigned>& s) { std::printf("%s:", n); for (unsigned x : s) std::printf(" %u", x); std::printf("\n"); };
    pr("se", se); pr("sh", sh); pr("cu", cu); pr("simd", simd); pr("wave", wave); pr("xcc", xcc);
    std::printf("distinct (xcc, se, sh, cu, simd): %zu\n", key.size());
    std::set<unsigned> full;
    for (int b = 0; b < B; ++b) {
        unsigned v = h[2 * b];
        full.insert(((h[2 * b + 1] & 15) << 20) | (((v >> 13) & 7) << 11) | (((v >> 12) & 1) << 10) | (((v >> 8) & 15) << 6) | (((v >> 4) & 3) << 4) | (v & 15));
    }
    std::printf("distinct (xcc, se, sh, cu, simd, wave): %zu\n", full.size());
    return 0;
}
