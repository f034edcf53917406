// LDS allocation granularity on the device (diagnostic): the workgroups per CU the occupancy
// calculator grants a 64-thread kernel at a range of dynamic LDS sizes.
#include <hip/hip_runtime.h>
#include <cstdio>
extern __shared__ double dyn[];
__global__ void __launch_bounds__(64) k(double* o) { dyn[threadIdx.x] = 1; o[threadIdx.x] = dyn[(threadIdx.x + 1) & 63]; }
int main() {
    hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    const int sizes[] = {13312, 13600, 13648, 13653, 13696, 14336, 18204, 18432, 20480, 26624, 27136, 27296, 27304, 27392, 27648, 29536, 32768};
    for (int s : sizes) {
        int n = 0;
        hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, (const void*)k, 64, s);
        printf("lds %6d B -> %d workgroups per CU (%s)\n", s, n, hipGetErrorString(e));
    }
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    printf("sharedMemPerMultiprocessor %zu, maxSharedMemoryPerMultiProcessor %zu, sharedMemPerBlock %zu\n",
           p.sharedMemPerMultiprocessor, p.maxSharedMemoryPerMultiProcessor, p.sharedMemPerBlock);
    return 0;
}
