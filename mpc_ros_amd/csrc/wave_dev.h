// mpc_ros_amd/csrc/wave_dev.h -- CDNA4 wavefront context of the wide solver (wide_core.h).
//
// Lane index, the wavefront's LDS base, and the cross-lane primitives:
//   sync()          order LDS accesses across lanes of the wavefront.  LDS
//                   instructions of one wavefront execute in issue order, so a
//                   compiler barrier (wave-scope fence) is all that is needed;
//   bcast8<q>(v)    lane q of the lane's group of 8 (ds_swizzle bit mode, no LDS memory);
//   rpart<s>(v)     partner of reduction step s: xor 1, xor 2 (DPP quad_perm), mirror
//                   within 8, mirror within 16 (DPP row_half_mirror / row_mirror),
//                   xor 16 (ds_swizzle), xor 32 (ds_bpermute).  Pairs are symmetric, so
//                   a commutative op leaves every lane with identical bits;
//   up1(v), dn1(v)  value of lane t-1 / t+1 (DPP wave_shr:1 / wave_shl:1; lanes 0 / 63: undefined);
//   up8(x, y), dn6(x, y)  x := y of lane t-1 (t+1); lane 0 (63) keeps x (the systolic
//                   recursions);
//   lo_half(v)      v of lane t & 31 (v_permlane32_swap);
//   xor32_pair(v, a, b)  {a, b} = {v, v of lane t ^ 32} (v_permlane32_swap);
//   any(b), uni(i), uni_d(x)  wave vote; wave-uniform (scalar) copy of lane 0's value;
//   ballot_prefix(b, &n)  lanes below with b set (stream compaction of the filter), n = total;
//   lane()          the lane index, recomputed by a volatile v_mbcnt pair: each solver phase
//                   derives its per-lane LDS offsets from it, so the compiler cannot hoist
//                   them out of the iteration loop (they were kept live across every phase
//                   and 60-70 VGPRs spilled to scratch);
//   S()             the LDS base (address 0); ld2(i, a, b) / st2(i, a, b): 16-byte LDS load /
//                   store of two doubles (i even).
#ifndef MPCG_WAVE_DEV_H
#define MPCG_WAVE_DEV_H

#include <hip/hip_runtime.h>

namespace mpcg {

#if defined(__HIP_DEVICE_COMPILE__)
#define MPCG_LDS __attribute__((address_space(3)))
#else
#define MPCG_LDS
#endif

// The workgroup's dynamic LDS (one problem per workgroup).  The solver kernels use no
// static LDS, so the dynamic segment starts at LDS address 0 and is addressed from a
// literal 0 base: every access is then one DS instruction on the lane's own offset
// (through the symbol, the late-resolved base costs a v_add per per-lane address --
// 3 % of the kernel time).  launch_wide_solve checks that the kernel has no static LDS.
extern __shared__ double mpcg_dyn_lds[];

struct DevWaveBase {
    typedef MPCG_LDS double ldsT;
    typedef MPCG_LDS double2 ldsT2;
    int t;
    __device__ __forceinline__ static ldsT* S() { return (ldsT*)(__SIZE_TYPE__)0; }
    // the LDS base as an array of U (double: the fp64 solver; float: the fp32 solver)
    template <class U>
    __device__ __forceinline__ static MPCG_LDS U* Sp() { return (MPCG_LDS U*)(__SIZE_TYPE__)0; }

    __device__ __forceinline__ void sync() const {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    // order global-memory accesses across the lanes of the wavefront (the restoration
    // phase's HBM records written by one lane and read by another): workgroup-scope release
    // and acquire -- the vector memory operations of a workgroup share the CU's L1
    __device__ __forceinline__ void gsync() const {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
    __device__ __forceinline__ void ld2(int i, double& a, double& b) const {
        const double2 v = *(const ldsT2*)(S() + i);
        a = v.x;
        b = v.y;
    }
    __device__ __forceinline__ void st2(int i, double a, double b) const {
        *(ldsT2*)(S() + i) = double2{a, b};
    }
    // (fp32 solver: 8-byte pair loads)
    __device__ __forceinline__ void ld2(int i, float& a, float& b) const {
        const float2 v = *(const MPCG_LDS float2*)(Sp<float>() + i);
        a = v.x;
        b = v.y;
    }
    template <int pat>
    __device__ __forceinline__ static float swz(float v) {
        return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), pat));
    }
    template <int ctrl>
    __device__ __forceinline__ static float dpp(float v) {
        return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), ctrl, 0xF, 0xF, false));
    }
    template <int s>
    __device__ __forceinline__ float rpart(float v) const {
        if (s == 0) return dpp<0xB1>(v);
        if (s == 1) return dpp<0x4E>(v);
        if (s == 2) return dpp<0x141>(v);
        if (s == 3) return dpp<0x140>(v);
        if (s == 4) return swz<0x1F | (0x10 << 10)>(v);
        return __shfl_xor(v, 32, 64);
    }
    __device__ __forceinline__ float up1(float v) const { return dpp<0x138>(v); }
    __device__ __forceinline__ float dn1(float v) const { return dpp<0x130>(v); }
    template <bool UP, int n>
    __device__ __forceinline__ static void shift(float* x, const float* y) {
#pragma unroll
        for (int q = 0; q < n; ++q)
            x[q] = __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(x[q]), __float_as_int(y[q]),
                                                              UP ? 0x138 : 0x130, 0xF, 0xF, false));
    }
    __device__ __forceinline__ void up8(float* x, const float* y) const { shift<true, 8>(x, y); }
    __device__ __forceinline__ void dn6(float* x, const float* y) const { shift<false, 6>(x, y); }
    __device__ __forceinline__ float lo_half(float v) const {
        const auto r = __builtin_amdgcn_permlane32_swap(__float_as_int(v), __float_as_int(v), false, false);
        return __int_as_float((int)r[0]);
    }
    __device__ __forceinline__ void xor32_pair(float v, float& a, float& b) const {
        const auto r = __builtin_amdgcn_permlane32_swap(__float_as_int(v), __float_as_int(v), false, false);
        a = __int_as_float((int)r[0]);
        b = __int_as_float((int)r[1]);
    }
    __device__ __forceinline__ float uni_d(float v) const {
        return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
    }
    template <int pat>
    __device__ __forceinline__ static double swz(double v) {
        const int lo = __builtin_amdgcn_ds_swizzle(__double2loint(v), pat);
        const int hi = __builtin_amdgcn_ds_swizzle(__double2hiint(v), pat);
        return __hiloint2double(hi, lo);
    }
    template <int ctrl>
    __device__ __forceinline__ static double dpp(double v) {
        const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), ctrl, 0xF, 0xF, false);
        const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), ctrl, 0xF, 0xF, false);
        return __hiloint2double(hi, lo);
    }
    // ds_swizzle bit mode: lane = ((lane & and) | or) ^ xor within 32 lanes
    template <int q>
    __device__ __forceinline__ double bcast8(double v) const {
        return swz<0x18 | (q << 5)>(v);
    }
    template <int s>
    __device__ __forceinline__ double rpart(double v) const {
        if (s == 0) return dpp<0xB1>(v);           // quad_perm [1,0,3,2]
        if (s == 1) return dpp<0x4E>(v);           // quad_perm [2,3,0,1]
        if (s == 2) return dpp<0x141>(v);          // row_half_mirror
        if (s == 3) return dpp<0x140>(v);          // row_mirror
        if (s == 4) return swz<0x1F | (0x10 << 10)>(v);  // xor 16
        return __shfl_xor(v, 32, 64);
    }
    // DPP wave_shr:1 (a gfx9-family DPP control): lane t reads lane t-1
    __device__ __forceinline__ double up1(double v) const { return dpp<0x138>(v); }
    // DPP wave_shl:1: lane t reads lane t+1
    __device__ __forceinline__ double dn1(double v) const { return dpp<0x130>(v); }
    // x[q] := y[q] of lane t-1 (UP: DPP wave_shr:1) / t+1 (wave_shl:1), n doubles.  Lane 0
    // (63), whose source lane does not exist, keeps x[q]: the DPP move with bound_ctrl off
    // does not write it.  One v_mov_b32_dpp per dword, the old value tied to the result.
    template <bool UP, int n>
    __device__ __forceinline__ static void shift(double* x, const double* y) {
#pragma unroll
        for (int q = 0; q < n; ++q) {
            const int lo = __builtin_amdgcn_update_dpp(__double2loint(x[q]), __double2loint(y[q]),
                                                       UP ? 0x138 : 0x130, 0xF, 0xF, false);
            const int hi = __builtin_amdgcn_update_dpp(__double2hiint(x[q]), __double2hiint(y[q]),
                                                       UP ? 0x138 : 0x130, 0xF, 0xF, false);
            x[q] = __hiloint2double(hi, lo);
        }
    }
    // the step recursion (8 doubles up) and the multiplier recursion (6 doubles down)
    __device__ __forceinline__ void up8(double* x, const double* y) const { shift<true, 8>(x, y); }
    __device__ __forceinline__ void dn6(double* x, const double* y) const { shift<false, 6>(x, y); }
    // v of lane t & 31: the lower half-wave's value in both halves (v_permlane32_swap of v
    // with itself moves the lower half into the upper)
    __device__ __forceinline__ double lo_half(double v) const {
        const auto lo = __builtin_amdgcn_permlane32_swap(__double2loint(v), __double2loint(v), false, false);
        const auto hi = __builtin_amdgcn_permlane32_swap(__double2hiint(v), __double2hiint(v), false, false);
        return __hiloint2double((int)hi[0], (int)lo[0]);
    }
    // {a, b} = {v, v of lane t ^ 32} in some order (v_permlane32_swap per dword: the lower
    // half-wave receives the upper half's values and vice versa)
    __device__ __forceinline__ void xor32_pair(double v, double& a, double& b) const {
        const auto lo = __builtin_amdgcn_permlane32_swap(__double2loint(v), __double2loint(v), false, false);
        const auto hi = __builtin_amdgcn_permlane32_swap(__double2hiint(v), __double2hiint(v), false, false);
        a = __hiloint2double((int)hi[0], (int)lo[0]);
        b = __hiloint2double((int)hi[1], (int)lo[1]);
    }
    __device__ __forceinline__ bool any(bool b) const { return __any(b); }
    // the value of lane 63 / lane 0 (wave-uniform; the two-block recursions)
    __device__ __forceinline__ double lane63(double v) const {
        return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), 63),
                                __builtin_amdgcn_readlane(__double2loint(v), 63));
    }
    __device__ __forceinline__ double lane0(double v) const {
        return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), 0),
                                __builtin_amdgcn_readlane(__double2loint(v), 0));
    }
    // the value of lane l (l wave-uniform)
    __device__ __forceinline__ double lanev(double v, int l) const {
        return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l),
                                __builtin_amdgcn_readlane(__double2loint(v), l));
    }
    __device__ __forceinline__ float lanev(float v, int l) const {
        return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
    }
    __device__ __forceinline__ float lane63(float v) const {
        return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
    }
    __device__ __forceinline__ float lane0(float v) const {
        return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
    }
    // number of lanes below this one with b set, and (total) the count over the wavefront
    __device__ __forceinline__ int ballot_prefix(bool b, int* total) const {
        const unsigned long long m = __ballot(b);
        *total = __builtin_amdgcn_readfirstlane(__popcll(m));
        return __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
    }
    // the lane index, recomputed (volatile: the compiler cannot hoist it or values derived
    // from it out of the solver's loops)
    __device__ __forceinline__ int lane() const {
        int r;
        asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(r));
        return r;
    }
    __device__ __forceinline__ int uni(int v) const { return __builtin_amdgcn_readfirstlane(v); }
    // scheduling barrier: instructions are not moved across it (no wait is inserted)
    __device__ __forceinline__ void sched_fence() const { __builtin_amdgcn_sched_barrier(0); }
    __device__ __forceinline__ double uni_d(double v) const {
        return __hiloint2double(__builtin_amdgcn_readfirstlane(__double2hiint(v)),
                                __builtin_amdgcn_readfirstlane(__double2loint(v)));
    }
};

struct DevWave : DevWaveBase {
    __device__ __forceinline__ void mark(int) const {}
};

}  // namespace mpcg
#endif
