// mpc_ros_amd/csrc/mpcg_wide.hip -- one problem per wavefront (wide_core.h) on CDNA4.
//
// One workgroup = one wavefront = one problem; the problem's whole state lives in
// the workgroup's LDS (WideLayout: 19.9 KB at N = 20, i.e. 8 problems resident per
// CU).  Workgroups are dispatched by the hardware as CUs free up, so a slow problem
// occupies one wavefront slot while the rest of the batch streams past it.
#include <hip/hip_runtime.h>
#include <hipcub/device/device_radix_sort.hpp>

#include "mpcg_internal.h"
#include "wave_dev.h"
#include "wide_core.h"

namespace mpcg {

struct WideArgs {
    IpmParams P;
    int64_t B;
    const int32_t* order;  // workgroup -> problem (NULL: identity)
    const double* state;
    const double* coeffs;
    double* u0;
    double* traj;
    int32_t* status;
    double* obj;
    int32_t* iters;
    int32_t* diag;         // [B][4] restoration phases, filter overflows, parked, 0 (or null)
    void* slots;           // nslots workspaces of slot_elems elements of T (the rare paths' copies)
    int32_t* slot_flags;   // 1 while a resident wavefront holds the slot
    int32_t nslots;        // kXcds partitions of nslots / kXcds slots, one per XCD
    int32_t slot_elems;    // WideLayout::spill() rounded up to whole 128-byte lines
    // parked problems (the restoration phase, continued by k_resume_wide while the batch
    // kernel runs): count, capacity, problem index, ready flag and state of each; the entries
    // taken by the resume workers; the batch kernel's finished workgroups
    int32_t* park_count;
    int32_t park_cap;
    int64_t* park_idx;
    int32_t* park_ready;
    int32_t* park_taken;
    int32_t* done;
    void* park;
    int64_t park_stride;   // elements of T per park entry (WideSolver::park_elems, whole 128-byte lines)
};
// the wavefront's end in k_solve_wide (after its results / its parked state are written).
// No fence: the count only tells the resume workers when every workgroup has finished, and
// a parking workgroup has released its entry (agent scope) before it counts itself.
__device__ __forceinline__ void block_done(int32_t* done) {
    __builtin_amdgcn_wave_barrier();
    if (threadIdx.x == 0) atomicAdd(done, 1);
}

// The XCD the wavefront runs on (HW_REG_XCC_ID, 0..7 on MI355X).
constexpr int kXcds = 8;
__device__ __forceinline__ int xcc_id() {
    unsigned v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
    return (int)(v & 15) % kXcds;
}

// A workspace slot for the wavefront's problem, from the partition of the XCD it runs on:
// the first free one from blockIdx on (a partition holds 4x the wavefronts an XCD keeps
// resident, so the first probe normally succeeds; with fewer, a wavefront waits for a
// resident one on its XCD to finish and release its slot).  A slot is therefore only ever
// touched through one XCD's L2, and every owner writes a slot location before it reads it
// (the watchdog, acceptable-point, SOC and soft-restoration copies, the filter's workspace
// entries): no data crosses wavefronts, so claim and release need no acquire / release
// fence (an agent-scope release is a write-back of the whole XCD L2, buffer_wbl2, per
// wavefront: 1.6 GB of write traffic per B = 65,536 launch when it was there).  Slot
// lines are whole 128-byte lines, so two XCDs never share one.  Vector atomics (device
// scope) on the flags.
__device__ __forceinline__ int claim_slot(int32_t* flags, int nslots, int64_t hint) {
    const int per = nslots / kXcds, base = xcc_id() * per;
    int s = (int)(hint % per);
    int r = 0;
    if (threadIdx.x == 0) {
        for (;;) {
            if (atomicCAS(&flags[base + s], 0, 1) == 0) break;
            s = s + 1 == per ? 0 : s + 1;
            if (s == (int)(hint % per)) __builtin_amdgcn_s_sleep(8);
        }
        r = base + s;
    }
    return __builtin_amdgcn_readfirstlane(__shfl(r, 0, 64));
}
__device__ __forceinline__ void release_slot(int32_t* flags, int s) {
    __builtin_amdgcn_wave_barrier();
    if (threadIdx.x == 0) atomicExch(&flags[s], 0);
}

// 2 wavefronts per SIMD: 19 KB of LDS per problem allows 8 problems per CU, the register
// budget of 256 per lane lets all of them be resident
// SPLIT (N <= 32): the recursions and the step statistics use both half-waves (wide_core.h)
// T: the solver's arithmetic type (double; float for precision 1).  Inputs and outputs
// stay double at the boundary.
// NB: stage blocks (2 for 64 < N <= 128, lane t owning stages t and 64 + t).
// DEFOPT: the Ipopt options are the reference's defaults (ipopt_default_options), compiled
// as constants.
template <class Solver>
__device__ __forceinline__ void write_out(const WideArgs& a, Solver& S, int64_t p, int parked);

// WPE: wavefronts per SIMD the register allocation is for -- 2 (256 VGPRs), or 1 (512) for
// the instances whose LDS per problem allows at most 4 problems per CU anyway (wide_kernel)
template <int MODEL, bool SPLIT, class T, int NB, bool DEFOPT = false, int WPE = 2>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE, WPE))) k_solve_wide(WideArgs a) {
    if ((int64_t)blockIdx.x >= a.B) return;
    const int64_t p = a.order ? (int64_t)a.order[blockIdx.x] : (int64_t)blockIdx.x;
    const int t = threadIdx.x;
    IpmProblem<T> pr;
#pragma unroll
    for (int j = 0; j < 6; ++j) pr.init[j] = (T)a.state[p * 6 + j];
#pragma unroll
    for (int j = 0; j < 4; ++j) pr.c[j] = (T)a.coeffs[p * 4 + j];
    DevWave wv;
    wv.t = t;
    IpmParams Pk = a.P;
    if constexpr (DEFOPT) ipopt_default_options(Pk);
    const int slot = claim_slot(a.slot_flags, a.nslots, (int64_t)blockIdx.x);
    typedef WideSolver<DevWave, MODEL, SPLIT, T, NB> Solver;
    Solver S(Pk, pr, wv, (T*)a.slots + (int64_t)slot * a.slot_elems);
    S.solve();
    if (S.status == Solver::NEED_RESTO) {
        // the restoration phase runs in k_resume_wide: park the problem
        int e = 0;
        if (t == 0) e = atomicAdd(a.park_count, 1);
        e = __builtin_amdgcn_readfirstlane(__shfl(e, 0, 64));
        if (e < a.park_cap) {
            S.park((T*)a.park + (int64_t)e * a.park_stride);
            if (t == 0) a.park_idx[e] = p;
            // the entry is complete: its ready flag after the stores (release, device scope)
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            __builtin_amdgcn_wave_barrier();
            if (t == 0) atomicExch(&a.park_ready[e], 1);
            release_slot(a.slot_flags, slot);
            block_done(a.done);
            return;
        }
        S.status = IPM_RESTORATION_FAILURE;  // (more parked problems than the park area holds)
    }
    write_out(a, S, p, 0);
    release_slot(a.slot_flags, slot);
    block_done(a.done);
}

// results of problem p (u0, status, iterations, objective, trajectory; honor_original_bounds)
template <class Solver>
__device__ __forceinline__ void write_out(const WideArgs& a, Solver& S, int64_t p, int parked) {
    const int t = threadIdx.x;
    if (a.diag && t == 0) {
        a.diag[p * 4 + 0] = S.n_resto;
        a.diag[p * 4 + 1] = S.n_fover;
        a.diag[p * 4 + 2] = parked;
        a.diag[p * 4 + 3] = S.nf_peak;
    }
    const double o = (double)S.objective_out();
    const int N = a.P.N;
    if (t == 0) {
        a.u0[p * 2 + 0] = (double)S.x_ctrl(0, 0);
        a.u0[p * 2 + 1] = (double)S.x_ctrl(1, 0);
        if (a.status) a.status[p] = S.status;
        if (a.iters) a.iters[p] = S.iter;
        if (a.obj) a.obj[p] = o;
    }
    if (a.traj) {
        double* tr = a.traj + p * 3 * N;
        for (int k = t; k < N; k += 64) {
            tr[k] = (double)S.x_state(0, k);
            tr[N + k] = (double)S.x_state(1, k);
            tr[2 * N + k] = (double)S.x_state(2, k);
        }
    }
}

// The parked problems: the restoration phase (WideSolver<..., RESTO> out of line) and the
// rest of the solve, from the state k_solve_wide parked -- the same solver instance, so the
// iterates are those the first kernel would have continued with.  A separate kernel keeps
// the call out of the batch kernel's register allocation.  It runs on a second stream
// alongside the batch kernel: a few workers take parked problems as they appear (a problem
// that parks early in the batch is resumed while the batch still runs) and exit once every
// workgroup of the batch kernel has finished and every parked problem is taken.  A worker
// that sees no progress of the batch kernel for 20 s exits (the batch kernel failed).
__device__ __forceinline__ int take_parked(const WideArgs& a) {
    int r = -1;
    if (threadIdx.x == 0) {
        uint64_t t0 = wall_clock64();
        int last_done = -1;
        for (;;) {
            const int d = __hip_atomic_load(a.done, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
            int c = __hip_atomic_load(a.park_count, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
            c = c < a.park_cap ? c : a.park_cap;
            const int tk = __hip_atomic_load(a.park_taken, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
            if (tk < c) {
                if (atomicCAS(a.park_taken, tk, tk + 1) == tk) {
                    r = tk;
                    break;
                }
                continue;
            }
            // (a workgroup parks before it counts itself done: all parked once done == B)
            if ((int64_t)d >= a.B && tk >= c) break;
            if (d != last_done) {
                last_done = d;
                t0 = wall_clock64();
            } else if (wall_clock64() - t0 > (uint64_t)2000000000) {  // 20 s at 100 MHz
                break;
            }
            __builtin_amdgcn_s_sleep(32);
        }
        if (r >= 0) {  // the entry's stores are visible once its ready flag is
            while (__hip_atomic_load(&a.park_ready[r], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == 0)
                __builtin_amdgcn_s_sleep(8);
        }
    }
    r = __builtin_amdgcn_readfirstlane(__shfl(r, 0, 64));
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    return r;
}

// (one wavefront per SIMD: the restoration phase and the resumed solve get the whole
// register file -- the workers are few, and the drain runs after the batch kernel)
template <int MODEL, bool SPLIT, class T, int NB>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 1))) k_resume_wide(WideArgs a) {
    const int t = threadIdx.x;
    const WideLayout Lw(a.P.N, a.P.filter_cap, MODEL);
    typedef WideSolver<DevWave, MODEL, SPLIT, T, NB> Solver;
    for (;;) {
        const int e = take_parked(a);
        if (e < 0) return;
        const int64_t p = a.park_idx[e];
        IpmProblem<T> pr;
#pragma unroll
        for (int j = 0; j < 6; ++j) pr.init[j] = (T)a.state[p * 6 + j];
#pragma unroll
        for (int j = 0; j < 4; ++j) pr.c[j] = (T)a.coeffs[p * 4 + j];
        DevWave wv;
        wv.t = t;
        T* ent = (T*)a.park + (int64_t)e * a.park_stride;
        Solver S(a.P, pr, wv, ent + Solver::PARK_SCALARS + Lw.total());
        S.unpark(ent);
        S.finish_resto();
        write_out(a, S, p, 1);
    }
}

// Scheduling key: workgroups are dispatched roughly in index order, so a slow problem
// dispatched late extends the launch (its iterations run at the lone-wavefront rate
// after the rest of the batch is done).  The curvature of the reference polynomial
// predicts the slow tail (infinity set: 36 of the 39 problems above p99 in iterations
// are in the top decile of |c1| + |c2| + |c3|), so problems are solved in descending
// order of it.  Results do not depend on the order.
__global__ void __launch_bounds__(256) k_sched_key(int64_t B, const double* coeffs, float* key, int32_t* idx) {
    const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= B) return;
    const double* c = coeffs + p * 4;
    key[p] = (float)(fabs(c[1]) + fabs(c[2]) + fabs(c[3]));
    idx[p] = (int32_t)p;
}

size_t wide_sched_bytes(int64_t B) {
    size_t temp = 0;
    hipcub::DeviceRadixSort::SortPairsDescending(nullptr, temp, (const float*)nullptr, (float*)nullptr,
                                                 (const int32_t*)nullptr, (int32_t*)nullptr, (int)B);
    return 2 * sizeof(float) * B + 2 * sizeof(int32_t) * B + temp + 256;
}

hipError_t launch_wide_order(int64_t B, const double* coeffs, void* buf, size_t bytes, int32_t** order,
                             hipStream_t stream) {
    char* b = (char*)buf;
    float* k0 = (float*)b;
    float* k1 = k0 + B;
    int32_t* v0 = (int32_t*)(k1 + B);
    int32_t* v1 = v0 + B;
    void* temp = (void*)(((uintptr_t)(v1 + B) + 255) & ~(uintptr_t)255);
    size_t temp_bytes = bytes - ((char*)temp - b);
    hipLaunchKernelGGL(k_sched_key, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, stream, B, coeffs, k0, v0);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    e = hipcub::DeviceRadixSort::SortPairsDescending(temp, temp_bytes, k0, k1, v0, v1, (int)B, 0, 32, stream);
    *order = v1;
    return e;
}

static size_t elem_bytes(const IpmParams& P) { return P.precision == 1 ? sizeof(float) : sizeof(double); }
size_t wide_lds_bytes(const IpmParams& P) {
    return (size_t)WideLayout(P.N, P.filter_cap, P.model).total() * elem_bytes(P);
}

// the resume kernel of a solve kernel's instance (the general-options instance also for the
// default-options one: the two compute bitwise the same)
static const void* resume_kernel(const IpmParams& P) {
    const bool split = P.N <= 32;
    const bool f32 = P.precision == 1;
    const int nb = P.N > 64 ? 2 : 1;
    if (P.N > 128 || (f32 && P.model != 0)) return nullptr;
    if (f32)
        return nb == 2 ? (const void*)k_resume_wide<0, false, float, 2>
             : split ? (const void*)k_resume_wide<0, true, float, 1> : (const void*)k_resume_wide<0, false, float, 1>;
    if (P.model == 1)
        return nb == 2 ? (const void*)k_resume_wide<1, false, double, 2>
             : split ? (const void*)k_resume_wide<1, true, double, 1> : (const void*)k_resume_wide<1, false, double, 1>;
    return nb == 2 ? (const void*)k_resume_wide<0, false, double, 2>
         : split ? (const void*)k_resume_wide<0, true, double, 1> : (const void*)k_resume_wide<0, false, double, 1>;
}

// (model, split, precision, blocks, default options, waves per SIMD) -> kernel instance;
// null if none.  An fp64 problem of more than 32 KB of LDS (N >= 35; every N > 64) leaves
// room for at most 4 problems per CU (160 KB), one wavefront per SIMD: its instance is
// register-allocated for one (512 VGPRs, no spills) instead of two.
// A batch the device holds at one wavefront per SIMD (B <= kLoneBatch: 4 x 256 CUs) runs
// the benchmark configuration's instance allocated for one wavefront per SIMD as well.
constexpr int64_t kLoneBatch = 1024;
static const void* wide_kernel(const IpmParams& P, int64_t B) {
    const bool split = P.N <= 32;
    const bool f32 = P.precision == 1;
    const int nb = P.N > 64 ? 2 : 1;
    if (P.N > 128) return nullptr;
    if (f32 && P.model != 0) return nullptr;  // (fp32: the differential drive)
    if (f32)
        return nb == 2 ? (const void*)k_solve_wide<0, false, float, 2>
             : split ? (const void*)k_solve_wide<0, true, float, 1> : (const void*)k_solve_wide<0, false, float, 1>;
    const bool one = wide_lds_bytes(P) > 32768;
    if (P.model == 1)
        return nb == 2 ? (const void*)k_solve_wide<1, false, double, 2, false, 1>
             : split ? (const void*)k_solve_wide<1, true, double, 1>
             : one   ? (const void*)k_solve_wide<1, false, double, 1, false, 1>
                     : (const void*)k_solve_wide<1, false, double, 1>;
    if (split && ipopt_options_are_default(P))  // (the benchmark configuration)
        return B <= kLoneBatch ? (const void*)k_solve_wide<0, true, double, 1, true, 1>
                               : (const void*)k_solve_wide<0, true, double, 1, true>;
    return nb == 2 ? (const void*)k_solve_wide<0, false, double, 2, false, 1>
         : split ? (const void*)k_solve_wide<0, true, double, 1>
         : one   ? (const void*)k_solve_wide<0, false, double, 1, false, 1>
                 : (const void*)k_solve_wide<0, false, double, 1>;
}

// Workspace slots for a batch of B: four times the wavefronts the device can hold resident at
// once (occupancy of the instance at its LDS size times the CUs), at most B (at least 32 per
// XCD), in kXcds equal partitions.  A wavefront claims slot blockIdx mod the partition size
// in its XCD's partition, or the next free one: with the margin, a slow problem still
// holding a slot rarely makes a later wavefront probe further.
int64_t wide_slots(const IpmParams& P, int64_t B) {
    if (B <= 0) return 0;
    int64_t n = 4096;  // (fallback if the runtime cannot say)
    const void* fn = wide_kernel(P, B);
    int dev = 0, cus = 0, per = 0;
    if (fn && hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
        hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)wide_lds_bytes(P)) == hipSuccess &&
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, fn, 64, wide_lds_bytes(P)) == hipSuccess && per > 0 &&
        cus > 0)
        n = 4 * (int64_t)per * cus;
    n = n < B ? n : B;
    int64_t part = (n + kXcds - 1) / kXcds;
    const int64_t floor_ = B < 32 ? B : 32;
    part = part > floor_ ? part : floor_;
    return part * kXcds;
}
// a slot's elements: WideLayout::spill() rounded up to whole 128-byte lines
static int64_t slot_elems(const IpmParams& P) {
    const int64_t e = P.precision == 1 ? 4 : 8, per_line = 128 / e;
    const int64_t n = WideLayout(P.N, P.filter_cap, P.model).spill();
    return (n + per_line - 1) / per_line * per_line;
}
static size_t slot_flag_bytes(int64_t nslots) { return ((size_t)nslots * sizeof(int32_t) + 255) & ~(size_t)255; }
// the park area: problems that enter the restoration phase (rare: ~5e-5 of the infinity set at
// N = 20, 5e-4 at N = 40, ~4e-3 with the fp32 solver at N = 40); beyond its capacity (B / 128,
// at least 256) a problem ends with restoration_failure
int64_t wide_park_cap(int64_t B) {
    const int64_t c = B / 128 > 256 ? B / 128 : 256;
    return c < B ? c : B;
}
static size_t park_elems(const IpmParams& P) {
    const WideLayout L(P.N, P.filter_cap, P.model);
    const size_t n = (size_t)(32 + L.total() + L.slot()), per_line = 128 / elem_bytes(P);  // (WideSolver::park_elems)
    return (n + per_line - 1) / per_line * per_line;
}
size_t wide_spill_bytes(const IpmParams& P, int64_t B) {
    const int64_t ns = wide_slots(P, B), pc = wide_park_cap(B);
    return slot_flag_bytes(ns) + 256 + ((size_t)pc * sizeof(int64_t) + 255 & ~(size_t)255) + slot_flag_bytes(pc) +
           (size_t)slot_elems(P) * elem_bytes(P) * (size_t)ns +
           park_elems(P) * elem_bytes(P) * (size_t)pc;
}

// Concurrent resume workers (parked problems in flight while the batch kernel runs): each
// holds a wavefront slot and a problem's LDS for the whole batch kernel (32 workers cost
// the batch kernel ~7 %, 2 under 1 %), and problems park rarely (~5e-5 of the infinity set
// at N = 20, ~5e-4 at N = 40; ~4e-3 with the fp32 solver): two, and one more per 65536
// problems.  What is still parked when the batch ends goes to the drain launch.
#ifndef MPCG_RESUME_WORKERS
#define MPCG_RESUME_WORKERS 2
#endif
static int64_t resume_workers(int64_t B) { return MPCG_RESUME_WORKERS + B / 65536; }

hipError_t launch_wide_solve(const IpmParams& P, int64_t B, const double* state, const double* coeffs, double* u0,
                             double* traj, int32_t* status, double* obj, int32_t* iters, int32_t* diag,
                             const int32_t* order, void* spill, size_t spill_bytes, hipStream_t stream,
                             hipStream_t aux, hipEvent_t ev_fork, hipEvent_t ev_join) {
    if (B <= 0) return hipSuccess;
    if (!spill) return hipErrorInvalidValue;
    const size_t lds = wide_lds_bytes(P);
    const void* fn = wide_kernel(P, B);
    if (!fn) return hipErrorInvalidValue;
    // the solver addresses its dynamic LDS from address 0 (wave_dev.h): no static LDS
    hipFuncAttributes fa;
    hipError_t e = hipFuncGetAttributes(&fa, fn);
    if (e != hipSuccess) return e;
    if (fa.sharedSizeBytes != 0) return hipErrorInvalidKernelFile;
    e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    // the workspace (wide_spill_bytes): slot flags | park count, taken, done (256 B) | park
    // indices | park ready flags | slots | park area
    const int64_t ns = wide_slots(P, B), pc = wide_park_cap(B);
    if (ns < 1 || wide_spill_bytes(P, B) > spill_bytes) return hipErrorInvalidValue;
    char* w = (char*)spill;
    int32_t* flags = (int32_t*)w;
    w += slot_flag_bytes(ns);
    int32_t* pcount = (int32_t*)w;
    w += 256;
    int64_t* pidx = (int64_t*)w;
    w += (size_t)pc * sizeof(int64_t) + 255 & ~(size_t)255;
    int32_t* pready = (int32_t*)w;
    w += slot_flag_bytes(pc);
    void* slots = w;
    w += (size_t)slot_elems(P) * elem_bytes(P) * (size_t)ns;
    void* park = w;
    e = hipMemsetAsync(flags, 0, slot_flag_bytes(ns) + 256, stream);  // (slot flags, park counters)
    if (e == hipSuccess) e = hipMemsetAsync(pready, 0, slot_flag_bytes(pc), stream);
    if (e != hipSuccess) return e;
    const WideArgs a{P,      B,          order,      state,  coeffs, u0,  traj, status, obj, iters, diag, slots, flags,
                     (int32_t)ns, (int32_t)slot_elems(P), pcount, (int32_t)pc, pidx, pready, pcount + 1, pcount + 2,
                     park, (int64_t)park_elems(P)};
    void* args[] = {(void*)&a};
    const void* rf = resume_kernel(P);
    e = hipFuncGetAttributes(&fa, rf);
    if (e != hipSuccess) return e;
    if (fa.sharedSizeBytes != 0) return hipErrorInvalidKernelFile;
    e = hipFuncSetAttribute(rf, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    // fork: the resume workers on the aux stream alongside the batch kernel; join: the
    // stream continues after both (no host synchronisation; graph-capturable)
    const bool fork = aux && aux != stream && ev_fork && ev_join;
    if (fork) {
        e = hipEventRecord(ev_fork, stream);
        if (e == hipSuccess) e = hipStreamWaitEvent(aux, ev_fork, 0);
        if (e != hipSuccess) return e;
    }
    e = hipLaunchKernel(fn, dim3((unsigned)B), dim3(64), args, lds, stream);
    if (e != hipSuccess) return e;
    if (fork) {  // the concurrent workers
        const unsigned workers = (unsigned)(pc < resume_workers(B) ? pc : resume_workers(B));
        e = hipLaunchKernel(rf, dim3(workers), dim3(64), args, lds, aux);
        if (e != hipSuccess) return e;
    }
    // the drain, after the batch kernel: one worker per park entry, so the problems still
    // parked when the batch ends run side by side (a worker finding nothing left exits at
    // once) -- the tail is the longest restoration, not their sum over a few workers
    e = hipLaunchKernel(rf, dim3((unsigned)pc), dim3(64), args, lds, stream);
    if (e != hipSuccess) return e;
    if (fork) {
        e = hipEventRecord(ev_join, aux);
        if (e == hipSuccess) e = hipStreamWaitEvent(stream, ev_join, 0);
        if (e != hipSuccess) return e;
    }
    return hipGetLastError();
}

}  // namespace mpcg
