// mpc_ros_amd/csrc/mpcg_wide_kern.h -- the solver kernels of mpcg_wide.hip (one problem per
// wavefront, wide_core.h) as templates.  Each instance is compiled in its own translation
// unit (mpcg_wide_inst.hip, one group per MPCG_INST value, built in parallel); the
// dispatcher in mpcg_wide.hip reaches them through solve_kernel_fn / resume_kernel_fn.
//
// One workgroup = one wavefront = one problem; the problem's whole state lives in
// the workgroup's LDS (WideLayout: 19.0 KB at N = 20, i.e. 8 problems resident per
// CU).  Workgroups are dispatched by the hardware as CUs free up, so a slow problem
// occupies one wavefront slot while the rest of the batch streams past it.
#ifndef MPCG_WIDE_KERN_H
#define MPCG_WIDE_KERN_H
#include <hip/hip_runtime.h>

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
    int32_t* diag;         // [B][4] restoration phases, filter overflows, parked (1) / re-solved (2), filter peak (or null)
    int64_t n_prob;        // problems in state / coeffs / the outputs (the caller's batch; B is this launch's share)
    void* slots;           // nslots workspaces of slot_elems elements of T (the rare paths' copies)
    int32_t* slot_flags;   // 1 while a resident wavefront holds the slot
    int32_t nslots;        // nxcc partitions of nslots / nxcc slots, one per XCD
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
    int32_t* started;      // set by the batch kernel's first workgroup (the resume workers' liveness test)
    // problems that needed the restoration phase while the park area was full: their indices,
    // solved again from the start by the overflow launch (phase 1 of k_resume_wide)
    int32_t* ovf_count;
    int32_t* ovf_taken;
    int64_t* ovf_idx;
    int32_t nxcc;          // XCDs of the device (hipDeviceAttributeNumberOfXccs): slot partitions
    // k_resume_wide: 0 parked problems; 1 the overflow list (solved from the start, in park
    // entry ent0 + blockIdx.x; diag[:, 2] = ovf_mark, 2: park-area overflow)
    int32_t phase;
    int32_t ent0;
    int32_t ovf_mark;
    // the fp32 configuration's hand-over (WideSolver::handoff_out): written by the fp32 batch
    // kernel, read by k_warm_wide and its resume workers; handoff_stride floats per problem
    float* handoff;
    int64_t handoff_stride;
};
// Always-on range checks of the indices a kernel reads from device memory (the solve order, the
// park area's problem indices, the overflow list, a parked entry's counts) or derives from the
// workspace's counters (slot, park entry): a value out of range is reported and the kernel
// traps, before the value addresses anything.  One check per problem and index, wave-uniform.
// (The round-5 illegal address -- a captured graph replayed with the workspace resets as memset
// nodes the executor ran unordered with the solver kernels, DESIGN.md "Data layout in HBM" --
// was a use of such a value before its reset.)
__device__ __noinline__ void index_fault(const char* what, long long v, long long lim) {
    printf("mpcg: %s %lld outside [0, %lld) (block %d)\n", what, v, lim, (int)blockIdx.x);
    __builtin_trap();
}
__device__ __forceinline__ void check_index(const char* what, int64_t v, int64_t lim) {
    if (__builtin_expect(v < 0 || v >= lim, 0)) index_fault(what, (long long)v, (long long)lim);
}
// (the batch kernel: the same test without the report -- a printf call site costs the solver's
// register allocation 11 SGPR spill slots; the trap still stops the wavefront before the access)
__device__ __forceinline__ void check_index_quiet(int64_t v, int64_t lim) {
    if (__builtin_expect(v < 0 || v >= lim, 0)) __builtin_trap();
}

// the wavefront's end in k_solve_wide (after its results / its parked state are written).
// No fence: the count only tells the resume workers when every workgroup has finished, and
// a parking workgroup has released its entry (agent scope) before it counts itself.
__device__ __forceinline__ void block_done(int32_t* done) {
    __builtin_amdgcn_wave_barrier();
    if (threadIdx.x == 0) atomicAdd(done, 1);
}

constexpr int kXcds = 8;  // (MI355X; the runtime's count is used where it can say: device_xccs)
// The XCD the wavefront runs on (HW_REG_XCC_ID; 0..7 on MI355X in SPX mode), reduced to the
// device's nxcc XCDs (a partitioned device reports fewer)
__device__ __forceinline__ int xcc_id(int nxcc) {
    unsigned v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
    return (int)(v & 15) % nxcc;
}

// A workspace slot for the wavefront's problem, from the partition of the XCD it runs on:
// the first free one from blockIdx on (a partition holds 4x the wavefronts an XCD keeps
// resident, so the first probe normally succeeds; with fewer, a wavefront waits for a
// resident one on its XCD to finish and release its slot).  A slot is therefore only ever
// touched through one XCD's L2, so handing it over needs no agent-scope fence (an agent
// release is a write-back of the whole XCD L2, buffer_wbl2, per wavefront: 1.6 GB of write
// traffic per B = 65,536 launch when it was there).  The hand-over is ordered within the
// XCD: release_slot waits for the owner's stores to complete (they are in the XCD's L2
// then; the vector L1 is write-through) before the flag is cleared, and claim_slot
// invalidates the claiming CU's vector L1 after the flag is taken, so no line a previous
// owner wrote through another CU is read stale.  Slot lines are whole 128-byte lines, so two
// XCDs never share one.  Vector atomics (device scope) on the flags.  (Measured in round 5
// without gain: a per-XCD LIFO free list -- a new problem in the slot its XCD released last --
// made the headline launch 5x slower, 2,048 wavefronts CAS-ing 8 heads; the slot of the
// hardware wave slot (HW_REG_HW_ID) kept the time and moved the written bytes per launch
// both ways: N = 40 763 -> 1,072 MB, bicycle 732 -> 565 MB, fp32 N = 40 1,097 -> 1,176 MB.)
__device__ __forceinline__ int claim_slot(int32_t* flags, int nslots, int nxcc, int64_t hint) {
    const int per = nslots / nxcc, base = xcc_id(nxcc) * per;
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
    r = __builtin_amdgcn_readfirstlane(__shfl(r, 0, 64));
    asm volatile("s_waitcnt vmcnt(0)\n\tbuffer_inv sc0" ::: "memory");  // (acquire: the CU's L1)
    return r;
}
__device__ __forceinline__ void release_slot(int32_t* flags, int s) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (release: the slot's stores are in L2)
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

// WPE: wavefronts per SIMD the register allocation is for -- 2 (256 VGPRs), 1 (512) for the
// instances whose LDS per problem allows at most 4 problems per CU anyway (wide_kernel), or
// 3 (168 VGPRs) for the fp32 solver (N <= 64), whose LDS per problem leaves room for more
// than 8 problems per CU (N = 20: 9.5 KB, 12 per CU; N = 40: 14.8 KB, 11): with 68 VGPRs
// spilled the split instance is still 13 % faster than at 2 per SIMD
// The batch kernels' body: one problem per wavefront.  WARM (the fp64 phase of the fp32
// configuration, k_warm_wide): the problem continues from the fp32 solver's hand-over
// (WideSolver::solve_warm) where the fp32 solve converged, else it is solved from the start.
template <int MODEL, bool SPLIT, class T, int NB, bool DEFOPT, bool WARM>
__device__ __forceinline__ void solve_body(const WideArgs& a) {
    if ((int64_t)blockIdx.x >= a.B) return;
    const int64_t p = a.order ? (int64_t)a.order[blockIdx.x] : (int64_t)blockIdx.x;
    check_index_quiet(p, a.n_prob);
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
    if (blockIdx.x == 0 && t == 0) atomicExch(a.started, 1);
    const int slot = claim_slot(a.slot_flags, a.nslots, a.nxcc, (int64_t)blockIdx.x);
    check_index_quiet(slot, a.nslots);
    typedef WideSolver<DevWave, MODEL, SPLIT, T, NB> Solver;
    Solver S(Pk, pr, wv, (T*)a.slots + (int64_t)slot * a.slot_elems);
    if constexpr (WARM) {
        const float* h = a.handoff + p * a.handoff_stride;
        if (__builtin_amdgcn_readfirstlane(h[0] != 0.0f ? 1 : 0))
            S.init_warm(h);
        else
            S.init();
        S.run();  // (one call site of the solver's loop)
    } else {
        S.solve();
    }
    // the fp32 phase of the fp32 configuration: its ending goes to the fp64 phase (k_warm_wide)
    if constexpr (sizeof(T) == 4) {
        if (a.handoff) {
            S.handoff_out(a.handoff + p * a.handoff_stride);
            release_slot(a.slot_flags, slot);
            block_done(a.done);
            return;
        }
    }
    if (S.status == Solver::NEED_RESTO) {
        // the restoration phase runs in k_resume_wide: park the problem
        int e = 0;
        if (t == 0) e = atomicAdd(a.park_count, 1);
        e = __builtin_amdgcn_readfirstlane(__shfl(e, 0, 64));
        if (e < a.park_cap) {
            check_index_quiet(e, a.park_cap);
            S.park((T*)a.park + (int64_t)e * a.park_stride, p);
            if (t == 0) a.park_idx[e] = p;
            // the entry is complete: its ready flag after the stores (release, device scope)
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            __builtin_amdgcn_wave_barrier();
            if (t == 0) atomicExch(&a.park_ready[e], 1);
            release_slot(a.slot_flags, slot);
            block_done(a.done);
            return;
        }
        // the park area is full: the problem is solved again from the start by the overflow
        // launch after the drain (the same iterates; its outputs are written there)
        // (the index is published by an atomic store: a worker on another XCD may take the
        // entry while the batch runs -- the list starts as -1, written by the launch)
        if (t == 0) {
            const int o = atomicAdd(a.ovf_count, 1);
            check_index_quiet(o, a.B);
            atomicExch((unsigned long long*)&a.ovf_idx[o], (unsigned long long)p);
        }
        release_slot(a.slot_flags, slot);
        block_done(a.done);
        return;
    }
    write_out(a, S, p, 0);
    release_slot(a.slot_flags, slot);
    block_done(a.done);
}

template <int MODEL, bool SPLIT, class T, int NB, bool DEFOPT = false, int WPE = 2>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE, WPE))) k_solve_wide(WideArgs a) {
    solve_body<MODEL, SPLIT, T, NB, DEFOPT, false>(a);
}
// the fp64 phase of the fp32 configuration (mpcg_params.precision 1): every problem again, from
// the fp32 solver's converged iterate (WideSolver::solve_warm) or, where the fp32 solve did not
// converge, from the start
template <int MODEL, bool SPLIT, class T, int NB, bool DEFOPT = false, int WPE = 2>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE, WPE))) k_warm_wide(WideArgs a) {
    solve_body<MODEL, SPLIT, T, NB, DEFOPT, true>(a);
}

// results of problem p (u0, status, iterations, objective, trajectory; honor_original_bounds)
template <class Solver>
__device__ __forceinline__ void write_out(const WideArgs& a, Solver& S, int64_t p, int parked) {
    const int t = threadIdx.x;
    if (a.diag && t == 0) {
        // (the fp64 phase of the fp32 configuration: 4 continued from the fp32 iterate, 3 solved
        // again from the start)
        if (a.handoff && sizeof(typename Solver::T) == 8) parked = a.handoff[p * a.handoff_stride] != 0.0f ? 4 : 3;
        a.diag[p * 4 + 0] = S.n_resto;
        a.diag[p * 4 + 1] = S.n_fover;
        a.diag[p * 4 + 2] = parked;
        a.diag[p * 4 + 3] = S.nf_peak;
#ifdef MPCG_DEBUG_MU
        // (diagnostic build: the barrier parameter at the end of the solve, -100 log10 mu, and
        // the unscaled complementarity, -100 log10)
        a.diag[p * 4 + 1] = (int)(-100.0 * log10((double)S.mu));
        a.diag[p * 4 + 3] = (int)(-100.0 * log10((double)S.compl0 + 1e-300));
#endif
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
// exits early when the batch kernel has not started within ~2 ms (the two launches do not
// run concurrently, e.g. a graph executor that orders the fork's branches: the drain launch
// after the batch kernel takes every parked problem then), and when the batch kernel makes
// no progress for 20 s (it failed).
__device__ __forceinline__ int take_parked(const WideArgs& a) {
    int r = -1;
    if (threadIdx.x == 0) {
        const uint64_t t_start = wall_clock64();
        uint64_t t0 = t_start;
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
            const uint64_t now = wall_clock64();
            if (d == 0 && now - t_start > (uint64_t)200000 &&  // 2 ms at 100 MHz
                __hip_atomic_load(a.started, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0)
                break;
            if (d != last_done) {
                last_done = d;
                t0 = now;
            } else if (now - t0 > (uint64_t)2000000000) {  // 20 s at 100 MHz
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
// phase 1: the next problem of the overflow list, -1 when none is left.  The overflow launch
// runs after the batch kernel, so the list is complete then; the protocol would also serve a
// list that grows while the batch kernel runs: an entry is taken by a CAS on the taken count,
// its index awaited until the batch kernel has published it; the worker exits once every
// workgroup of the batch has finished and every entry is taken (or, as take_parked, when the
// batch kernel has not started within ~2 ms or makes no progress for 20 s).
__device__ __forceinline__ int64_t take_overflow(const WideArgs& a) {
    int64_t p = -1;
    if (threadIdx.x == 0) {
        const uint64_t t_start = wall_clock64();
        uint64_t t0 = t_start;
        int last_done = -1;
        int o = -1;
        for (;;) {
            const int d = __hip_atomic_load(a.done, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
            const int c = __hip_atomic_load(a.ovf_count, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
            const int tk = __hip_atomic_load(a.ovf_taken, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
            if (tk < c) {
                if (atomicCAS(a.ovf_taken, tk, tk + 1) == tk) {
                    o = tk;
                    break;
                }
                continue;
            }
            if ((int64_t)d >= a.B) break;  // (a workgroup lists itself before it counts itself done)
            const uint64_t now = wall_clock64();
            if (d == 0 && now - t_start > (uint64_t)200000 &&
                __hip_atomic_load(a.started, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0)
                break;
            if (d != last_done) {
                last_done = d;
                t0 = now;
            } else if (now - t0 > (uint64_t)2000000000) {
                break;
            }
            __builtin_amdgcn_s_sleep(32);
        }
        if (o >= 0) {
            for (;;) {
                p = (int64_t)__hip_atomic_load((unsigned long long*)&a.ovf_idx[o], __ATOMIC_ACQUIRE,
                                               __HIP_MEMORY_SCOPE_AGENT);
                if (p >= 0) break;
                __builtin_amdgcn_s_sleep(8);
            }
        }
    }
    const int lo = __builtin_amdgcn_readfirstlane(__shfl((int)(p & 0xffffffff), 0, 64));
    const int hi = __builtin_amdgcn_readfirstlane(__shfl((int)(p >> 32), 0, 64));
    return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

// (one wavefront per SIMD: the restoration phase and the resumed solve get the whole
// register file -- the workers are few, and the drain runs after the batch kernel)
template <int MODEL, bool SPLIT, class T, int NB>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 1))) k_resume_wide(WideArgs a) {
    const int t = threadIdx.x;
    const WideLayout Lw(a.P.N, a.P.filter_cap, MODEL);
    typedef WideSolver<DevWave, MODEL, SPLIT, T, NB> Solver;
    for (;;) {
        int64_t p;
        T* ent;
        if (a.phase == 0) {
            const int e = take_parked(a);
            if (e < 0) return;
            check_index("parked entry", e, a.park_cap);
            p = a.park_idx[e];
            check_index("parked problem", p, a.n_prob);
            ent = (T*)a.park + (int64_t)e * a.park_stride;
        } else {
            // the whole solve, in park entry ent0 + blockIdx.x (this worker's own)
            p = take_overflow(a);
            if (p < 0) return;
            check_index("overflow problem", p, a.n_prob);
            check_index("overflow worker's park entry", (int64_t)a.ent0 + blockIdx.x, a.park_cap);
            ent = (T*)a.park + (int64_t)(a.ent0 + blockIdx.x) * a.park_stride;
        }
        IpmProblem<T> pr;
#pragma unroll
        for (int j = 0; j < 6; ++j) pr.init[j] = (T)a.state[p * 6 + j];
#pragma unroll
        for (int j = 0; j < 4; ++j) pr.c[j] = (T)a.coeffs[p * 4 + j];
        DevWave wv;
        wv.t = t;
        Solver S(a.P, pr, wv, ent + Solver::PARK_SCALARS + Lw.total());
        if (a.phase == 0) {
            if (!S.park_entry_ok(ent, p)) index_fault("parked entry's tag / counts: problem", p, a.n_prob);
            S.unpark(ent);
        } else {
            if (a.handoff && a.handoff[p * a.handoff_stride] != 0.0f)
                S.init_warm(a.handoff + p * a.handoff_stride);  // (the fp32 configuration's fp64 phase)
            else
                S.init();
            S.run();
        }
        S.finish_resto();
        write_out(a, S, p, a.phase == 0 ? 1 : a.ovf_mark);
    }
}

// Kernel instances (host stubs), defined in mpcg_wide_inst.hip: the instance of
// k_solve_wide<MODEL, SPLIT, T, NB, DEFOPT, WPE> / k_resume_wide<MODEL, SPLIT, T, NB>.
template <int MODEL, bool SPLIT, class T, int NB, bool DEFOPT, int WPE>
const void* solve_kernel_fn();
// (the dispatcher's choice: the instance and its name, "k_solve_wide<M,S,T,NB,D,W>")
struct WideInst {
    const void* fn;
    const char* name;
};
WideInst wide_kernel(const IpmParams& P, int64_t B);
int device_xccs();
template <int MODEL, bool SPLIT, class T, int NB>
const void* resume_kernel_fn();
template <int MODEL, bool SPLIT, class T, int NB, bool DEFOPT, int WPE>
const void* warm_kernel_fn();

// (group, model, split, type, blocks, default options, waves per SIMD): the instances the
// library carries; group = the MPCG_INST translation unit that compiles it
#define MPCG_WIDE_SOLVE_INSTANCES(X)          \
    X(0, 0, true, double, 1, true, 2)         \
    X(0, 0, true, double, 1, true, 1)         \
    X(1, 0, true, double, 1, false, 2)        \
    X(2, 0, false, double, 1, false, 2)       \
    X(2, 0, false, double, 1, false, 1)       \
    X(5, 0, false, double, 1, true, 2)        \
    X(3, 0, false, double, 2, false, 1)       \
    X(1, 0, false, double, 2, true, 1)        \
    X(6, 0, false, double, 1, true, 1)        \
    X(4, 0, true, float, 1, false, 3)         \
    X(5, 0, false, float, 1, false, 3)        \
    X(6, 0, false, float, 2, false, 2)        \
    X(7, 1, true, double, 1, false, 2)        \
    X(4, 1, true, double, 1, true, 2)         \
    X(8, 1, false, double, 1, false, 2)       \
    X(7, 1, false, double, 1, true, 2)        \
    X(8, 1, false, double, 1, false, 1)       \
    X(9, 1, false, double, 2, false, 1)
// (the fp32 solver's problems that need the restoration phase are solved again in fp64: its
// resume kernel is the fp64 instance of the same horizon)
#define MPCG_WIDE_RESUME_INSTANCES(X)         \
    X(1, 0, true, double, 1)                  \
    X(2, 0, false, double, 1)                 \
    X(3, 0, false, double, 2)                 \
    X(7, 1, true, double, 1)                  \
    X(8, 1, false, double, 1)                 \
    X(9, 1, false, double, 2)
// the fp64 phase of the fp32 configuration (k_warm_wide), default options: per horizon class
#define MPCG_WIDE_WARM_INSTANCES(X)           \
    X(10, 0, true, double, 1, true, 2)        \
    X(10, 0, false, double, 1, true, 2)       \
    X(11, 0, false, double, 1, true, 1)       \
    X(11, 0, false, double, 2, true, 1)
#define MPCG_DECL_SOLVE(g, M, S, T, NB, D, W) template <> const void* solve_kernel_fn<M, S, T, NB, D, W>();
#define MPCG_DECL_WARM(g, M, S, T, NB, D, W) template <> const void* warm_kernel_fn<M, S, T, NB, D, W>();
#define MPCG_DECL_RESUME(g, M, S, T, NB) template <> const void* resume_kernel_fn<M, S, T, NB>();
MPCG_WIDE_SOLVE_INSTANCES(MPCG_DECL_SOLVE)
MPCG_WIDE_RESUME_INSTANCES(MPCG_DECL_RESUME)
MPCG_WIDE_WARM_INSTANCES(MPCG_DECL_WARM)
#undef MPCG_DECL_SOLVE
#undef MPCG_DECL_WARM
#undef MPCG_DECL_RESUME

}  // namespace mpcg
#endif
