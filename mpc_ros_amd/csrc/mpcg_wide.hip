// mpc_ros_amd/csrc/mpcg_wide.hip -- one problem per wavefront (wide_core.h) on CDNA4: the
// launch side (solve order, instance choice, workspace, batch kernel + resume workers).
// The kernels are in mpcg_wide_kern.h, their instances in mpcg_wide_inst.hip.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <hipcub/device/device_radix_sort.hpp>

#include "mpcg_wide_kern.h"

namespace mpcg {

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

// the workspace's per-launch state: the slot flags, the 64 counters (park count / taken / done /
// started, the overflow count / taken), the park ready flags, the overflow list (-1: not yet
// published)
__global__ void __launch_bounds__(256) k_reset_ws(int32_t* flags, int64_t nflags, int32_t* cnt, int32_t* pready,
                                                  int64_t npready, int64_t* ovf, int64_t novf) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < nflags) flags[i] = 0;
    if (i < 64) cnt[i] = 0;
    if (i < npready) pready[i] = 0;
    if (i < novf) ovf[i] = -1;
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

// The instances (solve_kernel_fn / resume_kernel_fn, mpcg_wide_inst.hip).  A diagnostic
// build with MPCG_HEADLINE_ONLY links only the benchmark configuration's group (tools/).
template <int M, bool S, class T, int NB, bool D, int W>
static WideInst sk(const char* name) {
#ifdef MPCG_HEADLINE_ONLY
    if constexpr (!(M == 0 && S && sizeof(T) == 8 && NB == 1 && D))
        return WideInst{nullptr, name};
    else
#endif
        return WideInst{solve_kernel_fn<M, S, T, NB, D, W>(), name};
}
// (the instance and its name: mpcg_last_kernel() reports the name of the one a solve launched)
#define SK(M, S, T, NB, D, W) sk<M, S, T, NB, D, W>("k_solve_wide<" #M "," #S "," #T "," #NB "," #D "," #W ">")
template <int M, bool S, class T, int NB>
static const void* rk() {
#ifdef MPCG_HEADLINE_ONLY
    if constexpr (!(M == 0 && S && sizeof(T) == 8 && NB == 1))
        return nullptr;
    else
#endif
        return resume_kernel_fn<M, S, T, NB>();
}

// The fp32 configuration (mpcg_params.precision 1) runs in two phases: the fp32 solver on the
// whole batch (its stated options), then the fp64 solver with the reference's Ipopt options on
// the whole batch again (k_warm_wide) -- from the fp32 solver's converged iterate (a few fp64
// iterations to Ipopt's tolerance), or from the start where the fp32 solve did not converge
// (its line search fails where Ipopt would enter the restoration phase, a tiny step, the
// iteration limit: a float iterate's noise floor).  mpcg_params.no_restoration = 1 keeps the
// fp32 solver's own ending instead (status 9 where Ipopt would restore).
static bool two_phase(const IpmParams& P) { return P.precision == 1 && !P.no_resto; }
static IpmParams fp64_params(const IpmParams& P) {
    IpmParams q = P;
    q.precision = 0;
    ipopt_default_options(q);
    return q;
}

// the resume kernel of a solve kernel's instance (the general-options instance also for the
// default-options one: the two compute bitwise the same); for the fp32 solver the fp64
// instance of the same horizon (a precision-1 launch parks nothing -- the fp32 phase hands every
// ending to the fp64 phase, no_restoration = 1 keeps it -- so its workers find nothing and exit)
static const void* resume_kernel(const IpmParams& P) {
    const bool split = P.N <= 32;
    const int nb = P.N > 64 ? 2 : 1;
    if (P.N > 128 || (P.precision == 1 && P.model != 0)) return nullptr;
    if (P.model == 1)
        return nb == 2 ? rk<1, false, double, 2>() : split ? rk<1, true, double, 1>() : rk<1, false, double, 1>();
    return nb == 2 ? rk<0, false, double, 2>() : split ? rk<0, true, double, 1>() : rk<0, false, double, 1>();
}

// (model, split, precision, blocks, default options, waves per SIMD) -> kernel instance;
// null if none.  An fp64 problem of more than 32 KB of LDS (N >= 35; every N > 64) leaves
// room for at most 4 problems per CU (160 KB), one wavefront per SIMD: its instance is
// register-allocated for one (512 VGPRs, no spills) instead of two.
// A small batch (B <= kLoneBatch) runs the benchmark configuration's instance allocated for
// one wavefront per SIMD as well: its time is set by its longest problem at the
// lone-wavefront rate, which the 512-VGPR allocation (no spills) shortens (B = 4,096, the
// BASELINE's configs[1]: 3.02 -> 2.93 ms; B = 1,024 is held at one wavefront per SIMD).
constexpr int64_t kLoneBatch = 4096;
WideInst wide_kernel(const IpmParams& P, int64_t B) {
    const bool split = P.N <= 32;
    const bool f32 = P.precision == 1;
    const int nb = P.N > 64 ? 2 : 1;
    if (P.N > 128) return WideInst{nullptr, ""};
    if (f32 && P.model != 0) return WideInst{nullptr, ""};  // (fp32: the differential drive)
    if (f32)  // (N <= 64: 3 wavefronts per SIMD, mpcg_wide_kern.h)
        return nb == 2 ? SK(0, false, float, 2, false, 2)
             : split ? SK(0, true, float, 1, false, 3) : SK(0, false, float, 1, false, 3);
    const bool one = wide_lds_bytes(P) > 32768;
    // (default Ipopt options: the instances that compile them as constants -- the benchmark
    // configuration, configs[4]'s bicycle, and every fp64 horizon of the differential drive
    // and the bicycle's 33..64 stages at two wavefronts per SIMD)
    const bool dflt = ipopt_options_are_default(P);
    if (P.model == 1)
        return nb == 2 ? SK(1, false, double, 2, false, 1)
             : split ? (dflt ? SK(1, true, double, 1, true, 2) : SK(1, true, double, 1, false, 2))
             : one   ? SK(1, false, double, 1, false, 1)
                     : (dflt ? SK(1, false, double, 1, true, 2) : SK(1, false, double, 1, false, 2));
    if (split && dflt)  // (the benchmark configuration)
        return B <= kLoneBatch ? SK(0, true, double, 1, true, 1) : SK(0, true, double, 1, true, 2);
    return nb == 2 ? (dflt ? SK(0, false, double, 2, true, 1) : SK(0, false, double, 2, false, 1))
         : split ? SK(0, true, double, 1, false, 2)
         : one   ? (dflt ? SK(0, false, double, 1, true, 1) : SK(0, false, double, 1, false, 1))
                 : (dflt ? SK(0, false, double, 1, true, 2) : SK(0, false, double, 1, false, 2));
}

// XCDs of the current device (HW_REG_XCC_ID partitions of the workspace slots); 8 on an
// MI355X in SPX mode, fewer on a partitioned device
int device_xccs() {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeNumberOfXccs, dev) != hipSuccess ||
        n < 1)
        return kXcds;
    return n > 16 ? 16 : n;
}

// Workspace slots for a batch of B: four times the wavefronts the device can hold resident at
// once (occupancy of the instance at its LDS size times the CUs), at most B (at least 32 per
// XCD), in one equal partition per XCD (device_xccs).  A wavefront claims slot blockIdx mod the
// partition size in its XCD's partition, or the next free one: with the margin, a slow problem
// still holding a slot rarely makes a later wavefront probe further.
int64_t wide_slots(const IpmParams& P, int64_t B) {
    if (B <= 0) return 0;
    int64_t n = 4096;  // (fallback if the runtime cannot say)
    const void* fn = wide_kernel(P, B).fn;
    int dev = 0, cus = 0, per = 0;
    if (fn && hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
        hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)wide_lds_bytes(P)) == hipSuccess &&
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, fn, 64, wide_lds_bytes(P)) == hipSuccess && per > 0 &&
        cus > 0)
        n = 4 * (int64_t)per * cus;
    n = n < B ? n : B;
    const int nx = device_xccs();
    int64_t part = (n + nx - 1) / nx;
    const int64_t floor_ = B < 32 ? B : 32;
    part = part > floor_ ? part : floor_;
    return part * nx;
}
// a slot's elements: WideLayout::spill() rounded up to whole 128-byte lines
static int64_t slot_elems(const IpmParams& P) {
    const int64_t e = P.precision == 1 ? 4 : 8, per_line = 128 / e;
    const int64_t n = WideLayout(P.N, P.filter_cap, P.model).spill();
    return (n + per_line - 1) / per_line * per_line;
}
static size_t slot_flag_bytes(int64_t nslots) { return ((size_t)nslots * sizeof(int32_t) + 255) & ~(size_t)255; }
// the park area: problems that enter the restoration phase (rare: ~5e-5 of the infinity set at
// N = 20, 5e-4 at N = 40, ~4e-3 with the fp32 solver at N = 40); its capacity is B / 128, at
// least 256 (P.park_cap > 0: that many, mpcg_set_park_capacity).  Beyond it a problem goes to
// the overflow list and is solved again from the start after the drain.
int64_t wide_park_cap(const IpmParams& P, int64_t B) {
    int64_t c = B / 128 > 256 ? B / 128 : 256;
    if (P.park_cap > 0) c = P.park_cap;
    return c < B ? c : B;
}
// the overflow list: one index per problem (only where the park area can overflow)
static size_t ovf_bytes(const IpmParams& P, int64_t B) {
    return wide_park_cap(P, B) < B ? ((size_t)B * sizeof(int64_t) + 255) & ~(size_t)255 : 0;
}
static size_t park_elems(const IpmParams& P);
static size_t park_entry_bytes(const IpmParams& P) { return park_elems(P) * elem_bytes(P); }
static size_t park_elems(const IpmParams& P) {
    const WideLayout L(P.N, P.filter_cap, P.model);
    const size_t n = (size_t)(32 + L.total() + L.slot()), per_line = 128 / elem_bytes(P);  // (WideSolver::park_elems)
    return (n + per_line - 1) / per_line * per_line;
}
// one phase's workspace: slot flags | counters | park indices | park ready flags | overflow list
// | slots | park area
static size_t phase_bytes(const IpmParams& P, int64_t B) {
    const int64_t ns = wide_slots(P, B), pc = wide_park_cap(P, B);
    return slot_flag_bytes(ns) + 256 + ((size_t)pc * sizeof(int64_t) + 255 & ~(size_t)255) + slot_flag_bytes(pc) +
           ovf_bytes(P, B) + (size_t)slot_elems(P) * elem_bytes(P) * (size_t)ns + park_entry_bytes(P) * (size_t)pc;
}
// (the fp32 configuration: the larger phase's workspace -- the phases run one after the other --
// then the hand-over, WideSolver::handoff_elems floats per problem)
static size_t handoff_offset(const IpmParams& P, int64_t B) {
    const size_t a = phase_bytes(P, B), b = phase_bytes(fp64_params(P), B);
    return ((a > b ? a : b) + 255) & ~(size_t)255;
}
static int64_t handoff_stride(const IpmParams& P) {
    return ((int64_t)(4 + 30 * P.N) + 31) / 32 * 32;  // (WideSolver::handoff_elems, whole lines)
}
// The fp32 configuration's head: the problems the solve order ranks longest (ordered batches only,
// B / 1024 of them) are solved by the fp64 solver from the start on the aux stream while the fp32
// phase runs the others -- the longest fp64 solves (through the restoration phase) would otherwise
// start only with the fp64 phase and set its length (problem 19,304 of the infinity set at N = 40:
// rank 2 of the order, 217 fp64 iterations, 11.5 ms alone).
static int64_t head_count(int64_t B) {
    int64_t div = 1024;
#ifdef MPCG_HEAD_ENV
    // (diagnostic builds only: the head's share of the batch, B / MPCG_HEAD_DIV; 0: no head)
    if (const char* d = getenv("MPCG_HEAD_DIV")) div = atol(d);
    if (div <= 0) return 0;
#endif
    return B > kOrderMinBatch ? B / div : 0;
}
static size_t order2_offset(const IpmParams& P, int64_t B) {
    return handoff_offset(P, B) + (size_t)handoff_stride(P) * sizeof(float) * (size_t)B;
}
// the head's parameters: the fp64 solver's, with a park entry for every head problem (no
// park-area overflow: the head's stream never waits for its resume workers' stream)
static IpmParams head_params(const IpmParams& P, int64_t K) {
    IpmParams q = fp64_params(P);
    q.park_cap = (int)K;
    return q;
}
static size_t head_offset(const IpmParams& P, int64_t B) {
    return (order2_offset(P, B) + ((size_t)(B + 63) / 64 * 64 + 64) * sizeof(int32_t) + 255) & ~(size_t)255;
}
size_t wide_spill_bytes(const IpmParams& P, int64_t B) {
    // (+ the fp64 phase's solve order: B indices and two counters, + the head's workspace)
    if (two_phase(P)) {
        const int64_t K = head_count(B);
        return head_offset(P, B) + (K > 0 ? phase_bytes(head_params(P, K), K) : 0);
    }
    return phase_bytes(P, B);
}

// diag[p][2] = mark for the problems p = order[0, K) (of n_prob)
__global__ void __launch_bounds__(256) k_mark_rows(int64_t K, const int32_t* order, int32_t* diag, int32_t mark,
                                                   int64_t n_prob) {
    const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (b >= K) return;
    const int64_t p = order[b];
    check_index("head order: problem", p, n_prob);
    diag[p * 4 + 2] = mark;
}

// The fp64 phase's solve order: the problems the fp32 phase did not converge on (solved from the
// start: full-length fp64 solves, some through the restoration phase) first, then the others (a
// few fp64 iterations each), so the long solves do not trail the batch.  Positions by two atomic
// counters (from the front, and from the back): results do not depend on the order.
__global__ void __launch_bounds__(256) k_cold_first(int64_t B, const float* h, int64_t stride, const int32_t* order,
                                                    int32_t* out, int32_t* cnt, int64_t n_prob) {
    const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (b >= B) return;
    const int32_t p = order ? order[b] : (int32_t)b;
    check_index("fp64 phase order: problem", p, n_prob);
    if (h[(int64_t)p * stride] != 0.0f)
        out[B - 1 - atomicAdd(&cnt[1], 1)] = p;
    else
        out[atomicAdd(&cnt[0], 1)] = p;
}

// Concurrent resume workers (parked problems in flight while the batch kernel runs): each
// holds a wavefront slot and a problem's LDS for the whole batch kernel (32 workers cost
// the batch kernel ~7 %, 2 under 1 %), and problems park rarely (~5e-5 of the infinity set
// at N = 20, ~5e-4 at N = 40; ~4e-3 with the fp32 solver): two, and one more per 65536
// problems.  What is still parked when the batch ends goes to the drain launch.
#ifndef MPCG_RESUME_WORKERS
#define MPCG_RESUME_WORKERS 2
#endif
// (MPCG_RESUME_WORKERS in the environment overrides the count: a tuning knob, read once)
static int64_t resume_workers(int64_t B) {
    static const int64_t env = [] {
        const char* s = getenv("MPCG_RESUME_WORKERS");
        return s ? (int64_t)atoll(s) : (int64_t)-1;
    }();
    return env > 0 ? env : MPCG_RESUME_WORKERS + B / 65536;
}
// One batch launch (with its resume workers, drain and overflow launches) of the instance inst
// for parameters P on the workspace at spill.  handoff: the fp32 configuration's hand-over
// buffer (the fp32 phase writes it, the fp64 phase -- inst a k_warm_wide instance -- reads it).
// origin (the fp32 configuration's head): &the caller's stream (a pointer: the caller's stream may
// be the null stream) -- the workspace reset runs there,
// then both `stream` and (with workers) `aux` fork from it (ev_fork), and the caller joins them
// (*forked_out: whether aux received work); no stream forks from a forked stream, which a
// captured graph does not survive.
static hipError_t launch_phase(const IpmParams& P, const WideInst& inst, int64_t B, const double* state,
                               const double* coeffs, double* u0, double* traj, int32_t* status, double* obj,
                               int32_t* iters, int32_t* diag, const int32_t* order, void* spill, float* handoff,
                               hipStream_t stream, hipStream_t aux, hipEvent_t ev_fork, hipEvent_t ev_join,
                               int64_t nworkers = -1, const hipStream_t* origin = nullptr,
                               bool* forked_out = nullptr, int64_t n_prob = -1) {
    size_t lds = wide_lds_bytes(P);
#ifdef MPCG_LDS_PAD_ENV
    // (diagnostic builds only: extra LDS per workgroup, fewer problems per CU)
    if (const char* pad = getenv("MPCG_LDS_PAD")) lds += (size_t)atol(pad);
#endif
    const void* fn = inst.fn;
    if (!fn) return hipErrorInvalidValue;
    // the solver addresses its dynamic LDS from address 0 (wave_dev.h): no static LDS
    hipFuncAttributes fa;
    hipError_t e = hipFuncGetAttributes(&fa, fn);
    if (e != hipSuccess) return e;
    if (fa.sharedSizeBytes != 0) return hipErrorInvalidKernelFile;
    e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    const bool fp32_phase = P.precision == 1 && handoff;  // (parks nothing: its endings go to the hand-over)
    // (every host-side call before the first launch: the device does not wait for the host
    // between the reset kernel and the solver -- ~15 us of a B = 1 solve otherwise)
    const void* rf = fp32_phase ? nullptr : resume_kernel(P);
    const size_t rlds = lds;
    if (rf) {
        e = hipFuncGetAttributes(&fa, rf);
        if (e != hipSuccess) return e;
        if (fa.sharedSizeBytes != 0) return hipErrorInvalidKernelFile;
        e = hipFuncSetAttribute(rf, hipFuncAttributeMaxDynamicSharedMemorySize, (int)rlds);
        if (e != hipSuccess) return e;
    }
    // the workspace (phase_bytes): slot flags | counters: park count, taken, done, started,
    // overflow count, overflow taken (256 B) | park indices | park ready flags | overflow list |
    // slots | park area
    const int64_t ns = wide_slots(P, B), pc = wide_park_cap(P, B);
    char* w = (char*)spill;
    int32_t* flags = (int32_t*)w;
    w += slot_flag_bytes(ns);
    int32_t* cnt = (int32_t*)w;
    w += 256;
    int64_t* pidx = (int64_t*)w;
    w += (size_t)pc * sizeof(int64_t) + 255 & ~(size_t)255;
    int32_t* pready = (int32_t*)w;
    w += slot_flag_bytes(pc);
    int64_t* ovf = (int64_t*)w;
    w += ovf_bytes(P, B);
    void* slots = w;
    w += (size_t)slot_elems(P) * elem_bytes(P) * (size_t)ns;
    void* park = w;
    // (the per-launch state -- slot flags, counters, park ready flags, the overflow list at -1 --
    // reset by a kernel, not by memset nodes: a captured graph replayed a second time ran its
    // small memsets unordered with the solver kernels)
    {
        const int64_t npr = pc, nov = ovf_bytes(P, B) ? B : 0;
        int64_t n = npr > 64 ? npr : 64;
        n = n > nov ? n : nov;
        n = n > ns ? n : ns;
        hipLaunchKernelGGL(k_reset_ws, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, origin ? *origin : stream,
                           flags, ns, cnt, pready, npr, ovf, nov);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    if (origin) {
        e = hipEventRecord(ev_fork, *origin);
        if (e == hipSuccess) e = hipStreamWaitEvent(stream, ev_fork, 0);
        if (e != hipSuccess) return e;
    }
    WideArgs a{P,      B,          order,      state,  coeffs, u0,  traj, status, obj, iters, diag,
               n_prob > 0 ? n_prob : B, slots, flags,
               (int32_t)ns, (int32_t)slot_elems(P), cnt, fp32_phase ? 0 : (int32_t)pc, pidx, pready, cnt + 1, cnt + 2,
               park, (int64_t)park_elems(P), cnt + 3, cnt + 4, cnt + 5, ovf, (int32_t)device_xccs(), 0, 0, 2,
               handoff, handoff ? handoff_stride(P) : 0};
    void* args[] = {(void*)&a};
    if (fp32_phase) {
        e = hipLaunchKernel(fn, dim3((unsigned)B), dim3(64), args, lds, stream);
        return e != hipSuccess ? e : hipGetLastError();
    }
    // the resume workers: parked problems (the restoration phase) continued by k_resume_wide
    // fork: the resume workers on the aux stream alongside the batch kernel (the fork point is
    // before the batch kernel); join: the stream continues after both (no host
    // synchronisation).  Under graph capture the two branches need not run concurrently: the
    // workers then exit at once (take_parked) and the drain takes every parked problem.  No
    // worker, no fork (a captured fork whose branch held no work deadlocked the second replay of
    // the graph).
    const int64_t nw = nworkers > 0 ? nworkers : resume_workers(B);
    // (B = 1: a parked problem is the whole batch, the drain continues it as soon as a worker
    // would -- no fork, no worker spinning beside the solve)
    const bool can_fork = B > 1 && aux && aux != stream && ev_fork && ev_join;
    const unsigned workers = can_fork ? (unsigned)(pc < nw ? pc : nw) : 0u;
    const bool fork = workers > 0;
    if (forked_out) *forked_out = fork;
    if (fork) {
        e = origin ? hipSuccess : hipEventRecord(ev_fork, stream);
        if (e == hipSuccess) e = hipStreamWaitEvent(aux, ev_fork, 0);
        if (e != hipSuccess) return e;
    }
    e = hipLaunchKernel(fn, dim3((unsigned)B), dim3(64), args, lds, stream);
    if (e != hipSuccess) return e;
    if (fork) {
        e = hipLaunchKernel(rf, dim3(workers), dim3(64), args, rlds, aux);
        if (e != hipSuccess) return e;
    }
    // the drain, after the batch kernel: one worker per park entry, so the problems still
    // waiting when the batch ends run side by side (a worker finding nothing left exits at once)
    // -- the tail is the longest restoration, not their sum over a few workers
    e = hipLaunchKernel(rf, dim3((unsigned)pc), dim3(64), args, rlds, stream);
    if (e != hipSuccess) return e;
    if (fork && !origin) {
        e = hipEventRecord(ev_join, aux);
        if (e == hipSuccess) e = hipStreamWaitEvent(stream, ev_join, 0);
        if (e != hipSuccess) return e;
    }
    // the park-area overflow (only where it can occur: pc < B), after every worker that holds a
    // park entry: problems solved again from the start, one per park entry at a time
    if (pc < B) {
        WideArgs ao = a;
        ao.phase = 1;
        ao.ent0 = 0;
        void* oargs[] = {(void*)&ao};
        e = hipLaunchKernel(rf, dim3((unsigned)pc), dim3(64), oargs, rlds, stream);
        if (e != hipSuccess) return e;
    }
    return hipGetLastError();
}

// the fp64 phase's instance (k_warm_wide, default options) for the horizon class of P
static WideInst warm_kernel(const IpmParams& Pr) {
#ifdef MPCG_HEADLINE_ONLY
    (void)Pr;
    return WideInst{nullptr, ""};  // (not linked into the timing tool)
#else
    const bool split = Pr.N <= 32;
    const int nb = Pr.N > 64 ? 2 : 1;
    if (Pr.N > 128 || Pr.model != 0) return WideInst{nullptr, ""};
    if (nb == 2) return WideInst{warm_kernel_fn<0, false, double, 2, true, 1>(), "k_warm_wide<0,false,double,2,true,1>"};
    if (split) return WideInst{warm_kernel_fn<0, true, double, 1, true, 2>(), "k_warm_wide<0,true,double,1,true,2>"};
    if (wide_lds_bytes(Pr) > 32768)
        return WideInst{warm_kernel_fn<0, false, double, 1, true, 1>(), "k_warm_wide<0,false,double,1,true,1>"};
    return WideInst{warm_kernel_fn<0, false, double, 1, true, 2>(), "k_warm_wide<0,false,double,1,true,2>"};
#endif
}

hipError_t launch_wide_solve(const IpmParams& P, int64_t B, const double* state, const double* coeffs, double* u0,
                             double* traj, int32_t* status, double* obj, int32_t* iters, int32_t* diag,
                             const int32_t* order, void* spill, size_t spill_bytes, hipStream_t stream,
                             const WideStreams& ws, const char** kernel_name) {
    if (B <= 0) return hipSuccess;
    if (!spill) return hipErrorInvalidValue;
    if (wide_spill_bytes(P, B) > spill_bytes) return hipErrorInvalidValue;
    const WideInst inst = wide_kernel(P, B);
    if (!inst.fn) return hipErrorInvalidValue;
    if (kernel_name) *kernel_name = inst.name;
    if (!two_phase(P))
        return launch_phase(P, inst, B, state, coeffs, u0, traj, status, obj, iters, diag, order, spill, nullptr,
                            stream, ws.aux, ws.ev_fork, ws.ev_join);
    // the fp32 configuration: [the head on aux, in fp64 from the start] the fp32 phase (hand-over,
    // no outputs), then the fp64 phase, over the problems outside the head
    IpmParams Pr = fp64_params(P);
    const bool can_head = order && ws.aux && ws.aux != stream && ws.aux2 && ws.aux2 != ws.aux &&
                          ws.aux2 != stream && ws.ev_fork && ws.ev_join && ws.ev_join2;
    const int64_t K = can_head ? head_count(B) : 0;
    hipError_t e;
    bool head_workers = false;
    if (K > 0) {
        // (after the solve order: the head is order[0, K), on its own workspace; aux and the
        // head's resume workers on aux2 both fork from the caller's stream -- no fork of a forked
        // stream, which a captured graph does not survive -- and both join it after the fp32 phase)
        const IpmParams Ph = head_params(P, K);
        const WideInst hi = wide_kernel(Ph, B);  // (the fp64 solver's batch instance)
        if (!hi.fn) return hipErrorInvalidValue;
        e = launch_phase(Ph, hi, K, state, coeffs, u0, traj, status, obj, iters, diag, order,
                         (char*)spill + head_offset(P, B), nullptr, ws.aux, ws.aux2, ws.ev_fork, ws.ev_join2, -1,
                         &stream, &head_workers, B);
        if (e != hipSuccess) return e;
    }
    const int64_t Bm = B - K;
    const int32_t* om = order ? order + K : nullptr;
    float* handoff = (float*)((char*)spill + handoff_offset(P, B));
    e = launch_phase(P, inst, Bm, state, coeffs, u0, traj, status, obj, iters, diag, om, spill, handoff, stream,
                     ws.aux, ws.ev_fork, ws.ev_join, -1, nullptr, nullptr, B);
    if (e != hipSuccess) return e;
    if (K > 0) {  // (the head joins before the fp64 phase forks its own workers onto aux)
        if (head_workers) {
            e = hipEventRecord(ws.ev_join2, ws.aux2);
            if (e == hipSuccess) e = hipStreamWaitEvent(stream, ws.ev_join2, 0);
            if (e != hipSuccess) return e;
        }
        e = hipEventRecord(ws.ev_join, ws.aux);
        if (e == hipSuccess) e = hipStreamWaitEvent(stream, ws.ev_join, 0);
        if (e != hipSuccess) return e;
        if (diag) {  // (solved from the start by the fp64 solver: diag[:, 2] = 3, after the head's last write)
            hipLaunchKernelGGL(k_mark_rows, dim3((unsigned)((K + 255) / 256)), dim3(256), 0, stream, K, order, diag, 3, B);
            e = hipGetLastError();
            if (e != hipSuccess) return e;
        }
    }
    const WideInst wi = warm_kernel(Pr);
    int32_t* order2 = (int32_t*)((char*)spill + order2_offset(P, B));
    int32_t* cnt2 = order2 + ((B + 63) / 64) * 64;
    hipLaunchKernelGGL(k_reset_ws, dim3(1), dim3(256), 0, stream, cnt2, (int64_t)0, cnt2, nullptr, (int64_t)0,
                       nullptr, (int64_t)0);
    hipLaunchKernelGGL(k_cold_first, dim3((unsigned)((Bm + 255) / 256)), dim3(256), 0, stream, Bm,
                       (const float*)handoff, handoff_stride(P), om, order2, cnt2, B);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    // (the problems solved from the start come first and some of them enter the restoration
    // phase early in the launch: more concurrent resume workers than a batch of the fp64 solver
    // needs, so they are continued while the rest of the batch runs)
    return launch_phase(Pr, wi, Bm, state, coeffs, u0, traj, status, obj, iters, diag, order2, spill, handoff, stream,
                        ws.aux, ws.ev_fork, ws.ev_join, 8 + B / 2048, nullptr, nullptr, B);
}

}  // namespace mpcg
