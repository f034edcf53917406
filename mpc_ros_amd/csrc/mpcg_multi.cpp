// mpc_ros_amd/csrc/mpcg_multi.cpp -- one process, several GPUs, RCCL gather: the persistent
// context mpcg_multi (create once, solve many batches, destroy) and mpcg_solve_multi (the
// same for one batch).
//
// the B problems are independent, so they are split into contiguous
// shards (mpcg_shard_range: the first B % G GPUs take one extra problem), each GPU solves
// its shard with its own handle and stream, and the per-problem results are gathered to
// the first GPU with one grouped RCCL send/recv per output array (mpcg_multi_gather_plan:
// rank r sends its shard, the root receives every shard at its offset -- point-to-point
// over xGMI, the north star's "RCCL used only for the final gather"), then copied to the
// caller's host buffers.  The context holds the communicator, a handle, stream and device
// buffers per GPU, pinned host staging for the inputs of each shard and the root's outputs,
// and each handle's solver workspace reserved for the largest shard: a solve allocates
// nothing.  The shards' inputs are staged and their copies and solves queued by one host
// thread per GPU, so no GPU waits for another's host-to-device copy (a copy from the caller's
// pageable memory returns only once it has completed).  Every HIP and RCCL return is checked; a failure sets
// mpcg_last_error(); a failure inside the gather group aborts the communicators (an
// unmatched send must not be waited for) and marks the context broken.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "mpcg.h"
#include "mpcg_internal.h"

namespace {
struct Shard {
    int dev = 0;
    mpcg_handle* h = nullptr;
    hipStream_t s = nullptr;
    int64_t start = 0, count = 0;
    double* in = nullptr;   // state [count][6] | coeffs [count][4]
    char* out = nullptr;    // root: gathered outputs of all B problems; others: their shard
    double* hin = nullptr;  // pinned host staging of `in` (the largest shard)
    char* hout = nullptr;   // root only: pinned host staging of the gathered outputs
};

// output record layout of B problems: u0 [B][2] | traj [B][3N] | obj [B] | status [B] | iters [B]
struct OutLayout {
    int64_t B;
    int N;
    size_t u0() const { return 0; }
    size_t traj() const { return u0() + sizeof(double) * 2 * B; }
    size_t obj() const { return traj() + sizeof(double) * 3 * N * B; }
    size_t status() const { return obj() + sizeof(double) * B; }
    size_t iters() const { return status() + sizeof(int32_t) * B; }
    size_t total() const { return iters() + sizeof(int32_t) * B; }
};

int nccl_fail(ncclResult_t e, const char* what) {
    return mpcg::set_error(-4, std::string(what) + ": " + ncclGetErrorString(e));
}
int hip_fail(hipError_t e, const char* what) {
    return mpcg::set_error(-2, std::string(what) + ": " + hipGetErrorString(e));
}
}  // namespace

extern "C" {

int mpcg_shard_range(int64_t B, int ngpu, int r, int64_t* start, int64_t* count) {
    if (B < 0 || ngpu < 1 || r < 0 || r >= ngpu || !start || !count)
        return mpcg::set_error(-1, "mpcg_shard_range: B >= 0, 0 <= r < ngpu and non-null outputs");
    const int64_t base = B / ngpu, rem = B % ngpu;
    *count = base + (r < rem ? 1 : 0);
    *start = r * base + (r < rem ? r : rem);
    return 0;
}

int mpcg_multi_gather_plan(int64_t B, int32_t N, int ngpu, int r, mpcg_xfer* xfers) {
    if (N < 1 || !xfers) return mpcg::set_error(-1, "mpcg_multi_gather_plan: N >= 1 and non-null xfers");
    int64_t start = 0, count = 0;
    if (int rc = mpcg_shard_range(B, ngpu, r, &start, &count)) return rc;
    const OutLayout G{B, N}, L{r == 0 ? B : count, N};
    // rank 0 solves in place into its slot of the gathered arrays (src == dst, nothing moves)
    const int64_t so = r == 0 ? start : 0;
    const size_t src[MPCG_GATHER_ARRAYS] = {L.u0(), L.traj(), L.obj(), L.status(), L.iters()};
    const size_t dst[MPCG_GATHER_ARRAYS] = {G.u0(), G.traj(), G.obj(), G.status(), G.iters()};
    const size_t per[MPCG_GATHER_ARRAYS] = {sizeof(double) * 2, sizeof(double) * 3 * (size_t)N, sizeof(double),
                                            sizeof(int32_t), sizeof(int32_t)};
    for (int k = 0; k < MPCG_GATHER_ARRAYS; ++k) {
        xfers[k].src_offset = src[k] + per[k] * (size_t)so;
        xfers[k].dst_offset = dst[k] + per[k] * (size_t)start;
        xfers[k].bytes = per[k] * (size_t)count;
    }
    return 0;
}

size_t mpcg_multi_out_bytes(int64_t B, int32_t N) {
    return B < 0 || N < 1 ? 0 : OutLayout{B, N}.total();
}

// the context's device buffers on GPU r for batches of up to B_max: the inputs of its largest
// shard, and its outputs (the root: the gathered outputs of B_max problems); the solver
// workspace its handle reserves comes on top (mpcg_workspace_bytes of the largest shard)
size_t mpcg_multi_buffer_bytes(int64_t B_max, int32_t N, int ngpu, int r) {
    if (B_max < 0 || N < 1 || ngpu < 1 || r < 0 || r >= ngpu) return 0;
    int64_t start = 0, count = 0;
    mpcg_shard_range(B_max, ngpu, 0, &start, &count);  // (GPU 0's shard is a largest one)
    const size_t in = sizeof(double) * 10 * (size_t)(count > 0 ? count : 1);
    const size_t out = OutLayout{r == 0 ? B_max : count, N}.total();
    return in + (out > 0 ? out : 1);
}

}  // extern "C"

struct mpcg_multi {
    int ngpu = 0;
    int N = 0;
    int64_t B_max = 0;
    bool broken = false;  // a gather failed inside its group: the communicators were aborted
    std::vector<Shard> sh;
    std::vector<ncclComm_t> comms;
};

namespace {
// (drains every stream before it frees: a failure may leave work queued; aborted
// communicators first, so that no stream waits for an unmatched transfer)
void multi_free(mpcg_multi* m) {
    if (m->broken)
        for (auto& c : m->comms)
            if (c) {
                ncclCommAbort(c);
                c = nullptr;
            }
    for (auto& s : m->sh) {
        hipSetDevice(s.dev);
        if (s.s) hipStreamSynchronize(s.s);
        if (s.h) mpcg_destroy(s.h);
        if (s.in) hipFree(s.in);
        if (s.out) hipFree(s.out);
        if (s.hin) hipHostFree(s.hin);
        if (s.hout) hipHostFree(s.hout);
        if (s.s) hipStreamDestroy(s.s);
        s = Shard{};
    }
    for (auto c : m->comms)
        if (c) ncclCommDestroy(c);
    m->comms.clear();
}
}  // namespace

extern "C" {

int mpcg_multi_create(int ngpu, const int* devices, const mpcg_params* params, int64_t B_max, mpcg_multi** out) {
    if (!out) return mpcg::set_error(-1, "mpcg_multi_create: null out");
    *out = nullptr;
    if (ngpu < 1 || !devices || !params) return mpcg::set_error(-1, "mpcg_multi_create: ngpu >= 1, devices, params");
    if (B_max < 1) return mpcg::set_error(-1, "mpcg_multi_create: B_max >= 1");
    int rc = mpcg_params_check(params);
    if (rc) return rc;
    int ndev = 0;
    hipError_t he = hipGetDeviceCount(&ndev);
    if (he != hipSuccess) return hip_fail(he, "hipGetDeviceCount");
    for (int r = 0; r < ngpu; ++r) {
        if (devices[r] < 0 || devices[r] >= ndev) return mpcg::set_error(-3, "mpcg_multi_create: device out of range");
        for (int q = 0; q < r; ++q)
            if (devices[q] == devices[r]) return mpcg::set_error(-1, "mpcg_multi_create: devices repeat");
    }
    mpcg_multi* m = new mpcg_multi();
    m->ngpu = ngpu;
    m->N = params->steps;
    m->B_max = B_max;
    m->sh.resize(ngpu);
    m->comms.assign(ngpu, nullptr);
    int64_t start = 0, cmax = 0;
    mpcg_shard_range(B_max, ngpu, 0, &start, &cmax);
    int result = 0;
    do {
        ncclResult_t ne = ncclCommInitAll(m->comms.data(), ngpu, devices);
        if (ne != ncclSuccess) { result = nccl_fail(ne, "ncclCommInitAll"); break; }
        for (int r = 0; r < ngpu && !result; ++r) {
            Shard& s = m->sh[r];
            s.dev = devices[r];
            if ((rc = mpcg_create(s.dev, &s.h)) != 0) { result = rc; break; }
            if ((rc = mpcg_set_params(s.h, params)) != 0) { result = rc; break; }
            if ((rc = mpcg_reserve(s.h, cmax)) != 0) { result = rc; break; }
            if ((he = hipSetDevice(s.dev)) != hipSuccess) { result = hip_fail(he, "hipSetDevice"); break; }
            if ((he = hipStreamCreateWithFlags(&s.s, hipStreamNonBlocking)) != hipSuccess) {
                result = hip_fail(he, "hipStreamCreateWithFlags");
                break;
            }
            const size_t in_bytes = sizeof(double) * 10 * (size_t)(cmax > 0 ? cmax : 1);
            const size_t out_bytes = mpcg_multi_buffer_bytes(B_max, m->N, ngpu, r) - in_bytes;
            if ((he = hipMalloc((void**)&s.in, in_bytes)) != hipSuccess ||
                (he = hipMalloc((void**)&s.out, out_bytes)) != hipSuccess) {
                result = hip_fail(he, "hipMalloc");
                break;
            }
            if ((he = hipHostMalloc((void**)&s.hin, in_bytes, hipHostMallocDefault)) != hipSuccess ||
                (r == 0 && (he = hipHostMalloc((void**)&s.hout, out_bytes, hipHostMallocDefault)) != hipSuccess)) {
                result = hip_fail(he, "hipHostMalloc");
                break;
            }
        }
    } while (false);
    if (result) {
        multi_free(m);
        delete m;
        return result;
    }
    *out = m;
    return 0;
}

void mpcg_multi_destroy(mpcg_multi* m) {
    if (!m) return;
    multi_free(m);
    delete m;
}

int mpcg_multi_solve(mpcg_multi* m, int64_t B, const double* state, const double* coeffs, double* u0, double* traj,
                     int32_t* status, double* obj, int32_t* iters) {
    if (!m) return mpcg::set_error(-1, "mpcg_multi_solve: null context");
    if (m->broken) return mpcg::set_error(-4, "mpcg_multi_solve: the context's communicators were aborted");
    if (B < 0 || B > m->B_max) return mpcg::set_error(-1, "mpcg_multi_solve: 0 <= B <= the context's B_max");
    if (B == 0) return 0;
    if (!state || !coeffs || !u0) return mpcg::set_error(-1, "mpcg_multi_solve: null state / coeffs / u0");
    const int ngpu = m->ngpu, N = m->N;
    std::vector<Shard>& sh = m->sh;
    for (int r = 0; r < ngpu; ++r) mpcg_shard_range(B, ngpu, r, &sh[r].start, &sh[r].count);
    hipError_t he;
    int rc;
    // shards: stage the inputs in pinned memory, copy in, solve -- one host thread per GPU, so
    // each GPU's copy and solve are queued without waiting for another GPU's copy
    auto enqueue = [&](int r) -> int {
        Shard& s = sh[r];
        if (s.count == 0) return 0;
        hipError_t e;
        if ((e = hipSetDevice(s.dev)) != hipSuccess) return hip_fail(e, "hipSetDevice");
        std::memcpy(s.hin, state + 6 * s.start, sizeof(double) * 6 * s.count);
        std::memcpy(s.hin + 6 * s.count, coeffs + 4 * s.start, sizeof(double) * 4 * s.count);
        double* din = s.in;
        if ((e = hipMemcpyAsync(din, s.hin, sizeof(double) * 10 * s.count, hipMemcpyHostToDevice, s.s)) != hipSuccess)
            return hip_fail(e, "hipMemcpyAsync (inputs)");
        // the root solves into its own slot of the gathered arrays (the plan's src offsets)
        mpcg_xfer x[MPCG_GATHER_ARRAYS];
        int c;
        if ((c = mpcg_multi_gather_plan(B, N, ngpu, r, x)) != 0) return c;
        char* o = s.out;
        return mpcg_solve_device(s.h, s.count, din, din + 6 * s.count, (double*)(o + x[0].src_offset),
                                 (double*)(o + x[1].src_offset), (int32_t*)(o + x[3].src_offset),
                                 (double*)(o + x[2].src_offset), (int32_t*)(o + x[4].src_offset), s.s);
    };
    std::vector<int> rcs(ngpu, 0);
    std::vector<std::string> errs(ngpu);
    if (ngpu == 1) {
        rcs[0] = enqueue(0);
    } else {
        // (mpcg_last_error() is per thread: a worker's message is carried back)
        std::vector<std::thread> th;
        for (int r = 0; r < ngpu; ++r)
            th.emplace_back([&, r] {
                rcs[r] = enqueue(r);
                if (rcs[r]) errs[r] = mpcg_last_error();
            });
        for (auto& t : th) t.join();
    }
    for (int r = 0; r < ngpu; ++r)
        if (rcs[r]) return ngpu == 1 ? rcs[r] : mpcg::set_error(rcs[r], errs[r]);
    // the gather: rank r > 0 sends each of its output arrays, the root receives them at their
    // offsets (grouped point-to-point: every shard moves once over xGMI).  The plan is checked
    // before the group opens; a failing call inside it closes the group (not launched: it has a
    // recorded error) and then aborts the communicators, so no unmatched send is waited for.
    std::vector<mpcg_xfer> plan((size_t)ngpu * MPCG_GATHER_ARRAYS);
    for (int r = 1; r < ngpu; ++r)
        if ((rc = mpcg_multi_gather_plan(B, N, ngpu, r, &plan[(size_t)r * MPCG_GATHER_ARRAYS])) != 0) return rc;
    ncclResult_t ne = ncclGroupStart();
    if (ne != ncclSuccess) return nccl_fail(ne, "ncclGroupStart");
    int grc = 0;
    for (int r = 1; r < ngpu && !grc; ++r) {
        const Shard& s = sh[r];
        if (s.count == 0) continue;
        for (int k = 0; k < MPCG_GATHER_ARRAYS && !grc; ++k) {
            const mpcg_xfer& p = plan[(size_t)r * MPCG_GATHER_ARRAYS + k];
            if ((ne = ncclSend(s.out + p.src_offset, p.bytes, ncclChar, 0, m->comms[r], s.s)) != ncclSuccess)
                grc = nccl_fail(ne, "ncclSend");
            else if ((ne = ncclRecv(sh[0].out + p.dst_offset, p.bytes, ncclChar, r, m->comms[0], sh[0].s)) != ncclSuccess)
                grc = nccl_fail(ne, "ncclRecv");
        }
    }
    if (grc) {
        // close the group first (it still holds the communicators; a group with a recorded
        // error is not launched), then abort them
        m->broken = true;
        ncclGroupEnd();
        for (auto& c : m->comms) ncclCommAbort(c), c = nullptr;
        return grc;
    }
    if ((ne = ncclGroupEnd()) != ncclSuccess) {
        m->broken = true;
        for (auto& c : m->comms) ncclCommAbort(c), c = nullptr;
        return nccl_fail(ne, "ncclGroupEnd");
    }
    // results to the host from the root, through its pinned staging
    if ((he = hipSetDevice(sh[0].dev)) != hipSuccess) return hip_fail(he, "hipSetDevice");
    const OutLayout G{B, N};
    const char* o = sh[0].out;
    hipStream_t s0 = sh[0].s;
    struct { void* host; size_t off, bytes; } back[MPCG_GATHER_ARRAYS] = {
        {u0, G.u0(), sizeof(double) * 2 * B}, {traj, G.traj(), sizeof(double) * 3 * N * B},
        {obj, G.obj(), sizeof(double) * B}, {status, G.status(), sizeof(int32_t) * B},
        {iters, G.iters(), sizeof(int32_t) * B}};
    for (const auto& b : back) {
        if (!b.host) continue;
        if ((he = hipMemcpyAsync(sh[0].hout + b.off, o + b.off, b.bytes, hipMemcpyDeviceToHost, s0)) != hipSuccess)
            return hip_fail(he, "hipMemcpyAsync (results)");
    }
    for (auto& s : sh)
        if ((he = hipSetDevice(s.dev)) != hipSuccess || (he = hipStreamSynchronize(s.s)) != hipSuccess)
            return hip_fail(he, "hipStreamSynchronize");
    for (const auto& b : back)
        if (b.host) std::memcpy(b.host, sh[0].hout + b.off, b.bytes);
    return 0;
}

int mpcg_solve_multi(int ngpu, const int* devices, const mpcg_params* params, int64_t B, const double* state,
                     const double* coeffs, double* u0, double* traj, int32_t* status, double* obj, int32_t* iters) {
    if (ngpu < 1 || !devices || !params) return mpcg::set_error(-1, "mpcg_solve_multi: ngpu >= 1, devices, params");
    if (B < 0) return mpcg::set_error(-1, "mpcg_solve_multi: B < 0");
    if (B == 0) return 0;
    if (!state || !coeffs || !u0) return mpcg::set_error(-1, "mpcg_solve_multi: null state / coeffs / u0");
    mpcg_multi* m = nullptr;
    int rc = mpcg_multi_create(ngpu, devices, params, B, &m);
    if (rc) return rc;
    rc = mpcg_multi_solve(m, B, state, coeffs, u0, traj, status, obj, iters);
    mpcg_multi_destroy(m);
    return rc;
}

}  // extern "C"
