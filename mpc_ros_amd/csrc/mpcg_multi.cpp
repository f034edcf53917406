// mpc_ros_amd/csrc/mpcg_multi.cpp -- mpcg_solve_multi: one process, several GPUs, RCCL gather.
//
// the B problems are independent, so they are split into contiguous
// shards (the first B % G GPUs take one extra problem), each GPU solves its shard with
// its own handle and stream, and the per-problem results are gathered to the first GPU
// with one grouped RCCL send/recv per output array (rank r sends its shard, the root
// receives every shard at its offset: point-to-point over xGMI, the north star's "RCCL
// used only for the final gather"), then copied to the caller's host buffers.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <string>
#include <vector>

#include "mpcg.h"

namespace {
struct Shard {
    int dev = 0;
    mpcg_handle* h = nullptr;
    hipStream_t s = nullptr;
    int64_t start = 0, count = 0;
    double* in = nullptr;   // state [count][6] | coeffs [count][4]
    double* out = nullptr;  // root: gathered outputs of all B problems; others: their shard
    size_t out_bytes = 0;
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
}  // namespace

extern "C" int mpcg_solve_multi(int ngpu, const int* devices, const mpcg_params* params, int64_t B,
                                const double* state, const double* coeffs, double* u0, double* traj,
                                int32_t* status, double* obj, int32_t* iters) {
    if (ngpu < 1 || !devices || !params) return -1;
    if (B < 0) return -1;
    if (B == 0) return 0;
    if (!state || !coeffs || !u0) return -1;
    int rc = mpcg_params_check(params);
    if (rc) return rc;
    const int N = params->steps;
    std::vector<Shard> sh(ngpu);
    const int64_t base = B / ngpu, rem = B % ngpu;
    for (int r = 0; r < ngpu; ++r) {
        sh[r].dev = devices[r];
        sh[r].count = base + (r < rem ? 1 : 0);
        sh[r].start = r * base + (r < rem ? r : rem);
    }
    std::vector<ncclComm_t> comms(ngpu, nullptr);
    auto cleanup = [&]() {
        for (auto& s : sh) {
            if (s.h) mpcg_destroy(s.h);
            hipSetDevice(s.dev);
            if (s.in) hipFree(s.in);
            if (s.out) hipFree(s.out);
            if (s.s) hipStreamDestroy(s.s);
        }
        for (auto c : comms)
            if (c) ncclCommDestroy(c);
    };
    int result = 0;
    do {
        if (ncclCommInitAll(comms.data(), ngpu, devices) != ncclSuccess) { result = -4; break; }
        // shards: copy in, solve (each on its own GPU and stream, queued without waiting)
        for (int r = 0; r < ngpu && !result; ++r) {
            Shard& s = sh[r];
            if ((rc = mpcg_create(s.dev, &s.h)) != 0) { result = rc; break; }
            if ((rc = mpcg_set_params(s.h, params)) != 0) { result = rc; break; }
            hipSetDevice(s.dev);
            if (hipStreamCreateWithFlags(&s.s, hipStreamNonBlocking) != hipSuccess) { result = -2; break; }
            const OutLayout L{r == 0 ? B : s.count, N};
            s.out_bytes = L.total();
            if (hipMalloc((void**)&s.in, sizeof(double) * 10 * (s.count > 0 ? s.count : 1)) != hipSuccess ||
                hipMalloc((void**)&s.out, s.out_bytes) != hipSuccess) { result = -2; break; }
            if (s.count == 0) continue;
            double* din = s.in;
            hipMemcpyAsync(din, state + 6 * s.start, sizeof(double) * 6 * s.count, hipMemcpyHostToDevice, s.s);
            hipMemcpyAsync(din + 6 * s.count, coeffs + 4 * s.start, sizeof(double) * 4 * s.count,
                           hipMemcpyHostToDevice, s.s);
            // the root solves into its own slot of the gathered arrays
            const OutLayout G{B, N};
            char* o = (char*)s.out;
            const int64_t off = r == 0 ? s.start : 0;
            const OutLayout& Lr = r == 0 ? G : L;
            rc = mpcg_solve_device(s.h, s.count, din, din + 6 * s.count, (double*)(o + Lr.u0()) + 2 * off,
                                   (double*)(o + Lr.traj()) + (size_t)3 * N * off, (int32_t*)(o + Lr.status()) + off,
                                   (double*)(o + Lr.obj()) + off, (int32_t*)(o + Lr.iters()) + off, s.s);
            if (rc) { result = rc; break; }
        }
        if (result) break;
        // the gather: rank r > 0 sends each of its output arrays, the root receives them
        // at their offsets (grouped point-to-point: every shard moves once over xGMI)
        const OutLayout G{B, N};
        if (ncclGroupStart() != ncclSuccess) { result = -4; break; }
        for (int r = 1; r < ngpu; ++r) {
            const Shard& s = sh[r];
            if (s.count == 0) continue;
            const OutLayout L{s.count, N};
            char* src = (char*)s.out;
            char* dst = (char*)sh[0].out;
            struct { size_t so, go, per; } parts[5] = {
                {L.u0(), G.u0(), sizeof(double) * 2}, {L.traj(), G.traj(), sizeof(double) * 3 * N},
                {L.obj(), G.obj(), sizeof(double)}, {L.status(), G.status(), sizeof(int32_t)},
                {L.iters(), G.iters(), sizeof(int32_t)}};
            for (const auto& p : parts) {
                const size_t bytes = p.per * (size_t)s.count;
                ncclSend(src + p.so, bytes, ncclChar, 0, comms[r], s.s);
                ncclRecv(dst + p.go + p.per * (size_t)s.start, bytes, ncclChar, r, comms[0], sh[0].s);
            }
        }
        if (ncclGroupEnd() != ncclSuccess) { result = -4; break; }
        // results to the host from the root
        hipSetDevice(sh[0].dev);
        const char* o = (const char*)sh[0].out;
        hipStream_t s0 = sh[0].s;
        hipMemcpyAsync(u0, o + G.u0(), sizeof(double) * 2 * B, hipMemcpyDeviceToHost, s0);
        if (traj) hipMemcpyAsync(traj, o + G.traj(), sizeof(double) * 3 * N * B, hipMemcpyDeviceToHost, s0);
        if (obj) hipMemcpyAsync(obj, o + G.obj(), sizeof(double) * B, hipMemcpyDeviceToHost, s0);
        if (status) hipMemcpyAsync(status, o + G.status(), sizeof(int32_t) * B, hipMemcpyDeviceToHost, s0);
        if (iters) hipMemcpyAsync(iters, o + G.iters(), sizeof(int32_t) * B, hipMemcpyDeviceToHost, s0);
        for (auto& s : sh) {
            hipSetDevice(s.dev);
            if (hipStreamSynchronize(s.s) != hipSuccess) result = -2;
        }
    } while (false);
    cleanup();
    return result;
}
