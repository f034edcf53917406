// mpc_ros_amd/csrc/mpcg_internal.h -- declarations shared by the kernels and the C-ABI layer.
#ifndef MPCG_INTERNAL_H
#define MPCG_INTERNAL_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "ipm_core.h"

namespace mpcg {

// mpcg_last_error()'s message for this thread; returns code
int set_error(int code, const std::string& msg);

// One problem per wavefront (mpcg_wide.hip): LDS bytes per problem, launch.
size_t wide_lds_bytes(const IpmParams& P);
// HBM workspace of a batch of B (watchdog, acceptable point, second-order corrections,
// soft restoration, the restoration phase: rare paths that must not cost LDS): one slot
// per wavefront the device holds resident (wide_slots), claimed by each problem's wavefront
size_t wide_spill_bytes(const IpmParams& P, int64_t B);
int64_t wide_slots(const IpmParams& P, int64_t B);
// batches beyond the resident wavefronts are solved in expected-longest-first order
constexpr int64_t kOrderMinBatch = 2048;
// The streams and events a solve forks work onto (each joined back into the caller's stream
// before the launch returns): aux -- the resume workers of the restoration phase, and the fp32
// configuration's head (the problems the solve order ranks longest, solved in fp64 while the
// fp32 phase runs); aux2 -- the head's own resume workers.
struct WideStreams {
    hipStream_t aux = nullptr, aux2 = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr, ev_join2 = nullptr;
};
hipError_t launch_wide_solve(const IpmParams& P, int64_t B, const double* state, const double* coeffs, double* u0,
                             double* traj, int32_t* status, double* obj, int32_t* iters, int32_t* diag,
                             const int32_t* order, void* spill, size_t spill_bytes, hipStream_t stream,
                             const WideStreams& ws = WideStreams(), const char** kernel_name = nullptr);
// park-area capacity of a batch of B (problems that enter the restoration phase)
int64_t wide_park_cap(const IpmParams& P, int64_t B);
// Solve order (expected-longest first): device buffer bytes for B problems, and the
// launch that writes the workgroup -> problem map into `buf` (returned in *order).
size_t wide_sched_bytes(int64_t B);
hipError_t launch_wide_order(int64_t B, const double* coeffs, void* buf, size_t bytes, int32_t** order,
                             hipStream_t stream);

// findBestPath preprocessing and post-processing (mpcg_track.hip).
// (M > 64: ws holds find_best_path_ws_bytes(B, M) bytes of device scratch)
size_t find_best_path_ws_bytes(int64_t B, int M);
hipError_t launch_find_best_path(int64_t B, int M, double dt, int delay_mode, const double* pose, const double* vel,
                                 const double* plan, double* state, double* coeffs, double* ws, hipStream_t stream);
hipError_t launch_post(int64_t B, double dt, double ref_v, const double* vel, const double* u0, double* cmd,
                       hipStream_t stream);

// The benchmark's synthetic robots (mpcg_synth.hip): the lemniscate's arc-length table (host,
// once) and the per-robot pose / velocities / plan from (seed, global index)
void synth_arc_table(std::vector<double>& t, std::vector<double>& s);
int synth_arc_len();
hipError_t launch_synth_infinity(uint64_t seed, int64_t start, int64_t B, int M, const double* arc_t,
                                 const double* arc_s, double* pose, double* vel, double* plan, hipStream_t stream);

}  // namespace mpcg
#endif
