// mpc_ros_amd/csrc/mpcg_internal.h -- declarations shared by the kernels and the C-ABI layer.
#ifndef MPCG_INTERNAL_H
#define MPCG_INTERNAL_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ipm_core.h"

namespace mpcg {

hipError_t launch_ipm_solve(const IpmParams& P, int64_t B, const double* state, const double* coeffs, double* u0,
                            double* traj, int32_t* status, double* obj, int32_t* iters, double* ws,
                            hipStream_t stream);

}  // namespace mpcg
#endif
