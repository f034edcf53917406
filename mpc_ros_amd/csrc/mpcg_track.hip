// mpc_ros_amd/csrc/mpcg_track.hip -- the caller side of MPC::Solve on the device.
//
// Tracking::findBestPath (mpc_ros/src/driving_state.cpp:175-271) for B robots, one
// robot per lane:
//   waypoints to the vehicle frame (:196-207), cubic polyfit by Householder QR
//   (:210, polyfit :283-300), cte = polyeval(c, 0) (:211), path heading from the
//   first int(0.3 M) waypoint increments (:214-235), delay-mode state prediction
//   (:242-256);
// and the post-processing of the solve (:262-269): w = w0, throttle = a0,
// speed = min(v_fb + throttle dt, REF_V).
//
// The QR runs on MAXM-row arrays (the M waypoint rows followed by zero rows, which
// change no norm or inner product), unrolled so they stay in registers for M <= 16;
// a second instance with MAXM = 64 covers longer plans, and plans beyond 64 waypoints
// (findBestPath takes any length) run the same QR with the matrix in an HBM workspace
// (k_find_best_path_long).  Same operation order as oracle/preprocess.c.
#include <hip/hip_runtime.h>

#include <math.h>

#include "mpcg_internal.h"

namespace mpcg {

template <int MAXM>
__device__ __forceinline__ void polyfit3(int M, const double* xs, const double* ys, double* c) {
    constexpr int n = 4;
    double A[MAXM][n], b[MAXM];
#pragma unroll
    for (int i = 0; i < MAXM; ++i) {
        const bool in = i < M;
        A[i][0] = in ? 1.0 : 0.0;
#pragma unroll
        for (int j = 0; j < n - 1; ++j) A[i][j + 1] = A[i][j] * (in ? xs[i] : 0.0);
        b[i] = in ? ys[i] : 0.0;
    }
#pragma unroll
    for (int k = 0; k < n; ++k) {
        double nrm = 0.0;
#pragma unroll
        for (int i = k; i < MAXM; ++i) nrm += A[i][k] * A[i][k];
        nrm = sqrt(nrm);
        const double alpha = (A[k][k] > 0) ? -nrm : nrm;
        double vv[MAXM];
#pragma unroll
        for (int i = k; i < MAXM; ++i) vv[i] = (i == k) ? A[k][k] - alpha : A[i][k];
        double vnorm2 = 0.0;
#pragma unroll
        for (int i = k; i < MAXM; ++i) vnorm2 += vv[i] * vv[i];
        const bool skip = (nrm == 0.0) || (vnorm2 == 0.0);
#pragma unroll
        for (int j = k; j < n; ++j) {
            double s = 0.0;
#pragma unroll
            for (int i = k; i < MAXM; ++i) s += vv[i] * A[i][j];
            s = 2.0 * s / vnorm2;
#pragma unroll
            for (int i = k; i < MAXM; ++i) A[i][j] = skip ? A[i][j] : A[i][j] - s * vv[i];
        }
        double s = 0.0;
#pragma unroll
        for (int i = k; i < MAXM; ++i) s += vv[i] * b[i];
        s = 2.0 * s / vnorm2;
#pragma unroll
        for (int i = k; i < MAXM; ++i) b[i] = skip ? b[i] : b[i] - s * vv[i];
    }
#pragma unroll
    for (int k = n - 1; k >= 0; --k) {
        double s = b[k];
#pragma unroll
        for (int j = k + 1; j < n; ++j) s -= A[k][j] * c[j];
        c[k] = s / A[k][k];
    }
}

struct TrackArgs {
    int64_t B;
    int M;
    double dt;
    int delay_mode;
    const double* pose;   // [B][3] x, y, yaw
    const double* vel;    // [B][3] v feedback, previous w, previous throttle
    const double* plan;   // [B][M][2]
    double* state;        // [B][6]
    double* coeffs;       // [B][4]
};

__device__ __forceinline__ void finish_state(const TrackArgs& a, int64_t p, double theta, double v, double w,
                                             double throttle, const double* c);

template <int MAXM>
__global__ void __launch_bounds__(64) k_find_best_path(TrackArgs a) {
    const int64_t p = (int64_t)blockIdx.x * 64 + threadIdx.x;
    if (p >= a.B) return;
    const int M = a.M;
    const double px = a.pose[p * 3 + 0], py = a.pose[p * 3 + 1], theta = a.pose[p * 3 + 2];
    const double v = a.vel[p * 3 + 0], w = a.vel[p * 3 + 1], throttle = a.vel[p * 3 + 2];
    const double dt = a.dt;
    const double* pl = a.plan + p * (int64_t)M * 2;
    const double ct = cos(theta), st = sin(theta);
    double xv[MAXM], yv[MAXM];
#pragma unroll
    for (int i = 0; i < MAXM; ++i) {
        double dx = 0, dy = 0;
        if (i < M) {
            dx = pl[2 * i] - px;
            dy = pl[2 * i + 1] - py;
        }
        xv[i] = dx * ct + dy * st;
        yv[i] = dy * ct - dx * st;
    }
    double c[4];
    polyfit3<MAXM>(M, xv, yv, c);
    finish_state(a, p, theta, v, w, throttle, c);
}

// Plans of more than 64 waypoints: polyfit3's Householder QR, same operations in the same
// order, on the M x 4 matrix, the right-hand side and the reflector held in HBM
// (element (i, j) of robot p at ws[(6 i + j) B + p]: a wavefront's lanes touch 64
// consecutive doubles); zero rows past M change nothing, so the loops stop at M.
__global__ void __launch_bounds__(64) k_find_best_path_long(TrackArgs a, double* ws) {
    const int64_t p = (int64_t)blockIdx.x * 64 + threadIdx.x;
    if (p >= a.B) return;
    const int M = a.M;
    const int64_t B = a.B;
    double* e = ws + p;
#define E(i, j) e[((int64_t)(i) * 6 + (j)) * B]
    const double px = a.pose[p * 3 + 0], py = a.pose[p * 3 + 1], theta = a.pose[p * 3 + 2];
    const double v = a.vel[p * 3 + 0], w = a.vel[p * 3 + 1], throttle = a.vel[p * 3 + 2];
    const double* pl = a.plan + p * (int64_t)M * 2;
    const double ct = cos(theta), st = sin(theta);
    for (int i = 0; i < M; ++i) {
        const double dx = pl[2 * i] - px, dy = pl[2 * i + 1] - py;
        const double xv = dx * ct + dy * st;
        E(i, 0) = 1.0;
        double q = 1.0;
        for (int j = 0; j < 3; ++j) {
            q = q * xv;
            E(i, j + 1) = q;
        }
        E(i, 4) = dy * ct - dx * st;
    }
    for (int k = 0; k < 4; ++k) {
        double nrm = 0.0;
        for (int i = k; i < M; ++i) nrm += E(i, k) * E(i, k);
        nrm = sqrt(nrm);
        const double akk = E(k, k);
        const double alpha = (akk > 0) ? -nrm : nrm;
        double vnorm2 = 0.0;
        for (int i = k; i < M; ++i) {
            const double vi = (i == k) ? akk - alpha : E(i, k);
            E(i, 5) = vi;
            vnorm2 += vi * vi;
        }
        if (nrm == 0.0 || vnorm2 == 0.0) continue;
        for (int j = k; j < 5; ++j) {  // columns k..3, then the right-hand side
            double s = 0.0;
            for (int i = k; i < M; ++i) s += E(i, 5) * E(i, j);
            s = 2.0 * s / vnorm2;
            for (int i = k; i < M; ++i) E(i, j) = E(i, j) - s * E(i, 5);
        }
    }
    double c[4];
    for (int k = 3; k >= 0; --k) {
        double s = E(k, 4);
        for (int j = k + 1; j < 4; ++j) s -= E(k, j) * c[j];
        c[k] = s / E(k, k);
    }
#undef E
    finish_state(a, p, theta, v, w, throttle, c);
}

// cte, the path heading and the (delayed) state from the fitted polynomial
// (driving_state.cpp:211-256)
__device__ __forceinline__ void finish_state(const TrackArgs& a, int64_t p, double theta, double v, double w,
                                             double throttle, const double* c) {
    const int M = a.M;
    const double dt = a.dt;
    const double* pl = a.plan + p * (int64_t)M * 2;
    // polyeval(coeffs, 0.0) with pow(0, k) (driving_state.cpp:302-309): pow(0, 0) = 1
    const double cte = c[0];
    double gx = 0.0, gy = 0.0;
    const int nsample = (int)(M * 0.3);
    for (int i = 1; i < nsample; ++i) {
        gx += pl[2 * i] - pl[2 * (i - 1)];
        gy += pl[2 * i + 1] - pl[2 * (i - 1) + 1];
    }
    double temp_theta = theta;
    const double traj_deg = atan2(gy, gx);
    const double PI = M_PI;
    if (temp_theta <= -PI + traj_deg) temp_theta = temp_theta + 2 * PI;
    double etheta;
    if (gx != 0.0 && gy != 0.0 && temp_theta - traj_deg < 1.8 * PI)
        etheta = temp_theta - traj_deg;
    else
        etheta = 0;
    double* s = a.state + p * 6;
    if (a.delay_mode) {
        const double theta_act = w * dt;
        s[0] = v * dt;
        s[1] = 0;
        s[2] = theta_act;
        s[3] = v + throttle * dt;
        s[4] = cte + v * sin(etheta) * dt;
        s[5] = etheta - theta_act;
    } else {
        s[0] = 0;
        s[1] = 0;
        s[2] = 0;
        s[3] = v;
        s[4] = cte;
        s[5] = etheta;
    }
    double* co = a.coeffs + p * 4;
    co[0] = c[0];
    co[1] = c[1];
    co[2] = c[2];
    co[3] = c[3];
}

// driving_state.cpp:262-269 -> cmd[B][3] = (speed, w, throttle)
__global__ void __launch_bounds__(64) k_post(int64_t B, double dt, double ref_v, const double* vel, const double* u0,
                                            double* cmd) {
    const int64_t p = (int64_t)blockIdx.x * 64 + threadIdx.x;
    if (p >= B) return;
    const double w = u0[p * 2 + 0], thr = u0[p * 2 + 1];
    double speed = vel[p * 3 + 0] + thr * dt;
    if (speed >= ref_v) speed = ref_v;
    cmd[p * 3 + 0] = speed;
    cmd[p * 3 + 1] = w;
    cmd[p * 3 + 2] = thr;
}

hipError_t launch_find_best_path(int64_t B, int M, double dt, int delay_mode, const double* pose, const double* vel,
                                 const double* plan, double* state, double* coeffs, double* ws, hipStream_t stream) {
    if (B <= 0) return hipSuccess;
    const TrackArgs a{B, M, dt, delay_mode, pose, vel, plan, state, coeffs};
    const dim3 grid((unsigned)((B + 63) / 64)), block(64);
    if (M <= 16)
        hipLaunchKernelGGL(k_find_best_path<16>, grid, block, 0, stream, a);
    else if (M <= 64)
        hipLaunchKernelGGL(k_find_best_path<64>, grid, block, 0, stream, a);
    else if (!ws)
        return hipErrorInvalidValue;
    else
        hipLaunchKernelGGL(k_find_best_path_long, grid, block, 0, stream, a, ws);
    return hipGetLastError();
}

size_t find_best_path_ws_bytes(int64_t B, int M) { return M > 64 ? sizeof(double) * 6 * (size_t)M * (size_t)B : 0; }

hipError_t launch_post(int64_t B, double dt, double ref_v, const double* vel, const double* u0, double* cmd,
                       hipStream_t stream) {
    if (B <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_post, dim3((unsigned)((B + 63) / 64)), dim3(64), 0, stream, B, dt, ref_v, vel, u0, cmd);
    return hipGetLastError();
}

}  // namespace mpcg
