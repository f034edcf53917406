// mpc_ros_amd/csrc/mpcg_synth.hip -- the benchmark's synthetic robots, generated on the device.
//
// every problem of the "infinity set" (mpc_ros_amd/infinity.py) is a pure
// function of (seed, global index): six counter-based uniforms (splitmix64 of the index, the
// seed and the draw number) give the scenario -- the position along a lemniscate of Gerono
// (A = 3 m), a lateral offset, a heading error, the speed and the previous controls -- and the
// reference plan is M waypoints 0.5 m apart along the course from the robot's arc length.  A
// rank of the multi-GPU benchmark generates exactly its own slice on its GPU; the robots then
// go through the device preprocessing (findBestPath, mpcg_track.hip) to become MPC::Solve's
// (state, coeffs).  Same formulas and operation order as infinity.py (the integer hash
// bitwise; the trigonometry is the device's, within an ulp of the host's libm).  Not part of
// the reference's interface: a data generator for benchmarks and tests.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>

#include <vector>

#include "mpcg_internal.h"

namespace mpcg {

namespace {
constexpr double kA = 3.0;          // LEMNISCATE_A
constexpr double kPathLength = 5.0;  // path_length, MPCPlanner.cfg:19
constexpr int kArcN = 200001;        // arc-length table over t in [0, 4 pi)

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
    z = z + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
// U[0,1) draw k of problem idx (infinity.uniforms)
__device__ __forceinline__ double uniform(uint64_t idx, int k, uint64_t seed) {
    uint64_t z = idx * 0xD1B54A32D192ED03ull;
    z = z ^ (seed * 0x9E3779B97F4A7C15ull) ^ ((uint64_t)(k + 1) * 0xA24BAED4963EE407ull);
    z = splitmix64(splitmix64(z));
    return (double)(z >> 11) * (1.0 / 9007199254740992.0);
}
// numpy.interp(x, xp, fp) on an increasing table
__device__ __forceinline__ double interp(double x, const double* xp, const double* fp, int n) {
    if (!(x > xp[0])) return fp[0];
    if (!(x < xp[n - 1])) return fp[n - 1];
    int lo = 0, hi = n - 1;  // xp[lo] <= x < xp[hi]
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (xp[mid] <= x)
            lo = mid;
        else
            hi = mid;
    }
    if (x == xp[lo]) return fp[lo];
    const double slope = (fp[lo + 1] - fp[lo]) / (xp[lo + 1] - xp[lo]);
    return slope * (x - xp[lo]) + fp[lo];
}
}  // namespace

// one robot per thread: pose [B][3], vel [B][3] (v, previous w, previous throttle), plan [B][M][2]
__global__ void __launch_bounds__(256) k_synth_infinity(uint64_t seed, int64_t start, int64_t B, int M,
                                                        const double* arc_t, const double* arc_s, double* pose,
                                                        double* vel, double* plan) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= B) return;
    const uint64_t g = (uint64_t)(start + i);
    const double t = 2.0 * M_PI * uniform(g, 0, seed);
    const double lateral = -0.45 + 0.75 * uniform(g, 1, seed);
    const double heading_err = -0.85 + 1.95 * uniform(g, 2, seed);
    const double v = 0.8 * uniform(g, 3, seed);
    const double w_prev = -1.0 + 2.0 * uniform(g, 4, seed);
    const double a_prev = -1.0 + 2.0 * uniform(g, 5, seed);
    // scenario_poses
    const double st = sin(t);
    double px = kA * st, py = kA * st * cos(t);
    const double hd = atan2(kA * cos(2.0 * t), kA * cos(t));
    px = px - sin(hd) * lateral;
    py = py + cos(hd) * lateral;
    double yaw = hd + heading_err;
    yaw = atan2(sin(yaw), cos(yaw));
    const double s0 = interp(t, arc_t, arc_s, kArcN);
    const double ds = kPathLength / (double)(M - 1);
    for (int j = 0; j < M; ++j) {
        const double tj = interp(s0 + ds * (double)j, arc_s, arc_t, kArcN);
        const double sj = sin(tj);
        plan[(i * M + j) * 2 + 0] = kA * sj;
        plan[(i * M + j) * 2 + 1] = kA * sj * cos(tj);
    }
    pose[i * 3 + 0] = px;
    pose[i * 3 + 1] = py;
    pose[i * 3 + 2] = yaw;
    vel[i * 3 + 0] = v;
    vel[i * 3 + 1] = w_prev;
    vel[i * 3 + 2] = a_prev;
}

// The arc-length table of the lemniscate (infinity._Arc): t = linspace(0, 4 pi, n), speed
// |p'(t)| = hypot(A cos t, A cos 2t), s = cumulative trapezoid -- built on the host once, in
// numpy's operation order
void synth_arc_table(std::vector<double>& t, std::vector<double>& s) {
    t.resize(kArcN);
    s.resize(kArcN);
    const double stop = 4.0 * M_PI, step = stop / (double)(kArcN - 1);
    for (int i = 0; i < kArcN; ++i) t[i] = (double)i * step;
    t[kArcN - 1] = stop;
    std::vector<double> sp(kArcN);
    for (int i = 0; i < kArcN; ++i) sp[i] = hypot(kA * cos(t[i]), kA * cos(2.0 * t[i]));
    s[0] = 0.0;
    double acc = 0.0;
    for (int i = 1; i < kArcN; ++i) {
        acc += 0.5 * (sp[i] + sp[i - 1]) * (t[i] - t[i - 1]);
        s[i] = acc;
    }
}
int synth_arc_len() { return kArcN; }

hipError_t launch_synth_infinity(uint64_t seed, int64_t start, int64_t B, int M, const double* arc_t,
                                 const double* arc_s, double* pose, double* vel, double* plan, hipStream_t stream) {
    if (B <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_synth_infinity, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, stream, seed, start, B, M,
                       arc_t, arc_s, pose, vel, plan);
    return hipGetLastError();
}

}  // namespace mpcg
