/*
 * include/mpcg.h -- C-ABI of the MI355X batched NMPC solver (libmpcg.so).
 *
 * Drop-in boundary for the hot path of OkDoky/mpc_ros: the call
 *     vector<double> MPC::Solve(Eigen::VectorXd state, Eigen::VectorXd coeffs)
 * (mpc_ros/include/mpc_planner.h:31, mpc_ros/src/mpc_planner.cpp:265-402), which
 * tapes FG_eval with CppAD and solves the NLP with Ipopt 3.12.8 through
 * CppAD::ipopt::solve (mpc_ros/include/cppad/ipopt/solve.hpp:419-589).  Here a
 * batch of B independent problems is solved on one GPU by hand-written CDNA4 HIP
 * kernels running the same interior-point algorithm (mpc_ros_amd/csrc/ipm_core.h).
 *
 * Plain C types only; every pointer is caller-owned.  Return codes: 0 = ok,
 * negative = API / HIP error (message in mpcg_last_error()).  Per-problem solver
 * outcomes are reported in `status` with CppAD::ipopt::solve_result::status_type
 * numbering (mpc_ros/include/cppad/ipopt/solve_result.hpp:30-46): 1 success,
 * 2 maxiter_exceeded, 3 stop_at_tiny_step, 4 stop_at_acceptable_point,
 * 5 local_infeasibility and 7 feasible_point_found (the feasibility-restoration phase
 * converged without returning to the problem), 9 restoration_failure (the restoration
 * phase's line search failed), 10 error_in_step_computation, 11 invalid_number_detected,
 * 14 unknown (Ipopt's CPUTIME_EXCEEDED, solve_callback.hpp:1165-1167: the max_cpu_time
 * budget below).  As in the reference (mpc_planner.cpp:378, the status is computed and
 * then ignored), the last iterate is always returned.
 *
 * Device-side checks: every index a kernel reads from device memory (the solve order, the
 * workspace's slot and park-area counters and lists, a parked entry's problem tag) is
 * range-checked before use.  A value out of range -- a workspace corrupted or reused by
 * concurrent work outside stream order -- stops the kernel with a trap (the resume and
 * bookkeeping kernels print the value and its bound first); the stream then reports a HIP
 * error (a later call returns -2) and, as after any device fault, the process's HIP context
 * is unusable.
 *
 * Threading: one handle per thread; mpcg_set_params must not run concurrently with
 * a solve on the same handle (the reference has an unsynchronised writer here,
 * SURVEY.md §3.3 -- this API makes the ordering the caller's explicit job).  A handle's
 * device scratch (solve order, spill areas, staging) is used stream-ordered: a solve on a
 * different stream than the handle's previous one first waits for that previous work
 * (an event), so one thread may queue solves on several streams.
 *
 * Integration (cgo/ctypes/C++ stubs): INTEGRATION.md.
 */
#ifndef MPCG_H
#define MPCG_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MPCG_ABI_VERSION 2

/* The 15 keys of the reference's parameter map (DrivingStateContext::updateMpcConfigs,
 * mpc_ros/src/driving_state.cpp:65-79; MPC::LoadParams mpc_planner.cpp:243-262;
 * FG_eval::LoadParams mpc_planner.cpp:71-97), plus the Ipopt options the reference
 * leaves at their defaults (mpc_planner.cpp:356-368). */
typedef struct mpcg_params {
    int32_t steps;            /* "STEPS": horizon N (double truncated to int, :74, :247) */
    int32_t model;            /* 0 = differential drive (FG_eval); 1 = kinematic bicycle: the control
                                 w is the steering angle (|w| <= ANGVEL) and the heading rows turn
                                 by v w / wheelbase dt (strategy WAVE only) */
    double dt;                /* "DT" */
    double ref_cte;           /* "REF_CTE" */
    double ref_etheta;        /* "REF_ETHETA" */
    double ref_v;             /* "REF_V" */
    double w_cte;             /* "W_CTE" */
    double w_etheta;          /* "W_EPSI" */
    double w_v;               /* "W_V" */
    double w_angvel;          /* "W_ANGVEL" */
    double w_accel;           /* "W_A" */
    double w_angvel_d;        /* "W_DANGVEL" */
    double w_accel_d;         /* "W_DA" */
    double max_angvel;        /* "ANGVEL" */
    double max_throttle;      /* "MAXTHR" */
    double bound;             /* "BOUND" */
    /* Ipopt 3.12 defaults unless changed */
    double tol;               /* 1e-8 */
    int32_t max_iter;         /* 3000 */
    int32_t filter_cap;       /* filter entries held in LDS per problem (64); 448 more are kept in
                                 the HBM workspace, so the oldest entry is dropped only beyond
                                 filter_cap + 448 non-dominated entries (counted in diag[:, 1];
                                 Ipopt's filter is unbounded) */
    double bound_relax_factor;/* 1e-8 */
    double mu_init;           /* 0.1 */
    double wheelbase;         /* model 1 only: Lf [m] */
    /* "max_cpu_time" (the reference sets 0.5 s, mpc_planner.cpp:368): applied as the number of
     * iterations the reference's Solve affords in that time at this horizon, so that results
     * are deterministic: (max_cpu_time - CppAD taping) / (CppAD derivative evaluations + Ipopt's
     * own iteration work) -- taping and derivatives measured in the survey (1.52 ms and
     * 0.225 ms per iteration at N = 20), Ipopt's KKT factorisation, solve and line search
     * calibrated at 5.14 us per stage (0.103 ms at N = 20): 1,520 iterations at N = 20, 737 at
     * N = 40.  Beyond it the status is 14 (unknown) with the last iterate.  >= 1e6: no budget
     * (Ipopt's "no limit"). */
    double max_cpu_time;
    /* Ipopt 3.12 defaults (the reference leaves them untouched) */
    double acceptable_tol;             /* 1e-6 */
    double acceptable_dual_inf_tol;    /* 1e10 */
    double acceptable_constr_viol_tol; /* 1e-2 */
    double acceptable_compl_inf_tol;   /* 1e-2 */
    double acceptable_obj_change_tol;  /* 1e20 */
    double kappa_soc;                  /* 0.99 */
    double soft_resto_pderror_reduction_factor; /* 0.9999 (0: no soft restoration) */
    double obj_max_inc;                /* 5 */
    double tiny_step_tol;              /* 10 eps */
    double tiny_step_y_tol;            /* 1e-2 */
    double dual_inf_tol;               /* 1 (unscaled dual infeasibility at termination) */
    double constr_viol_tol;            /* 1e-4 (unscaled constraint violation; caps the bound relaxation) */
    double compl_inf_tol;              /* 1e-4 (unscaled complementarity; mu_min = min(tol, this) / 11) */
    int32_t acceptable_iter;           /* 15 (0: no acceptable termination) */
    int32_t max_soc;                   /* 4 (0: no second-order corrections) */
    int32_t watchdog_shortened_iter_trigger; /* 10 (0: no watchdog) */
    int32_t watchdog_trial_iter_max;   /* 3 */
    int32_t max_soft_resto_iters;      /* 10 */
    int32_t max_filter_resets;         /* 5 */
    int32_t filter_reset_trigger;      /* 5 */
    /* Arithmetic of the solve: 0 = fp64 (the reference's double, the default); 1 = fp32
     * (BASELINE configs[2]; differential drive only): iterate, multipliers and Newton systems
     * in float -- state a tolerance a float iterate can meet (tol ~1e-5 instead of 1e-8;
     * tiny_step_tol 10 FLT_EPSILON).  Inputs and outputs stay double.
     * Two phases (precision 1, no_restoration 0): the fp32 solver on the whole batch with these
     * params' options, then the fp64 solver with the reference's Ipopt options (the 3.12
     * defaults of the fields above; max_cpu_time and the problem parameters are kept) on the
     * whole batch again -- from the fp32 iterate, multipliers and barrier parameter where the
     * fp32 solve converged (status 1 or 4; diag[:, 2] = 4), from the start where it did not (its
     * line search failed where Ipopt would enter the restoration phase, a tiny step, the
     * iteration limit; diag[:, 2] = 3, bitwise the fp64 solver's result).  The outputs are the
     * fp64 phase's; iters counts both phases' iterations for a continued row, the fp64 solve's
     * for a row solved from the start.  Batches of more than 2,048 (solved in expected-longest-
     * first order): the B / 1024 problems ranked longest are solved by the fp64 solver from the
     * start (diag[:, 2] = 3) while the fp32 phase runs the others.  Which rows form this head
     * depends on the batch (its size and the other rows' ranks), so re-batching or sharding the
     * same problems can move a row between the head (the fp64 solve from the start) and the fp32
     * path (the fp64 continuation of its fp32 iterate); every other row's result, and every
     * result of the fp64 configuration, is independent of the batch. */
    int32_t precision;
    /* 0 (default): Ipopt's feasibility-restoration phase where the line search fails (fp32:
     * the two phases above); 1: stop there with RESTORATION_FAILURE (9) instead, and for
     * precision 1 the fp32 phase alone (its ending kept).  Occupies the struct's padding:
     * sizeof(mpcg_params) is unchanged. */
    int32_t no_restoration;
} mpcg_params;

typedef struct mpcg_handle mpcg_handle;

int mpcg_abi_version(void);
/* Hash of the sources the library was built from (mpc_ros_amd/build.py source_hash()). */
const char* mpcg_build_id(void);
const char* mpcg_last_error(void);

/* Defaults of an MPC object before LoadParams: MPC::MPC() (mpc_planner.cpp:223-241)
 * + FG_eval constructor (:42-68). */
int mpcg_params_default(mpcg_params* p);
/* Defaults the move_base plugin loads (mpc_ros/cfg/MPCPlanner.cfg:22-37, DT 0.1). */
int mpcg_params_plugin_default(mpcg_params* p);
/* One LoadParams map entry: key is one of the 15 reference keys, or one of the
 * extension keys MODEL (0 differential drive, 1 kinematic bicycle) and LF (wheelbase).
 * Returns 0 if applied, 1 if the key is unknown (ignored, as LoadParams ignores it). */
int mpcg_params_set(mpcg_params* p, const char* key, double value);
/* Validate a parameter set (steps >= 2, dt > 0, bounds > 0, weights >= 0). */
int mpcg_params_check(const mpcg_params* p);

/* Handle bound to one GPU (HIP device ordinal). */
int mpcg_create(int device, mpcg_handle** out);
void mpcg_destroy(mpcg_handle* h);
int mpcg_set_params(mpcg_handle* h, const mpcg_params* p);
int mpcg_get_params(const mpcg_handle* h, mpcg_params* p);
/* Device workspace for B problems (bytes): 4 slots per wavefront the GPU holds resident
 * (not per problem: the rare solver paths' copies), the park area of problems that enter the
 * restoration phase (max(256, B/128) entries, at most B; each holds the problem's state and
 * the restoration phase's records), the park-area overflow list (8 B per problem where the
 * area can overflow), and the solve-order buffers (B > 2048); reserve it ahead of graph
 * capture (a solve that must grow it allocates and synchronises the device). */
size_t mpcg_workspace_bytes(const mpcg_params* p, int64_t B);
/* The same for a handle: its parameters, its park capacity (mpcg_set_park_capacity) and the XCD
 * count of its device (the slot partitions) -- what mpcg_reserve(h, B) allocates. */
size_t mpcg_handle_workspace_bytes(const mpcg_handle* h, int64_t B);
int mpcg_reserve(mpcg_handle* h, int64_t B);
/* Park-area entries of the handle's solves (0 = the default max(256, B/128)).  A problem that
 * enters the restoration phase while every entry is taken goes to an overflow list and is
 * solved again from the start after the batch (the same iterates, diag[:, 2] = 2): results do
 * not depend on the capacity, only the tail does.  A tuning and test knob.  Set it before
 * mpcg_reserve: a larger capacity grows the workspace, and the next solve would otherwise
 * allocate it (with a device synchronisation -- not during graph capture). */
int mpcg_set_park_capacity(mpcg_handle* h, int64_t cap);
/* The solver kernel instance the handle's last solve launched, "k_solve_wide<model, split,
 * type, stage blocks, default options, waves per SIMD>" ("" before the first solve). */
const char* mpcg_last_kernel(const mpcg_handle* h);
/* 1 if the handle's last solve ran its problems in expected-longest-first order (batches of
 * B > 2048: a radix sort of the path curvature before the batch kernel), 0 otherwise. */
int mpcg_last_solve_order(const mpcg_handle* h);

/* Batched solve, host buffers, synchronous (copies in, solves, copies out).
 *   state  [B][6]  x, y, theta, v, cte, etheta   (MPC::Solve `state`)
 *   coeffs [B][4]  c0..c3                        (MPC::Solve `coeffs`)
 *   u0     [B][2]  omega_0, a_0                  (MPC::Solve return value)
 *   traj   [B][3][N] mpc_x | mpc_y | mpc_theta   (MPC::mpc_x/mpc_y/mpc_theta) or NULL
 *   status [B] or NULL, obj [B] or NULL, iters [B] or NULL */
int mpcg_solve(mpcg_handle* h, int64_t B, const double* state, const double* coeffs, double* u0,
               double* traj, int32_t* status, double* obj, int32_t* iters);

/* Batched solve on device-resident buffers (same layouts), queued on `stream` (a
 * hipStream_t; NULL = the null stream, as everywhere in HIP) without any host
 * synchronisation: the solve-order sort (B > 2048), a workspace reset, the batch kernel and
 * the restoration phase's resume kernels; work forked onto the handle's own streams (resume
 * workers, the fp32 configuration's head) is joined back into `stream` by events, so the
 * sequence can be captured in a HIP graph.  Synchronise the stream before reading the outputs
 * on the host.  No allocation if mpcg_reserve(h, B) was called. */
int mpcg_solve_device(mpcg_handle* h, int64_t B, const double* d_state, const double* d_coeffs, double* d_u0,
                      double* d_traj, int32_t* d_status, double* d_obj, int32_t* d_iters, void* stream);

/* mpcg_solve / mpcg_solve_device with per-problem solver diagnostics diag [B][4] (int32,
 * may be NULL): restoration phases entered, filter entries dropped beyond its capacity
 * (filter_cap in LDS plus 448 in the workspace; Ipopt's filter is unbounded, so any nonzero
 * value marks a solve that may differ from Ipopt's), 1 if the problem was continued by the
 * parked-problem kernel (2 if it was solved again after a park-area overflow; precision 1: 4 if
 * the fp64 phase continued from the fp32 iterate, 3 if it solved the problem from the start;
 * 0 otherwise), the
 * most filter entries held at once (the original problem). */
int mpcg_solve_ex(mpcg_handle* h, int64_t B, const double* state, const double* coeffs, double* u0, double* traj,
                  int32_t* status, double* obj, int32_t* iters, int32_t* diag);
int mpcg_solve_device_ex(mpcg_handle* h, int64_t B, const double* d_state, const double* d_coeffs, double* d_u0,
                         double* d_traj, int32_t* d_status, double* d_obj, int32_t* d_iters, int32_t* d_diag,
                         void* stream);

/* Multi-GPU batched solves from one process, host buffers as
 * mpcg_solve: the B problems are split into ngpu contiguous shards (the first B % ngpu
 * GPUs take one more), solved on devices[r] with the given parameters, and the results are
 * gathered to devices[0] by grouped RCCL send/recv (one message per output array and GPU,
 * point-to-point over xGMI), then copied to the host.
 *
 * mpcg_multi: a persistent context for a serving loop -- the RCCL communicator
 * (ncclCommInitAll), a handle, stream and device buffers per GPU, and each handle's solver
 * workspace reserved for the largest shard of B_max problems, all created once by
 * mpcg_multi_create; mpcg_multi_solve then allocates nothing (batches of B <= B_max; the
 * parameters are the context's).  A failure inside the gather group aborts the communicators
 * and marks the context broken (later solves return -4; destroy and create it again).
 * mpcg_solve_multi = create + solve + destroy for one batch.  Returns 0, or < 0 with
 * mpcg_last_error() set (-1 arguments, -2 HIP, -3 device ordinal, -4 RCCL). */
typedef struct mpcg_multi mpcg_multi;
int mpcg_multi_create(int ngpu, const int* devices, const mpcg_params* params, int64_t B_max, mpcg_multi** out);
int mpcg_multi_solve(mpcg_multi* m, int64_t B, const double* state, const double* coeffs, double* u0, double* traj,
                     int32_t* status, double* obj, int32_t* iters);
void mpcg_multi_destroy(mpcg_multi* m);
int mpcg_solve_multi(int ngpu, const int* devices, const mpcg_params* params, int64_t B, const double* state,
                     const double* coeffs, double* u0, double* traj, int32_t* status, double* obj, int32_t* iters);

/* mpcg_solve_multi's arithmetic, pure functions (no GPU):
 * mpcg_shard_range: GPU r of ngpu solves problems [start, start + count) -- contiguous,
 *   the first B % ngpu GPUs one more, empty shards when B < ngpu.
 * mpcg_multi_gather_plan: the MPCG_GATHER_ARRAYS messages GPU r sends to devices[0]
 *   (u0, traj, obj, status, iters): byte offsets in its own output buffer and in the root's
 *   gathered buffer of mpcg_multi_out_bytes(B, N) bytes, and sizes (count x 32 + 24 N bytes
 *   in all; 0 for an empty shard).  For r = 0 src_offset == dst_offset: the root solves in
 *   place and sends nothing. */
#define MPCG_GATHER_ARRAYS 5
typedef struct mpcg_xfer {
    size_t src_offset, dst_offset, bytes;
} mpcg_xfer;
int mpcg_shard_range(int64_t B, int ngpu, int r, int64_t* start, int64_t* count);
int mpcg_multi_gather_plan(int64_t B, int32_t N, int ngpu, int r, mpcg_xfer* xfers);
size_t mpcg_multi_out_bytes(int64_t B, int32_t N);
/* mpcg_multi_buffer_bytes: the device buffers a context for batches of up to B_max holds on
 * GPU r (inputs of the largest shard; outputs of that shard, or on the root the gathered
 * outputs of B_max problems), besides the handle's solver workspace (mpcg_workspace_bytes of
 * the largest shard).  0 for invalid arguments. */
size_t mpcg_multi_buffer_bytes(int64_t B_max, int32_t N, int ngpu, int r);

/* Tracking::findBestPath's preprocessing (mpc_ros/src/driving_state.cpp:175-256) on the
 * device for B robots: waypoints to the vehicle frame, cubic polyfit (Householder QR),
 * cte, heading error from the first int(0.3 M) waypoint increments, delay-mode
 * prediction.  M waypoints per robot, the same for the batch: M >= 4 (polyfit asserts
 * order 3 <= M - 1, driving_state.cpp:286); plans beyond 64 waypoints take a handle-owned
 * device scratch of 48 M B bytes (used stream-ordered).
 *   pose [B][3]  x, y, yaw                       (global_pose)
 *   vel  [B][3]  v feedback, previous w, previous throttle (feedback_vel.linear.x, _w, _throttle)
 *   plan [B][M][2] waypoints x, y                (ref_plan)
 *   state [B][6], coeffs [B][4]                  the arguments of MPC::Solve (outputs)
 * dt = the handle's DT.  Queued on `stream`; no solve. */
int mpcg_preprocess_device(mpcg_handle* h, int64_t B, int32_t M, const double* d_pose, const double* d_vel,
                           const double* d_plan, int32_t delay_mode, double* d_state, double* d_coeffs,
                           void* stream);

/* One control tick of Tracking::findBestPath for B robots: preprocessing, the solve,
 * and the post-processing of driving_state.cpp:262-269.
 *   cmd [B][3]  speed = min(v + throttle dt, REF_V), w = w0, throttle = a0
 *   traj [B][3][N], status [B]: as mpcg_solve_device (may be NULL).
 * Intermediate state/coeffs/controls live in handle-owned device buffers. */
int mpcg_track_device(mpcg_handle* h, int64_t B, int32_t M, const double* d_pose, const double* d_vel,
                      const double* d_plan, int32_t delay_mode, double* d_cmd, double* d_traj, int32_t* d_status,
                      void* stream);

/* The benchmark's synthetic robots (the "infinity set", mpc_ros_amd/infinity.py) generated on
 * the device: robot start + i of the set (i < B) is a pure function of (seed, start + i) --
 * a pose near a lemniscate course, its speed and previous controls, and a plan of M waypoints
 * along the course -- so a rank of a multi-GPU run generates exactly its own slice on its GPU.
 * Outputs as mpcg_preprocess_device takes them: pose [B][3], vel [B][3], plan [B][M][2].  Not
 * part of the reference's interface (a data generator for benchmarks and tests); queued on
 * `stream` (the first call uploads a 3.2 MB table synchronously). */
int mpcg_synth_infinity_device(mpcg_handle* h, uint64_t seed, int64_t start, int64_t B, int32_t M, double* d_pose,
                               double* d_vel, double* d_plan, void* stream);

/* Kernel strategy of the handle's solves.  Since ABI 2 there is one: one problem per
 * wavefront, the whole problem state in LDS (AUTO and WAVE select it).  LANE (the round-1
 * one-problem-per-lane kernels) was removed; selecting it is an error. */
#define MPCG_STRATEGY_AUTO 0
#define MPCG_STRATEGY_LANE 1
#define MPCG_STRATEGY_WAVE 2
int mpcg_set_strategy(mpcg_handle* h, int32_t strategy);
/* The strategy a solve of the handle's current parameters would use (never AUTO). */
int mpcg_get_strategy(const mpcg_handle* h);

/* Wait for all work queued on the handle's stream. */
int mpcg_synchronize(mpcg_handle* h);

#ifdef __cplusplus
}
#endif
#endif
