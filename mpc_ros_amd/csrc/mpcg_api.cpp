// mpc_ros_amd/csrc/mpcg_api.cpp -- the C-ABI of include/mpcg.h.
//
// Owns device buffers and a stream per handle; translates the reference's
// parameter map semantics (MPC::LoadParams / FG_eval::LoadParams,
// mpc_ros/src/mpc_planner.cpp:71-97, 243-262) into the kernel's IpmParams.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>

#include "mpcg.h"
#include "mpcg_internal.h"

namespace {
thread_local std::string g_err;
}  // namespace

namespace mpcg {
int set_error(int code, const std::string& msg) {
    g_err = msg;
    return code;
}
}  // namespace mpcg

namespace {
int fail(int code, const std::string& msg) { return mpcg::set_error(code, msg); }
int hip_fail(hipError_t e, const char* what) {
    return fail(-2, std::string(what) + ": " + hipGetErrorString(e));
}
}  // namespace

struct mpcg_handle {
    int device = 0;
    hipStream_t stream = nullptr;
    // the restoration phase's resume workers run on aux alongside the batch kernel (fork /
    // join events on the caller's stream)
    hipStream_t aux = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    // (the fp32 configuration's head runs on aux, its resume workers on aux2)
    hipStream_t aux2 = nullptr;
    hipEvent_t ev_join2 = nullptr;
    mpcg_params params{};
    // staging buffers for mpcg_solve (host pointers)
    double* d_io = nullptr;
    size_t io_bytes = 0;
    int strategy = MPCG_STRATEGY_AUTO;
    // mpcg_track_device intermediates: state [B][6] | coeffs [B][4] | u0 [B][2]
    double* d_trk = nullptr;
    size_t trk_bytes = 0;
    // preprocessing scratch of plans longer than 64 waypoints
    double* d_pp = nullptr;
    size_t pp_bytes = 0;
    // solve-order buffers (keys, indices, sort scratch)
    void* d_sched = nullptr;
    size_t sched_bytes = 0;
    // HBM workspace slots of the solver's rare paths and restoration phase (one per resident wavefront)
    double* d_spill = nullptr;
    size_t spill_bytes = 0;
    // stream ordering of the scratch above: the last stream that used it and an event
    // recorded after that use
    hipStream_t last_stream = nullptr;
    hipEvent_t last_ev = nullptr;
    bool have_last = false;
    // the solver kernel instance the last solve launched (mpcg_last_kernel)
    const char* last_kernel = "";
    // 1 if the last solve ran in expected-longest-first order (B > kOrderMinBatch)
    int last_ordered = 0;
    // park-area entries (0: the default, max(256, B / 128))
    int64_t park_cap = 0;
    // the synthetic robots' arc-length table (mpcg_synth_infinity_device), uploaded once
    double* d_arc = nullptr;
};

#ifndef MPCG_BUILD_ID
#define MPCG_BUILD_ID "unversioned"
#endif

extern "C" {

int mpcg_abi_version(void) { return MPCG_ABI_VERSION; }
const char* mpcg_build_id(void) {
    static const char kId[] = MPCG_BUILD_ID;  // "MPCG-BUILD-ID:<source hash>" (mpc_ros_amd/build.py)
    return std::strncmp(kId, "MPCG-BUILD-ID:", 14) == 0 ? kId + 14 : kId;
}
const char* mpcg_last_error(void) { return g_err.c_str(); }

static void ipopt_defaults(mpcg_params* p) {
    p->tol = 1e-8;
    p->max_iter = 3000;
    p->filter_cap = 64;
    p->bound_relax_factor = 1e-8;
    p->mu_init = 0.1;
    p->wheelbase = 0.5;
    p->model = 0;
    p->max_cpu_time = 0.5;  // mpc_planner.cpp:368
    p->acceptable_tol = 1e-6;
    p->acceptable_dual_inf_tol = 1e10;
    p->acceptable_constr_viol_tol = 1e-2;
    p->acceptable_compl_inf_tol = 1e-2;
    p->acceptable_obj_change_tol = 1e20;
    p->kappa_soc = 0.99;
    p->soft_resto_pderror_reduction_factor = 0.9999;
    p->obj_max_inc = 5.0;
    p->tiny_step_tol = 10.0 * 2.220446049250313e-16;
    p->tiny_step_y_tol = 1e-2;
    p->dual_inf_tol = 1.0;
    p->constr_viol_tol = 1e-4;
    p->compl_inf_tol = 1e-4;
    p->acceptable_iter = 15;
    p->max_soc = 4;
    p->watchdog_shortened_iter_trigger = 10;
    p->watchdog_trial_iter_max = 3;
    p->max_soft_resto_iters = 10;
    p->max_filter_resets = 5;
    p->filter_reset_trigger = 5;
}

// max_cpu_time as the iterations the reference's Solve affords in that time at horizon
// N: CppAD taping 1.52 ms (N = 20) / 3.93 ms (N = 40) and derivative cost 0.225 / 0.467 ms
// per iteration, measured in the survey, plus Ipopt's own per-iteration
// work (KKT factorisation and solve, line search): the structured oracle's iteration on
// one EPYC 9575F core, 0.103 ms at N = 20 (profiles/r3/cpu_iter_cost.json), taken linear
// in N (5.14 us per stage).  0.5 s -> 1520 iterations at N = 20, 737 at N = 40.  -1: no
// budget.  (oracle/ipm.c ora_cpu_iter_budget restates the same model for the checker.)
static int cpu_iter_budget(double max_cpu_time, int steps) {
    if (!(max_cpu_time > 0) || max_cpu_time >= 999999.0) return -1;
    const double setup = std::fmax(0.0, 0.1205e-3 * steps - 0.89e-3);
    const double per = std::fmax(0.0121e-3 * steps - 0.017e-3, 1e-5) + 5.14e-6 * steps;
    const double b = std::floor((max_cpu_time - setup) / per);
    return b < 0 ? 0 : (b > 1e9 ? 1000000000 : (int)b);
}

int mpcg_params_default(mpcg_params* p) {
    if (!p) return fail(-1, "null params");
    std::memset(p, 0, sizeof *p);
    // MPC::MPC() (mpc_planner.cpp:223-241)
    p->steps = 20;
    p->max_angvel = 3.0;
    p->max_throttle = 1.0;
    p->bound = 1.0e3;
    // FG_eval::FG_eval (mpc_planner.cpp:42-68)
    p->dt = 0.1;
    p->ref_cte = 0.0;
    p->ref_etheta = 0.0;
    p->ref_v = 0.5;
    p->w_cte = 100;
    p->w_etheta = 100;
    p->w_v = 1;
    p->w_angvel = 100;
    p->w_accel = 50;
    p->w_angvel_d = 0;
    p->w_accel_d = 0;
    ipopt_defaults(p);
    return 0;
}

int mpcg_params_plugin_default(mpcg_params* p) {
    if (!p) return fail(-1, "null params");
    std::memset(p, 0, sizeof *p);
    // mpc_ros/cfg/MPCPlanner.cfg:22-37; DT = 1/controller_frequency (driving_state.cpp:28)
    p->steps = 20;
    p->dt = 0.1;
    p->ref_cte = 0.0;
    p->ref_etheta = 0.0;
    p->ref_v = 1.0;
    p->w_cte = 1000;
    p->w_etheta = 1000;
    p->w_v = 100;
    p->w_angvel = 100;
    p->w_accel = 50;
    p->w_angvel_d = 0;
    p->w_accel_d = 10;
    p->max_angvel = 1.0;
    p->max_throttle = 1.0;
    p->bound = 1000;
    ipopt_defaults(p);
    return 0;
}

int mpcg_params_set(mpcg_params* p, const char* key, double v) {
    if (!p || !key) return fail(-1, "null argument");
    const std::string k(key);
    if (k == "DT") p->dt = v;
    else if (k == "STEPS") p->steps = (int32_t)v;  // double -> int truncation, as the reference
    else if (k == "REF_CTE") p->ref_cte = v;
    else if (k == "REF_ETHETA") p->ref_etheta = v;
    else if (k == "REF_V") p->ref_v = v;
    else if (k == "W_CTE") p->w_cte = v;
    else if (k == "W_EPSI") p->w_etheta = v;
    else if (k == "W_V") p->w_v = v;
    else if (k == "W_ANGVEL") p->w_angvel = v;
    else if (k == "W_A") p->w_accel = v;
    else if (k == "W_DANGVEL") p->w_angvel_d = v;
    else if (k == "W_DA") p->w_accel_d = v;
    else if (k == "ANGVEL") p->max_angvel = v;
    else if (k == "MAXTHR") p->max_throttle = v;
    else if (k == "BOUND") p->bound = v;
    // extension keys (not in the reference map): dynamics model and wheelbase
    else if (k == "MODEL") p->model = (int32_t)v;
    else if (k == "LF") p->wheelbase = v;
    else return 1;
    return 0;
}

int mpcg_params_check(const mpcg_params* p) {
    if (!p) return fail(-1, "null params");
    if (p->steps < 2 || p->steps > 4096) return fail(-1, "STEPS must be in [2, 4096]");
    if (!(p->max_cpu_time > 0)) return fail(-1, "max_cpu_time must be > 0");
    if (p->acceptable_iter < 0 || p->max_soc < 0 || p->watchdog_shortened_iter_trigger < 0 ||
        p->watchdog_trial_iter_max < 0 || p->max_soft_resto_iters < 0 || p->max_filter_resets < 0 ||
        p->filter_reset_trigger < 1)
        return fail(-1, "invalid Ipopt integer option");
    if (!(p->soft_resto_pderror_reduction_factor >= 0) || !(p->tiny_step_tol >= 0) || !(p->kappa_soc > 0) ||
        !(p->dual_inf_tol > 0) || !(p->constr_viol_tol > 0) || !(p->compl_inf_tol > 0))
        return fail(-1, "invalid Ipopt option");
    if (!(p->dt > 0) || !std::isfinite(p->dt)) return fail(-1, "DT must be > 0");
    if (!(p->max_angvel > 0) || !(p->max_throttle > 0) || !(p->bound > 0)) return fail(-1, "bounds must be > 0");
    const double w[] = {p->w_cte, p->w_etheta, p->w_v, p->w_angvel, p->w_accel, p->w_angvel_d, p->w_accel_d};
    for (double x : w)
        if (!(x >= 0) || !std::isfinite(x)) return fail(-1, "weights must be finite and >= 0");
    if (!(p->tol > 0)) return fail(-1, "tol must be > 0");
    if (p->max_iter < 0) return fail(-1, "max_iter must be >= 0");
    if (p->filter_cap < 1 || p->filter_cap > 1024) return fail(-1, "filter_cap must be in [1, 1024]");
    if (!(p->bound_relax_factor >= 0) || !(p->mu_init > 0)) return fail(-1, "invalid Ipopt options");
    if (p->model != 0 && p->model != 1) return fail(-1, "model must be 0 (differential drive) or 1 (bicycle)");
    if (p->model == 1 && !(p->wheelbase > 0)) return fail(-1, "model 1 needs wheelbase (LF) > 0");
    if (p->precision != 0 && p->precision != 1) return fail(-1, "precision must be 0 (fp64) or 1 (fp32)");
    if (p->precision == 1 && p->model != 0) return fail(-1, "precision 1 (fp32) runs the differential drive only");
    if (p->no_restoration != 0 && p->no_restoration != 1) return fail(-1, "no_restoration must be 0 or 1");
    return 0;
}

static mpcg::IpmParams to_ipm(const mpcg_params& p) {
    mpcg::IpmParams q{};
    q.N = p.steps;
    q.dt = p.dt;
    q.ref_cte = p.ref_cte;
    q.ref_eth = p.ref_etheta;
    q.ref_v = p.ref_v;
    q.w_cte = p.w_cte;
    q.w_eth = p.w_etheta;
    q.w_v = p.w_v;
    q.w_w = p.w_angvel;
    q.w_a = p.w_accel;
    q.w_dw = p.w_angvel_d;
    q.w_da = p.w_accel_d;
    q.max_w = p.max_angvel;
    q.max_a = p.max_throttle;
    q.bound = p.bound;
    q.tol = p.tol;
    q.bound_relax_factor = p.bound_relax_factor;
    q.mu_init = p.mu_init;
    q.max_iter = p.max_iter;
    q.filter_cap = p.filter_cap;
    q.model = p.model;
    q.lf = p.wheelbase;
    q.acceptable_tol = p.acceptable_tol;
    q.acceptable_iter = p.acceptable_iter;
    q.acceptable_dual_inf_tol = p.acceptable_dual_inf_tol;
    q.acceptable_constr_viol_tol = p.acceptable_constr_viol_tol;
    q.acceptable_compl_inf_tol = p.acceptable_compl_inf_tol;
    q.acceptable_obj_change_tol = p.acceptable_obj_change_tol;
    q.max_soc = p.max_soc;
    q.kappa_soc = p.kappa_soc;
    q.watchdog_trigger = p.watchdog_shortened_iter_trigger;
    q.watchdog_trial_max = p.watchdog_trial_iter_max;
    q.soft_resto_factor = p.soft_resto_pderror_reduction_factor;
    q.max_soft_resto_iters = p.max_soft_resto_iters;
    q.obj_max_inc = p.obj_max_inc;
    q.max_filter_resets = p.max_filter_resets;
    q.filter_reset_trigger = p.filter_reset_trigger;
    q.tiny_step_tol = p.tiny_step_tol;
    q.tiny_step_y_tol = p.tiny_step_y_tol;
    q.dual_inf_tol = p.dual_inf_tol;
    q.constr_viol_tol = p.constr_viol_tol;
    q.compl_inf_tol = p.compl_inf_tol;
    q.cpu_iter_budget = cpu_iter_budget(p.max_cpu_time, p.steps);
    q.precision = p.precision;
    q.no_resto = p.no_restoration;
    return q;
}

// solve-order buffers (batches beyond the resident wavefronts)
using mpcg::kOrderMinBatch;
static mpcg::IpmParams handle_ipm(const mpcg_handle* h);

size_t mpcg_workspace_bytes(const mpcg_params* p, int64_t B) {
    if (!p || B <= 0) return 0;
    const mpcg::IpmParams P = to_ipm(*p);
    return mpcg::wide_spill_bytes(P, B) + (B > kOrderMinBatch ? mpcg::wide_sched_bytes(B) : 0);
}

// (the handle's own: its parameters, park capacity and device -- the slot partitions follow the
// device's XCD count)
size_t mpcg_handle_workspace_bytes(const mpcg_handle* h, int64_t B) {
    if (!h || B <= 0) return 0;
    int prev = -1;
    const bool sw = hipGetDevice(&prev) == hipSuccess && prev != h->device;
    if (sw && hipSetDevice(h->device) != hipSuccess) return 0;
    const size_t n = mpcg::wide_spill_bytes(handle_ipm(h), B) + (B > kOrderMinBatch ? mpcg::wide_sched_bytes(B) : 0);
    if (sw) hipSetDevice(prev);
    return n;
}

int mpcg_create(int device, mpcg_handle** out) {
    if (!out) return fail(-1, "null out");
    *out = nullptr;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) return hip_fail(e, "hipGetDeviceCount");
    if (device < 0 || device >= n) return fail(-3, "device ordinal out of range (no GPU?)");
    e = hipSetDevice(device);
    if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
    mpcg_handle* h = new mpcg_handle();
    h->device = device;
    e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete h;
        return hip_fail(e, "hipStreamCreate");
    }
    mpcg_params_plugin_default(&h->params);
    e = hipEventCreateWithFlags(&h->last_ev, hipEventDisableTiming);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&h->aux, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&h->ev_fork, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&h->ev_join, hipEventDisableTiming);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&h->aux2, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&h->ev_join2, hipEventDisableTiming);
    if (e != hipSuccess) {
        mpcg_destroy(h);
        return hip_fail(e, "hipEventCreate / hipStreamCreate");
    }
    *out = h;
    return 0;
}

void mpcg_destroy(mpcg_handle* h) {
    if (!h) return;
    hipSetDevice(h->device);
    if (h->stream) hipStreamSynchronize(h->stream);
    if (h->have_last) hipEventSynchronize(h->last_ev);
    if (h->d_io) hipFree(h->d_io);
    if (h->d_trk) hipFree(h->d_trk);
    if (h->d_pp) hipFree(h->d_pp);
    if (h->d_sched) hipFree(h->d_sched);
    if (h->d_spill) hipFree(h->d_spill);
    if (h->d_arc) hipFree(h->d_arc);
    if (h->aux) hipStreamSynchronize(h->aux);
    if (h->aux2) hipStreamSynchronize(h->aux2);
    if (h->last_ev) hipEventDestroy(h->last_ev);
    if (h->ev_fork) hipEventDestroy(h->ev_fork);
    if (h->ev_join) hipEventDestroy(h->ev_join);
    if (h->ev_join2) hipEventDestroy(h->ev_join2);
    if (h->aux) hipStreamDestroy(h->aux);
    if (h->aux2) hipStreamDestroy(h->aux2);
    if (h->stream) hipStreamDestroy(h->stream);
    delete h;
}

int mpcg_set_params(mpcg_handle* h, const mpcg_params* p) {
    if (!h || !p) return fail(-1, "null argument");
    int rc = mpcg_params_check(p);
    if (rc) return rc;
    h->params = *p;
    return 0;
}

int mpcg_get_params(const mpcg_handle* h, mpcg_params* p) {
    if (!h || !p) return fail(-1, "null argument");
    *p = h->params;
    return 0;
}

static mpcg::IpmParams handle_ipm(const mpcg_handle* h) {
    mpcg::IpmParams P = to_ipm(h->params);
    P.park_cap = (int)h->park_cap;
    return P;
}

static int ensure_spill(mpcg_handle* h, int64_t B) {
    const size_t need = mpcg::wide_spill_bytes(handle_ipm(h), B);
    if (need <= h->spill_bytes) return 0;
    hipSetDevice(h->device);
    if (h->d_spill) {
        hipDeviceSynchronize();  // may be in use on any stream
        hipFree(h->d_spill);
        h->d_spill = nullptr;
        h->spill_bytes = 0;
    }
    hipError_t e = hipMalloc((void**)&h->d_spill, need);
    if (e != hipSuccess) return hip_fail(e, "hipMalloc(spill areas)");
    h->spill_bytes = need;
    return 0;
}

static int ensure_sched(mpcg_handle* h, int64_t B) {
    const size_t need = mpcg::wide_sched_bytes(B);
    if (need <= h->sched_bytes) return 0;
    hipSetDevice(h->device);
    if (h->d_sched) {
        hipDeviceSynchronize();  // may be in use on any stream
        hipFree(h->d_sched);
        h->d_sched = nullptr;
        h->sched_bytes = 0;
    }
    hipError_t e = hipMalloc(&h->d_sched, need);
    if (e != hipSuccess) return hip_fail(e, "hipMalloc(schedule buffers)");
    h->sched_bytes = need;
    return 0;
}

// 160 KiB of LDS per CU: up to N = 64 a problem leaves room for a second wavefront (and
// eight fit at N = 20); up to N = 128 (two stage blocks) one problem may take the CU's LDS
static const size_t kWideLdsMax = 160 * 1024;

// The handle's scratch (solve order, spill areas, track intermediates) is used
// stream-ordered: work queued on stream s first waits for the scratch's last use on
// another stream, and an event marks each use.
static int order_on(mpcg_handle* h, hipStream_t s) {
    if (h->have_last && h->last_stream != s) {
        hipError_t e = hipStreamWaitEvent(s, h->last_ev, 0);
        if (e != hipSuccess) return hip_fail(e, "hipStreamWaitEvent");
    }
    return 0;
}
static int record_on(mpcg_handle* h, hipStream_t s) {
    hipError_t e = hipEventRecord(h->last_ev, s);
    if (e != hipSuccess) return hip_fail(e, "hipEventRecord");
    h->last_stream = s;
    h->have_last = true;
    return 0;
}

static bool wave_fits(const mpcg::IpmParams& P) { return P.N <= 128 && mpcg::wide_lds_bytes(P) <= kWideLdsMax; }

int mpcg_reserve(mpcg_handle* h, int64_t B) {
    if (!h) return fail(-1, "null handle");
    if (B < 0) return fail(-1, "negative batch");
    if (B == 0) return 0;
    int rc = ensure_spill(h, B);
    if (rc) return rc;
    return B > kOrderMinBatch ? ensure_sched(h, B) : 0;
}

int mpcg_set_strategy(mpcg_handle* h, int32_t strategy) {
    if (!h) return fail(-1, "null handle");
    if (strategy == MPCG_STRATEGY_LANE) return fail(-1, "strategy LANE was removed in ABI 2 (one solver: WAVE)");
    if (strategy != MPCG_STRATEGY_AUTO && strategy != MPCG_STRATEGY_WAVE) return fail(-1, "unknown strategy");
    h->strategy = strategy;
    return 0;
}

int mpcg_get_strategy(const mpcg_handle* h) {
    if (!h) return fail(-1, "null handle");
    return MPCG_STRATEGY_WAVE;
}

int mpcg_solve_device(mpcg_handle* h, int64_t B, const double* d_state, const double* d_coeffs, double* d_u0,
                      double* d_traj, int32_t* d_status, double* d_obj, int32_t* d_iters, void* stream) {
    return mpcg_solve_device_ex(h, B, d_state, d_coeffs, d_u0, d_traj, d_status, d_obj, d_iters, nullptr, stream);
}

int mpcg_solve_device_ex(mpcg_handle* h, int64_t B, const double* d_state, const double* d_coeffs, double* d_u0,
                         double* d_traj, int32_t* d_status, double* d_obj, int32_t* d_iters, int32_t* d_diag,
                         void* stream) {
    if (!h) return fail(-1, "null handle");
    if (B < 0) return fail(-1, "negative batch");
    if (B == 0) return 0;
    if (!d_state || !d_coeffs || !d_u0) return fail(-1, "state, coeffs and u0 are required");
    int rc = mpcg_params_check(&h->params);
    if (rc) return rc;
    hipError_t e = hipSetDevice(h->device);
    if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
    hipStream_t s = (hipStream_t)stream;  // NULL = the null stream, as in HIP
    const mpcg::IpmParams P = handle_ipm(h);
    if (!wave_fits(P)) return fail(-1, "STEPS must be <= 128 (the problem state must fit the CU's 160 KiB of LDS)");
    rc = ensure_spill(h, B);
    if (rc) return rc;
    if (B > kOrderMinBatch) {
        rc = ensure_sched(h, B);
        if (rc) return rc;
    }
    rc = order_on(h, s);
    if (rc) return rc;
    // batches larger than the resident wavefronts (8 per CU) are solved in
    // expected-longest-first order (launch_wide_order)
    const int32_t* order = nullptr;
    if (B > kOrderMinBatch) {
        int32_t* ord = nullptr;
        e = mpcg::launch_wide_order(B, d_coeffs, h->d_sched, h->sched_bytes, &ord, s);
        if (e != hipSuccess) return hip_fail(e, "solve-order sort");
        order = ord;
    }
    mpcg::WideStreams ws;
    ws.aux = h->aux;
    ws.aux2 = h->aux2;
    ws.ev_fork = h->ev_fork;
    ws.ev_join = h->ev_join;
    ws.ev_join2 = h->ev_join2;
    e = mpcg::launch_wide_solve(P, B, d_state, d_coeffs, d_u0, d_traj, d_status, d_obj, d_iters, d_diag, order,
                                (void*)h->d_spill, h->spill_bytes, s, ws, &h->last_kernel);
    if (e != hipSuccess) return hip_fail(e, "wide solve launch");
    h->last_ordered = order != nullptr;
    return record_on(h, s);
}

int mpcg_solve(mpcg_handle* h, int64_t B, const double* state, const double* coeffs, double* u0, double* traj,
               int32_t* status, double* obj, int32_t* iters) {
    return mpcg_solve_ex(h, B, state, coeffs, u0, traj, status, obj, iters, nullptr);
}

int mpcg_solve_ex(mpcg_handle* h, int64_t B, const double* state, const double* coeffs, double* u0, double* traj,
                  int32_t* status, double* obj, int32_t* iters, int32_t* diag) {
    if (!h) return fail(-1, "null handle");
    if (B < 0) return fail(-1, "negative batch");
    if (B == 0) return 0;
    if (!state || !coeffs || !u0) return fail(-1, "state, coeffs and u0 are required");
    int rc = mpcg_params_check(&h->params);
    if (rc) return rc;
    const int N = h->params.steps;
    // io block: state 6 | coeffs 4 | u0 2 | traj 3N | obj 1 | status+iters (2 int32 = 1 double) |
    // diag (4 int32 = 2 doubles)
    const size_t per = (size_t)(6 + 4 + 2 + 3 * N + 1 + 1 + 2);
    const size_t need = per * sizeof(double) * (size_t)B;
    hipError_t e = hipSetDevice(h->device);
    if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
    if (need > h->io_bytes) {
        if (h->d_io) {
            hipStreamSynchronize(h->stream);
            hipFree(h->d_io);
            h->d_io = nullptr;
            h->io_bytes = 0;
        }
        e = hipMalloc((void**)&h->d_io, need);
        if (e != hipSuccess) return hip_fail(e, "hipMalloc(io)");
        h->io_bytes = need;
    }
    double* ds = h->d_io;
    double* dc = ds + 6 * B;
    double* du = dc + 4 * B;
    double* dt = du + 2 * B;
    double* dob = dt + (size_t)3 * N * B;
    int32_t* dst = (int32_t*)(dob + B);
    int32_t* dit = dst + B;
    int32_t* ddg = dit + B;
    e = hipMemcpyAsync(ds, state, sizeof(double) * 6 * B, hipMemcpyHostToDevice, h->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(dc, coeffs, sizeof(double) * 4 * B, hipMemcpyHostToDevice, h->stream);
    if (e != hipSuccess) return hip_fail(e, "hipMemcpy H2D");
    rc = mpcg_solve_device_ex(h, B, ds, dc, du, dt, dst, dob, dit, diag ? ddg : nullptr, h->stream);
    if (rc) return rc;
    e = hipMemcpyAsync(u0, du, sizeof(double) * 2 * B, hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess && traj)
        e = hipMemcpyAsync(traj, dt, sizeof(double) * 3 * N * B, hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess && obj) e = hipMemcpyAsync(obj, dob, sizeof(double) * B, hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess && status)
        e = hipMemcpyAsync(status, dst, sizeof(int32_t) * B, hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess && iters)
        e = hipMemcpyAsync(iters, dit, sizeof(int32_t) * B, hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess && diag)
        e = hipMemcpyAsync(diag, ddg, sizeof(int32_t) * 4 * B, hipMemcpyDeviceToHost, h->stream);
    if (e != hipSuccess) return hip_fail(e, "hipMemcpy D2H");
    e = hipStreamSynchronize(h->stream);
    if (e != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
    return 0;
}

int mpcg_preprocess_device(mpcg_handle* h, int64_t B, int32_t M, const double* d_pose, const double* d_vel,
                           const double* d_plan, int32_t delay_mode, double* d_state, double* d_coeffs,
                           void* stream) {
    if (!h) return fail(-1, "null handle");
    if (B < 0) return fail(-1, "negative batch");
    if (B == 0) return 0;
    // findBestPath returns without solving for an empty plan (driving_state.cpp:182-185);
    // polyfit asserts order 3 <= M - 1 (:286); any longer plan is taken (beyond 64
    // waypoints through an HBM workspace)
    if (M < 4) return fail(-1, "M (waypoints per robot) must be >= 4");
    if (!d_pose || !d_vel || !d_plan || !d_state || !d_coeffs) return fail(-1, "null buffer");
    hipError_t e = hipSetDevice(h->device);
    if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
    hipStream_t s = (hipStream_t)stream;
    const size_t need = mpcg::find_best_path_ws_bytes(B, M);
    if (need > h->pp_bytes) {
        if (h->d_pp) {
            hipDeviceSynchronize();  // the old scratch may be in use on any stream
            hipFree(h->d_pp);
            h->d_pp = nullptr;
            h->pp_bytes = 0;
        }
        e = hipMalloc((void**)&h->d_pp, need);
        if (e != hipSuccess) return hip_fail(e, "hipMalloc(preprocessing scratch)");
        h->pp_bytes = need;
    }
    int rc = need ? order_on(h, s) : 0;
    if (rc) return rc;
    e = mpcg::launch_find_best_path(B, M, h->params.dt, delay_mode ? 1 : 0, d_pose, d_vel, d_plan, d_state,
                                    d_coeffs, h->d_pp, s);
    if (e != hipSuccess) return hip_fail(e, "find_best_path launch");
    return need ? record_on(h, s) : 0;
}

int mpcg_track_device(mpcg_handle* h, int64_t B, int32_t M, const double* d_pose, const double* d_vel,
                      const double* d_plan, int32_t delay_mode, double* d_cmd, double* d_traj, int32_t* d_status,
                      void* stream) {
    if (!h) return fail(-1, "null handle");
    if (B < 0) return fail(-1, "negative batch");
    if (B == 0) return 0;
    if (!d_cmd) return fail(-1, "cmd is required");
    hipError_t e = hipSetDevice(h->device);
    if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
    const size_t need = sizeof(double) * 12 * (size_t)B;
    if (need > h->trk_bytes) {
        if (h->d_trk) {
            hipDeviceSynchronize();  // the old buffers may be in use on any stream
            hipFree(h->d_trk);
            h->d_trk = nullptr;
            h->trk_bytes = 0;
        }
        e = hipMalloc((void**)&h->d_trk, need);
        if (e != hipSuccess) return hip_fail(e, "hipMalloc(track buffers)");
        h->trk_bytes = need;
    }
    double* st = h->d_trk;
    double* cf = st + 6 * B;
    double* u0 = cf + 4 * B;
    int rc = order_on(h, (hipStream_t)stream);
    if (rc) return rc;
    rc = mpcg_preprocess_device(h, B, M, d_pose, d_vel, d_plan, delay_mode, st, cf, stream);
    if (rc) return rc;
    rc = mpcg_solve_device(h, B, st, cf, u0, d_traj, d_status, nullptr, nullptr, stream);
    if (rc) return rc;
    e = mpcg::launch_post(B, h->params.dt, h->params.ref_v, d_vel, u0, d_cmd, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "post-processing launch");
    return record_on(h, (hipStream_t)stream);
}

const char* mpcg_last_kernel(const mpcg_handle* h) { return h ? h->last_kernel : ""; }
int mpcg_last_solve_order(const mpcg_handle* h) { return h ? h->last_ordered : 0; }

int mpcg_synth_infinity_device(mpcg_handle* h, uint64_t seed, int64_t start, int64_t B, int32_t M, double* d_pose,
                               double* d_vel, double* d_plan, void* stream) {
    if (!h) return fail(-1, "null handle");
    if (B < 0 || start < 0) return fail(-1, "negative batch or start");
    if (B == 0) return 0;
    if (M < 4) return fail(-1, "M (waypoints per robot) must be >= 4");
    if (!d_pose || !d_vel || !d_plan) return fail(-1, "null buffer");
    hipError_t e = hipSetDevice(h->device);
    if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
    const int n = mpcg::synth_arc_len();
    if (!h->d_arc) {
        std::vector<double> t, s;
        mpcg::synth_arc_table(t, s);
        e = hipMalloc((void**)&h->d_arc, sizeof(double) * 2 * n);
        if (e != hipSuccess) return hip_fail(e, "hipMalloc(arc table)");
        e = hipMemcpy(h->d_arc, t.data(), sizeof(double) * n, hipMemcpyHostToDevice);
        if (e == hipSuccess) e = hipMemcpy(h->d_arc + n, s.data(), sizeof(double) * n, hipMemcpyHostToDevice);
        if (e != hipSuccess) {
            hipFree(h->d_arc);
            h->d_arc = nullptr;
            return hip_fail(e, "hipMemcpy(arc table)");
        }
    }
    e = mpcg::launch_synth_infinity(seed, start, B, M, h->d_arc, h->d_arc + n, d_pose, d_vel, d_plan,
                                    (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "synthetic robots launch");
    return 0;
}

int mpcg_set_park_capacity(mpcg_handle* h, int64_t cap) {
    if (!h) return fail(-1, "null handle");
    if (cap < 0 || cap > (int64_t)1 << 30) return fail(-1, "park capacity must be in [0, 2^30]");
    h->park_cap = cap;
    return 0;
}

int mpcg_synchronize(mpcg_handle* h) {
    if (!h) return fail(-1, "null handle");
    hipSetDevice(h->device);
    hipError_t e = hipStreamSynchronize(h->stream);
    if (e != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
    return 0;
}

}  // extern "C"
