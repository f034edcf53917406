// mpc_ros_amd/csrc/mpc_planner.cpp -- the drop-in class MPC (include/mpc_planner.h).
//
// Same behaviour as mpc_ros/src/mpc_planner.cpp:
//  * constructor defaults of MPC::MPC() (:223-241);
//  * LoadParams stores the map and re-reads STEPS/ANGVEL/MAXTHR/BOUND, keeping the
//    previous value of each that is absent (:243-262);
//  * every Solve builds the FG_eval parameters from the FG_eval constructor
//    defaults (:42-68) overridden by the stored map (:351-352);
//  * Solve returns {w0, a0} and fills mpc_x/mpc_y/mpc_theta with N values
//    (:388-401); the solver status is not raised (:378) -- the last iterate is
//    returned, and the status is available through last_status().
// The solve itself runs on the GPU through the C-ABI (one problem per call here;
// SolveBatch for many).
#include "mpc_planner.h"

#include <cstdio>

MPC::MPC()
    : _max_angvel(3.0), _max_throttle(1.0), _bound_value(1.0e3), _mpc_steps(20), _device(0), _handle(nullptr),
      _last_status(0), _last_iters(0), _last_obj(0.0) {
    _x_start = 0;
    _y_start = _x_start + _mpc_steps;
    _theta_start = _y_start + _mpc_steps;
    _v_start = _theta_start + _mpc_steps;
    _cte_start = _v_start + _mpc_steps;
    _etheta_start = _cte_start + _mpc_steps;
    _angvel_start = _etheta_start + _mpc_steps;
    _a_start = _angvel_start + _mpc_steps - 1;
}

MPC::~MPC() {
    if (_handle) mpcg_destroy(_handle);
}

MPC::MPC(const MPC& o)
    : mpc_x(o.mpc_x), mpc_y(o.mpc_y), mpc_theta(o.mpc_theta), _max_angvel(o._max_angvel),
      _max_throttle(o._max_throttle), _bound_value(o._bound_value), _mpc_steps(o._mpc_steps), _x_start(o._x_start),
      _y_start(o._y_start), _theta_start(o._theta_start), _v_start(o._v_start), _cte_start(o._cte_start),
      _etheta_start(o._etheta_start), _angvel_start(o._angvel_start), _a_start(o._a_start), _params(o._params),
      _device(o._device), _handle(nullptr), _last_status(o._last_status), _last_iters(o._last_iters),
      _last_obj(o._last_obj) {}

MPC& MPC::operator=(const MPC& o) {
    if (this == &o) return *this;
    MPC tmp(o);
    std::swap(mpc_x, tmp.mpc_x);
    std::swap(mpc_y, tmp.mpc_y);
    std::swap(mpc_theta, tmp.mpc_theta);
    _max_angvel = o._max_angvel;
    _max_throttle = o._max_throttle;
    _bound_value = o._bound_value;
    _mpc_steps = o._mpc_steps;
    _x_start = o._x_start;
    _y_start = o._y_start;
    _theta_start = o._theta_start;
    _v_start = o._v_start;
    _cte_start = o._cte_start;
    _etheta_start = o._etheta_start;
    _angvel_start = o._angvel_start;
    _a_start = o._a_start;
    _params = o._params;
    _device = o._device;
    _last_status = o._last_status;
    _last_iters = o._last_iters;
    _last_obj = o._last_obj;
    return *this;  // keeps its own GPU handle
}

void MPC::LoadParams(const std::map<string, double>& params) {
    _params = params;
    auto it = _params.find("STEPS");
    if (it != _params.end()) _mpc_steps = (int)it->second;
    it = _params.find("ANGVEL");
    if (it != _params.end()) _max_angvel = it->second;
    it = _params.find("MAXTHR");
    if (it != _params.end()) _max_throttle = it->second;
    it = _params.find("BOUND");
    if (it != _params.end()) _bound_value = it->second;
    _x_start = 0;
    _y_start = _x_start + _mpc_steps;
    _theta_start = _y_start + _mpc_steps;
    _v_start = _theta_start + _mpc_steps;
    _cte_start = _v_start + _mpc_steps;
    _etheta_start = _cte_start + _mpc_steps;
    _angvel_start = _etheta_start + _mpc_steps;
    _a_start = _angvel_start + _mpc_steps - 1;
}

mpcg_params MPC::effective_params() const {
    mpcg_params p;
    mpcg_params_default(&p);  // FG_eval constructor defaults for the FG keys
    for (const auto& kv : _params) {
        if (kv.first == "STEPS" || kv.first == "ANGVEL" || kv.first == "MAXTHR" || kv.first == "BOUND") continue;
        mpcg_params_set(&p, kv.first.c_str(), kv.second);
    }
    p.steps = _mpc_steps;
    p.max_angvel = _max_angvel;
    p.max_throttle = _max_throttle;
    p.bound = _bound_value;
    return p;
}

int MPC::ensure_handle() {
    if (!_handle) {
        int rc = mpcg_create(_device, &_handle);
        if (rc) {
            std::fprintf(stderr, "[MPC] mpcg_create failed: %s\n", mpcg_last_error());
            _handle = nullptr;
            return rc;
        }
    }
    mpcg_params p = effective_params();
    int rc = mpcg_set_params(_handle, &p);
    if (rc) std::fprintf(stderr, "[MPC] invalid parameters: %s\n", mpcg_last_error());
    return rc;
}

vector<double> MPC::SolveRaw(const double* state, const double* coeffs) {
    vector<double> result(2, 0.0);
    if (ensure_handle() != 0) {
        _last_status = 13;  // internal_error
        return result;
    }
    const int N = _mpc_steps;
    vector<double> traj(3 * (size_t)N);
    double u0[2] = {0, 0}, obj = 0;
    int32_t status = 0, iters = 0;
    int rc = mpcg_solve(_handle, 1, state, coeffs, u0, traj.data(), &status, &obj, &iters);
    if (rc) {
        std::fprintf(stderr, "[MPC] solve failed: %s\n", mpcg_last_error());
        _last_status = 13;
        return result;
    }
    _last_status = status;
    _last_iters = iters;
    _last_obj = obj;
    mpc_x.assign(traj.begin(), traj.begin() + N);
    mpc_y.assign(traj.begin() + N, traj.begin() + 2 * N);
    mpc_theta.assign(traj.begin() + 2 * N, traj.end());
    result[0] = u0[0];
    result[1] = u0[1];
    return result;
}

int MPC::SolveBatch(int64_t B, const double* state, const double* coeffs, double* u0, double* traj,
                    int32_t* status) {
    int rc = ensure_handle();
    if (rc) return rc;
    return mpcg_solve(_handle, B, state, coeffs, u0, traj, status, nullptr, nullptr);
}
