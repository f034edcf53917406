/*
 * include/mpc_planner.h -- drop-in replacement of the reference's
 * mpc_ros/include/mpc_planner.h (class MPC, :26-47), backed by libmpcg.so.
 *
 * The move_base plugin (mpc_ros/src/mpc_planner_ros.cpp) and the driving-state
 * FSM (mpc_ros/src/driving_state.cpp:260) compile against this header unchanged:
 *   MPC();  void LoadParams(const std::map<string,double>&);
 *   vector<double> Solve(Eigen::VectorXd state, Eigen::VectorXd coeffs);  -> {w0, a0}
 *   vector<double> mpc_x, mpc_y, mpc_theta;
 * Solve is a template over the vector type so that Eigen::VectorXd (when the caller
 * has Eigen) and std::vector<double> both work; arguments are taken by value, as in
 * the reference.  Extensions: SolveBatch (B robots per call) and the last solve's
 * status / iteration count / objective.
 */
#ifndef MPCG_MPC_PLANNER_H
#define MPCG_MPC_PLANNER_H

#include <map>
#include <string>
#include <vector>

#include "mpcg.h"

using namespace std;  // the reference header does this (mpc_planner.h:24); kept for source compatibility

class MPC {
   public:
    MPC();
    ~MPC();
    MPC(const MPC& o);             // DrivingStateContext::getMpc() copies (driving_state.h:79)
    MPC& operator=(const MPC& o);

    // Solve the model given an initial state and polynomial coefficients.
    // Return the first actuations {angular velocity, acceleration}.
    template <class Vec>
    vector<double> Solve(Vec state, Vec coeffs) {
        double s[6], c[4];
        for (int i = 0; i < 6; ++i) s[i] = static_cast<double>(state[i]);
        for (int i = 0; i < 4; ++i) c[i] = static_cast<double>(coeffs[i]);
        return SolveRaw(s, c);
    }
    vector<double> mpc_x;
    vector<double> mpc_y;
    vector<double> mpc_theta;

    void LoadParams(const std::map<string, double>& params);

    // ---- extensions (not in the reference) ----
    // B problems in one GPU launch; state [B][6], coeffs [B][4], u0 [B][2],
    // traj [B][3][N] (or null), status [B] (or null).  Returns 0 or a negative mpcg code.
    int SolveBatch(int64_t B, const double* state, const double* coeffs, double* u0, double* traj,
                   int32_t* status);
    int last_status() const { return _last_status; }
    int last_iters() const { return _last_iters; }
    double last_obj() const { return _last_obj; }
    int steps() const { return _mpc_steps; }
    // GPU the solver runs on (default 0); call before the first Solve.
    void set_device(int device) { _device = device; }

   private:
    vector<double> SolveRaw(const double* state, const double* coeffs);
    int ensure_handle();
    mpcg_params effective_params() const;

    // Parameters for mpc solver (same members as the reference, mpc_planner.h:40-43)
    double _max_angvel, _max_throttle, _bound_value;
    int _mpc_steps, _x_start, _y_start, _theta_start, _v_start, _cte_start, _etheta_start, _angvel_start, _a_start;
    std::map<string, double> _params;

    int _device;
    mpcg_handle* _handle;
    int _last_status, _last_iters;
    double _last_obj;
};

#endif /* MPCG_MPC_PLANNER_H */
