// tests/native/mpc_class_check.cpp -- exercises the drop-in class MPC (include/mpc_planner.h)
// exactly as the reference's caller does (driving_state.cpp:65-80 builds the map,
// :260 calls Solve, :262-269 reads the result), with std::vector in place of
// Eigen::VectorXd (the Solve template accepts either).
//
// stdin: lines of state[6] coeffs[4]; stdout per line: w0 a0 mpc_x[N] last_status
#include <cstdio>
#include <map>
#include <string>
#include <vector>

#include "mpc_planner.h"

int main() {
    std::map<std::string, double> mpc_params;  // MPCPlanner.cfg defaults, DT = 0.1
    mpc_params["DT"] = 0.1;
    mpc_params["STEPS"] = 20;
    mpc_params["REF_CTE"] = 0.0;
    mpc_params["REF_ETHETA"] = 0.0;
    mpc_params["REF_V"] = 1.0;
    mpc_params["W_CTE"] = 1000;
    mpc_params["W_EPSI"] = 1000;
    mpc_params["W_V"] = 100;
    mpc_params["W_ANGVEL"] = 100;
    mpc_params["W_A"] = 50;
    mpc_params["W_DANGVEL"] = 0;
    mpc_params["W_DA"] = 10;
    mpc_params["ANGVEL"] = 1.0;
    mpc_params["MAXTHR"] = 1.0;
    mpc_params["BOUND"] = 1000;
    MPC mpc;
    mpc.LoadParams(mpc_params);
    std::vector<double> state(6), coeffs(4);
    while (true) {
        for (double& v : state)
            if (std::scanf("%lf", &v) != 1) return 0;
        for (double& v : coeffs)
            if (std::scanf("%lf", &v) != 1) return 1;
        std::vector<double> r = mpc.Solve(state, coeffs);
        std::printf("%.17g %.17g", r[0], r[1]);
        for (double x : mpc.mpc_x) std::printf(" %.17g", x);
        std::printf(" %d\n", mpc.last_status());
        std::fflush(stdout);
    }
}
