// tests/native/ipm_host_check.cpp -- TEST HARNESS ONLY.
//
// Runs the device solver core (mpc_ros_amd/csrc/ipm_core.h) on the host, one
// problem at a time, so the CPU test suite can check the algorithm against the
// oracle (oracle/ipm.c) without a GPU.  Compiled by tests/ into a temporary
// directory; never part of the product library (the product has no CPU path).
//
// stdin:  N dt ref_cte ref_eth ref_v w_cte w_eth w_v w_w w_a w_dw w_da max_w max_a bound tol max_iter
//         B, then B x (state[6], coeffs[4])
// stdout: per problem: status iters obj u0[2] traj[3N]
#include <cmath>
#include <cstdio>
#include <vector>

#include "../../mpc_ros_amd/csrc/ipm_core.h"

// single-problem workspace: the pair-interleaved layout degenerates to identity
struct HostWs {
    double* base;
    double ld(int e) const { return base[e]; }
    void st(int e, double v) const { base[e] = v; }
    void ld2(int e, double& a, double& b) const { a = base[e]; b = base[e + 1]; }
    void st2(int e, double a, double b) const { base[e] = a; base[e + 1] = b; }
};

int main() {
    mpcg::IpmParams P{};
    if (std::scanf("%d %lf %lf %lf %lf %lf %lf %lf %lf %lf %lf %lf %lf %lf %lf %lf %d", &P.N, &P.dt, &P.ref_cte,
                   &P.ref_eth, &P.ref_v, &P.w_cte, &P.w_eth, &P.w_v, &P.w_w, &P.w_a, &P.w_dw, &P.w_da, &P.max_w,
                   &P.max_a, &P.bound, &P.tol, &P.max_iter) != 17)
        return 1;
    P.bound_relax_factor = 1e-8;
    P.mu_init = 0.1;
    P.filter_cap = 64;
    P.model = 0;
    P.lf = 0.5;
    int model;
    if (std::scanf("%d %lf", &model, &P.lf) != 2) return 1;
    if (model != 0) return 2;  // the lane solver implements the differential drive only
    long B;
    if (std::scanf("%ld", &B) != 1) return 1;
    mpcg::IpmLayout L{P.N};
    (void)L;
    std::vector<double> buf(L.total(P.filter_cap));
    for (long b = 0; b < B; ++b) {
        mpcg::IpmProblem<double> pr;
        for (double& v : pr.init) std::scanf("%lf", &v);
        for (double& v : pr.c) std::scanf("%lf", &v);
        HostWs ws{buf.data()};
        mpcg::IpmSolver<double, HostWs> S(P, pr, ws);
        mpcg::IpmResult r = S.solve();
        std::printf("%d %d %.17g %.17g %.17g", r.status, r.iters, S.objective_out(), S.x_ctrl(0, 0),
                    S.x_ctrl(1, 0));
        for (int s = 0; s < 3; ++s)
            for (int k = 0; k < P.N; ++k) std::printf(" %.17g", S.x_state(s, k));
        std::printf("\n");
    }
    return 0;
}
