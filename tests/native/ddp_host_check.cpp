// tests/native/ddp_host_check.cpp -- TEST HARNESS ONLY.
//
// Runs the device solver core (mpc_ros_amd/csrc/ddp_core.h) on the host, one
// problem at a time, so the CPU test suite can check the algorithm against the
// oracle without a GPU.  It is compiled by tests/ into a temporary directory and is
// never part of the product library (the product has no CPU path).
//
// stdin:  N dt ref_cte ref_eth ref_v w_cte w_eth w_v w_w w_a w_dw w_da max_w max_a bound tol max_iter
//         B, then B x (state[6], coeffs[4])
// stdout: per problem: status iters obj u0[2] traj[3N]
#include <cmath>
#include <cstdio>
#include <vector>

#include "../../mpc_ros_amd/csrc/ddp_core.h"

int main() {
    mpcg::SolverParams P{};
    if (std::scanf("%d %lf %lf %lf %lf %lf %lf %lf %lf %lf %lf %lf %lf %lf %lf %lf %d", &P.N, &P.dt, &P.ref_cte,
                   &P.ref_eth, &P.ref_v, &P.w_cte, &P.w_eth, &P.w_v, &P.w_w, &P.w_a, &P.w_dw, &P.w_da, &P.max_w,
                   &P.max_a, &P.bound, &P.tol, &P.max_iter) != 17)
        return 1;
    P.relax = 1e-8;
    P.max_ls = 12;
    long B;
    if (std::scanf("%ld", &B) != 1) return 1;
    mpcg::Layout L{P.N};
    std::vector<double> buf(L.total());
    for (long b = 0; b < B; ++b) {
        double s[6], c[4];
        for (double& v : s) std::scanf("%lf", &v);
        for (double& v : c) std::scanf("%lf", &v);
        mpcg::Problem<double> pr{s[0], s[1], s[2], s[3], s[4], s[5], c[0], c[1], c[2], c[3], 0, 0, 0};
        pr.ce = s[5] - s[2];
        pr.sce = std::sin(pr.ce);
        pr.cce = std::cos(pr.ce);
        mpcg::Ws<double> ws{buf.data(), 1};
        int cur;
        double obj;
        mpcg::SolveOut o = mpcg::solve_one(P, pr, ws, &cur, &obj);
        double w0 = ws[L.W(cur, 0)], a0 = ws[L.A(cur, 0)];
        w0 = std::fmin(std::fmax(w0, -P.max_w), P.max_w);
        a0 = std::fmin(std::fmax(a0, -P.max_a), P.max_a);
        std::printf("%d %d %.17g %.17g %.17g", o.status, o.iters, obj, w0, a0);
        for (int k = 0; k < P.N; ++k) std::printf(" %.17g", ws[L.X(cur, k)]);
        for (int k = 0; k < P.N; ++k) std::printf(" %.17g", ws[L.Y(cur, k)]);
        for (int k = 0; k < P.N; ++k) std::printf(" %.17g", ws[L.TH(cur, k)]);
        std::printf("\n");
    }
    return 0;
}
