// oracle/ref_probe/cppad_fg.cpp -- derivative probe (TEST INFRASTRUCTURE ONLY).
//
// The reference's MPC path (mpc_ros/src/mpc_planner.cpp) does not build here: it
// needs Eigen/Core and Ipopt's coin/ headers, neither of which is in the image
// (SURVEY.md §8c).  Its AD layer -- the vendored CppAD cppad-20180000.0
// (mpc_ros/include/cppad/configure.hpp:63) -- does build standalone, so this probe
// tapes the NLP of FG_eval::operator() (mpc_planner.cpp:102-217) with the
// reference's own CppAD and prints f, g, grad f, J_g and the Lagrangian Hessian at
// given points.  tests/golden/make_goldens.py turns the output into fixtures that
// pin oracle/nlp_mpc.c's analytic derivatives (and, through the same fixtures,
// the GPU kernel's cost/constraint evaluation).
//
// Built by `make -C oracle ref` into oracle/_ref/ with -I/root/reference/mpc_ros/include;
// nothing from the reference tree is copied.
//
// stdin:  N dt ref_cte ref_eth ref_v w_cte w_eth w_v w_w w_a w_dw w_da   (12 numbers)
//         K                                                              (number of points)
//         K x [ c0 c1 c2 c3 | vars (8N-2) | sigma | lambda (6N) ]
// stdout: per point: fg (1+6N), jac of fg ((1+6N) x (8N-2), row 0 = grad f), hess (nx x nx)
#include <cppad/cppad.hpp>
#include <cstdio>
#include <vector>

using CppAD::AD;

struct Weights {
    int N;
    double dt, ref_cte, ref_eth, ref_v, w_cte, w_eth, w_v, w_w, w_a, w_dw, w_da;
};

// Same objective/constraint vector as FG_eval::operator(), written over a generic
// scalar so that CppAD records it.  CppAD::pow(AD, int) is used where the reference
// uses it (pow_int, cppad/utility/pow_int.hpp), including the k = 0 term of f(x).
template <class S>
static void nlp_fg(const Weights& P, const double* c, const std::vector<S>& z, std::vector<S>& out) {
    const int N = P.N;
    const int X = 0, Y = N, TH = 2 * N, V = 3 * N, CTE = 4 * N, ETH = 5 * N, W = 6 * N, A = 7 * N - 1;
    S cost = 0.0;
    for (int i = 0; i < N; ++i) {
        cost += P.w_cte * CppAD::pow(z[CTE + i] - P.ref_cte, 2);
        cost += P.w_eth * CppAD::pow(z[ETH + i] - P.ref_eth, 2);
        cost += P.w_v * CppAD::pow(z[V + i] - P.ref_v, 2);
    }
    for (int i = 0; i + 1 < N; ++i) cost += P.w_w * CppAD::pow(z[W + i], 2) + P.w_a * CppAD::pow(z[A + i], 2);
    for (int i = 0; i + 2 < N; ++i)
        cost += P.w_dw * CppAD::pow(z[W + i + 1] - z[W + i], 2) + P.w_da * CppAD::pow(z[A + i + 1] - z[A + i], 2);
    out[0] = cost;
    const int starts[6] = {X, Y, TH, V, CTE, ETH};
    for (int s = 0; s < 6; ++s) out[1 + starts[s]] = z[starts[s]];
    for (int i = 0; i + 1 < N; ++i) {
        S poly = 0.0;
        for (int k = 0; k < 4; ++k) poly += c[k] * CppAD::pow(z[X + i], k);
        out[2 + X + i] = z[X + i + 1] - (z[X + i] + z[V + i] * CppAD::cos(z[TH + i]) * P.dt);
        out[2 + Y + i] = z[Y + i + 1] - (z[Y + i] + z[V + i] * CppAD::sin(z[TH + i]) * P.dt);
        out[2 + TH + i] = z[TH + i + 1] - (z[TH + i] + z[W + i] * P.dt);
        out[2 + V + i] = z[V + i + 1] - (z[V + i] + z[A + i] * P.dt);
        out[2 + CTE + i] = z[CTE + i + 1] - ((poly - z[Y + i]) + z[V + i] * CppAD::sin(z[ETH + i]) * P.dt);
        out[2 + ETH + i] = z[ETH + i + 1] - (z[ETH + i] + z[W + i] * P.dt);
    }
}

int main() {
    Weights P;
    if (std::scanf("%d %lf %lf %lf %lf %lf %lf %lf %lf %lf %lf %lf", &P.N, &P.dt, &P.ref_cte, &P.ref_eth,
                   &P.ref_v, &P.w_cte, &P.w_eth, &P.w_v, &P.w_w, &P.w_a, &P.w_dw, &P.w_da) != 12)
        return 1;
    int K;
    if (std::scanf("%d", &K) != 1) return 1;
    const int nx = 8 * P.N - 2, ng = 6 * P.N;
    for (int k = 0; k < K; ++k) {
        double c[4];
        for (int i = 0; i < 4; ++i)
            if (std::scanf("%lf", &c[i]) != 1) return 2;
        std::vector<double> x(nx), w(1 + ng);
        for (int i = 0; i < nx; ++i)
            if (std::scanf("%lf", &x[i]) != 1) return 2;
        for (int i = 0; i < 1 + ng; ++i)
            if (std::scanf("%lf", &w[i]) != 1) return 2;
        std::vector<AD<double>> ax(nx), afg(1 + ng);
        for (int i = 0; i < nx; ++i) ax[i] = x[i];
        CppAD::Independent(ax);
        nlp_fg(P, c, ax, afg);
        CppAD::ADFun<double> F(ax, afg);
        F.optimize();
        std::vector<double> fg = F.Forward(0, x);
        std::vector<double> jac = F.Jacobian(x);
        std::vector<double> hes = F.Hessian(x, w);
        for (double v : fg) std::printf("%.17g\n", v);
        for (double v : jac) std::printf("%.17g\n", v);
        for (double v : hes) std::printf("%.17g\n", v);
    }
    return 0;
}
