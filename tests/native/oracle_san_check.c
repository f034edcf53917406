/* tests/native/oracle_san_check.c -- the oracle's C code under AddressSanitizer and
 * UndefinedBehaviorSanitizer (tests/test_sanitizers.py builds it with
 * -fsanitize=address,undefined; test infrastructure only).
 *
 * Runs HS071, a few MPC problems through the dense and the structured (envelope) KKT
 * paths with every Ipopt mechanism on, one problem that enters the restoration phase
 * path (a huge finite state), and findBestPath on a plan longer than 64 waypoints
 * (heap arrays).  Prints one line per case; exits non-zero on a failed solve. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include "ora.h"

int main(void) {
    ora_ipm_opts o;
    ora_ipm_default_opts(&o);
    double x[4], zl[4], zu[4];
    int it = 0;
    int st = ora_hs071_solve(&o, x, zl, zu, &it);
    printf("hs071 status %d iters %d x %.6f %.6f %.6f %.6f\n", st, it, x[0], x[1], x[2], x[3]);
    if (st != ORA_SUCCESS) return 1;

    ora_mpc_params p = {20, 0.1, 0.0, 0.0, 1.0, 1000, 1000, 100, 100, 50, 0, 10, 1.0, 1.0, 1000, 0, 0.5};
    const double states[3][6] = {{0.05, 0.0, 0.02, 0.4, 0.1, 0.05}, {0.1, 0.0, 0.2, 0.9, -0.3, 0.4},
                                 {1e300, 0.0, 0.0, 0.5, 0.0, 0.0}};
    const double coeffs[4] = {0.1, 0.02, -0.01, 0.001};
    for (int mode = 0; mode < 2; ++mode) {
        o.kkt_structured = mode;
        for (int b = 0; b < 3; ++b) {
            double u0[2], traj[60], obj = 0, kkt = 0;
            int iters = 0;
            const int s = ora_mpc_solve(&p, &o, states[b], coeffs, u0, traj, &obj, &iters, &kkt, NULL);
            printf("mpc kkt_structured %d problem %d status %d iters %d u0 %.9f %.9f\n", mode, b, s, iters, u0[0], u0[1]);
            if (b < 2 && s != ORA_SUCCESS) return 2;
        }
    }
    const int M = 150;
    double* plan = (double*)malloc(sizeof(double) * 2 * M);
    for (int i = 0; i < M; ++i) {
        plan[2 * i] = 0.05 * i;
        plan[2 * i + 1] = 0.3 * sin(0.02 * i);
    }
    double state[6], c4[4];
    const int rc = ora_find_best_path(0.0, 0.0, 0.1, 0.5, 0.1, 0.2, 0.1, M, plan, 1, state, c4);
    printf("find_best_path M %d rc %d coeffs %.9f %.9f %.9f %.9f\n", M, rc, c4[0], c4[1], c4[2], c4[3]);
    free(plan);
    return rc == 0 ? 0 : 3;
}
