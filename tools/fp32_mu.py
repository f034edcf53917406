"""Diagnostic (a build with -DMPCG_DEBUG_MU): the fp32 solver's exit barrier parameter and
complementarity against |u0 - u0_fp64| on the first B infinity problems at N = 40."""
import sys
import numpy as np
sys.path.insert(0, ".")
from mpc_ros_amd import infinity, params  # noqa: E402
from mpc_ros_amd.solver import BatchSolver  # noqa: E402
from oracle import pyoracle as O  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
P = dict(params.PLUGIN_DEFAULTS, STEPS=40)
st, cf = infinity.make_problems(np.arange(B))
ref = O.mpc_solve_batch(P, st, cf, opts=O.ref_opts(40), nthreads=16)
r = BatchSolver(0, P, dtype="fp32").solve(st, cf)
du = np.abs(r["u0"] - ref["u0"]).max(1)
d = r["diag"]
fp32 = d[:, 2] != 3
mu = 10.0 ** (-d[:, 1] / 100.0)
cm = 10.0 ** (-d[:, 3] / 100.0)
print("rows", B, "escalated", int((~fp32).sum()))
for lo, hi in ((0, 1e-6), (1e-6, 1e-5), (1e-5, 3e-5), (3e-5, 1e-4), (1e-4, 3e-4), (3e-4, 1e-3), (1e-3, 1)):
    m = fp32 & (mu >= lo) & (mu < hi)
    if m.any():
        print(f"mu [{lo:.0e},{hi:.0e}): n {m.sum():5d}  du max {du[m].max():.2e} p99 {np.quantile(du[m], .99):.2e} "
              f">1e-4 {(du[m] > 1e-4).sum()} >1e-3 {(du[m] > 1e-3).sum()}")
for lo, hi in ((0, 1e-5), (1e-5, 1e-4), (1e-4, 1e-3), (1e-3, 3e-3), (3e-3, 1e-2), (1e-2, 1)):
    m = fp32 & (cm >= lo) & (cm < hi)
    if m.any():
        print(f"compl [{lo:.0e},{hi:.0e}): n {m.sum():5d}  du max {du[m].max():.2e} >1e-4 {(du[m] > 1e-4).sum()} "
              f">1e-3 {(du[m] > 1e-3).sum()}")
bad = np.flatnonzero(fp32 & (du > 1e-4))
for b in bad[:30]:
    print(b, "status", r["status"][b], "iters", r["iters"][b], "fp64 iters", ref["iters"][b], f"mu {mu[b]:.2e} compl {cm[b]:.2e} du {du[b]:.2e}")
