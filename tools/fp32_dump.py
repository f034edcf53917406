"""Dump fp32-solver results on the infinity set (status, iters, u0) for offline analysis."""
import sys

import numpy as np

sys.path.insert(0, ".")
from mpc_ros_amd import infinity, params  # noqa: E402
from mpc_ros_amd.solver import BatchSolver  # noqa: E402

B = int(sys.argv[1])
out = sys.argv[2]
kw = {}
for a in sys.argv[3:]:
    k, v = a.split("=")
    kw[k] = float(v) if ("." in v or "e" in v) else int(v)
res = {}
for N in (20, 40):
    P = dict(params.PLUGIN_DEFAULTS, STEPS=N)
    st, cf = infinity.make_problems(np.arange(B))
    r = BatchSolver(0, P, dtype="fp32", **kw).solve(st, cf)
    for k in ("status", "iters", "u0"):
        res[f"N{N}_{k}"] = r[k]
    u, c = np.unique(r["status"], return_counts=True)
    print(N, dict(zip(u.tolist(), c.tolist())), "iters mean", r["iters"].mean(), "max", r["iters"].max(), flush=True)
np.savez(out, **res)
