"""Per-iteration cost of the structured oracle (oracle/ipm.c with kkt_structured: Ipopt's
iteration with its KKT system factored in stage order within the band) on one host
thread, at N = 20 and N = 40 -- the Ipopt-side term of the max_cpu_time model
(mpcg_api.cpp cpu_iter_budget; the CppAD derivative term is SURVEY.md §6's).

    python tools/cpu_iter_cost.py [problems]
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpc_ros_amd import infinity, params  # noqa: E402
from oracle import pyoracle as O  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 400
O.build()
model = "unknown"
with open("/proc/cpuinfo") as f:
    for line in f:
        if line.startswith("model name"):
            model = line.split(":", 1)[1].strip()
            break
out = {"cpu_model": model, "problems": n, "ms_per_iter": {}}
for N in (20, 40):
    P = dict(params.PLUGIN_DEFAULTS, STEPS=N)
    st, cf = infinity.make_problems(np.arange(n))
    o = O.ref_opts(N)
    o.kkt_structured = 1
    best = None
    for _ in range(3):
        t0 = time.perf_counter()
        r = O.mpc_solve_batch(P, st, cf, opts=o, nthreads=1)
        v = (time.perf_counter() - t0) / r["iters"].sum() * 1e3
        best = v if best is None else min(best, v)
    out["ms_per_iter"][str(N)] = best
print(json.dumps(out))
