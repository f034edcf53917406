"""Diagnostic: the B = 1 device path (bench.py latency_b1) repeated, for a kernel trace
(rocprofv3 --kernel-trace): which launches one solve makes and the gaps between them."""
import sys
import time
import numpy as np
import torch
import os  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpc_ros_amd import infinity, params  # noqa: E402
from mpc_ros_amd.solver import BatchSolver  # noqa: E402

P = dict(params.PLUGIN_DEFAULTS)
st, cf = infinity.make_problems(np.arange(1))
dev = torch.device("cuda:0")
s = BatchSolver(0, P)
ts, tc = torch.from_numpy(st).to(dev), torch.from_numpy(cf).to(dev)
u = torch.empty((1, 2), dtype=torch.float64, device=dev)
it = torch.empty(1, dtype=torch.int32, device=dev)
ms = []
for r in range(60):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    s.solve_device(ts, tc, u, iters=it)
    torch.cuda.synchronize()
    ms.append((time.perf_counter() - t0) * 1e3)
print(f"B = 1: median {np.median(ms[10:]):.4f} ms, iterations {int(it.item())}, kernel {s.last_kernel}")
