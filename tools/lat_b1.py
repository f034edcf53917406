"""Diagnostic: the B = 1 device path (bench.py latency_b1) repeated, for a kernel trace
(rocprofv3 --kernel-trace): which launches one solve makes and the gaps between them."""
import sys
import time
import numpy as np
import torch
import os  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpc_ros_amd import params  # noqa: E402
from mpc_ros_amd.solver import BatchSolver  # noqa: E402

P = dict(params.PLUGIN_DEFAULTS)
idx = int(sys.argv[1]) if len(sys.argv) > 1 else 0  # (the bench's infinity-set problem, device generator)
dev = torch.device("cuda:0")
s = BatchSolver(0, P)
pose, vel, plan = s.synth_infinity_device(idx, 1)
ts = torch.empty((1, 6), dtype=torch.float64, device=dev)
tc = torch.empty((1, 4), dtype=torch.float64, device=dev)
s.preprocess_device(pose, vel, plan, ts, tc)
u = torch.empty((1, 2), dtype=torch.float64, device=dev)
it = torch.empty(1, dtype=torch.int32, device=dev)
ms = []
for r in range(60):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    s.solve_device(ts, tc, u, iters=it)
    torch.cuda.synchronize()
    ms.append((time.perf_counter() - t0) * 1e3)
print(f"B = 1, problem {idx}: median {np.median(ms[10:]):.4f} ms, iterations {int(it.item())}, kernel {s.last_kernel}")
