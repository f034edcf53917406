"""Diagnostic: a solve's fixed cost against its per-iteration cost (B = 65,536, N = 20 by default).

    python tools/fixed_cost_probe.py [N] [B] [bicycle]

Times the batch with max_iter = 0, 1, 2, 4, 8 and the reference's options (the iteration budget
stops every problem at that count; max_iter = 0 is set-up, the starting point, the least-squares
multipliers, one statistics sweep, the convergence test and the outputs)."""
import sys
import time
import numpy as np
import torch
sys.path.insert(0, ".")
from mpc_ros_amd import params  # noqa: E402
from mpc_ros_amd.solver import BatchSolver  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 20
B = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
P = dict(params.PLUGIN_DEFAULTS, STEPS=N)
if len(sys.argv) > 3 and sys.argv[3] == "bicycle":  # (bench.py's bicycle configuration)
    P.update(MODEL=1, LF=0.5, ANGVEL=0.5)
dev = torch.device("cuda:0")
for mi in (0, 1, 2, 4, 8, None):
    s = BatchSolver(0, P) if mi is None else BatchSolver(0, P, max_iter=mi)
    pose, vel, plan = s.synth_infinity_device(0, B)
    st = torch.empty((B, 6), dtype=torch.float64, device=dev)
    cf = torch.empty((B, 4), dtype=torch.float64, device=dev)
    s.preprocess_device(pose, vel, plan, st, cf)
    u0 = torch.empty((B, 2), dtype=torch.float64, device=dev)
    traj = torch.empty((B, 3, N), dtype=torch.float64, device=dev)
    iters = torch.empty(B, dtype=torch.int32, device=dev)
    s.reserve(B)
    ts = []
    for r in range(6):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        s.solve_device(st, cf, u0, traj=traj, iters=iters)
        torch.cuda.synchronize()
        if r:
            ts.append((time.perf_counter() - t0) * 1e3)
    it = iters.cpu().numpy()
    print(f"max_iter {mi}: {np.median(ts):.3f} ms, iters mean {it.mean():.2f} max {it.max()}, kernel {s.last_kernel}",
          flush=True)
