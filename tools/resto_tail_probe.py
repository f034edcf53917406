"""Diagnostic: configs[2]'s fp64-phase tail.  Finds the longest problems the fp64 phase solves from
the start (B = 65,536, N = 40, fp32 configuration) and times each alone in fp64 (B = 1), next to
the longest problems without a restoration phase, for the per-iteration cost of the parked
(k_resume_wide) part against the batch instance."""
import os
import sys
import time
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpc_ros_amd import params  # noqa: E402
from mpc_ros_amd.solver import BatchSolver  # noqa: E402

N, B = 40, 65536
P = dict(params.PLUGIN_DEFAULTS, STEPS=N)
dev = torch.device("cuda:0")


def batch(s):
    pose, vel, plan = s.synth_infinity_device(0, B)
    st = torch.empty((B, 6), dtype=torch.float64, device=dev)
    cf = torch.empty((B, 4), dtype=torch.float64, device=dev)
    s.preprocess_device(pose, vel, plan, st, cf)
    u0 = torch.empty((B, 2), dtype=torch.float64, device=dev)
    it = torch.empty(B, dtype=torch.int32, device=dev)
    dg = torch.empty((B, 4), dtype=torch.int32, device=dev)
    s.solve_device(st, cf, u0, iters=it, diag=dg)
    torch.cuda.synchronize()
    return it.cpu().numpy(), dg.cpu().numpy()


def alone(s, i, reps=5):
    pose, vel, plan = s.synth_infinity_device(int(i), 1)
    st = torch.empty((1, 6), dtype=torch.float64, device=dev)
    cf = torch.empty((1, 4), dtype=torch.float64, device=dev)
    s.preprocess_device(pose, vel, plan, st, cf)
    u0 = torch.empty((1, 2), dtype=torch.float64, device=dev)
    it = torch.empty(1, dtype=torch.int32, device=dev)
    dg = torch.empty((1, 4), dtype=torch.int32, device=dev)
    ts = []
    for r in range(reps + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        s.solve_device(st, cf, u0, iters=it, diag=dg)
        torch.cuda.synchronize()
        if r:
            ts.append((time.perf_counter() - t0) * 1e3)
    return float(np.median(ts)), int(it.item()), dg.cpu().numpy()[0].tolist()


s64 = BatchSolver(0, P)
it2, dg2 = batch(BatchSolver(0, P, dtype="fp32"))
it64, dg64 = batch(s64)
cold = np.flatnonzero(dg2[:, 2] == 3)
top = cold[np.argsort(-it2[cold])][:4]
plain = np.flatnonzero(dg64[:, 0] == 0)
topp = plain[np.argsort(-it64[plain])][:3]
for name, rows in (("from-start rows of the fp64 phase", top), ("longest fp64 rows without restoration", topp)):
    print(name, flush=True)
    for i in rows:
        ms, it, dg = alone(s64, i)
        print(f"  problem {i}: alone {ms:.3f} ms, {it} iterations ({1e3 * ms / max(it, 1):.1f} us each), "
              f"restoration phases {dg[0]}, parked {dg[2]}", flush=True)
