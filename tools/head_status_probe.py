"""Diagnostic: the fp32 configuration at B = 65,536, N = 40 -- rows not ending at status 1, with
their place in the solve order (head rows first), repeated solves."""
import os
import sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpc_ros_amd import params  # noqa: E402
from mpc_ros_amd.solver import BatchSolver  # noqa: E402

B = 65536
P = dict(params.PLUGIN_DEFAULTS, STEPS=40)
dev = torch.device("cuda:0")
s = BatchSolver(0, P, dtype="fp32")
pose, vel, plan = s.synth_infinity_device(0, B)
st = torch.empty((B, 6), dtype=torch.float64, device=dev)
cf = torch.empty((B, 4), dtype=torch.float64, device=dev)
s.preprocess_device(pose, vel, plan, st, cf)
c = cf.cpu().numpy()
key = (np.abs(c[:, 1]) + np.abs(c[:, 2]) + np.abs(c[:, 3])).astype(np.float32)
rank = np.empty(B, int)
rank[np.argsort(-key, kind="stable")] = np.arange(B)
resto0 = None
for rep in range(int(os.environ.get('REPS', '4'))):
    u0 = torch.full((B, 2), -7.0, dtype=torch.float64, device=dev)
    status = torch.full((B,), -1, dtype=torch.int32, device=dev)
    iters = torch.full((B,), -1, dtype=torch.int32, device=dev)
    diag = torch.full((B, 4), -1, dtype=torch.int32, device=dev)
    s.solve_device(st, cf, u0, status=status, iters=iters, diag=diag)
    torch.cuda.synchronize()
    sts, it, dg = status.cpu().numpy(), iters.cpu().numpy(), diag.cpu().numpy()
    bad = np.flatnonzero(sts != 1)
    if rep == 0:
        resto0 = set(np.flatnonzero(dg[:, 0] > 0).tolist())
        print("rows through the restoration phase in rep 0:", len(resto0), "of them in the head:",
              sum(rank[i] < B // 1024 for i in resto0), flush=True)
    else:
        print("   unwritten rows that entered the restoration phase in rep 0:",
              sum(i in resto0 for i in bad.tolist()), "of", len(bad), flush=True)
    print(f"head rows {sorted(np.flatnonzero(rank < B // 1024).tolist())[:8]}...", flush=True)
    print(f"rep {rep}: statuses {dict(zip(*[x.tolist() for x in np.unique(sts, return_counts=True)]))}", flush=True)
    for i in bad[:10]:
        print(f"   row {i} rank {rank[i]} status {sts[i]} iters {it[i]} diag {dg[i].tolist()}", flush=True)
