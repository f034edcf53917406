"""configs[2] (B = 65,536, N = 40, fp32 two-phase) with the fp32 phase's iteration limit lowered
(diagnostic, GPU): a row that reaches it is solved by the fp64 phase from the start.  Prints, per
limit, the launch time (HIP events, median of 5), the rows solved from the start, and the rows
whose objective differs from the fp64 solver's by more than 1e-6 relative (another local minimum).
With a diagnostic build (MPCG_EXTRA_CFLAGS=-DMPCG_HEAD_ENV) and HEAD_DIVS=1024,256,..., each limit
is also run with the head (the rows solved in fp64 from the start while the fp32 phase runs) at
B / div.

    [HEAD_DIVS=1024,256] python tools/fp32_maxiter_probe.py [limits, e.g. 300,100,80,60]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from mpc_ros_amd import params  # noqa: E402
from mpc_ros_amd.solver import BatchSolver  # noqa: E402


def main():
    limits = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "300,100,80,60").split(",")]
    B, N = 65536, 40
    dev = torch.device("cuda:0")
    P = dict(params.PLUGIN_DEFAULTS, STEPS=N)
    ref = BatchSolver(0, P)
    pose, vel, plan = ref.synth_infinity_device(0, B)
    st = torch.empty((B, 6), dtype=torch.float64, device=dev)
    cf = torch.empty((B, 4), dtype=torch.float64, device=dev)
    ref.preprocess_device(pose, vel, plan, st, cf)
    u0 = torch.empty((B, 2), dtype=torch.float64, device=dev)
    status = torch.empty(B, dtype=torch.int32, device=dev)
    obj = torch.empty(B, dtype=torch.float64, device=dev)
    iters = torch.empty(B, dtype=torch.int32, device=dev)
    diag = torch.empty((B, 4), dtype=torch.int32, device=dev)
    ref.solve_device(st, cf, u0, status=status, obj=obj, diag=diag)
    torch.cuda.synchronize()
    o64, u64 = obj.cpu().numpy(), u0.cpu().numpy()
    divs = [d for d in os.environ.get("HEAD_DIVS", "").split(",") if d] or [None]
    for div, lim in [(d, m) for d in divs for m in limits]:
        if div is not None:
            os.environ["MPCG_HEAD_DIV"] = div  # (read by the library at each solve and reserve)
        s = BatchSolver(0, P, dtype="fp32", max_iter=lim)
        s.reserve(B)
        ts = []
        for r in range(6):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            s.solve_device(st, cf, u0, status=status, obj=obj, iters=iters, diag=diag)
            e1.record()
            torch.cuda.synchronize()
            if r:
                ts.append(e0.elapsed_time(e1))
        o, u, dg = obj.cpu().numpy(), u0.cpu().numpy(), diag.cpu().numpy()
        om = np.flatnonzero(np.abs(o - o64) > 1e-6 * np.abs(o64))
        du = np.abs(u - u64).max(1)
        print(f"head B/{div or 1024}, max_iter {lim}: {np.median(ts):.2f} ms, from start {int((dg[:, 2] == 3).sum())}, continued "
              f"{int((dg[:, 2] == 4).sum())}, other minima {om.tolist()}, max |du0| {du.max():.2e}, "
              f"status {np.unique(status.cpu().numpy()).tolist()}", flush=True)
        s.close()


if __name__ == "__main__":
    main()
