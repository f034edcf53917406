"""fp32 solver (N = 40) against the fp64 oracle on the first B infinity problems: the rows whose
controls differ by more than 1e-3, with their status, iterations and diagnostics; then the
kernel time of a 65,536-problem batch (diagnostic).

    python tools/fp32_diag.py [B] [option=value ...]   (options: mpcg_params fields, e.g. compl_inf_tol=1e-3)"""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from mpc_ros_amd import infinity, params  # noqa: E402
from mpc_ros_amd.solver import BatchSolver  # noqa: E402
from oracle import pyoracle as O  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
opts = {k: float(v) if "." in v or "e" in v else int(v) for k, v in (a.split("=") for a in sys.argv[2:])}
print("options:", opts)
P = dict(params.PLUGIN_DEFAULTS, STEPS=40)
st, cf = infinity.make_problems(np.arange(B))
ref = O.mpc_solve_batch(P, st, cf, opts=O.ref_opts(40), nthreads=16)
r = BatchSolver(0, P, dtype="fp32", **opts).solve(st, cf)
du = np.abs(r["u0"] - ref["u0"]).max(1)
bad = np.flatnonzero(du > 1e-3)
print("within 1e-3:", np.mean(du <= 1e-3), "median", np.median(du), "status counts:",
      dict(zip(*np.unique(r["status"], return_counts=True))))
print("escalated:", int((r["diag"][:, 2] == 3).sum()))
for b in bad[:40]:
    print(b, "fp32 status", r["status"][b], "iters", r["iters"][b], "diag", r["diag"][b].tolist(), "| fp64 status",
          ref["status"][b], "iters", ref["iters"][b], "| du", du[b], "dobj", r["obj"][b] - ref["obj"][b])

# kernel time at the configs[2] batch
Bt = 65536
st, cf = infinity.make_problems(np.arange(Bt))
s = BatchSolver(0, P, dtype="fp32", **opts)
dev = torch.device("cuda", 0)
tst, tcf = torch.from_numpy(st).to(dev), torch.from_numpy(cf).to(dev)
u0 = torch.empty((Bt, 2), dtype=torch.float64, device=dev)
status = torch.empty(Bt, dtype=torch.int32, device=dev)
iters = torch.empty(Bt, dtype=torch.int32, device=dev)
diag = torch.zeros((Bt, 4), dtype=torch.int32, device=dev)
s.reserve(Bt)
stream = torch.cuda.current_stream(dev)
ms = []
for i in range(6):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    s.solve_device(tst, tcf, u0, None, status, None, iters, stream=stream, diag=diag)
    e1.record(stream)
    torch.cuda.synchronize()
    if i >= 2:
        ms.append(e0.elapsed_time(e1))
sts = status.cpu().numpy()
print(f"B={Bt}: kernel ms {np.mean(ms):.2f} ({min(ms):.2f}..{max(ms):.2f}), status 1/4 {np.mean(np.isin(sts, (1, 4))):.5f}",
      dict(zip(*np.unique(sts, return_counts=True))), "escalated", int((diag.cpu().numpy()[:, 2] == 3).sum()),
      "iters mean", float(iters.float().mean()))
