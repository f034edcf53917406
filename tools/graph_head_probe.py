"""Diagnostic: capture one solve in a HIP graph and replay it (mode: fp64 B / fp32 B), comparing
with the eager solve.  python tools/graph_head_probe.py fp32 4096"""
import os
import sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpc_ros_amd import infinity, params  # noqa: E402
from mpc_ros_amd.solver import BatchSolver  # noqa: E402

dt, B = sys.argv[1], int(sys.argv[2])
N = int(sys.argv[3]) if len(sys.argv) > 3 else 40
P = dict(params.PLUGIN_DEFAULTS, STEPS=N)
st, cf = infinity.make_problems(np.arange(B))
s = BatchSolver(0, P, dtype=dt)
a = s.solve(st, cf)
dev = torch.device("cuda:0")
s.reserve(B)
tst, tcf = torch.from_numpy(st).to(dev), torch.from_numpy(cf).to(dev)
u0 = torch.empty((B, 2), dtype=torch.float64, device=dev)
side = torch.cuda.Stream(dev)
with torch.cuda.stream(side):
    s.solve_device(tst, tcf, u0)
torch.cuda.synchronize()
print("capture", dt, B, flush=True)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=side):
    s.solve_device(tst, tcf, u0)
print("captured", flush=True)
for rep in range(2):
    u0.zero_()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    print("replay", rep, "equal", bool((u0.cpu().numpy() == a["u0"]).all()), flush=True)
