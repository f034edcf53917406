import sys, time, numpy as np, torch
sys.path.insert(0, '.')
from mpc_ros_amd import infinity, params
from mpc_ros_amd.solver import BatchSolver
dtype = sys.argv[1]
P = dict(params.PLUGIN_DEFAULTS, STEPS=40)
st, cf = infinity.make_problems(np.arange(4096))
s = BatchSolver(0, P, dtype=dtype)
a = s.solve(st, cf)
esc = np.flatnonzero(a["diag"][:, 2] >= 1)
i = int(esc[0]) if len(esc) else 0
print("row", i, a["diag"][i], flush=True)
if len(sys.argv) > 2:
    s.set_park_capacity(1)
    b = s.solve(st, cf)
    print("park 1 solved", (b["u0"] == a["u0"]).all(), flush=True)
    s.set_park_capacity(0)
    r = s.solve(st[i:i + 1], cf[i:i + 1])
    print("B = 1 after park 1", r["u0"], flush=True)
dev = torch.device("cuda:0")
s.reserve(1)
tst, tcf = torch.from_numpy(st[i:i + 1].copy()).to(dev), torch.from_numpy(cf[i:i + 1].copy()).to(dev)
u0 = torch.empty((1, 2), dtype=torch.float64, device=dev)
status = torch.empty(1, dtype=torch.int32, device=dev)
diag = torch.empty((1, 4), dtype=torch.int32, device=dev)
side = torch.cuda.Stream(dev)
with torch.cuda.stream(side):
    s.solve_device(tst, tcf, u0, status=status, diag=diag)
print("warm-up queued", flush=True)
torch.cuda.synchronize()
print("warm-up done", u0.cpu().numpy(), diag.cpu().numpy(), flush=True)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=side):
    s.solve_device(tst, tcf, u0, status=status, diag=diag)
print("captured", flush=True)
for rep in range(int(sys.argv[3]) if len(sys.argv) > 3 else 1):
    u0.zero_()
    torch.cuda.synchronize()
    g.replay()
    print("replay queued", rep, flush=True)
    torch.cuda.synchronize()
    print("replay done", rep, u0.cpu().numpy(), a["u0"][i], diag.cpu().numpy(), flush=True)
