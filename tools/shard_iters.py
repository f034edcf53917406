"""Per-shard iteration statistics and kernel time of the multi-GPU benchmark's shards,
solved one after another on one GPU (diagnostic: the 8-GPU weak-scaling run takes the
slowest rank's time, so a shard with a pathological iteration tail would show here).

    python tools/shard_iters.py [world=8] [per_gpu=65536]
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpc_ros_amd import dist as D  # noqa: E402
from mpc_ros_amd import infinity, params  # noqa: E402
from mpc_ros_amd.solver import BatchSolver  # noqa: E402

world = int(sys.argv[1]) if len(sys.argv) > 1 else 8
B = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
dev = torch.device("cuda", 0)
s = BatchSolver(0, params.PLUGIN_DEFAULTS)
s.reserve(B)
u0 = torch.empty((B, 2), dtype=torch.float64, device=dev)
status = torch.empty(B, dtype=torch.int32, device=dev)
iters = torch.empty(B, dtype=torch.int32, device=dev)
for r in range(world):
    start, count = D.shard(B * world, r, world)
    st, cf = infinity.make_problems(np.arange(start, start + count))
    tst = torch.from_numpy(st).to(dev)
    tcf = torch.from_numpy(cf).to(dev)
    s.solve_device(tst, tcf, u0, None, status, None, iters)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    s.solve_device(tst, tcf, u0, None, status, None, iters)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3
    it = iters.cpu().numpy()
    stv = status.cpu().numpy()
    top = np.sort(it)[-5:][::-1]
    print(f"rank {r}: {ms:7.2f} ms  iters mean {it.mean():.3f} max {it.max()} top5 {top.tolist()} "
          f"success {np.mean(stv == 1):.5f} statuses {dict(zip(*np.unique(stv, return_counts=True)))}", flush=True)
