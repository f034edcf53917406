"""Multi-rank path on CPU: world_size 2 over gloo.  Each rank solves its shard
(with the oracle standing in for the GPU kernel), rank 0 gathers; the result must
equal the single-process solve of the whole batch, in order."""
from __future__ import annotations

import os

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT

TOTAL = 23  # not divisible by the world size on purpose


def _worker(rank, world, port, out_path):
    import sys

    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mpc_ros_amd import dist as D, infinity, params
    from oracle import pyoracle as O

    P = params.PLUGIN_DEFAULTS

    def make_inputs(start, count):
        st, cf = infinity.make_problems(np.arange(start, start + count))
        return torch.from_numpy(st), torch.from_numpy(cf)

    def solve(st, cf):
        r = O.mpc_solve_batch(P, st.numpy(), cf.numpy(), opts=O.ref_opts(int(P["STEPS"])), nthreads=1)
        return torch.from_numpy(r["u0"]), torch.from_numpy(r["status"])

    u0, status = D.solve_sharded(TOTAL, solve, make_inputs)
    if rank == 0:
        np.savez(out_path, u0=u0.numpy(), status=status.numpy())
    else:
        assert u0 is None and status is None
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_shard_and_gather(tmp_path, oracle):
    out = str(tmp_path / "r0.npz")
    port = 29500 + os.getpid() % 2000
    mp.spawn(_worker, args=(2, port, out), nprocs=2, join=True)
    from mpc_ros_amd import infinity, params

    st, cf = infinity.make_problems(np.arange(TOTAL))
    ref = oracle.mpc_solve_batch(params.PLUGIN_DEFAULTS, st, cf, opts=oracle.ref_opts(20))
    with np.load(out) as z:
        np.testing.assert_array_equal(z["status"], ref["status"])
        np.testing.assert_array_equal(z["u0"], ref["u0"])
