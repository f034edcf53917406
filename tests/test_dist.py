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


def _gather_worker(rank, world, port, total, out_path):
    import sys

    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mpc_ros_amd import dist as D

    start, count = D.shard(total, rank, world)
    idx = torch.arange(start, start + count, dtype=torch.float64)
    rows = torch.stack([idx, -idx, idx * 0.5], 1)  # [count, 3]
    g = D.gather_rows(rows, total)
    g_st = D.gather_rows(torch.full((count,), rank, dtype=torch.int32), total)
    if rank == 0:
        np.savez(out_path, rows=g.numpy(), owner=g_st.numpy())
    else:
        assert g is None and g_st is None
    dist.barrier()
    dist.destroy_process_group()


def test_gather_to_rank0_ragged_and_empty_shards(tmp_path):
    """gather_rows: a gather to rank 0 only, ragged (B % G != 0) and with empty shards (B < G),
    rows land in global order and each row comes from the rank shard() assigns it to."""
    from mpc_ros_amd import dist as D

    for world, total in ((3, 7), (4, 2)):
        out = str(tmp_path / f"g{world}_{total}.npz")
        port = 31500 + (os.getpid() + world) % 2000
        mp.spawn(_gather_worker, args=(world, port, total, out), nprocs=world, join=True)
        with np.load(out) as z:
            idx = np.arange(total, dtype=np.float64)
            np.testing.assert_array_equal(z["rows"], np.stack([idx, -idx, idx * 0.5], 1))
            owner = np.concatenate([np.full(D.shard(total, r, world)[1], r) for r in range(world)])
            np.testing.assert_array_equal(z["owner"], owner)


def test_shard_and_gather_plan_arithmetic():
    """shard(): contiguous, balanced, covering [0, B) once, the first B % G ranks one more,
    empty shards for B < G; gather_plan(): rank 0 sends nothing, the others max_shard rows."""
    from mpc_ros_amd import dist as D

    for total in (0, 1, 2, 7, 23, 65536, 524288, 524289):
        for world in (1, 2, 3, 4, 7, 8):
            sl = [D.shard(total, r, world) for r in range(world)]
            assert sum(c for _, c in sl) == total
            nxt = 0
            for r, (s, c) in enumerate(sl):
                assert s == nxt and c >= 0
                assert c == total // world + (1 if r < total % world else 0)
                nxt = s + c
            plan = D.gather_plan(total, world, 16)
            assert plan[0]["send_bytes"] == 0
            assert all(p["send_bytes"] == D.max_shard(total, world) * 16 for p in plan[1:])
    with __import__("pytest").raises(ValueError):
        D.shard(10, 2, 2)
