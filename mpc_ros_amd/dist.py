"""Data-parallel sharding of a batch of NMPC problems over the GPUs of a node.

The B problems are independent: rank r of W solves the contiguous
slice [start, start + count) with no communication, then the per-problem results
are gathered to rank 0 -- the only exchange on the path (RCCL over xGMI with the
"nccl" backend; gloo on CPU in tests).  Inputs are regenerated on every rank from
(seed, global index), so no input is ever sent.
"""
from __future__ import annotations

import os


def shard(total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous, balanced slice of `total` problems for `rank` (first ranks get the remainder)."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError("bad rank/world")
    base, rem = divmod(int(total), int(world))
    count = base + (1 if rank < rem else 0)
    start = rank * base + min(rank, rem)
    return start, count


def max_shard(total: int, world: int) -> int:
    return -(-int(total) // int(world))


def env_rank_world() -> tuple[int, int, int]:
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def gather_rows(t, total: int, group=None):
    """Gather every rank's slice (rows of `t`, shard() layout) into a [total, ...] tensor on rank 0.

    Shards are padded to the largest shard so that one all_gather_into_tensor moves
    everything (RCCL all-gather: every rank sends its slice once over xGMI).  Returns
    the assembled tensor on rank 0 and None elsewhere."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    m = max_shard(total, world)
    pad = torch.zeros((m,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    pad[: t.shape[0]] = t
    out = torch.empty((world * m,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    dist.all_gather_into_tensor(out, pad, group=group)
    if rank != 0:
        return None
    parts = []
    for r in range(world):
        _, cnt = shard(total, r, world)
        parts.append(out[r * m: r * m + cnt])
    return torch.cat(parts, 0)


def solve_sharded(total: int, solve_fn, make_inputs, group=None, device="cpu"):
    """One data-parallel pass: this rank generates and solves its slice, then the
    controls and statuses are gathered to rank 0.

    solve_fn(state, coeffs) -> (u0 [n,2] float64 tensor, status [n] int32 tensor) on `device`;
    make_inputs(start, count) -> (state [n,6], coeffs [n,4]) tensors on `device`.
    Returns (u0_all, status_all) on rank 0, (None, None) elsewhere."""
    import torch.distributed as dist

    rank, world = dist.get_rank(group), dist.get_world_size(group)
    start, count = shard(total, rank, world)
    state, coeffs = make_inputs(start, count)
    u0, status = solve_fn(state, coeffs)
    return gather_rows(u0, total, group), gather_rows(status, total, group)
