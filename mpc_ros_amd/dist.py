"""Data-parallel sharding of a batch of NMPC problems over the GPUs of a node.

The B problems are independent: rank r of W solves the contiguous
slice [start, start + count) with no communication, then the per-problem results
are gathered to rank 0 -- the only exchange on the path (one gather per output array,
RCCL point-to-point over xGMI with the "nccl" backend; gloo on CPU in tests).  Inputs are regenerated on every rank from
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


def gather_plan(total: int, world: int, row_bytes: int) -> list[dict]:
    """Per rank: its slice and the bytes gather_rows moves for one array of `row_bytes`-byte
    rows -- rank r > 0 sends max_shard rows (its slice, padded by at most one row) to rank 0
    only; rank 0 sends nothing over the link."""
    m = max_shard(total, world) if world > 0 else 0
    out = []
    for r in range(world):
        start, count = shard(total, r, world)
        out.append(dict(rank=r, start=start, count=count, send_bytes=0 if r == 0 else m * row_bytes))
    return out


def gather_rows(t, total: int, group=None):
    """Gather every rank's slice (rows of `t`, shard() layout) into a [total, ...] tensor on rank 0.

    One torch.distributed.gather to rank 0 (RCCL point-to-point under "nccl": each rank
    sends only its own slice, padded to the largest shard so the messages are equal-sized;
    no rank but 0 receives anything).  Returns the assembled tensor on rank 0 and None
    elsewhere."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    start, count = shard(total, rank, world)
    if t.shape[0] != count:
        raise ValueError(f"rank {rank}: {t.shape[0]} rows, its shard holds {count}")
    m = max_shard(total, world)
    tail = tuple(t.shape[1:])
    if t.shape[0] == m:
        send = t.contiguous()
    else:
        send = torch.zeros((m,) + tail, dtype=t.dtype, device=t.device)
        send[:count] = t
    root = dist.get_global_rank(group, 0) if group is not None else 0
    if rank != 0:
        dist.gather(send, None, dst=root, group=group)
        return None
    buf = torch.empty((world * m,) + tail, dtype=t.dtype, device=t.device)
    dist.gather(send, list(buf.split(m, 0)), dst=root, group=group)
    parts = []
    for r in range(world):
        _, cnt = shard(total, r, world)
        parts.append(buf[r * m: r * m + cnt])
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
