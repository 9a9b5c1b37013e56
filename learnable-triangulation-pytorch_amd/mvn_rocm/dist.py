"""Frame sharding across GPUs of one node.

Frames are independent in every hot-path op (op.py:107 loops per frame, op.py:89
reduces per (b, j), multiview.py:166 per (b, j)), so a batch splits into contiguous
per-rank frame ranges with NO collective on the data path.  The only exchange is one
all-gather of the (frames, J, 3) joints at the end — RCCL over xGMI when the process
group is "nccl" (== RCCL on ROCm), gloo on CPU for tests.  The payload is a few KB:
latency-bound, one collective per batch.
"""
from __future__ import annotations

from typing import Callable, Tuple

import torch
import torch.distributed as dist


def shard(global_batch: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous [start, start + count) frame range of `rank`; ragged tails go to the
    lowest ranks, so counts differ by at most one."""
    if not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world of {world}")
    base, extra = divmod(global_batch, world)
    count = base + (1 if rank < extra else 0)
    start = rank * base + min(rank, extra)
    return start, count


def gather_joints(local: torch.Tensor, global_batch: int, group=None) -> torch.Tensor:
    """All-gather every rank's (count, J, 3) joints into (global_batch, J, 3) in frame
    order.  One collective: ragged shards are padded to the largest shard."""
    world = dist.get_world_size(group)
    if world == 1:
        return local
    if local.is_cuda and dist.get_backend(group) == "gloo":
        # gloo collectives take host tensors (tests: several ranks sharing one GPU)
        return gather_joints(local.cpu(), global_batch, group).to(local.device)
    per = -(-global_batch // world)
    J = local.shape[1]
    send = local.new_zeros((per, J, 3))
    send[: local.shape[0]] = local
    recv = local.new_empty((world * per, J, 3))
    dist.all_gather_into_tensor(recv, send, group=group)
    out = []
    for r in range(world):
        _, count = shard(global_batch, world, r)
        out.append(recv[r * per: r * per + count])
    return torch.cat(out, 0)


def run_sharded(global_batch: int, make_frames: Callable[[int, int], object],
                compute: Callable[[object], torch.Tensor], group=None) -> torch.Tensor:
    """Generic driver: this rank builds its own frames [start, start+count) with
    `make_frames(start, count)`, runs `compute` on them, and the joints of all ranks
    are gathered.  Returns (global_batch, J, 3) on every rank."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    start, count = shard(global_batch, world, rank)
    local = compute(make_frames(start, count))
    return gather_joints(local, global_batch, group) if world > 1 else local
