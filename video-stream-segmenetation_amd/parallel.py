"""Data parallelism over frames.

The forward is independent per frame, so the batch is sharded by contiguous
frame ranges across ranks (one process per GPU) and the only exchange is one
all-gather of the f32 masks, after which every rank — in particular the
compositing consumer — holds all N masks in frame order.  On ROCm the "nccl"
backend of torch.distributed is RCCL (over xGMI within a node); the same code
runs on "gloo" for the CPU tests.

Ragged batches (N % world != 0) are padded to ceil(N / world) frames per rank
for the collective (all_gather_into_tensor needs equal counts) and the padding
rows are dropped afterwards, so the gathered masks are exactly the masks of
the N real frames.  The reference itself has no parallelism at all
(SURVEY.md §2 row 16): this module is the build's addition.
"""
from __future__ import annotations


def shard_range(n_total: int, rank: int, world: int) -> tuple[int, int]:
    """(start, count) of rank's contiguous shard; the first n % world ranks get one more."""
    if world < 1 or not 0 <= rank < world or n_total < 0:
        raise ValueError("bad shard arguments")
    base, rem = divmod(n_total, world)
    count = base + (1 if rank < rem else 0)
    start = rank * base + min(rank, rem)
    return start, count


def shard_capacity(n_total: int, world: int) -> int:
    return -(-n_total // world)


def gather_masks(local, n_total: int, group=None, out=None):
    """All-gather every rank's masks ([count, H*W] float32 tensor, this rank's
    shard in frame order) into [n_total, H*W] on every rank, in frame order."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    cap = shard_capacity(n_total, world)
    start, count = shard_range(n_total, rank, world)
    if local.shape[0] != count:
        raise ValueError(f"rank {rank} holds {local.shape[0]} masks, shard is {count}")
    hw = local.shape[1]
    if count == cap:
        send = local.contiguous()
    else:
        send = torch.zeros((cap, hw), dtype=local.dtype, device=local.device)
        send[:count] = local
    buf = torch.empty((world * cap, hw), dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(buf, send, group=group)
    if n_total == world * cap:
        res = buf
    else:
        idx = []
        for r in range(world):
            s, c = shard_range(n_total, r, world)
            idx.extend(range(r * cap, r * cap + c))
        res = buf[torch.tensor(idx, device=buf.device)]
    if out is not None:
        out.copy_(res)
        return out
    return res
