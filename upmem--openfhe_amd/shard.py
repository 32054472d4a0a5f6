"""Multi-GPU plumbing for the RNS path.

The pipeline is independent per (batch, tower), so ranks shard the batch with no
data-path collective.  The only exchange the north star names is the
evaluation-key broadcast, done with torch.distributed (backend "nccl" is RCCL
over xGMI on ROCm; "gloo" in CPU tests).
"""
from __future__ import annotations


def shard_batch(global_batch: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous batch range [start, start + count) owned by `rank`; the
    remainder goes to the lowest ranks so counts differ by at most one."""
    if world < 1 or not (0 <= rank < world) or global_batch < 0:
        raise ValueError("bad shard arguments")
    base, rem = divmod(global_batch, world)
    count = base + (1 if rank < rem else 0)
    start = rank * base + min(rank, rem)
    return start, count


def shard_towers(towers: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous tower range for per-tower sharding (configs[3]: T=32 over 8 GPUs)."""
    return shard_batch(towers, rank, world)


def evalkey_words(towers: int, log_n: int, dnum: int = 3) -> int:
    """Size of a hybrid key-switching key: 2 polynomials x dnum digits x
    (Q + P) towers x N words, with P = ceil(T / dnum) (keyswitch-hybrid.cpp:330-414)."""
    p = (towers + dnum - 1) // dnum
    return 2 * dnum * (towers + p) << log_n


def broadcast_evalkey(key, src: int = 0, group=None):
    """Broadcast an evaluation key tensor from `src` to every rank (in place)."""
    import torch.distributed as dist

    dist.broadcast(key, src=src, group=group)
    return key


def max_over_ranks(value: float, device=None) -> float:
    """Max of a per-rank float (timing is reported as the slowest rank)."""
    import torch
    import torch.distributed as dist

    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
