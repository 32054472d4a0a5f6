"""Multi-GPU plumbing for the RNS path.

The pipeline is independent per (batch, tower), so ranks shard the batch with no
data-path collective.  The only exchange the north star names is the
evaluation-key broadcast: through the library's own RCCL communicator
(ofhe_hip_comm_init / ofhe_hip_bcast_evalkey, open_comm + bcast_evalkey_capi
below), or with torch.distributed (backend "nccl" is RCCL over xGMI on ROCm;
"gloo" in CPU tests).
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


def _host_staged() -> bool:
    """gloo moves host tensors: device tensors are staged through the host."""
    import torch.distributed as dist

    return dist.get_backend() == "gloo"


def broadcast_evalkey(key, src: int = 0, group=None):
    """Broadcast an evaluation key tensor from `src` to every rank (in place)."""
    import torch.distributed as dist

    if key.is_cuda and _host_staged():
        h = key.cpu()
        dist.broadcast(h, src=src, group=group)
        key.copy_(h)
        return key
    dist.broadcast(key, src=src, group=group)
    return key


def open_comm(ctx, rank: int, world: int):
    """The C ABI's RCCL communicator for this rank's device; rank 0's unique id
    travels over the default torch.distributed group.  Collective."""
    import torch.distributed as dist

    import ofhe_hip as H

    # rank 0 always broadcasts: the id, or the reason it has none, so a failed
    # ofhe_hip_comm_unique_id never leaves the peers waiting in this broadcast
    # while rank 0 has moved on to the next collective
    uid = [None]
    if rank == 0:
        try:
            uid[0] = H.comm_unique_id()
        except Exception as e:  # noqa: BLE001  (library missing or RCCL refused: fall back, never hang)
            uid[0] = "unique id failed on rank 0: " + str(e)
    dist.broadcast_object_list(uid, src=0)
    if isinstance(uid[0], str):
        raise H.MathError(uid[0])
    return H.Comm(ctx, world, rank, uid[0])


def bcast_evalkey_capi(comm, key, src: int = 0):
    """In-place key broadcast through ofhe_hip_bcast_evalkey on the tensor's
    current stream (key: contiguous int64/uint64 device tensor)."""
    import torch

    assert key.is_contiguous() and key.element_size() == 8
    comm.bcast_evalkey(key.data_ptr(), key.numel(), src, torch.cuda.current_stream(key.device).cuda_stream)
    return key


def same_on_all_ranks(t) -> bool:
    """True when a tensor's word checksum agrees across ranks (broadcast check)."""
    import torch
    import torch.distributed as dist

    h = torch.stack([t.sum(), (t * 3).bitwise_xor(t >> 7).sum()]).to(torch.int64)
    if h.is_cuda and _host_staged():
        h = h.cpu()
    lo, hi = h.clone(), h.clone()
    dist.all_reduce(lo, op=dist.ReduceOp.MIN)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX)
    return bool(torch.equal(lo, hi))


def key_broadcaster(ctx, rank: int, world: int):
    """(broadcast function, backend label, communicator or None): the C-ABI
    communicator when it comes up, else torch.distributed's own RCCL group
    (the failure is named).  Close the communicator (comm.close()) before
    destroying the process group, not at interpreter exit.

    The ranks agree on the backend: each reports whether its communicator
    came up (all_reduce MIN of an ok flag), and unless every rank succeeded
    they all close theirs and use torch.distributed -- a rank never calls
    ncclBroadcast while a peer sits in dist.broadcast.  Every rank's own
    outcome (communicator up or the error it raised) is gathered onto the
    returned function as `.per_rank`, one {"rank", "comm", "error"} per rank,
    so a fallback names the rank that caused it."""
    import torch
    import torch.distributed as dist

    import ofhe_hip as H

    comm, err = None, None
    try:
        if ctx is None:
            raise H.MathError("no device context (CPU rehearsal)")
        comm = open_comm(ctx, rank, world)
    except Exception as e:  # noqa: BLE001
        err = str(e)
    backend = dist.get_backend()
    dev = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
    ok = torch.tensor([1 if comm is not None else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    per_rank = [None] * dist.get_world_size()
    dist.all_gather_object(per_rank, {"rank": rank, "comm": comm is not None, "error": err})
    if int(ok.item()) == 1:
        fn = lambda key, src=0: bcast_evalkey_capi(comm, key, src)  # noqa: E731
        fn.per_rank = per_rank
        return fn, "ofhe_hip_bcast_evalkey (RCCL)", comm
    if comm is not None:
        comm.close()
    why = err if err else "a peer rank's C-ABI communicator failed"
    fn = lambda key, src=0: broadcast_evalkey(key, src)  # noqa: E731
    fn.per_rank = per_rank
    return fn, f"torch.distributed {backend} (C-ABI comm: {why})", None


def max_over_ranks(value: float, device=None) -> float:
    """Max of a per-rank float (timing is reported as the slowest rank)."""
    import torch
    import torch.distributed as dist

    t = torch.tensor([value], dtype=torch.float64, device=None if _host_staged() else device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
