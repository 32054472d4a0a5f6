"""Multi-rank check of the C-ABI key broadcast (ofhe_hip_bcast_evalkey):

    python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port 29533 tools/comm_check.py

Each rank drives GPU LOCAL_RANK % device_count.  The 128-byte RCCL id goes
from rank 0 to the others over a gloo (CPU) group; the root's key is an
arithmetic sequence, every other rank starts from its own fill, and after the
broadcast every rank must hold the root's words.  Prints one JSON line per
rank (status, GB/s of the timed broadcast).  RCCL refuses two ranks on one
GPU; that case reports "init_failed" and exits 0 when there are fewer devices
than ranks, so the script is safe on a one-GPU box.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "upmem--openfhe_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import ofhe_hip as H  # noqa: E402
import shard  # noqa: E402


def main() -> int:
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    ndev = torch.cuda.device_count()
    d = int(os.environ.get("LOCAL_RANK", rank)) % ndev
    torch.cuda.set_device(d)
    ctx = H.Context(d)
    uid = [H.comm_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(uid, src=0)
    try:
        comm = H.Comm(ctx, world, rank, uid[0])
    except H.MathError as e:
        print(json.dumps({"rank": rank, "status": "init_failed", "devices": ndev, "error": str(e)[:200]}), flush=True)
        return 0 if ndev < world else 1
    words = shard.evalkey_words(int(os.environ.get("COMM_TOWERS", "32")), 16, 3)
    dv = torch.device("cuda", d)
    want = torch.arange(words, dtype=torch.int64, device=dv) * 3 + 7
    key = want.clone() if rank == 0 else torch.full((words,), -1 - rank, dtype=torch.int64, device=dv)
    s = torch.cuda.current_stream()
    comm.bcast_evalkey(key.data_ptr(), words, 0, s.cuda_stream)
    torch.cuda.synchronize()
    ok = bool(torch.equal(key, want))
    # timed repeat (same root buffer; the others overwrite theirs again)
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(5):
        comm.bcast_evalkey(key.data_ptr(), words, 0, s.cuda_stream)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 5
    print(json.dumps({"rank": rank, "status": "ok" if ok else "MISMATCH", "devices": ndev, "bytes": words * 8,
                      "ms": dt * 1e3, "GBps": words * 8 / dt / 1e9}), flush=True)
    comm.close()
    dist.destroy_process_group()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
