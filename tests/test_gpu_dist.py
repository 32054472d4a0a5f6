"""Multi-process GPU tests of the sharded product path:
two ranks on the box's one MI355X, each computing its shard with the HIP
library (not the oracle), the shards gathered over gloo (host) and compared
bit for bit with the oracle's single-rank result.  Covers both partitions the
bench uses: ciphertext batch (configs[2] / [4]) and contiguous tower ranges
(configs[3])."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT  # noqa: F401  (sets sys.path)
import shard
from test_dist import _free_port

pytestmark = pytest.mark.gpu


def _worker(rank, world, port, mode, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        try:
            import ofhe_hip as H
            import oracle as O

            log_n, T, B = 13, 8, 4
            n = 1 << log_n
            qs, rs = O.moduli_chain(log_n, T)
            a = O.uniform_dcrt(B, T, n, qs, 41)
            b = O.uniform_dcrt(B, T, n, qs, 42)
            if mode == "towers":
                t0, tc = shard.shard_towers(T, rank, world)
                b0, bc = 0, B
            else:
                t0, tc = 0, T
                b0, bc = shard.shard_batch(B, rank, world)
            ctx = H.Context(0)
            plan = H.NTTPlan(ctx, log_n, qs[t0:t0 + tc], rs[t0:t0 + tc])
            xa = torch.from_numpy(np.ascontiguousarray(a[b0:b0 + bc, t0:t0 + tc]).view(np.int64)).cuda()
            xb = torch.from_numpy(np.ascontiguousarray(b[b0:b0 + bc, t0:t0 + tc]).view(np.int64)).cuda()
            xc = torch.empty_like(xa)
            s = torch.cuda.current_stream()
            plan.ntt_mul_intt(xa.data_ptr(), xb.data_ptr(), xc.data_ptr(), bc, s.cuda_stream)
            s.synchronize()
            local = xc.cpu().numpy().view(np.uint64)
            plan.close()
            parts = [None] * world
            dist.all_gather_object(parts, ((b0, t0), local))
            parts.sort(key=lambda x: x[0])
            got = np.concatenate([p[1] for p in parts], axis=1 if mode == "towers" else 0)
            want = O.ntt_mul_intt(a, b, O.Tables(n, qs, rs))
            q.put((rank, bool(got.shape == want.shape and np.array_equal(got, want))))
            ctx.close()
        finally:
            dist.destroy_process_group()
    except Exception as e:
        q.put((rank, repr(e)))
        raise


@pytest.mark.parametrize("mode", ["towers", "batch"])
def test_two_ranks_one_gpu_shards_equal_oracle(mode):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, mode, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(r[1] is True for r in res), res
