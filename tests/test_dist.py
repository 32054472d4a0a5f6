"""Multi-process (world_size 2, gloo, CPU) tests of the sharded path: batch
shards cover the global batch exactly, the per-rank pipeline results gathered
equal the single-process result, and the evaluation-key broadcast delivers
identical keys (the only collective)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT  # noqa: F401  (sets sys.path)
import shard


def test_shard_batch_partitions():
    for gb in (0, 1, 7, 1024, 1031):
        for world in (1, 2, 3, 8):
            ranges = [shard.shard_batch(gb, r, world) for r in range(world)]
            covered = []
            for s, c in ranges:
                covered.extend(range(s, s + c))
            assert covered == list(range(gb))
            assert max(c for _, c in ranges) - min(c for _, c in ranges) <= 1
    with pytest.raises(ValueError):
        shard.shard_batch(4, 2, 2)


def test_evalkey_size():
    # configs[3]: T = 32 towers at N = 2^16, dnum = 3 -> P = 11
    assert shard.evalkey_words(32, 16, 3) == 2 * 3 * 43 * 65536


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    try:
        _work(rank, world, port, q)
    except Exception as e:  # report instead of leaving the parent waiting
        q.put((rank, False, False, repr(e)))
        raise


def _work(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle as O

        log_n, T, GB = 10, 3, 3 * world  # gloo all_gather needs equal shard sizes
        n = 1 << log_n
        qs, rs = O.moduli_chain(log_n, T)
        a = O.uniform_dcrt(GB, T, n, qs, 1)
        b = O.uniform_dcrt(GB, T, n, qs, 2)
        start, count = shard.shard_batch(GB, rank, world)
        local = O.ntt_mul_intt(a[start:start + count], b[start:start + count], O.Tables(n, qs, rs))
        # gather shards (test-side check only; the product path has no gather)
        sizes = [shard.shard_batch(GB, r, world)[1] for r in range(world)]
        buf = [torch.zeros((s, T, n), dtype=torch.int64) for s in sizes]
        dist.all_gather(buf, torch.from_numpy(np.ascontiguousarray(local).view(np.int64)))
        full = torch.cat(buf).numpy().view(np.uint64)
        ok_pipeline = bool(np.array_equal(full, O.ntt_mul_intt(a, b, O.Tables(n, qs, rs))))
        # evaluation-key broadcast
        key = torch.zeros(shard.evalkey_words(T, 6, 2), dtype=torch.int64)
        if rank == 0:
            key.random_(0, 2**40, generator=torch.Generator().manual_seed(9))
        shard.broadcast_evalkey(key, src=0)
        ref = torch.zeros_like(key).random_(0, 2**40, generator=torch.Generator().manual_seed(9))
        ok_bcast = bool(torch.equal(key, ref))
        # the bench's cross-rank check of a broadcast key
        ok_bcast = ok_bcast and shard.same_on_all_ranks(key) and not shard.same_on_all_ranks(key + rank)
        slowest = shard.max_over_ranks(float(rank + 1))
        q.put((rank, ok_pipeline, ok_bcast, slowest))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_shard_and_broadcast(world):
    """world_size 2 (the N > 1 contract) and 4 (a rehearsal of more ranks on
    gloo): batch shards, the key broadcast and the max-over-ranks timing."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert sorted(r[0] for r in res) == list(range(world))
    assert all(r[1] and r[2] for r in res), res
    assert all(r[3] == float(world) for r in res)


def _ks_worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        try:
            import keyswitch as K
            import oracle as O

            # configs[4] in miniature: ciphertext batch sharded, the evaluation
            # key generated on rank 0 and broadcast (bench.py --workload keyswitch)
            log_n, sq, sp, dnum, GB = 5, 4, 2, 2, 4
            n = 1 << log_n
            m, r = O.moduli_chain(log_n, sq + sp)
            kp = K.KeySwitchParams(n, m[:sq], r[:sq], m[sq:], r[sq:], dnum)
            rng = np.random.default_rng(3)
            c = np.stack([np.stack([rng.integers(0, x, size=n, dtype=np.uint64) for x in m[:sq]])
                          for _ in range(GB)])
            kb = torch.zeros((dnum, sq + sp, n), dtype=torch.int64)
            ka = torch.zeros_like(kb)
            if rank == 0:
                krng = np.random.default_rng(11)
                for t, x in enumerate(m):
                    kb[:, t] = torch.from_numpy(krng.integers(0, x, size=(dnum, n), dtype=np.uint64).view(np.int64))
                    ka[:, t] = torch.from_numpy(krng.integers(0, x, size=(dnum, n), dtype=np.uint64).view(np.int64))
            shard.broadcast_evalkey(kb, src=0)
            shard.broadcast_evalkey(ka, src=0)
            kbn, kan = kb.numpy().view(np.uint64), ka.numpy().view(np.uint64)
            start, count = shard.shard_batch(GB, rank, world)
            o0, o1 = K.ks_core(kp, c[start:start + count], kbn, kan)
            buf = [torch.zeros((2, count, sq, n), dtype=torch.int64) for _ in range(world)]
            dist.all_gather(buf, torch.from_numpy(np.ascontiguousarray(np.stack([o0, o1])).view(np.int64)))
            got = torch.cat(buf, dim=1).numpy().view(np.uint64)
            r0, r1 = K.ks_core(kp, c, kbn, kan)
            q.put((rank, bool(np.array_equal(got[0], r0) and np.array_equal(got[1], r1))))
        finally:
            dist.destroy_process_group()
    except Exception as e:
        q.put((rank, repr(e)))
        raise


def test_two_rank_sharded_keyswitch_with_broadcast_key():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ks_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert sorted(r[0] for r in res) == [0, 1]
    assert all(r[1] is True for r in res), res


def _uid_fail_worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        try:
            import ofhe_hip as H

            def no_uid():
                raise H.MathError("ncclGetUniqueId refused (test)")

            H.comm_unique_id = no_uid  # rank 0's id fails before its broadcast
            bfn, label, comm = shard.key_broadcaster(object(), rank, world)
            key = torch.arange(32, dtype=torch.int64) if rank == 0 else torch.zeros(32, dtype=torch.int64)
            bfn(key, 0)
            q.put((rank, comm is None, label, bool(torch.equal(key, torch.arange(32, dtype=torch.int64)))))
        finally:
            dist.destroy_process_group()
    except Exception as e:
        q.put((rank, False, repr(e), False))
        raise


def test_two_rank_unique_id_failure_falls_back_without_hanging():
    """rank 0's ofhe_hip_comm_unique_id failing must not leave the
    peers in broadcast_object_list while rank 0 enters the all_reduce: every
    rank reaches the fallback, the key still arrives, the reason is named."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_uid_fail_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert sorted(r[0] for r in res) == [0, 1]
    for rank, fell_back, label, key_ok in res:
        assert fell_back and key_ok, res
        assert "torch.distributed gloo" in label and "unique id failed on rank 0" in label, label


def _tower_worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        try:
            import oracle as O

            # configs[3] in miniature: 32 towers split into contiguous ranges
            # over the ranks (shard.shard_towers, bench.py --shard towers /
            # bench_configs3), each rank's plan over its own sub-basis of the
            # global chain; inputs drawn per GLOBAL tower index.  The oracle
            # stands in for the device compute on CPU.
            log_n, T, B = 8, 32, 2
            n = 1 << log_n
            qs, rs = O.moduli_chain(log_n, T)
            a = O.uniform_dcrt(B, T, n, qs, 31)
            b = O.uniform_dcrt(B, T, n, qs, 32)
            t0, cnt = shard.shard_towers(T, rank, world)
            local = O.ntt_mul_intt(a[:, t0:t0 + cnt], b[:, t0:t0 + cnt], O.Tables(n, qs[t0:t0 + cnt], rs[t0:t0 + cnt]))
            parts = [None] * world
            dist.all_gather_object(parts, (t0, local))  # test-side check only: the product path has no gather
            parts.sort(key=lambda x: x[0])
            got = np.concatenate([p[1] for p in parts], axis=1)
            want = O.ntt_mul_intt(a, b, O.Tables(n, qs, rs))
            q.put((rank, bool(got.shape == want.shape and np.array_equal(got, want)),
                   [p[0] for p in parts]))
        finally:
            dist.destroy_process_group()
    except Exception as e:
        q.put((rank, repr(e), None))
        raise


@pytest.mark.parametrize("world", [2, 3])
def test_tower_sharded_pipeline_matches_single_rank(world):
    """configs[3]: T = 32 towers split over `world` ranks (16 + 16; 11 + 11 + 10),
    every rank's tower range through the pipeline on its own sub-basis, the
    shards gathered along the tower axis equal the single-rank result bit for
    bit."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_tower_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(r[1] is True for r in res), res
    starts = [shard.shard_towers(32, r, world)[0] for r in range(world)]
    assert all(r[2] == starts for r in res)
