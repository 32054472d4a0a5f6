"""GPU tests of the RCCL key broadcast through the C ABI
(ofhe_hip_comm_* / ofhe_hip_bcast_evalkey, SURVEY.md §8(b),(e)).  One GPU:
a single-rank communicator (the broadcast is the identity on the root) and
the argument checks.  The two-rank exchange runs under torch.distributed.run
in tools/comm_check.py (ranks on distinct GPUs when there are several)."""
import numpy as np
import pytest

from test_gpu_parity import dev, host, stream

pytestmark = pytest.mark.gpu


def test_single_rank_broadcast_is_identity(hip):
    H, ctx = hip
    import shard

    uid = H.comm_unique_id()
    assert len(uid) == H.COMM_ID_BYTES
    comm = H.Comm(ctx, 1, 0, uid)
    words = shard.evalkey_words(2, 12, 3)
    rng = np.random.default_rng(9)
    key = rng.integers(0, 1 << 60, size=words, dtype=np.uint64)
    d = dev(key)
    comm.bcast_evalkey(d.data_ptr(), words, 0, stream())
    assert np.array_equal(host(d), key)
    comm.bcast_evalkey(d.data_ptr(), 0, 0, stream())  # empty: no-op
    with pytest.raises(H.MathError):
        comm.bcast_evalkey(d.data_ptr(), words, 1, stream())  # root outside [0, nranks)
    with pytest.raises(H.MathError):
        comm.bcast_evalkey(0, words, 0, stream())
    comm.close()
    with pytest.raises(H.MathError):
        comm.bcast_evalkey(d.data_ptr(), words, 0, stream())


def test_comm_init_rejects_bad_ranks(hip):
    H, ctx = hip
    uid = H.comm_unique_id()
    with pytest.raises(H.MathError):
        H.Comm(ctx, 2, 2, uid)
    with pytest.raises(H.MathError):
        H.Comm(ctx, 0, 0, uid)
    with pytest.raises(H.MathError):
        H.Comm(ctx, 1, 0, uid[:16])


def test_comm_init_times_out_without_peers(hip, monkeypatch):
    """A communicator whose peers never arrive fails with an error after
    OFHE_COMM_INIT_TIMEOUT_S instead of hanging (non-blocking init polled
    against a deadline); shard.key_broadcaster then falls back on every rank."""
    import time

    H, ctx = hip
    monkeypatch.setenv("OFHE_COMM_INIT_TIMEOUT_S", "3")
    uid = H.comm_unique_id()
    t0 = time.monotonic()
    with pytest.raises(H.MathError, match="timed out"):
        H.Comm(ctx, 2, 0, uid)
    assert time.monotonic() - t0 < 60
