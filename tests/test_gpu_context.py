"""GPU tests of the device context's lifetime rules (ofhe_hip_init /
ofhe_hip_finalize, the PimManager::getPim analogue, PimManager.h:23-29):
ofhe_hip_alloc_async blocks come from the context's own pool, so finalize must
refuse while any of them is still allocated (destroying the pool would free
them under the caller), and succeed once they are freed."""
import pytest

from test_gpu_parity import stream

pytestmark = pytest.mark.gpu


def test_finalize_refused_while_async_blocks_live():
    import torch

    import ofhe_hip as H

    ctx = H.Context(0)
    s = stream()
    p1 = ctx.alloc_async(1 << 20, s)
    p2 = ctx.alloc_async(4096, s)
    with pytest.raises(H.MathError, match="still allocated"):
        ctx.close()
    # the context is still usable: a block can be written and read back
    t = torch.arange(512, dtype=torch.int64, device="cuda")
    ctx.copy_device(p2, t.data_ptr(), 4096, s)
    back = torch.empty_like(t)
    ctx.copy_device(back.data_ptr(), p2, 4096, s)
    torch.cuda.synchronize()
    assert torch.equal(back, t)
    ctx.free_async(p1, s)
    with pytest.raises(H.MathError, match="1 ofhe_hip_alloc_async"):
        ctx.close()
    ctx.free_async(p2, s)
    ctx.free_async(0, s)  # NULL: no-op, not counted
    torch.cuda.synchronize()
    ctx.close()
    with pytest.raises(H.MathError):
        ctx.alloc_async(64, s)


def test_closed_context_rejects_use():
    import ofhe_hip as H

    ctx = H.Context(0)
    ctx.close()
    ctx.close()  # idempotent on the Python side
    with pytest.raises(H.MathError):
        _ = ctx.handle


def test_free_async_refuses_foreign_and_double_frees():
    """ofhe_hip_free_async accepts only live ofhe_hip_alloc_async blocks of its
    context: a hipMalloc'd pointer or a second free of the same block is an
    argument error and leaves the live-block accounting (and so finalize's
    refusal) intact (round-4 advisor finding)."""
    import ofhe_hip as H

    ctx = H.Context(0)
    s = stream()
    p = ctx.alloc_async(4096, s)
    plain = ctx.alloc(4096)
    with pytest.raises(H.MathError, match="not a live"):
        ctx.free_async(plain, s)
    ctx.free(plain)
    ctx.free_async(p, s)
    with pytest.raises(H.MathError, match="not a live"):
        ctx.free_async(p, s)
    q = ctx.alloc_async(64, s)
    with pytest.raises(H.MathError, match="1 ofhe_hip_alloc_async"):
        ctx.close()
    ctx.free_async(q, s)
    ctx.sync(s)
    ctx.close()


def test_event_marks_stream_work_and_outlives_its_context():
    """ofhe_hip_event_* (the adapter's staged-copy ordering): an event recorded
    after a copy on the stream, synchronised, sees the copy done; an event made
    before ofhe_hip_finalize is still destroyed cleanly after it (it keeps the
    device id, not the freed context)."""
    import ctypes

    import torch

    import ofhe_hip as H

    L = H.lib()
    vp = ctypes.c_void_p
    ctx = H.Context(0)
    s = stream()
    ev = vp()
    H._check(L.ofhe_hip_event_create(ctx.handle, ctypes.byref(ev)))
    src = torch.arange(1 << 20, dtype=torch.int64, device="cuda")
    dst = torch.empty_like(src)
    ctx.copy_device(dst.data_ptr(), src.data_ptr(), src.numel() * 8, s)
    H._check(L.ofhe_hip_event_record(ev, vp(s or None)))
    H._check(L.ofhe_hip_event_sync(ev))
    assert torch.equal(dst, src)
    ctx.close()  # frees the context
    H._check(L.ofhe_hip_event_destroy(ev))
