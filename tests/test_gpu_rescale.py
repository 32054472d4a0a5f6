"""GPU parity for the rescaling callers (ofhe_hip_drop_last_and_scale,
ofhe_hip_mod_reduce; DCRTPolyImpl::DropLastElementAndScale / ModReduce,
dcrtpoly-impl.h:746-812) through the C ABI, bit-exact against
oracle/keyswitch.py (itself checked against exact big-integer semantics in
tests/test_rescale_oracle.py).  Shapes cover the small-N path (k_small /
k_sub_scale), the fused forward-subtract block pass (N >= 2^12), N = 2^16's
k_tcols split and N = 2^17; both forms; in place and with padded strides."""
import numpy as np
import pytest

import keyswitch as K
import oracle as O
from test_gpu_parity import dev, host, stream

pytestmark = pytest.mark.gpu

SHAPES = [(10, 3, 2), (12, 4, 1), (14, 5, 3), (16, 3, 2), (17, 2, 1)]


def _case(log_n, T, B, seed):
    n = 1 << log_n
    q, r = O.moduli_chain(log_n, T)
    rng = np.random.default_rng(seed)
    x = np.stack([np.stack([rng.integers(0, qi, size=n, dtype=np.uint64) for qi in q]) for _ in range(B)])
    return n, q, r, x


@pytest.mark.parametrize("log_n,T,B", SHAPES)
@pytest.mark.parametrize("eval_form", [True, False])
def test_drop_last_and_scale_vs_oracle(hip, log_n, T, B, eval_form):
    import torch

    H, ctx = hip
    n, q, r, x = _case(log_n, T, B, 40 + log_n)
    c, a = K.rescale_tables(q)
    want = K.drop_last_and_scale(x, q, r, eval_form, c, a)
    plan = H.NTTPlan(ctx, log_n, q, r)
    dx = dev(x)
    out = torch.zeros((B, T - 1, n), dtype=torch.int64, device="cuda")
    plan.drop_last_and_scale(T, dx.data_ptr(), T * n, out.data_ptr(), (T - 1) * n, eval_form, c, a, B, stream())
    assert np.array_equal(host(out), want)
    # in place: the result in the first T - 1 towers of each batch entry
    plan.drop_last_and_scale(T, dx.data_ptr(), T * n, dx.data_ptr(), T * n, eval_form, c, a, B, stream())
    assert np.array_equal(host(dx)[:, :T - 1], want)


@pytest.mark.parametrize("log_n,T,B", SHAPES)
@pytest.mark.parametrize("eval_form", [True, False])
@pytest.mark.parametrize("t", [2, 65537])
def test_mod_reduce_vs_oracle(hip, log_n, T, B, eval_form, t):
    import torch

    H, ctx = hip
    n, q, r, x = _case(log_n, T, B, 70 + log_n + t)
    _, a = K.rescale_tables(q)
    negtinv = (-pow(t, -1, q[-1])) % q[-1]
    want = K.mod_reduce(x, q, r, eval_form, t, negtinv, a)
    plan = H.NTTPlan(ctx, log_n, q, r)
    dx = dev(x)
    # padded output stride: one spare tower per batch entry
    out = torch.zeros((B, T, n), dtype=torch.int64, device="cuda")
    plan.mod_reduce(T, dx.data_ptr(), T * n, out.data_ptr(), T * n, eval_form, t, negtinv, a, B, stream())
    got = host(out)
    assert np.array_equal(got[:, :T - 1], want)
    assert not got[:, T - 1].any()


def test_rescale_lower_level_and_edges(hip):
    """A lower level of a longer chain (the first 3 of 5 plan towers), all-(q-1)
    inputs, and the argument errors of DropLastElement (one tower)."""
    import torch

    H, ctx = hip
    log_n, B = 13, 2
    n = 1 << log_n
    qa, ra = O.moduli_chain(log_n, 5)
    T = 3
    q, r = qa[:T], ra[:T]
    x = np.broadcast_to(np.array(q, np.uint64)[None, :, None] - np.uint64(1), (B, T, n)).copy()
    c, a = K.rescale_tables(q)
    plan = H.NTTPlan(ctx, log_n, qa, ra)
    for ev in (True, False):
        dx = dev(x)
        out = torch.zeros((B, T - 1, n), dtype=torch.int64, device="cuda")
        plan.drop_last_and_scale(T, dx.data_ptr(), T * n, out.data_ptr(), (T - 1) * n, ev, c, a, B, stream())
        assert np.array_equal(host(out), K.drop_last_and_scale(x, q, r, ev, c, a))
    dx = dev(x)
    with pytest.raises(H.MathError):
        plan.drop_last_and_scale(1, dx.data_ptr(), n, dx.data_ptr(), n, True, c, a, B, stream())
    with pytest.raises(H.MathError):  # qlInvModq must be invertible in evaluation form
        plan.drop_last_and_scale(T, dx.data_ptr(), T * n, dx.data_ptr(), T * n, True, c, [0] * (T - 1), B, stream())


def test_rescale_rejects_unsafe_aliasing(hip):
    """out may be x only in place with equal strides.  A packed
    output over the input (out_stride = (towers-1)N < x_stride, batch >= 2)
    would overwrite towers of the previous entry that other workgroups still
    read, so it is refused; so is a partial overlap.  In place with equal
    strides still matches the oracle, and the context's scratch pool can be
    trimmed afterwards."""
    H, ctx = hip
    log_n, T, B = 13, 4, 3
    n, q, r, x = _case(log_n, T, B, 99)
    c, a = K.rescale_tables(q)
    plan = H.NTTPlan(ctx, log_n, q, r)
    dx = dev(x)
    for ev in (True, False):
        with pytest.raises(H.MathError, match="overlaps"):
            plan.drop_last_and_scale(T, dx.data_ptr(), T * n, dx.data_ptr(), (T - 1) * n, ev, c, a, B, stream())
        with pytest.raises(H.MathError, match="overlaps"):
            plan.drop_last_and_scale(T, dx.data_ptr(), T * n, dx.data_ptr() + 8 * n, T * n, ev, c, a, B, stream())
        with pytest.raises(H.MathError, match="overlaps"):
            plan.mod_reduce(T, dx.data_ptr(), T * n, dx.data_ptr(), (T - 1) * n, ev, 2, 1, a, B, stream())
    assert np.array_equal(host(dx), x)  # nothing was launched
    plan.drop_last_and_scale(T, dx.data_ptr(), T * n, dx.data_ptr(), T * n, True, c, a, B, stream())
    assert np.array_equal(host(dx)[:, :T - 1], K.drop_last_and_scale(x, q, r, True, c, a))
    ctx.trim(0)
