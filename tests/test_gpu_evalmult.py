"""GPU parity for the fused EvalMultCore tensor product (ofhe_hip_eval_mult_core;
LeveledSHEBase::EvalMultCore, base-leveledshe.cpp:667-672) through the C ABI:
bit-exact against the reference's own sequence of DCRTPoly ModMul / ModAdd
restated on the oracle (O.eltwise), on random, all-(q-1) and ragged shapes, and
the identity (c0 + c1 s)(d0 + d1 s) = o0 + o1 s + o2 s^2 that makes it the
ciphertext product."""
import numpy as np
import pytest

import oracle as O
from test_gpu_parity import dev, host, stream

pytestmark = pytest.mark.gpu


def _ref(c0, c1, d0, d1, q):
    o2 = O.eltwise("mul", c1, d1, q)                                   # cv1[1] * cv2[1]
    o1 = O.eltwise("mul", c1, d0, q)                                   # cv1[1] *= cv2[0]
    o0 = O.eltwise("mul", d0, c0, q)                                   # cv2[0] * cv1[0]
    o1 = O.eltwise("add", o1, O.eltwise("mul", c0, d1, q), q)          # += (cv1[0] *= cv2[1])
    return o0, o1, o2


@pytest.mark.parametrize("log_n,T,B,edge", [(4, 2, 3, False), (12, 3, 2, False), (16, 4, 1, False),
                                            (14, 2, 2, True)])
def test_eval_mult_core_vs_oracle(hip, log_n, T, B, edge):
    import torch

    H, ctx = hip
    n = 1 << log_n
    q, rq = O.moduli_chain(log_n, T)
    rng = np.random.default_rng(123 + log_n)
    if edge:
        xs = [np.broadcast_to(np.array(q, np.uint64)[None, :, None] - np.uint64(1), (B, T, n)).copy()
              for _ in range(4)]
    else:
        xs = [np.stack([np.stack([rng.integers(0, qi, size=n, dtype=np.uint64) for qi in q]) for _ in range(B)])
              for _ in range(4)]
    plan = H.NTTPlan(ctx, log_n, q, rq)
    dx = [dev(x) for x in xs]
    outs = [torch.empty_like(dx[0]) for _ in range(3)]
    plan.eval_mult_core(*(t.data_ptr() for t in dx), *(o.data_ptr() for o in outs), B, stream())
    want = _ref(*xs, q)
    for o, w in zip(outs, want):
        assert np.array_equal(host(o), w)
    if not edge:
        s = np.stack([np.stack([rng.integers(0, qi, size=n, dtype=np.uint64) for qi in q]) for _ in range(B)])
        mul = lambda a, b: O.eltwise("mul", a, b, q)  # noqa: E731
        add = lambda a, b: O.eltwise("add", a, b, q)  # noqa: E731
        lhs = mul(add(xs[0], mul(xs[1], s)), add(xs[2], mul(xs[3], s)))
        o = [host(t) for t in outs]
        assert np.array_equal(lhs, add(add(o[0], mul(o[1], s)), mul(o[2], mul(s, s))))
