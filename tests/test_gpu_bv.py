"""GPU parity for BV key switching with digitSize = 0 (ofhe_hip_bv_precompute,
ofhe_hip_bv_core; keyswitch-bv.cpp:302-340, dcrtpoly-impl.h:266-288) through
the C ABI, bit-exact against oracle/keyswitch.py (pinned by the identities of
tests/test_bv_oracle.py).  Shapes cover the unfused path (N <= 2^12: lift
kernel + transform), the fused lift in k_cols (2^13..2^15, 2^17) and in
k_tcols (2^16); a lower level uses the first towers of longer keys."""
import numpy as np
import pytest

import keyswitch as K
import oracle as O
from test_gpu_parity import dev, host, stream

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("log_n,T,B,key_extra", [(10, 3, 2, 0), (12, 2, 1, 1), (13, 4, 2, 0), (16, 3, 1, 1),
                                                 (17, 2, 1, 0)])
def test_bv_vs_oracle(hip, log_n, T, B, key_extra):
    import torch

    H, ctx = hip
    n = 1 << log_n
    qa, ra = O.moduli_chain(log_n, T + key_extra)
    q, rq = qa[:T], ra[:T]
    rng = np.random.default_rng(90 + log_n)
    c = np.stack([np.stack([rng.integers(0, qi, size=n, dtype=np.uint64) for qi in q]) for _ in range(B)])
    TK = T + key_extra
    kb = np.stack([np.stack([rng.integers(0, qi, size=n, dtype=np.uint64) for qi in qa]) for _ in range(T)])
    ka = np.stack([np.stack([rng.integers(0, qi, size=n, dtype=np.uint64) for qi in qa]) for _ in range(T)])
    want_d = K.crt_decompose0(c, q, rq)
    want0, want1 = K.bv_fast_core(want_d, kb, ka, q)
    plan = H.NTTPlan(ctx, log_n, qa, ra)
    dc = dev(c)
    dd = torch.empty((B, T, T, n), dtype=torch.int64, device="cuda")
    plan.bv_precompute(T, dc.data_ptr(), dd.data_ptr(), B, stream())
    assert np.array_equal(host(dd), want_d)
    dkb, dka = dev(kb), dev(ka)
    o0 = torch.empty((B, T, n), dtype=torch.int64, device="cuda")
    o1 = torch.empty_like(o0)
    plan.bv_core(T, dd.data_ptr(), dkb.data_ptr(), dka.data_ptr(), TK, o0.data_ptr(), o1.data_ptr(), B, stream())
    assert np.array_equal(host(o0), want0)
    assert np.array_equal(host(o1), want1)


def test_bv_semantic_and_max_sums(hip):
    """Real BV keys (KeySwitchGenInternal, digitSize = 0): ct0 + ct1 s_new =
    c s_old - sum_i d_i e_i on the device outputs; then all-(q-1) digits and keys
    (the 128-bit accumulation's largest sums)."""
    import torch

    H, ctx = hip
    log_n, T = 12, 4
    n = 1 << log_n
    q, rq = O.moduli_chain(log_n, T)
    rng = np.random.default_rng(17)
    c = np.stack([np.stack([rng.integers(0, qi, size=n, dtype=np.uint64) for qi in q])])
    s_old = K.small_poly_eval(rng.integers(-1, 2, size=n), q, rq)[0]
    s_new = K.small_poly_eval(rng.integers(-1, 2, size=n), q, rq)[0]
    kb, ka, es = K.bv_keygen(q, rq, s_old, s_new, rng)
    plan = H.NTTPlan(ctx, log_n, q, rq)
    dd = torch.empty((1, T, T, n), dtype=torch.int64, device="cuda")
    plan.bv_precompute(T, dev(c).data_ptr(), dd.data_ptr(), 1, stream())
    o0 = torch.empty((1, T, n), dtype=torch.int64, device="cuda")
    o1 = torch.empty_like(o0)
    dkb, dka = dev(kb), dev(ka)
    plan.bv_core(T, dd.data_ptr(), dkb.data_ptr(), dka.data_ptr(), T, o0.data_ptr(), o1.data_ptr(), 1, stream())
    d = host(dd)
    lhs = O.eltwise("add", host(o0), O.eltwise("mul", host(o1), s_new[None], q), q)
    noise = O.eltwise("mul", d[:, 0], es[0:1], q)
    for i in range(1, T):
        noise = O.eltwise("add", noise, O.eltwise("mul", d[:, i], es[i:i + 1], q), q)
    assert np.array_equal(lhs, O.eltwise("sub", O.eltwise("mul", c, s_old[None], q), noise, q))
    qm = np.array(q, np.uint64)[None, :, None] - np.uint64(1)
    big = np.broadcast_to(qm[:, None], (1, T, T, n)).copy()
    keys = np.broadcast_to(qm, (T, T, n)).copy()
    dbig, dkey = dev(big), dev(keys)
    plan.bv_core(T, dbig.data_ptr(), dkey.data_ptr(), dkey.data_ptr(), T, o0.data_ptr(), o1.data_ptr(), 1, stream())
    want, _ = K.bv_fast_core(big, keys, keys, q)
    assert np.array_equal(host(o0), want)
