"""CPU: the oracle's BV key switching with digitSize = 0 (oracle/keyswitch.py:
crt_decompose0, bv_fast_core; keyswitch-bv.cpp:302-340, dcrtpoly-impl.h:266-288)
against the algebra the reference's key generation (keyswitch-bv.cpp:99-111)
makes exact -- "parity unpinned" against reference-run data (none exists for
this path), pinned by identities instead:
  * every digit's tower i is c's tower i (CRTDecompose(0) keeps it);
  * digit i in coefficient form is tower i's coefficients re-centred into each
    tower (SwitchModulus);
  * with keys bv[i] = filtered_i - (a_i s_new + e_i):
    ct0 + ct1 s_new = c s_old - sum_i d_i e_i, exactly, tower by tower."""
import numpy as np
import pytest

import keyswitch as K
import oracle as O


@pytest.mark.parametrize("log_n,T", [(6, 2), (10, 3)])
def test_bv_identity(log_n, T):
    n = 1 << log_n
    q, rq = O.moduli_chain(log_n, T)
    rng = np.random.default_rng(3 + log_n)
    c = np.stack([np.stack([rng.integers(0, qi, size=n, dtype=np.uint64) for qi in q])])
    d = K.crt_decompose0(c, q, rq)
    for i in range(T):
        assert np.array_equal(d[0, i, i], c[0, i])
    coef_c = K.set_format(c, q, rq, False)
    coef_d1 = K.set_format(d[:, 1], q, rq, False)
    for k in range(T):
        assert np.array_equal(coef_d1[0, k], K.switch_modulus(coef_c[0, 1], q[1], q[k]))
    s_old = K.small_poly_eval(rng.integers(-1, 2, size=n), q, rq)[0]
    s_new = K.small_poly_eval(rng.integers(-1, 2, size=n), q, rq)[0]
    kb, ka, es = K.bv_keygen(q, rq, s_old, s_new, rng)
    o0, o1 = K.bv_fast_core(d, kb, ka, q)
    lhs = O.eltwise("add", o0, O.eltwise("mul", o1, s_new[None], q), q)
    noise = O.eltwise("mul", d[:, 0], es[0:1], q)
    for i in range(1, T):
        noise = O.eltwise("add", noise, O.eltwise("mul", d[:, i], es[i:i + 1], q), q)
    rhs = O.eltwise("sub", O.eltwise("mul", c, s_old[None], q), noise, q)
    assert np.array_equal(lhs, rhs)
