"""CPU: the oracle's restatement of the rescaling callers
(oracle/keyswitch.py: drop_last_and_scale, mod_reduce; dcrtpoly-impl.h:746-812)
against exact big-integer semantics -- parity unpinned against reference-run
data (the reference cannot be built here and its tests hold no vectors for
these), pinned instead by what the reference's constants make the operations
compute:
  * DropLastElementAndScale with ckksrns-cryptoparameters.cpp:65-86's tables
    is rounding division by q_l: |Y q_l - X| <= q_l / 2 for the centred CRT
    values X (input) and Y (output);
  * ModReduce with negtInvModq = -t^-1 mod q_l is exact division of X + t delta:
    Y q_l = X (mod t), |Y q_l - X| <= t q_l / 2;
  * evaluation-form and coefficient-form inputs give the same result (the
    reference's coefficient-form DropLastElementAndScale returns evaluation-form
    towers, dcrtpoly-impl.h:765-766).
"""
import numpy as np
import pytest

import keyswitch as K
import oracle as O


def _case(log_n, T, B, seed):
    n = 1 << log_n
    q, r = O.moduli_chain(log_n, T)
    rng = np.random.default_rng(seed)
    x = np.stack([np.stack([rng.integers(0, qi, size=n, dtype=np.uint64) for qi in q]) for _ in range(B)])
    return n, q, r, x


@pytest.mark.parametrize("log_n,T", [(6, 2), (10, 4), (12, 3)])
def test_rescale_is_rounding_division(log_n, T):
    n, q, r, x = _case(log_n, T, 2, 11 + log_n)
    c, a = K.rescale_tables(q)
    out = K.drop_last_and_scale(x, q, r, False, c, a)
    y = K.set_format(out, q[:-1], r[:-1], False)
    ql = q[-1]
    for b in range(x.shape[0]):
        X, Y = K.crt_centered(x[b], q), K.crt_centered(y[b], q[:-1])
        assert all(2 * abs(Y[i] * ql - X[i]) <= ql for i in range(n))
    xe = K.set_format(x, q, r, True)
    assert np.array_equal(K.drop_last_and_scale(xe, q, r, True, c, a), out)


@pytest.mark.parametrize("t", [2, 65537])
def test_mod_reduce_is_exact_division(t):
    n, q, r, x = _case(10, 4, 2, 7)
    ql = q[-1]
    _, a = K.rescale_tables(q)
    negtinv = (-pow(t, -1, ql)) % ql
    out = K.mod_reduce(x, q, r, False, t, negtinv, a)
    for b in range(x.shape[0]):
        X, Y = K.crt_centered(x[b], q), K.crt_centered(out[b], q[:-1])
        assert all((Y[i] * ql - X[i]) % t == 0 and 2 * abs(Y[i] * ql - X[i]) <= t * ql for i in range(n))
    xe = K.set_format(x, q, r, True)
    oe = K.mod_reduce(xe, q, r, True, t, negtinv, a)
    assert np.array_equal(K.set_format(oe, q[:-1], r[:-1], False), out)
