"""CPU checks of the oracle's restatement of ApproxModUp / ApproxModDown,
HYBRID key switching, SwitchModulus and AutomorphismTransform
(oracle/keyswitch.py).  There are no reference golden vectors for these
routines, so the restatement is pinned by exact algebraic identities and by a
semantic key-switching test with real keys (KeySwitchGenInternal,
keyswitch-hybrid.cpp:53-128): ct0 + ct1*s_new must equal c*s_old up to a small
error.  Its building blocks (NTT, ApproxSwitchCRTBasis) are pinned by the
reference's KATs in test_oracle.py.
"""
import numpy as np
import pytest

import keyswitch as K
import oracle as O


def _bases(log_n, sq, sp):
    m, r = O.moduli_chain(log_n, sq + sp)
    return m[:sq], r[:sq], m[sq:], r[sq:]


def _uniform(rng, batch, moduli, n):
    return np.stack([np.stack([rng.integers(0, m, size=n, dtype=np.uint64) for m in moduli])
                     for _ in range(batch)])


def test_switch_modulus_matches_reference_rule():
    # mubintvecnat.cpp:111-136, both branches, edge values
    for om, nm in [(97, 193), (193, 97), (1 << 20, 12289), (12289, 1 << 40), (1152921504606584833, 65537)]:
        v = np.array(sorted({0, 1, om // 2, om // 2 + 1, om - 1, om // 3}), dtype=np.uint64)
        got = K.switch_modulus(v, om, nm)
        for x, y in zip(v, got):
            x = int(x)
            if nm > om:
                e = x + (nm - om) if x > om // 2 else x
            else:
                e = x + (nm - om % nm) if x > om // 2 else x
                e = e % nm if e >= nm else e
            assert int(y) == e
        # centred value is preserved for |value| < min(om, nm)/2
        for x, y in zip(v, got):
            cx = int(x) - om if int(x) > om // 2 else int(x)
            if abs(cx) < min(om, nm) // 2:
                assert (int(y) - cx) % nm == 0


@pytest.mark.parametrize("log_n", [3, 5])
def test_automorphism_forms_agree(log_n):
    n = 1 << log_n
    q, r, _, _ = _bases(log_n, 1, 0)
    rng = np.random.default_rng(7)
    x = _uniform(rng, 1, q, n)
    for k in (1, 3, 5, 2 * n - 1, 2 * n + 3):
        ac = K.automorphism(x[0, 0], k, False, q[0])
        ac = np.where(ac == np.uint64(q[0]), np.uint64(0), ac)  # the reference leaves q for -0
        ev = K.set_format(x, q, r, True)
        ae = K.automorphism(ev[0, 0], k, True, q[0])
        assert np.array_equal(K.set_format(ac[None, None], q, r, True)[0, 0], ae), k
    with pytest.raises(ValueError):
        K.automorphism(x[0, 0], 2, True, q[0])


def test_automorphism_coefficient_rule():
    # X -> X^k on Z_q[X]/(X^n + 1), checked on monomials
    n, q = 8, 17
    for k in (3, 5, 7, 9, 15):
        for j in range(n):
            x = np.zeros(n, np.uint64)
            x[j] = 1
            y = K.automorphism(x, k, False, q)
            e = (j * k) % (2 * n)
            pos, sign = e % n, (e // n) % 2
            assert int(y[pos]) == (q - 1 if sign else 1)
            # zeros moved to a negated slot read q, as in the reference
            assert int(np.count_nonzero(y % np.uint64(q))) == 1


@pytest.mark.parametrize("eval_form", [False, True])
def test_mod_up_is_crt_lift(eval_form):
    log_n, sq, sp = 4, 3, 2
    n = 1 << log_n
    q, rq, p, rp = _bases(log_n, sq, sp)
    rng = np.random.default_rng(11)
    x = _uniform(rng, 2, q, n)
    xin = K.set_format(x, q, rq, True) if eval_form else x
    y = K.approx_mod_up(xin, q, rq, p, rp, eval_form)
    assert y.shape == (2, sq + sp, n)
    assert np.array_equal(y[:, :sq], K.set_format(x, q, rq, True))
    yp = K.set_format(y[:, sq:], p, rp, False)
    Q = int(np.prod([int(v) for v in q], dtype=object))
    qhinv, _ = K.switch_tables(q, p)
    for b in range(2):
        for c in range(n):
            # the un-reduced CRT sum  X + u*Q,  0 <= u < sizeQ
            lift = sum((int(x[b, i, c]) * qhinv[i] % q[i]) * (Q // q[i]) for i in range(sq))
            assert 0 <= lift // Q < sq
            for j in range(sp):
                assert int(yp[b, j, c]) == lift % p[j]


@pytest.mark.parametrize("t", [0, 65537])
def test_mod_down_inverts_p_times_mod_up(t):
    log_n, sq, sp = 5, 3, 2
    n = 1 << log_n
    q, rq, p, rp = _bases(log_n, sq, sp)
    rng = np.random.default_rng(12)
    x = K.set_format(_uniform(rng, 2, q, n), q, rq, True)
    up = K.approx_mod_up(x, q, rq, p, rp, True)
    Pm = int(np.prod([int(v) for v in p], dtype=object))
    scaled = O.mul_scalar(up, [Pm % m for m in q + p], q + p)
    assert not scaled[:, sq:].any()
    assert np.array_equal(K.approx_mod_down(scaled, q, rq, p, rp, t), x)


def test_key_switch_semantics():
    """ct0 + ct1 * s_new == c * s_old + small (mod Q), KeySwitchGenInternal keys."""
    log_n, sq, sp, dnum = 4, 4, 2, 2
    n = 1 << log_n
    q, rq, p, rp = _bases(log_n, sq, sp)
    kp = K.KeySwitchParams(n, q, rq, p, rp, dnum)
    rng = np.random.default_rng(2024)
    s_old, s_new = K.ternary(n, rng), K.ternary(n, rng)
    kb, ka = K.keyswitch_gen(kp, s_old, s_new, rng)
    c = K.set_format(_uniform(rng, 2, q, n), q, rq, True)
    o0, o1 = K.ks_core(kp, c, kb, ka)
    so = K.small_poly_eval(s_old, q, rq)
    sn = K.small_poly_eval(s_new, q, rq)
    B = c.shape[0]
    lhs = O.eltwise("add", o0, O.eltwise("mul", o1, np.repeat(sn, B, 0), q), q)
    rhs = O.eltwise("mul", c, np.repeat(so, B, 0), q)
    d = K.set_format(O.eltwise("sub", lhs, rhs, q), q, rq, False)
    for b in range(B):
        err = K.crt_centered(d[b], q)
        assert max(abs(e) for e in err) < 1 << 16, max(abs(e) for e in err)
    # and the result is not trivially small: c*s_old itself is Q-sized
    assert max(abs(e) for e in K.crt_centered(K.set_format(rhs, q, rq, False)[0], q)) > 1 << 200


def test_key_switch_lower_level_and_partial_digit():
    # alpha = 3: digits {0,1,2}, {3,4}; P needs >= alpha primes (sizeP = ceil(maxBits/auxBits))
    log_n, sq, sp, dnum = 3, 5, 3, 2
    n = 1 << log_n
    q, rq, p, rp = _bases(log_n, sq, sp)
    kp = K.KeySwitchParams(n, q, rq, p, rp, dnum)
    assert kp.alpha == 3 and kp.beta(5) == 2 and kp.beta(3) == 1 and kp.beta(4) == 2
    assert kp.complement(4, 1)[0] == q[:3] + p
    rng = np.random.default_rng(5)
    s_old, s_new = K.ternary(n, rng), K.ternary(n, rng)
    kb, ka = K.keyswitch_gen(kp, s_old, s_new, rng)
    for l in (5, 4, 2):
        c = K.set_format(_uniform(rng, 1, q[:l], n), q[:l], rq[:l], True)
        o0, o1 = K.ks_core(kp, c, kb, ka)
        sn = K.small_poly_eval(s_new, q[:l], rq[:l])
        so = K.small_poly_eval(s_old, q[:l], rq[:l])
        lhs = O.eltwise("add", o0, O.eltwise("mul", o1, sn, q[:l]), q[:l])
        d = K.set_format(O.eltwise("sub", lhs, O.eltwise("mul", c, so, q[:l]), q[:l]), q[:l], rq[:l], False)
        assert max(abs(e) for e in K.crt_centered(d[0], q[:l])) < 1 << 16


def test_key_switch_param_errors():
    q, rq, p, rp = _bases(3, 5, 1)
    with pytest.raises(ValueError):
        K.KeySwitchParams(8, q, rq, p, rp, 4)  # ceil(5/4)=2: 5 - 2*3 <= 0


def test_switch_modulus_reference_kat():
    """UnitTestPolyElements.cpp:265-305: {56,1,37,2} mod 73 -> mod 17 = {0,1,15,2};
    {56,43,35,28} mod 73 -> mod 193 = {176,163,35,28}."""
    from conftest import load_golden

    k = load_golden("reference_fixtures.json")["kat_switch_modulus"]
    for c in k["cases"]:
        got = K.switch_modulus(np.array(c["x"], np.uint64), k["q"], c["new_q"])
        assert got.tolist() == c["expected"]


def test_automorphism_reference_kat():
    """UnitTestPolyElements.cpp:500-523: AutomorphismTransform(3) of {56,1,37,2}
    mod 73 in coefficient form = {56,2,36,1}; and the evaluation-form map agrees
    with it through the NTT (q = 73, m = 8, root 22)."""
    from conftest import load_golden

    k = load_golden("reference_fixtures.json")["kat_automorphism"]
    x = np.array(k["x"], np.uint64)
    assert K.automorphism(x, k["k"], False, k["q"]).tolist() == k["expected"]
    tb = O.Tables(4, [k["q"]], [k["root"]])
    ev = O.ntt_fwd(x.reshape(1, 1, 4), tb).reshape(-1)
    back = O.ntt_inv(K.automorphism(ev, k["k"], True, k["q"]).reshape(1, 1, 4), tb).reshape(-1)
    assert back.tolist() == k["expected"]
    # UnitTestPolyElements.cpp:535-571: Transpose = AutomorphismTransform(m - 1), evaluation form
    t = k["transpose"]
    ev = O.ntt_fwd(np.array(t["x"], np.uint64).reshape(1, 1, 4), tb).reshape(-1)
    back = O.ntt_inv(K.automorphism(ev, t["k"], True, k["q"]).reshape(1, 1, 4), tb).reshape(-1)
    assert back.tolist() == t["expected"]


@pytest.mark.parametrize("log_n", [2, 5, 10])
@pytest.mark.parametrize("eval_form", [False, True])
def test_c_oracle_automorphism_equals_python(log_n, eval_form):
    """oracle_automorphism (C, used by tests/cpp/test_hooks.cpp) equals the
    Python restatement of PolyImpl::AutomorphismTransform (poly-impl.h:312-365)
    for every odd k below 2N, zeros included (a negated zero stays q)."""
    import ctypes

    n = 1 << log_n
    q, _ = O.moduli_chain(max(log_n, 2), 1)
    q = q[0]
    rng = np.random.default_rng(log_n)
    x = rng.integers(0, q, size=n, dtype=np.uint64)
    x[::3] = 0
    L = O.lib()
    for k in range(1, 2 * n, 2):
        out = np.zeros(n, np.uint64)
        L.oracle_automorphism(x.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                              out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), n, k, int(eval_form), q)
        assert np.array_equal(out, K.automorphism(x, k, eval_form, q)), k
