"""GPU parity for SURVEY.md §8(f) rows 1-3 through the C ABI: tower-range
NTTs, ApproxModUp / ApproxModDown, HYBRID key switching (precompute, inner
product, ModDown, KeySwitchCore), SwitchModulus and AutomorphismTransform.
Bit-exact against oracle/keyswitch.py, whose restatement is pinned by
tests/test_keyswitch_oracle.py (exact identities + a semantic key-switch test).
"""
import numpy as np
import pytest

import keyswitch as K
import oracle as O
from test_gpu_parity import dev, host, stream

pytestmark = pytest.mark.gpu


def _bases(log_n, sq, sp):
    m, r = O.moduli_chain(log_n, sq + sp)
    return m[:sq], r[:sq], m[sq:], r[sq:]


def _generic_bases(log_n, sq, sp):
    """moduli far from 2^60 (no special-prime form): exercises Mod<false>."""
    m = 2 << log_n
    qs, rs = [], []
    x = O.next_prime((1 << 50) + 1 + 12345 * m, m)  # candidates = 1 mod 2N
    while len(qs) < sq + sp:
        qs.append(x)
        rs.append(O.root_of_unity(m, x))
        x = O.next_prime(x + 977 * m, m)
    return qs[:sq], rs[:sq], qs[sq:], rs[sq:]


def _uniform(rng, batch, moduli, n):
    return np.stack([np.stack([rng.integers(0, m, size=n, dtype=np.uint64) for m in moduli])
                     for _ in range(batch)])


@pytest.mark.parametrize("log_n", [4, 11, 12, 13, 16])
def test_range_transforms_strided(hip, log_n):
    H, ctx = hip
    import torch

    n = 1 << log_n
    q, r = O.moduli_chain(log_n, 5)
    plan = H.NTTPlan(ctx, log_n, q, r)
    rng = np.random.default_rng(log_n)
    B = 2
    x = _uniform(rng, B, q, n)
    # towers [1, 4) of a 5-tower polynomial into a 7-tower-wide buffer at tower 2
    src = dev(x)
    dst = torch.zeros((B, 7, n), dtype=torch.int64, device="cuda")
    plan.forward_range(1, 3, src[:, 1].data_ptr(), dst[:, 2].data_ptr(), 5 * n, 7 * n, B, stream())
    got = host(dst)
    ref = K.set_format(x[:, 1:4], q[1:4], r[1:4], True)
    assert np.array_equal(got[:, 2:5], ref)
    assert not got[:, :2].any() and not got[:, 5:].any()
    back = torch.zeros((B, 3, n), dtype=torch.int64, device="cuda")
    plan.inverse_range(1, 3, dst[:, 2].data_ptr(), back.data_ptr(), 7 * n, 3 * n, B, stream())
    assert np.array_equal(host(back), x[:, 1:4])
    # in place on a strided view
    y = dev(x)
    plan.forward_range(4, 1, y[:, 4].data_ptr(), y[:, 4].data_ptr(), 5 * n, 5 * n, B, stream())
    g = host(y)
    assert np.array_equal(g[:, 4:], K.set_format(x[:, 4:], q[4:], r[4:], True))
    assert np.array_equal(g[:, :4], x[:, :4])


def test_range_errors(hip):
    H, ctx = hip
    import torch

    q, r = O.moduli_chain(6, 2)
    plan = H.NTTPlan(ctx, 6, q, r)
    x = torch.zeros((1, 2, 64), dtype=torch.int64, device="cuda")
    with pytest.raises(H.MathError):
        plan.forward_range(1, 2, x.data_ptr(), x.data_ptr(), 128, 128, 1, stream())
    with pytest.raises(H.MathError):
        plan.forward_range(0, 2, x.data_ptr(), x.data_ptr(), 64, 128, 1, stream())


def _converter(H, ctx, log_n, src, dst):
    qhinv, qhmodp = K.switch_tables(src, dst)
    return H.BaseConverter(ctx, log_n, src, dst, qhinv, [v for row in qhmodp for v in row])


@pytest.mark.parametrize("log_n,sq,sp,generic", [(5, 3, 2, False), (12, 4, 2, False), (13, 3, 3, True),
                                                 (16, 4, 2, False), (17, 16, 6, False), (17, 5, 9, True)])
@pytest.mark.parametrize("eval_form", [True, False])
def test_approx_mod_up(hip, log_n, sq, sp, generic, eval_form):
    H, ctx = hip
    import torch

    n = 1 << log_n
    q, rq, p, rp = (_generic_bases if generic else _bases)(log_n, sq, sp)
    pq, pp = H.NTTPlan(ctx, log_n, q, rq), H.NTTPlan(ctx, log_n, p, rp)
    bc = _converter(H, ctx, log_n, q, p)
    rng = np.random.default_rng(3 + log_n)
    B = 2
    x = _uniform(rng, B, q, n)
    if eval_form:
        x = K.set_format(x, q, rq, True)
    out = torch.empty((B, sq + sp, n), dtype=torch.int64, device="cuda")
    dx = dev(x)  # keep device inputs referenced until the stream has consumed them
    H.approx_mod_up(pq, pp, bc, eval_form, dx.data_ptr(), out.data_ptr(), B, stream())
    assert np.array_equal(host(out), K.approx_mod_up(x, q, rq, p, rp, eval_form))


@pytest.mark.parametrize("log_n,sq,sp,generic", [(5, 3, 2, False), (12, 4, 2, True), (14, 5, 3, False),
                                                 (17, 6, 16, False), (17, 7, 3, True)])
@pytest.mark.parametrize("t", [0, 65537])
def test_approx_mod_down(hip, log_n, sq, sp, generic, t):
    H, ctx = hip
    import torch

    n = 1 << log_n
    q, rq, p, rp = (_generic_bases if generic else _bases)(log_n, sq, sp)
    pq, pp = H.NTTPlan(ctx, log_n, q, rq), H.NTTPlan(ctx, log_n, p, rp)
    bc = _converter(H, ctx, log_n, p, q)
    T = K.moddown_tables(q, p, t)
    rng = np.random.default_rng(5 + log_n + t)
    B = 3
    x = _uniform(rng, B, q + p, n)
    out = torch.empty((B, sq, n), dtype=torch.int64, device="cuda")
    dx = dev(x)
    H.approx_mod_down(pq, pp, bc, T["pinv_modq"], t, dx.data_ptr(), out.data_ptr(), B, stream())
    assert np.array_equal(host(out), K.approx_mod_down(x, q, rq, p, rp, t))


@pytest.mark.parametrize("sq,reps,log_n", [(1, 1, 5), (7, 1, 5), (16, 1, 5), (17, 1, 5), (32, 1, 5), (33, 1, 5),
                                           (64, 1, 5), (16, 8, 5), (40, 24, 5), (65, 1, 5), (7, 1, 4)])
def test_base_conversion_max_sums(hip, sq, reps, log_n):
    """Extreme sums for every base-conversion kernel: inputs q_i - 1 (q_i up
    to 2^60 - 1) and 0x007F7F7F7F7F7F80 (seven signed base-256 digits of
    -128 in the matrix-core kernel's digit split), QHatInvModq = 1 and every
    QHatModp entry p_j - 1, for output moduli from 2 to 2^60 - 1 (powers of
    two included).  k_bconv_mma for size_q <= 64: K-steps 1, 2, 4, 5, 8 and
    the wide partial sums at 10 (33 sources) and 16 (64); 16 -> 72 and
    40 -> 216 targets run in several target chunks (blockIdx.y).  size_q = 65
    runs the 128-bit k_bconv, N = 16 (below one 32-coefficient group)
    k_bconv_limb.  Expected values by Python integers:
    out_j = sum_i x_i (p_j - 1) mod p_j."""
    H, ctx = hip
    import torch

    n = 1 << log_n
    q = [(1 << 60) - 1 - 2 * i for i in range(sq)]
    p = [2, 3, 1 << 31, (1 << 32) + 15, (1 << 45) + 7, (1 << 59) + 1, (1 << 60) - 1, 1 << 59, 97] * reps
    bc = H.BaseConverter(ctx, log_n, q, p, [1] * sq, [pj - 1 for _ in q for pj in p])
    rng = np.random.default_rng(sq)
    x = np.stack([np.full(n, qi - 1, np.uint64) for qi in q])
    x[:, 1::2] = np.stack([rng.integers(0, qi, size=n // 2, dtype=np.uint64) for qi in q])
    x[:, 2::4] = np.uint64(0x007F7F7F7F7F7F80)
    dx = dev(x[None])
    out = torch.zeros((1, len(p), n), dtype=torch.int64, device="cuda")
    bc.switch(dx.data_ptr(), out.data_ptr(), 1, stream())
    xs = [sum(int(x[i, k]) for i in range(sq)) for k in range(n)]
    want = np.array([[xs[k] * (pj - 1) % pj for k in range(n)] for pj in p], np.uint64)
    assert np.array_equal(host(out)[0], want)


@pytest.mark.parametrize("sq,sp,log_n", [(3, 5, 5), (16, 48, 6), (12, 4, 12)])
def test_base_conversion_kernel_options(hip, sq, sp, log_n):
    """Every base-conversion kernel the converter options select (matrix
    cores, 30-bit limbs, 128-bit sums) gives the oracle's ApproxSwitchCRTBasis
    on the same inputs (extreme residues q - 1 in half the positions)."""
    H, ctx = hip
    import torch

    n = 1 << log_n
    q, rq, p, rp = _bases(log_n, sq, sp)
    qhinv, qhmodp = K.switch_tables(q, p)
    rng = np.random.default_rng(sq * 100 + sp)
    x = _uniform(rng, 2, q, n)
    x[:, :, ::2] = np.array(q, np.uint64)[None, :, None] - np.uint64(1)
    want = K._switch_basis(x, q, p, qhinv, qhmodp)
    dx = dev(x)
    for kern in (H.BCONV_KERNEL_AUTO, H.BCONV_KERNEL_LIMB, H.BCONV_KERNEL_WIDE):
        bc = H.BaseConverter(ctx, log_n, q, p, qhinv, [v for row in qhmodp for v in row], kernel=kern)
        out = torch.zeros((2, sp, n), dtype=torch.int64, device="cuda")
        bc.switch(dx.data_ptr(), out.data_ptr(), 2, stream())
        assert np.array_equal(host(out), want), kern
        bc.close()


@pytest.mark.parametrize("sq", [3, 16])
def test_base_conversion_special_primes(hip, sq):
    """Targets that are all of the form 2^L - d (k_bconv_mma's shift fold,
    bm_reduce<.., SPQ>): d = 1 and d = 2^32 - 1 at L = 60, and the smallest L
    the host admits for a large d, with the same extreme inputs as
    test_base_conversion_max_sums.  Expected values by Python integers."""
    H, ctx = hip
    import torch

    log_n, n = 5, 32
    q = [(1 << 60) - 1 - 2 * i for i in range(sq)]
    p = [(1 << 60) - 1, (1 << 60) - (1 << 32) + 1, (1 << 58) - 12345, (1 << 55) - (1 << 23) + 5,
         (1 << 54) - (1 << 26) + 1, (1 << 60) - 93, (1 << 59) - 55, (1 << 57) - 3]
    bc = H.BaseConverter(ctx, log_n, q, p, [1] * sq, [pj - 1 for _ in q for pj in p])
    rng = np.random.default_rng(100 + sq)
    x = np.stack([np.full(n, qi - 1, np.uint64) for qi in q])
    x[:, 1::2] = np.stack([rng.integers(0, qi, size=n // 2, dtype=np.uint64) for qi in q])
    x[:, 2::4] = np.uint64(0x007F7F7F7F7F7F80)
    dx = dev(x[None])
    out = torch.zeros((1, len(p), n), dtype=torch.int64, device="cuda")
    bc.switch(dx.data_ptr(), out.data_ptr(), 1, stream())
    want = np.array([[sum(int(x[i, k]) * (pj - 1) for i in range(sq)) % pj for k in range(n)] for pj in p],
                    np.uint64)
    assert np.array_equal(host(out)[0], want)


@pytest.mark.parametrize("seed", range(8))
def test_base_conversion_random_shapes(hip, seed):
    """Seeded random ApproxSwitchCRTBasis shapes against the oracle
    (oracle/keyswitch.py, the reference's loop): 1..64 source towers, 1..90
    targets, special and generic moduli mixed or not, N = 2^5..2^8, batch
    1..3 -- every K-step count, target chunking and both reduction forms of
    k_bconv_mma, with the reference's own QHatInvModq / QHatModp tables."""
    H, ctx = hip
    import torch

    rng = np.random.default_rng(1000 + seed)
    log_n = int(rng.integers(5, 9))
    n = 1 << log_n
    sq, sp, batch = int(rng.integers(1, 65)), int(rng.integers(1, 91)), int(rng.integers(1, 4))
    special = seed % 2 == 0
    q, _, p, _ = (_bases if special else _generic_bases)(log_n, sq, sp)
    if seed % 4 == 2:  # one generic target among special ones: the generic reduction for all
        p = list(p[:-1]) + [_generic_bases(log_n, 0, 1)[2][0]]
    qhinv, qhmodp = K.switch_tables(q, p)
    bc = H.BaseConverter(ctx, log_n, q, p, qhinv, [v for row in qhmodp for v in row])
    x = _uniform(rng, batch, q, n)
    dx = dev(x)
    out = torch.zeros((batch, sp, n), dtype=torch.int64, device="cuda")
    bc.switch(dx.data_ptr(), out.data_ptr(), batch, stream())
    assert np.array_equal(host(out), K._switch_basis(x, q, p, qhinv, qhmodp))


def test_keyswitch_inner_max_values(hip):
    """Inner product with every digit and key word m - 1 (the largest limb sums
    of the batch-stationary kernel), against the oracle."""
    H, ctx = hip
    import torch

    n, q, rq, p, rp, kp, ks = _ks_case(H, ctx, 6, 5, 3, 2)
    l, B = 5, 3
    alpha, beta = ks.digits(l)
    mods = np.array(q[:l] + p, np.uint64)[None, :, None]
    digits = np.broadcast_to(mods - 1, (B * beta, l + len(p), n)).reshape(B, beta, l + len(p), n).copy()
    allm = np.array(q + p, np.uint64)[None, :, None]
    kb = np.broadcast_to(allm - 1, (2, len(q) + len(p), n)).copy()
    ka = kb.copy()
    ka[:, :, ::3] = 0
    c0 = torch.empty((B, l + len(p), n), dtype=torch.int64, device="cuda")
    c1 = torch.empty_like(c0)
    dd, dkb, dka = dev(digits), dev(kb), dev(ka)
    ks.fast_core_ext(l, dd.data_ptr(), dkb.data_ptr(), dka.data_ptr(), c0.data_ptr(), c1.data_ptr(), B, stream())
    r0, r1 = K.ks_fast_core_ext(kp, digits, kb, ka)
    assert np.array_equal(host(c0), r0) and np.array_equal(host(c1), r1)


def _ks_case(H, ctx, log_n, sq, sp, dnum, generic=False, options=None):
    n = 1 << log_n
    q, rq, p, rp = (_generic_bases if generic else _bases)(log_n, sq, sp)
    kp = K.KeySwitchParams(n, q, rq, p, rp, dnum)
    ks = H.KeySwitch(ctx, log_n, q, rq, p, rp, dnum, options)
    return n, q, rq, p, rp, kp, ks


KS_CASES = [
    (4, 4, 2, 2, False),    # tiny ring, two full digits
    (6, 5, 3, 2, False),    # partial last digit (alpha = 3)
    (12, 6, 2, 3, True),    # generic moduli
    (13, 8, 3, 3, False),   # alpha = 3, digits 3+3+2
    (16, 6, 2, 3, False),   # N = 2^16 (8|8 split transforms)
    (5, 8, 2, 4, False),    # beta = 4 (largest batch-stationary inner product)
    (5, 10, 2, 5, False),   # beta = 5 (generic inner product kernel)
    (10, 40, 4, 1, False),  # dnum = 1: a 40-tower digit (matrix-core conversion, wide partial sums)
]


@pytest.mark.parametrize("log_n,sq,sp,dnum,generic", KS_CASES)
def test_keyswitch_steps(hip, log_n, sq, sp, dnum, generic):
    H, ctx = hip
    import torch

    n, q, rq, p, rp, kp, ks = _ks_case(H, ctx, log_n, sq, sp, dnum, generic)
    rng = np.random.default_rng(100 + log_n)
    B = 2
    for l in sorted({sq, max(1, sq - 1), max(1, kp.alpha - 1)}, reverse=True):
        alpha, beta = ks.digits(l)
        assert (alpha, beta) == (kp.alpha, kp.beta(l))
        c = K.set_format(_uniform(rng, B, q[:l], n), q[:l], rq[:l], True)
        d = torch.empty((B, beta, l + sp, n), dtype=torch.int64, device="cuda")
        dc = dev(c)
        ks.precompute(l, dc.data_ptr(), d.data_ptr(), B, stream())
        dref = K.ks_precompute(kp, c)
        assert np.array_equal(host(d), dref), f"precompute level {l}"
        kb = _uniform(rng, dnum, q + p, n)
        ka = _uniform(rng, dnum, q + p, n)
        c0 = torch.empty((B, l + sp, n), dtype=torch.int64, device="cuda")
        c1 = torch.empty_like(c0)
        dd, dkb, dka = dev(dref), dev(kb), dev(ka)
        ks.fast_core_ext(l, dd.data_ptr(), dkb.data_ptr(), dka.data_ptr(), c0.data_ptr(), c1.data_ptr(), B,
                         stream())
        r0, r1 = K.ks_fast_core_ext(kp, dref, kb, ka)
        assert np.array_equal(host(c0), r0) and np.array_equal(host(c1), r1), f"inner product level {l}"
        for t in (0, 65537):
            o = torch.empty((B, l, n), dtype=torch.int64, device="cuda")
            dr = dev(r0)
            ks.mod_down(l, dr.data_ptr(), o.data_ptr(), t, B, stream())
            assert np.array_equal(host(o), K.ks_mod_down(kp, r0, t)), f"mod down level {l} t {t}"


@pytest.mark.parametrize("log_n,sq,sp,dnum,generic", KS_CASES)
def test_keyswitch_core_levels_and_t(hip, log_n, sq, sp, dnum, generic):
    """KeySwitchCore bit-exact against the oracle at full and lower levels, for
    t = 0 (CKKS / BFV) and t = 65537 (BGV), with an odd batch: covers the
    core's own-tower reads from c (beta <= 4), the merged ModUp launches at
    full level and the two ModDowns run as one 2 x batch launch set."""
    H, ctx = hip
    import torch

    n, q, rq, p, rp, kp, ks = _ks_case(H, ctx, log_n, sq, sp, dnum, generic)
    rng = np.random.default_rng(300 + log_n)
    B = 3 if log_n < 16 else 1
    kb = _uniform(rng, dnum, q + p, n)
    ka = _uniform(rng, dnum, q + p, n)
    dkb, dka = dev(kb), dev(ka)
    for l in sorted({sq, max(1, sq - 1), max(1, kp.alpha - 1)}, reverse=True):
        c = K.set_format(_uniform(rng, B, q[:l], n), q[:l], rq[:l], True)
        dc = dev(c)
        for t in (0, 65537):
            o0 = torch.empty((B, l, n), dtype=torch.int64, device="cuda")
            o1 = torch.empty_like(o0)
            ks.core(l, dc.data_ptr(), dkb.data_ptr(), dka.data_ptr(), o0.data_ptr(), o1.data_ptr(), t, B, stream())
            r0, r1 = K.ks_core(kp, c, kb, ka, t)
            assert np.array_equal(host(o0), r0) and np.array_equal(host(o1), r1), f"level {l} t {t}"


@pytest.mark.parametrize("log_n,sq,sp,dnum,generic", KS_CASES[:3])
def test_keyswitch_core_semantics(hip, log_n, sq, sp, dnum, generic):
    """KeySwitchCore on the GPU with real keys: equals the oracle bit for bit
    and satisfies ct0 + ct1*s_new = c*s_old + small."""
    H, ctx = hip
    import torch

    n, q, rq, p, rp, kp, ks = _ks_case(H, ctx, log_n, sq, sp, dnum, generic)
    rng = np.random.default_rng(7)
    s_old, s_new = K.ternary(n, rng), K.ternary(n, rng)
    kb, ka = K.keyswitch_gen(kp, s_old, s_new, rng)
    B = 2
    c = K.set_format(_uniform(rng, B, q, n), q, rq, True)
    o0 = torch.empty((B, sq, n), dtype=torch.int64, device="cuda")
    o1 = torch.empty_like(o0)
    dc, dkb, dka = dev(c), dev(kb), dev(ka)
    ks.core(sq, dc.data_ptr(), dkb.data_ptr(), dka.data_ptr(), o0.data_ptr(), o1.data_ptr(), 0, B, stream())
    g0, g1 = host(o0), host(o1)
    r0, r1 = K.ks_core(kp, c, kb, ka)
    assert np.array_equal(g0, r0) and np.array_equal(g1, r1)
    sn = np.repeat(K.small_poly_eval(s_new, q, rq), B, 0)
    so = np.repeat(K.small_poly_eval(s_old, q, rq), B, 0)
    lhs = O.eltwise("add", g0, O.eltwise("mul", g1, sn, q), q)
    d = K.set_format(O.eltwise("sub", lhs, O.eltwise("mul", c, so, q), q), q, rq, False)
    for b in range(B):
        assert max(abs(e) for e in K.crt_centered(d[b], q)) < 1 << 20


def test_keyswitch_bootstrap_shape(hip):
    """configs[4] shape: N = 2^17, 48 Q towers, dnum = 3 (alpha = 16), P = 16
    towers (sizeP = ceil(16*60 / 60)), one ciphertext, full level."""
    H, ctx = hip
    import torch

    log_n, sq, sp, dnum = 17, 48, 16, 3
    n, q, rq, p, rp, kp, ks = _ks_case(H, ctx, log_n, sq, sp, dnum)
    rng = np.random.default_rng(17)
    c = K.set_format(_uniform(rng, 1, q, n), q, rq, True)
    kb = _uniform(rng, dnum, q + p, n)
    ka = _uniform(rng, dnum, q + p, n)
    o0 = torch.empty((1, sq, n), dtype=torch.int64, device="cuda")
    o1 = torch.empty_like(o0)
    dc, dkb, dka = dev(c), dev(kb), dev(ka)
    ks.core(sq, dc.data_ptr(), dkb.data_ptr(), dka.data_ptr(), o0.data_ptr(), o1.data_ptr(), 0, 1, stream())
    r0, r1 = K.ks_core(kp, c, kb, ka)
    assert np.array_equal(host(o0), r0) and np.array_equal(host(o1), r1)


@pytest.mark.parametrize("sq,sp,dnum,generic,B,cases,fused", [
    (48, 16, 3, False, 2, ((48, 0), (47, 0)), "1"),   # configs[4]; level 47: ModDown fused, ModUp not
    (48, 16, 3, False, 1, ((48, 0),), "0"),           # the unfused kernels (options.separate_cols)
    (12, 4, 3, False, 1, ((12, 0), (12, 65537), (11, 0)), "1"),
    (8, 4, 2, True, 2, ((8, 0), (7, 65537)), "1"),     # generic moduli: Mod<false>, no special-prime fold
    (10, 6, 4, False, 1, ((10, 0), (10, 3)), "1"),     # digits of 3 / 3 / 3 / 1 towers, 6 special towers
    (24, 12, 2, False, 1, ((24, 0),), "1"),            # 12-tower digits and P: the KS = 3 conversion kernels
])
@pytest.mark.parametrize("icol", ["0", "1"])
def test_keyswitch_bconv_cols(hip, sq, sp, dnum, generic, B, cases, fused, icol):
    """N = 2^17 KeySwitchCore with ApproxSwitchCRTBasis fused with the targets'
    forward column pass (k_bconv_cols, the default) in ModUp (full level) and
    ModDown (t = 0), and with options.separate_cols, bit-exact against the
    oracle; lower levels and t > 0 take the unfused kernels in the same call.
    icol = 1 (the default; options.separate_icol = 0) also moves the sources'
    INTT column pass into k_bconv_cols."""
    H, ctx = hip
    import torch

    opt = H.KsOptions()
    opt.separate_cols = 0 if fused == "1" else 1
    opt.separate_icol = 0 if icol == "1" else 1
    n, q, rq, p, rp, kp, ks = _ks_case(H, ctx, 17, sq, sp, dnum, generic, opt)
    rng = np.random.default_rng(1700 + sq)
    kb = _uniform(rng, dnum, q + p, n)
    ka = _uniform(rng, dnum, q + p, n)
    dkb, dka = dev(kb), dev(ka)
    for l, t in cases:
        c = K.set_format(_uniform(rng, B, q[:l], n), q[:l], rq[:l], True)
        if l == sq and t == 0:
            c[0, :, : n // 2] = np.array(q[:l], np.uint64)[:, None] - np.uint64(1)  # largest digits
        dc = dev(c)
        o0 = torch.empty((B, l, n), dtype=torch.int64, device="cuda")
        o1 = torch.empty_like(o0)
        ks.core(l, dc.data_ptr(), dkb.data_ptr(), dka.data_ptr(), o0.data_ptr(), o1.data_ptr(), t, B, stream())
        r0, r1 = K.ks_core(kp, c, kb, ka, t)
        assert np.array_equal(host(o0), r0) and np.array_equal(host(o1), r1), f"level {l} t {t}"


@pytest.mark.parametrize("t", [0, 65537])
def test_mod_down_of_p_times_mod_up_full_size(hip, t):
    """Size-independent identity at N = 2^16, 16 towers: ModDown(P * ModUp(x)) = x."""
    H, ctx = hip
    import torch

    log_n, sq, sp = 16, 16, 4
    n = 1 << log_n
    q, rq, p, rp = _bases(log_n, sq, sp)
    pq, pp = H.NTTPlan(ctx, log_n, q, rq), H.NTTPlan(ctx, log_n, p, rp)
    pqp = H.NTTPlan(ctx, log_n, q + p, rq + rp)
    up_bc, down_bc = _converter(H, ctx, log_n, q, p), _converter(H, ctx, log_n, p, q)
    T = K.moddown_tables(q, p)
    B = 4
    x = torch.empty((B, sq, n), dtype=torch.int64, device="cuda")
    for t in range(sq):
        x[:, t].random_(0, q[t])
    up = torch.empty((B, sq + sp, n), dtype=torch.int64, device="cuda")
    H.approx_mod_up(pq, pp, up_bc, True, x.data_ptr(), up.data_ptr(), B, stream())
    Pm = int(np.prod([int(v) for v in p], dtype=object))
    pqp.mod_mul_scalar(up.data_ptr(), [Pm % m for m in q + p], up.data_ptr(), B, stream())
    out = torch.empty_like(x)
    H.approx_mod_down(pq, pp, down_bc, T["pinv_modq"], t, up.data_ptr(), out.data_ptr(), B, stream())
    torch.cuda.synchronize()
    assert torch.equal(out, x)


@pytest.mark.parametrize("om,nm", [(1152921504606584833, 1152921504598720513), (97, 1152921504606584833),
                                   (1152921504606584833, 65537), (1 << 40, 12289)])
def test_switch_modulus(hip, om, nm):
    H, ctx = hip
    import torch

    rng = np.random.default_rng(om % 1000)
    v = rng.integers(0, om, size=4099, dtype=np.uint64)
    v[:6] = [0, 1, om // 2, om // 2 + 1, om - 1, om - 2]
    x = dev(v)
    y = torch.empty_like(x)
    H.switch_modulus(ctx, x.data_ptr(), y.data_ptr(), v.size, om, nm, stream())
    assert np.array_equal(host(y), K.switch_modulus(v, om, nm))


@pytest.mark.parametrize("log_n", [3, 10, 16])
@pytest.mark.parametrize("eval_form", [True, False])
def test_automorphism(hip, log_n, eval_form):
    H, ctx = hip
    import torch

    n = 1 << log_n
    q, r = O.moduli_chain(log_n, 2)
    plan = H.NTTPlan(ctx, log_n, q, r)
    rng = np.random.default_rng(log_n)
    x = _uniform(rng, 2, q, n)
    x[0, 0, :4] = 0
    ks_ = (3, 5, 2 * n - 1, 25) if log_n <= 10 else (5, 2 * n - 1)
    for k in ks_:
        y = torch.empty((2, 2, n), dtype=torch.int64, device="cuda")
        dx = dev(x)
        plan.automorphism(k, eval_form, dx.data_ptr(), y.data_ptr(), 2, stream())
        got = host(y)
        if log_n <= 10:
            for b in range(2):
                for t in range(2):
                    assert np.array_equal(got[b, t], K.automorphism(x[b, t], k, eval_form, q[t])), (k, b, t)
        else:  # full size: permutation property against the closed form
            j = np.arange(n, dtype=np.uint64)
            if eval_form:
                rev = lambda v: np.array([int(format(int(a), f"0{log_n}b")[::-1], 2) for a in v], np.uint64)
                src = rev(((np.uint64(k) * (2 * j + 1)) % np.uint64(2 * n)) >> np.uint64(1))
                assert np.array_equal(got[:, :, rev(j)], x[:, :, src])
            else:
                jk = (j * np.uint64(k)) % np.uint64(2 * n)
                neg = (jk >> np.uint64(log_n)) & np.uint64(1)
                for t in range(2):
                    exp = np.where(neg == 1, np.uint64(q[t]) - x[:, t], x[:, t])
                    assert np.array_equal(got[:, t, jk % np.uint64(n)], exp)
    with pytest.raises(H.MathError):
        plan.automorphism(4, eval_form, dx.data_ptr(), y.data_ptr(), 2, stream())


def test_mod_down_t_after_plain_same_objects(hip):
    """ModDown with t = 0 and then t > 0 on the same plans / converter, N = 2^12
    (the C++ adapter test's sequence)."""
    H, ctx = hip
    import torch

    log_n, sq, sp = 12, 4, 2
    n = 1 << log_n
    q, rq, p, rp = _bases(log_n, sq, sp)
    pq, pp = H.NTTPlan(ctx, log_n, q, rq), H.NTTPlan(ctx, log_n, p, rp)
    pqp = H.NTTPlan(ctx, log_n, q + p, rq + rp)
    up_bc, down_bc = _converter(H, ctx, log_n, q, p), _converter(H, ctx, log_n, p, q)
    T = K.moddown_tables(q, p)
    B = 2
    rng = np.random.default_rng(1)
    x = _uniform(rng, B, q, n)
    dx = dev(x)
    up = torch.empty((B, sq + sp, n), dtype=torch.int64, device="cuda")
    H.approx_mod_up(pq, pp, up_bc, True, dx.data_ptr(), up.data_ptr(), B, stream())
    Pm = int(np.prod([int(v) for v in p], dtype=object))
    for t in (0, 65537, 0, 3):
        scaled = torch.empty_like(up)
        pqp.mod_mul_scalar(up.data_ptr(), [Pm % m for m in q + p], scaled.data_ptr(), B, stream())
        out = torch.zeros((B, sq, n), dtype=torch.int64, device="cuda")
        H.approx_mod_down(pq, pp, down_bc, T["pinv_modq"], t, scaled.data_ptr(), out.data_ptr(), B, stream())
        assert np.array_equal(host(out), x), t


def _centered_same_small(d, q, bound):
    """[T][N] residues: every tower holds the same integer e with |e| < bound
    (so the CRT value is e itself -- no big-integer lift needed)."""
    qa = np.array(q, np.uint64)[:, None]
    v = np.where(d > qa // np.uint64(2), d.astype(np.int64) - qa.astype(np.int64), d.astype(np.int64))
    return bool(np.all(np.abs(v) < bound) and np.all(v == v[0:1]))


@pytest.mark.parametrize("dnum", [1, 2, 3, 4])
def test_configs4_digit_split_identities(hip, dnum):
    """configs[4] shape (N = 2^17, Q = 48) at every digit split of
    keyswitch-hybrid.cpp:341-346 for dnum = 1..4 (alpha = 48 / 24 / 16 / 12),
    with P sized as OpenFHE sizes it for 60-bit towers (sizeP = alpha: P must
    exceed every digit's modulus, rns-cryptoparameters.cpp:126-135), i.e.
    P = 16 at the bench's dnum = 3:
    (1) each digit j of EvalKeySwitchPrecomputeCore is ApproxModUp of c's
        digit: on digit j's own towers it equals c, and
        ApproxModDown(P * digit_j) returns digit_j's Q part exactly
        (ApproxModDown of a multiple of P has a zero P part);
    (2) KeySwitchCore with a zero key is zero;
    (3) with keys built as KeySwitchGenInternal (keyswitch-hybrid.cpp:53-128)
        from ternary s_old, s_new: ct0 + ct1 s_new - c s_old is one small
        integer in all 48 towers.
    These are the reference's own identities; the reference holds no
    KeySwitchCore vector, so beyond them the key-switch oracle is parity
    unpinned."""
    H, ctx = hip
    import torch

    log_n, sq = 17, 48
    sp = (sq + dnum - 1) // dnum
    n, q, rq, p, rp, kp, ks = _ks_case(H, ctx, log_n, sq, sp, dnum)
    alpha, beta = ks.digits(sq)
    assert (alpha, beta) == ((sq + dnum - 1) // dnum, dnum)
    rng = np.random.default_rng(400 + dnum)
    c = K.set_format(_uniform(rng, 1, q, n), q, rq, True)
    dc = dev(c)
    digits = torch.empty((1, beta, sq + sp, n), dtype=torch.int64, device="cuda")
    ks.precompute(sq, dc.data_ptr(), digits.data_ptr(), 1, stream())
    qp = H.NTTPlan(ctx, log_n, q + p, rq + rp)
    Pm = 1
    for x in p:
        Pm *= x
    for j in range(beta):
        dj = digits[0, j].contiguous()
        got_dj = host(dj)
        st, en = j * alpha, min((j + 1) * alpha, sq)
        assert np.array_equal(got_dj[st:en], c[0, st:en]), f"digit {j} keeps its own towers"
        z = torch.empty_like(dj)
        qp.mod_mul_scalar(dj.data_ptr(), [Pm % m for m in q + p], z.data_ptr(), 1, stream())
        out = torch.empty((1, sq, n), dtype=torch.int64, device="cuda")
        ks.mod_down(sq, z.data_ptr(), out.data_ptr(), 0, 1, stream())
        assert np.array_equal(host(out)[0], got_dj[:sq]), f"ModDown(P * digit {j})"
    zero = torch.zeros((dnum, sq + sp, n), dtype=torch.int64, device="cuda")
    o0 = torch.empty((1, sq, n), dtype=torch.int64, device="cuda")
    o1 = torch.empty_like(o0)
    ks.core(sq, dc.data_ptr(), zero.data_ptr(), zero.data_ptr(), o0.data_ptr(), o1.data_ptr(), 0, 1, stream())
    assert not host(o0).any() and not host(o1).any(), "zero key"
    s_old, s_new = K.ternary(n, rng), K.ternary(n, rng)
    kb, ka = K.keyswitch_gen(kp, s_old, s_new, rng)
    dkb, dka = dev(kb), dev(ka)
    ks.core(sq, dc.data_ptr(), dkb.data_ptr(), dka.data_ptr(), o0.data_ptr(), o1.data_ptr(), 0, 1, stream())
    g0, g1 = host(o0), host(o1)
    sn = K.small_poly_eval(s_new, q, rq)
    so = K.small_poly_eval(s_old, q, rq)
    lhs = O.eltwise("add", g0, O.eltwise("mul", g1, sn, q), q)
    d = K.set_format(O.eltwise("sub", lhs, O.eltwise("mul", c, so, q), q), q, rq, False)
    assert _centered_same_small(d[0], q, 1 << 40), "ct0 + ct1 s_new - c s_old is small"
