"""Seeded randomized parity: every plan op and the base conversion on random
shapes, random moduli and edge-heavy inputs, bit-exact against the oracle.

The fixed-shape tests pin the benchmark configurations; these cases sweep
what they do not: ring dimensions 2^1 .. 2^17, ragged tower and batch counts,
moduli of 22 to 60 bits that are either near a power of two (the special
q = 2^L - d form the kernels detect per plan) or drawn anywhere in their
range (the generic kernels), and inputs whose words are 0, 1 and q - 1 at
random positions.  Each case is reproducible from its seed.  The oracle
follows the reference loops (transformnat-impl.h:300-354, 492-552;
mubintvecnat.cpp:245-367; dcrtpoly-impl.h:1034-1063)."""
import os

import numpy as np
import pytest

from test_gpu_parity import dev, host, stream

# OFHE_FUZZ_SCALE=k multiplies the case counts (a soak run: profiles/r03e_fuzz_soak.txt)
SCALE = int(os.environ.get("OFHE_FUZZ_SCALE", "1"))

pytestmark = pytest.mark.gpu

LOG_NS = list(range(1, 18))


def _random_prime(O, rng, bits, m, special):
    """A prime q = 1 mod m (m = 2N) below 2^60 with `bits` bits: the first
    below 2^bits (special form) or the next one above a random start."""
    if special:
        q = O.previous_prime(((1 << bits) // m) * m + 1, m)
    else:
        lo, hi = 1 << (bits - 1), (1 << bits) - 1
        start = int(rng.integers(lo, hi, dtype=np.uint64))
        q = O.next_prime(start - start % m + 1, m)
    if not (3 <= q < (1 << 60)) or q % m != 1:
        q = O.previous_prime(((1 << 60) - 1) // m * m + 1, m)
    return q


def _moduli(O, rng, log_n, towers):
    m = 2 << log_n
    qs, roots = [], []
    for _ in range(towers):
        bits = int(rng.integers(max(22, log_n + 4), 61))
        q = _random_prime(O, rng, bits, m, bool(rng.integers(0, 2)))
        qs.append(q)
        roots.append(O.root_of_unity(m, q))
    return qs, roots


def _edge_inputs(rng, B, qs, n):
    x = np.empty((B, len(qs), n), np.uint64)
    for t, q in enumerate(qs):
        x[:, t] = rng.integers(0, q, size=(B, n), dtype=np.uint64)
        for val in (0, 1, q - 1):
            k = max(1, n // 8)
            pos = rng.integers(0, n, size=(B, k))
            for b in range(B):
                x[b, t, pos[b]] = val
    return x


@pytest.mark.parametrize("seed", range(96 * SCALE))
def test_fuzz_plan_ops(hip, O, seed):
    import torch

    H, ctx = hip
    rng = np.random.default_rng(7000 + seed)
    log_n = LOG_NS[seed % len(LOG_NS)] if seed < len(LOG_NS) else int(rng.integers(1, 18))
    n = 1 << log_n
    big = log_n >= 15
    T = int(rng.integers(1, 4 if big else 10))
    B = int(rng.integers(1, 3 if big else 5))
    qs, roots = _moduli(O, rng, log_n, T)
    plan = H.NTTPlan(ctx, log_n, qs, roots)
    tb = O.Tables(n, qs, roots)
    a = _edge_inputs(rng, B, qs, n)
    b = _edge_inputs(rng, B, qs, n)
    ctx_msg = f"seed {seed}: log_n {log_n}, T {T}, B {B}, q {qs}"

    x = dev(a)
    plan.forward(x.data_ptr(), B, stream())
    assert np.array_equal(host(x), O.ntt_fwd(a, tb)), "forward " + ctx_msg
    x = dev(a)
    plan.inverse(x.data_ptr(), B, stream())
    assert np.array_equal(host(x), O.ntt_inv(a, tb)), "inverse " + ctx_msg
    for op in ("mul", "add", "sub"):
        xa, xb = dev(a), dev(b)
        xc = torch.empty_like(xa)
        getattr(plan, "mod_" + op)(xa.data_ptr(), xb.data_ptr(), xc.data_ptr(), B, stream())
        assert np.array_equal(host(xc), O.eltwise(op, a, b, qs)), op + " " + ctx_msg
    xa, xb = dev(a), dev(b)
    xc = torch.empty_like(xa)
    plan.ntt_mul_intt(xa.data_ptr(), xb.data_ptr(), xc.data_ptr(), B, stream())
    assert np.array_equal(host(xc), O.ntt_mul_intt(a, b, tb)), "pipeline " + ctx_msg
    # in place: c aliases a (the DCRTPoly *= pattern)
    xa, xb = dev(a), dev(b)
    plan.ntt_mul_intt(xa.data_ptr(), xb.data_ptr(), xa.data_ptr(), B, stream())
    assert np.array_equal(host(xa), O.ntt_mul_intt(a, b, tb)), "pipeline in place " + ctx_msg


@pytest.mark.parametrize("seed", range(48 * SCALE))
def test_fuzz_base_conversion(hip, O, seed):
    """ApproxSwitchCRTBasis (dcrtpoly-impl.h:1034-1063) with random source and
    target counts (1 .. 40 sources: the matrix-core kernel's K-step counts
    and its wide partial sums; up to 70 targets: several target chunks),
    random moduli and the tables the oracle derives from them."""
    import torch

    H, ctx = hip
    rng = np.random.default_rng(9000 + seed)
    log_n = int(rng.integers(3, 15))
    n = 1 << log_n
    sq = int(rng.integers(1, 41))
    sp = int(rng.integers(1, 71))
    m = 2 << log_n
    allq = []
    while len(allq) < sq + sp:
        bits = int(rng.integers(30, 61))
        q = _random_prime(O, rng, bits, m, bool(rng.integers(0, 2)))
        if q not in allq:
            allq.append(q)
    q, p = allq[:sq], allq[sq:]
    pre = O.base_conv_precompute(q, p)
    x = _edge_inputs(rng, 1, q, n)[0]
    want = O.approx_switch_crt_basis(x, q, p, pre)
    bc = H.BaseConverter(ctx, log_n, q, p, [int(v) for v in pre["qhinv"]], [int(v) for v in pre["qhmodp"]])
    dx = dev(x[None])
    out = torch.zeros((1, sp, n), dtype=torch.int64, device="cuda")
    bc.switch(dx.data_ptr(), out.data_ptr(), 1, stream())
    assert np.array_equal(host(out)[0], want), f"seed {seed}: log_n {log_n}, sizeQ {sq}, sizeP {sp}"


def _distinct_moduli(O, rng, log_n, count, lo_bits=30):
    m = 2 << log_n
    qs = []
    while len(qs) < count:
        q = _random_prime(O, rng, int(rng.integers(max(lo_bits, log_n + 4), 61)), m, bool(rng.integers(0, 2)))
        if q not in qs:
            qs.append(q)
    return qs, [O.root_of_unity(m, q) for q in qs]


@pytest.mark.parametrize("seed", range(48 * SCALE))
def test_fuzz_approx_mod_up_down(hip, O, seed):
    """ApproxModUp (dcrtpoly-impl.h:1085-1131, both input forms) and
    ApproxModDown (1134-1175, t = 0 or a random plaintext modulus) on random
    ring dimensions 2^4 .. 2^17 with random Q / P bases (mixed special and
    generic moduli), against oracle/keyswitch.py."""
    import torch

    import keyswitch as K

    H, ctx = hip
    rng = np.random.default_rng(11000 + seed)
    log_n = int(rng.integers(4, 18))
    n = 1 << log_n
    big = log_n >= 15
    sq = int(rng.integers(1, 5 if big else 9))
    sp = int(rng.integers(1, 4 if big else 7))
    allm, allr = _distinct_moduli(O, rng, log_n, sq + sp)
    q, rq, p, rp = allm[:sq], allr[:sq], allm[sq:], allr[sq:]
    pq, pp = H.NTTPlan(ctx, log_n, q, rq), H.NTTPlan(ctx, log_n, p, rp)
    B = int(rng.integers(1, 3 if big else 4))
    msg = f"seed {seed}: log_n {log_n}, q {q}, p {p}, B {B}"

    eval_form = bool(rng.integers(0, 2))
    qhinv, qhmodp = K.switch_tables(q, p)
    up = H.BaseConverter(ctx, log_n, q, p, qhinv, [v for row in qhmodp for v in row])
    x = _edge_inputs(rng, B, q, n)
    out = torch.empty((B, sq + sp, n), dtype=torch.int64, device="cuda")
    dx = dev(x)
    H.approx_mod_up(pq, pp, up, eval_form, dx.data_ptr(), out.data_ptr(), B, stream())
    assert np.array_equal(host(out), K.approx_mod_up(x, q, rq, p, rp, eval_form)), "mod up " + msg

    t = 0 if rng.integers(0, 2) else int(rng.choice([2, 3, 257, 65537]))
    T = K.moddown_tables(q, p, t)
    ph, pm = K.switch_tables(p, q)
    down = H.BaseConverter(ctx, log_n, p, q, ph, [v for row in pm for v in row])
    y = _edge_inputs(rng, B, q + p, n)
    out2 = torch.empty((B, sq, n), dtype=torch.int64, device="cuda")
    dy = dev(y)
    H.approx_mod_down(pq, pp, down, T["pinv_modq"], t, dy.data_ptr(), out2.data_ptr(), B, stream())
    assert np.array_equal(host(out2), K.approx_mod_down(y, q, rq, p, rp, t)), f"mod down t={t} " + msg
