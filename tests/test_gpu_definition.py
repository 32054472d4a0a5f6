"""GPU parity at the configs' full ring sizes against the mathematical
definition of the transform -- not against a restatement of the reference's
butterfly loops.

ChineseRemainderTransformFTT's forward transform (transformnat-impl.h:300-354,
tables of PreCompute 708-763: Table[rev(i)] = psi^i) leaves, at bit-reversed
slot i, the polynomial evaluated at an odd power of the primitive 2N-th root:

    y[i] = a(psi^(2 rev(i) + 1)) mod q.

tests/test_oracle.py::test_forward_is_evaluation_at_odd_powers checks that
identity on the oracle at small N, where the reference's own KAT
(UnitTestTransform.cpp:60-94) pins the oracle.  Here the GPU's forward
transform, inverse transform and the fused pipeline c = INTT(NTT(a) (.) b) are
checked at N = 2^16 and 2^17 (configs[2] / configs[4]) on sampled slots and
coefficients, with exact Python integers only (numpy object arrays):

  forward   y[i] = a(x_i),                  x_i = psi^(2 rev(i) + 1)
  inverse   a[j] = N^-1 sum_i y[i] x_i^-j
  pipeline  c(x_i) = a(x_i) * b[i]          (NTT(c) = NTT(a) (.) b)

Each sample is O(N) big-integer work, so this scales to the full sizes the
C oracle also covers, but shares no code with it."""
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _rev(x, bits):
    return int(format(x, f"0{bits}b")[::-1], 2)


def _powers(x, n, q):
    """[x^0, x^1, ..., x^(n-1)] mod q as a numpy object array (doubling)."""
    p = np.empty(n, dtype=object)
    p[0] = 1
    k = 1
    xk = x % q
    while k < n:
        m = min(k, n - k)
        p[k:k + m] = (p[:m] * xk) % q
        xk = xk * xk % q
        k += m
    return p


def _evaluate(coeffs_obj, x, q):
    return int((coeffs_obj * _powers(x, len(coeffs_obj), q)).sum() % q)


def _dev(x):
    import torch

    return torch.from_numpy(np.ascontiguousarray(x, dtype=np.uint64).view(np.int64)).cuda()


def _host(t):
    import torch

    torch.cuda.synchronize()
    return t.cpu().numpy().view(np.uint64)


def _stream():
    import torch

    return torch.cuda.current_stream().cuda_stream


def _setup(hip, log_n, towers, seed):
    H, ctx = hip
    import bench

    n = 1 << log_n
    qs, rs = bench.moduli_chain(log_n, towers)  # product-side setup (nbtheory semantics)
    rng = np.random.default_rng(seed)
    plan = H.NTTPlan(ctx, log_n, qs, rs)
    return plan, n, qs, rs, rng


def _samples(n, seed, k=12):
    r = random.Random(seed)
    return sorted({0, 1, n // 2, n - 1} | {r.randrange(n) for _ in range(k - 4)})


@pytest.mark.parametrize("log_n", [16, 17])
def test_forward_is_evaluation_full_size(hip, log_n):
    plan, n, qs, rs, rng = _setup(hip, log_n, 2, 100 + log_n)
    B = 2
    a = np.stack([np.stack([rng.integers(0, q, size=n, dtype=np.uint64) for q in qs]) for _ in range(B)])
    x = _dev(a)
    plan.forward(x.data_ptr(), B, _stream())
    y = _host(x)
    plan.close()
    for b in range(B):
        for t, (q, psi) in enumerate(zip(qs, rs)):
            coeffs = a[b, t].astype(object)
            for i in _samples(n, 7 * b + t):
                xi = pow(psi, 2 * _rev(i, log_n) + 1, q)
                assert int(y[b, t, i]) == _evaluate(coeffs, xi, q), (log_n, b, t, i)


@pytest.mark.parametrize("log_n", [16, 17])
def test_inverse_is_interpolation_full_size(hip, log_n):
    plan, n, qs, rs, rng = _setup(hip, log_n, 2, 200 + log_n)
    y = rng.integers(0, min(qs), size=(1, 2, n), dtype=np.uint64)
    x = _dev(y)
    plan.inverse(x.data_ptr(), 1, _stream())
    a = _host(x)
    plan.close()
    rev = np.array([_rev(i, log_n) for i in range(n)], dtype=np.int64)
    for t, (q, psi) in enumerate(zip(qs, rs)):
        ninv = pow(n, -1, q)
        yo = y[0, t].astype(object)
        for j in _samples(n, 31 + t, k=8):
            # x_i^-j = (psi^-2j)^rev(i) * psi^-j
            pinv = pow(psi, -j, q)
            w = _powers(pinv * pinv % q, n, q)[rev] * pinv % q
            want = int((yo * w).sum() % q) * ninv % q
            assert int(a[0, t, j]) == want, (log_n, t, j)


def test_pipeline_is_pointwise_product_at_configs2_ring(hip):
    """c = INTT(NTT(a) (.) b) at N = 2^16, 16 towers (configs[2]'s ring and
    tower count, batch 1): c(x_i) = a(x_i) * b[i] at sampled slots of every
    tower."""
    log_n, T = 16, 16
    plan, n, qs, rs, rng = _setup(hip, log_n, T, 300)
    import torch

    a = np.stack([rng.integers(0, q, size=n, dtype=np.uint64) for q in qs])[None]
    b = np.stack([rng.integers(0, q, size=n, dtype=np.uint64) for q in qs])[None]
    xa, xb = _dev(a), _dev(b)
    xc = torch.empty_like(xa)
    plan.ntt_mul_intt(xa.data_ptr(), xb.data_ptr(), xc.data_ptr(), 1, _stream())
    c = _host(xc)
    plan.close()
    assert all(int(c[0, t].max()) < q for t, q in enumerate(qs)), "outputs canonical"
    for t, (q, psi) in enumerate(zip(qs, rs)):
        ao, co = a[0, t].astype(object), c[0, t].astype(object)
        for i in _samples(n, 41 + t, k=4):
            xi = pow(psi, 2 * _rev(i, log_n) + 1, q)
            assert _evaluate(co, xi, q) == _evaluate(ao, xi, q) * int(b[0, t, i]) % q, (t, i)


@pytest.mark.parametrize("sq,sp", [(48, 16), (16, 48)])
def test_base_conversion_is_crt_sum_full_size(hip, sq, sp):
    """ApproxSwitchCRTBasis (dcrtpoly-impl.h:1034-1063) at configs[4]'s ring,
    N = 2^17: Q = 48 -> P = 16 (ModDown's direction, sizes swapped) and a
    16-tower digit -> 48 towers (ModUp's), on sampled coefficients against its
    definition with exact integers: out_j = (sum_i [x_i (Q/q_i)^-1]_{q_i} *
    (Q/q_i)) mod p_j -- one big-integer sum per coefficient, reduced once,
    against the kernel's per-term residues, 128-bit sums and Barrett
    reduction (matrix cores on this shape)."""
    import torch

    H, ctx = hip
    import bench

    log_n = 17
    n = 1 << log_n
    chain, _ = bench.moduli_chain(log_n, sq + sp)
    q, p = chain[:sq], chain[sq:]
    Q = 1
    for qi in q:
        Q *= qi
    qhat = [Q // qi for qi in q]
    qhinv = [pow(h % qi, -1, qi) for h, qi in zip(qhat, q)]
    qhmodp = [h % pj for h in qhat for pj in p]
    rng = np.random.default_rng(sq)
    x = np.stack([rng.integers(0, qi, size=n, dtype=np.uint64) for qi in q])[None]
    bc = H.BaseConverter(ctx, log_n, q, p, qhinv, qhmodp)
    out = torch.empty((1, sp, n), dtype=torch.int64, device="cuda")
    dx = _dev(x)
    bc.switch(dx.data_ptr(), out.data_ptr(), 1, _stream())
    got = _host(out)
    bc.close()
    for c in _samples(n, 5 + sq, k=24):
        s = sum(int(x[0, i, c]) * qhinv[i] % q[i] * qhat[i] for i in range(sq))
        assert [int(got[0, j, c]) for j in range(sp)] == [s % pj for pj in p], c
