"""GPU parity at the shapes the bench measures and at the round-2 EvalMultCore
failure's shapes, through the C ABI:

* configs[2] itself (N = 2^16, 16 towers, batch 1024: 8 GiB per operand, byte
  offsets far above 2^32): device-generated inputs equal the oracle's
  splitmix64 streams; rows {0, 511, 1023} x towers {0, 15} of the pipeline
  against the oracle (poly-benchmark-16k.cpp:89-96 moduli); and over the whole
  8 GiB buffers, INTT(NTT(x)) = x and NTT(a + b) = NTT(a) + NTT(b) on the
  device;
* configs[4]'s KeySwitchCore at batch 8 (the bench's shape: the batch walk of
  the inner product and the side-stream fork), ciphertexts {0, 7} against the
  oracle (keyswitch-hybrid.cpp:325-328);
* k_eltwise ModMul / ModAdd / ModSub, the scalar ops and the fused
  EvalMultCore at (N, towers, batch) = (2^16, 4, 1), (2^16, 4, 2), (2^16, 16, 2)
  -- where round 2's uncommitted grid-stride EvalMultCore returned wrong words
  (DESIGN.md "EvalMultCore failure in round 2") -- against the oracle."""
import numpy as np
import pytest

import keyswitch as K
import oracle as O
from test_gpu_parity import dev, host, stream

pytestmark = pytest.mark.gpu


def test_configs2_full_batch(hip):
    import torch

    H, ctx = hip
    log_n, T, B = 16, 16, 1024
    n = 1 << log_n
    qs, rs = O.moduli_chain(log_n, T)
    plan = H.NTTPlan(ctx, log_n, qs, rs)
    sp = stream()
    a = torch.empty((B, T, n), dtype=torch.int64, device="cuda")
    b = torch.empty_like(a)
    c = torch.empty_like(a)
    plan.fill_uniform(a.data_ptr(), B, 1, 0, sp)
    plan.fill_uniform(b.data_ptr(), B, 2, 0, sp)
    plan.ntt_mul_intt(a.data_ptr(), b.data_ptr(), c.data_ptr(), B, sp)
    torch.cuda.synchronize()
    for bi in (0, 511, 1023):
        for ti in (0, 15):
            aa = a[bi, ti].cpu().numpy().view(np.uint64)
            bb = b[bi, ti].cpu().numpy().view(np.uint64)
            want_a = O.splitmix_fill(n, qs[ti], O.U([0x5EED ^ (bi << 20) ^ (ti << 8) ^ 1]))
            assert np.array_equal(aa, want_a), (bi, ti)
            want = O.ntt_mul_intt(aa.reshape(1, 1, n), bb.reshape(1, 1, n), O.Tables(n, [qs[ti]], [rs[ti]]))
            assert np.array_equal(c[bi, ti].cpu().numpy().view(np.uint64), want.reshape(-1)), (bi, ti)
    # INTT(NTT(x)) = x over all 8 GiB
    x = a.clone()
    plan.forward(x.data_ptr(), B, sp)
    plan.inverse(x.data_ptr(), B, sp)
    assert torch.equal(x, a)
    # linearity: NTT(a + b) = NTT(a) + NTT(b), every word
    plan.mod_add(a.data_ptr(), b.data_ptr(), c.data_ptr(), B, sp)
    for t_ in (a, b, c):
        plan.forward(t_.data_ptr(), B, sp)
    plan.mod_add(a.data_ptr(), b.data_ptr(), x.data_ptr(), B, sp)
    assert torch.equal(x, c)
    del a, b, c, x
    plan.close()
    torch.cuda.empty_cache()


def test_configs4_keyswitch_batch8(hip):
    import torch

    H, ctx = hip
    log_n, sq, sp_, dnum, B = 17, 48, 16, 3, 8
    n = 1 << log_n
    m, r = O.moduli_chain(log_n, sq + sp_)
    q, rq, p, rp = m[:sq], r[:sq], m[sq:], r[sq:]
    kp = K.KeySwitchParams(n, q, rq, p, rp, dnum)
    ks = H.KeySwitch(ctx, log_n, q, rq, p, rp, dnum)
    pq, pqp = H.NTTPlan(ctx, log_n, q, rq), H.NTTPlan(ctx, log_n, q + p, rq + rp)
    s = stream()
    c = torch.empty((B, sq, n), dtype=torch.int64, device="cuda")
    pq.fill_uniform(c.data_ptr(), B, 5, 0, s)
    kb = torch.empty((dnum, sq + sp_, n), dtype=torch.int64, device="cuda")
    ka = torch.empty_like(kb)
    pqp.fill_uniform(kb.data_ptr(), dnum, 6, 0, s)
    pqp.fill_uniform(ka.data_ptr(), dnum, 7, 0, s)
    o0 = torch.empty((B, sq, n), dtype=torch.int64, device="cuda")
    o1 = torch.empty_like(o0)
    ks.core(sq, c.data_ptr(), kb.data_ptr(), ka.data_ptr(), o0.data_ptr(), o1.data_ptr(), 0, B, s)
    g0, g1 = host(o0), host(o1)
    hc, hkb, hka = host(c), host(kb), host(ka)
    r0, r1 = K.ks_core(kp, hc[[0, 7]], hkb, hka)
    assert np.array_equal(g0[[0, 7]], r0) and np.array_equal(g1[[0, 7]], r1)
    # the middle ciphertexts are the same function of their inputs: run them
    # again at batch 1 and compare (the batch walk must not mix ciphertexts)
    for bi in (3, 4):
        e0, e1 = torch.empty_like(o0[:1]), torch.empty_like(o1[:1])
        ks.core(sq, c[bi:bi + 1].data_ptr(), kb.data_ptr(), ka.data_ptr(), e0.data_ptr(), e1.data_ptr(), 0, 1, s)
        assert np.array_equal(host(e0)[0], g0[bi]) and np.array_equal(host(e1)[0], g1[bi])
    del c, kb, ka, o0, o1
    ks.close()
    pq.close()
    pqp.close()
    torch.cuda.empty_cache()


def _ref_evalmult(c0, c1, d0, d1, q):
    o2 = O.eltwise("mul", c1, d1, q)
    o1 = O.eltwise("add", O.eltwise("mul", c1, d0, q), O.eltwise("mul", c0, d1, q), q)
    o0 = O.eltwise("mul", d0, c0, q)
    return o0, o1, o2


@pytest.mark.parametrize("T,B", [(4, 1), (4, 2), (16, 2)])
def test_eltwise_and_evalmult_round2_shapes(hip, T, B):
    import torch

    H, ctx = hip
    log_n = 16
    n = 1 << log_n
    q, r = O.moduli_chain(log_n, T)
    rng = np.random.default_rng(1000 + T * 10 + B)
    xs = [np.stack([np.stack([rng.integers(0, qi, size=n, dtype=np.uint64) for qi in q]) for _ in range(B)])
          for _ in range(4)]
    plan = H.NTTPlan(ctx, log_n, q, r)
    dx = [dev(x) for x in xs]
    s = stream()
    for op in ("mul", "add", "sub"):
        out = torch.empty_like(dx[0])
        getattr(plan, "mod_" + op)(dx[1].data_ptr(), dx[3].data_ptr(), out.data_ptr(), B, s)
        assert np.array_equal(host(out), O.eltwise(op, xs[1], xs[3], q)), op
    sc = [int(v) for v in rng.integers(0, 2**63, size=T, dtype=np.uint64)]
    out = torch.empty_like(dx[0])
    plan.mod_mul_scalar(dx[0].data_ptr(), sc, out.data_ptr(), B, s)
    want = np.stack([np.stack([(xs[0][b, t].astype(object) * (sc[t] % q[t]) % q[t]).astype(np.uint64)
                               for t in range(T)]) for b in range(B)])
    assert np.array_equal(host(out), want)
    outs = [torch.empty_like(dx[0]) for _ in range(3)]
    plan.eval_mult_core(*(t.data_ptr() for t in dx), *(o.data_ptr() for o in outs), B, s)
    for o, w in zip(outs, _ref_evalmult(*xs, q)):
        assert np.array_equal(host(o), w)
