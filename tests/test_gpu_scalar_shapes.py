"""GPU parity, round 2 additions (all through the C ABI, bit-exact vs the oracle
or the reference's own known answers):

- scalar ModAdd / ModSub / ModMul / ModAddAtIndex per tower
  (mubintvecnat.cpp:198-231, 267-288, 310-332), including scalars >= q and
  plans wider than one kernel-argument pack (SCALAR_MAX towers);
- the reference's SwitchModulus and AutomorphismTransform KATs
  (UnitTestPolyElements.cpp:265-305, 500-523);
- the synthetic-input generator against the oracle's splitmix64 streams;
- configs[1] (N = 2^14, 8 towers) element-wise ModAdd / ModSub / ModMul;
- configs[3]'s per-rank workload: N = 2^16, 32 towers, every 4-tower shard
  through the tower-range transforms and the pipeline;
- ApproxModDown issued concurrently on two streams with different t (the
  cached constant tables; no call synchronises the device).
"""
import numpy as np
import pytest

import keyswitch as K
import oracle as O
from conftest import load_golden
from test_gpu_parity import dev, host, stream

pytestmark = pytest.mark.gpu

REF = load_golden("reference_fixtures.json")


def _uniform(rng, batch, moduli, n):
    return np.stack([np.stack([rng.integers(0, m, size=n, dtype=np.uint64) for m in moduli])
                     for _ in range(batch)])


@pytest.mark.parametrize("log_n,towers,batch", [(1, 3, 2), (4, 5, 3), (10, 4, 2), (14, 8, 2), (4, 130, 2)])
def test_scalar_ops(hip, log_n, towers, batch):
    H, ctx = hip
    import torch

    n = 1 << log_n
    q, r = O.moduli_chain(log_n, towers)
    plan = H.NTTPlan(ctx, log_n, q, r)
    rng = np.random.default_rng(log_n * 1000 + towers)
    a = _uniform(rng, batch, q, n)
    a[0, :, 0] = 0
    a[-1, :, -1] = np.array(q, np.uint64) - np.uint64(1)
    # scalars: 0, q-1, q, >= q, 2^64-1 and random, cycling over the towers
    special = [0, None, None, 2 ** 64 - 1, 1]
    s = []
    for t in range(towers):
        k = special[t % len(special)]
        if k is None:
            k = q[t] - 1 if t % 2 else q[t] + int(rng.integers(0, 1 << 62))
        s.append(k if t % 7 else int(rng.integers(0, q[t])))
    da = dev(a)
    for name, fn, ref in (("mul", plan.mod_mul_scalar, O.mul_scalar),
                          ("add", plan.mod_add_scalar, O.add_scalar),
                          ("sub", plan.mod_sub_scalar, O.sub_scalar)):
        c = torch.empty_like(da)
        fn(da.data_ptr(), s, c.data_ptr(), batch, stream())
        assert np.array_equal(host(c), ref(a, s, q)), name
        # in place (the *Eq form)
        x = dev(a)
        fn(x.data_ptr(), s, x.data_ptr(), batch, stream())
        assert np.array_equal(host(x), ref(a, s, q)), name + " in place"
    for idx in sorted({0, n - 1, n // 2}):
        x = dev(a)
        plan.mod_add_scalar_at(x.data_ptr(), idx, s, x.data_ptr(), batch, stream())
        assert np.array_equal(host(x), O.add_scalar_at(a, idx, s, q)), idx
    with pytest.raises(H.MathError):
        plan.mod_add_scalar_at(da.data_ptr(), n, s, da.data_ptr(), batch, stream())
    with pytest.raises(H.MathError):
        plan.mod_add_scalar(da.data_ptr(), s[:-1], da.data_ptr(), batch, stream())


def test_switch_modulus_reference_kat(hip):
    """UnitTestPolyElements.cpp:265-305 on the GPU."""
    H, ctx = hip
    import torch

    k = REF["kat_switch_modulus"]
    for c in k["cases"]:
        x = dev(np.array(c["x"], np.uint64))
        y = torch.empty_like(x)
        H.switch_modulus(ctx, x.data_ptr(), y.data_ptr(), 4, k["q"], c["new_q"], stream())
        assert host(y).tolist() == c["expected"]


def test_automorphism_reference_kat(hip):
    """UnitTestPolyElements.cpp:500-523 on the GPU: coefficient form directly, and
    evaluation form through the GPU NTT (q = 73, m = 8, root 22)."""
    H, ctx = hip
    import torch

    k = REF["kat_automorphism"]
    plan = H.NTTPlan(ctx, 2, [k["q"]], [k["root"]])
    x = dev(np.array(k["x"], np.uint64).reshape(1, 1, 4))
    y = torch.empty_like(x)
    plan.automorphism(k["k"], False, x.data_ptr(), y.data_ptr(), 1, stream())
    assert host(y).reshape(-1).tolist() == k["expected"]
    plan.forward(x.data_ptr(), 1, stream())
    plan.automorphism(k["k"], True, x.data_ptr(), y.data_ptr(), 1, stream())
    plan.inverse(y.data_ptr(), 1, stream())
    assert host(y).reshape(-1).tolist() == k["expected"]
    # UnitTestPolyElements.cpp:535-571: Transpose = AutomorphismTransform(m - 1), evaluation form
    t = k["transpose"]
    x = dev(np.array(t["x"], np.uint64).reshape(1, 1, 4))
    plan.forward(x.data_ptr(), 1, stream())
    plan.automorphism(t["k"], True, x.data_ptr(), y.data_ptr(), 1, stream())
    plan.inverse(y.data_ptr(), 1, stream())
    assert host(y).reshape(-1).tolist() == t["expected"]


@pytest.mark.parametrize("log_n,towers,batch,b0", [(3, 3, 4, 0), (14, 2, 3, 5), (16, 2, 2, 1021)])
def test_fill_uniform_matches_oracle(hip, log_n, towers, batch, b0):
    H, ctx = hip
    import torch

    n = 1 << log_n
    q, r = O.moduli_chain(log_n, towers)
    plan = H.NTTPlan(ctx, log_n, q, r)
    x = torch.empty((batch, towers, n), dtype=torch.int64, device="cuda")
    plan.fill_uniform(x.data_ptr(), batch, 7, b0, stream())
    got = host(x)
    want = np.stack([_oracle_row(O, b0 + i, towers, n, q, 7) for i in range(batch)])
    assert np.array_equal(got, want)


def _oracle_row(O, b, towers, n, q, seed):
    out = np.empty((towers, n), np.uint64)
    for t in range(towers):
        out[t] = O.splitmix_fill(n, q[t], O.U([0x5EED ^ (b << 20) ^ (t << 8) ^ seed]))
    return out


def test_configs1_eltwise(hip):
    """configs[1]: N = 2^14, 8 towers -- ModAdd, ModSub, ModMul against the oracle."""
    H, ctx = hip
    import torch

    log_n, T, B = 14, 8, 3
    n = 1 << log_n
    q, r = O.moduli_chain(log_n, T)
    plan = H.NTTPlan(ctx, log_n, q, r)
    a, b = O.uniform_dcrt(B, T, n, q, 11), O.uniform_dcrt(B, T, n, q, 12)
    a[0, :, :3] = np.array(q, np.uint64)[:, None] - np.uint64(1)
    b[0, :, :3] = np.array(q, np.uint64)[:, None] - np.uint64(1)
    da, db = dev(a), dev(b)
    for op in ("add", "sub", "mul"):
        c = torch.empty_like(da)
        getattr(plan, "mod_" + op)(da.data_ptr(), db.data_ptr(), c.data_ptr(), B, stream())
        assert np.array_equal(host(c), O.eltwise(op, a, b, q)), op


def test_configs3_tower_shards(hip):
    """configs[3]'s per-rank work: N = 2^16, 32 towers of the poly-benchmark
    chain split into eight 4-tower shards (what rank r of 8 owns,
    shard.shard_towers).  Each shard runs the forward and inverse range
    transforms on the full 32-tower layout and the pipeline on its own plan,
    all compared with the oracle."""
    H, ctx = hip
    import torch

    import shard

    log_n, T, B, W = 16, 32, 2, 8
    n = 1 << log_n
    q, r = O.moduli_chain(log_n, T)
    full = H.NTTPlan(ctx, log_n, q, r)
    a, b = O.uniform_dcrt(B, T, n, q, 21), O.uniform_dcrt(B, T, n, q, 22)
    da = dev(a)
    fwd = torch.empty_like(da)
    inv = torch.empty_like(da)
    tb_all = O.Tables(n, q, r)
    want_f = O.ntt_fwd(a, tb_all)
    want_i = O.ntt_inv(a, tb_all)
    for rank in range(W):
        t0, cnt = shard.shard_towers(T, rank, W)
        assert cnt == 4
        off = t0 * n
        full.forward_range(t0, cnt, da.data_ptr() + 8 * off, fwd.data_ptr() + 8 * off, T * n, T * n, B, stream())
        full.inverse_range(t0, cnt, da.data_ptr() + 8 * off, inv.data_ptr() + 8 * off, T * n, T * n, B, stream())
        sub = H.NTTPlan(ctx, log_n, q[t0:t0 + cnt], r[t0:t0 + cnt])
        sa, sb = dev(a[:, t0:t0 + cnt]), dev(b[:, t0:t0 + cnt])
        sc = torch.empty_like(sa)
        sub.ntt_mul_intt(sa.data_ptr(), sb.data_ptr(), sc.data_ptr(), B, stream())
        tb = O.Tables(n, q[t0:t0 + cnt], r[t0:t0 + cnt])
        assert np.array_equal(host(sc), O.ntt_mul_intt(a[:, t0:t0 + cnt], b[:, t0:t0 + cnt], tb)), rank
        sub.close()
    assert np.array_equal(host(fwd), want_f)
    assert np.array_equal(host(inv), want_i)


def test_mod_down_concurrent_streams(hip):
    """ApproxModDown with t = 0 and t = 65537 issued back to back on two
    streams on the same objects, twice: the per-(t, P^-1) constant tables are
    cached in the converter, so neither call drains the device or rewrites a
    table the other stream is reading."""
    H, ctx = hip
    import torch

    log_n, sq, sp, B = 12, 6, 3, 2
    n = 1 << log_n
    m, rr = O.moduli_chain(log_n, sq + sp)
    q, rq, p, rp = m[:sq], rr[:sq], m[sq:], rr[sq:]
    pq, pp = H.NTTPlan(ctx, log_n, q, rq), H.NTTPlan(ctx, log_n, p, rp)
    qhinv, qhmodp = K.switch_tables(p, q)
    bc = H.BaseConverter(ctx, log_n, p, q, qhinv, [v for row in qhmodp for v in row])
    rng = np.random.default_rng(9)
    x = _uniform(rng, B, q + p, n)
    dx = dev(x)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    outs = []
    for rep in range(2):
        for t, s in ((0, s1), (65537, s2)):
            o = torch.empty((B, sq, n), dtype=torch.int64, device="cuda")
            H.approx_mod_down(pq, pp, bc, K.moddown_tables(q, p, t)["pinv_modq"], t, dx.data_ptr(), o.data_ptr(),
                              B, s.cuda_stream)
            outs.append((t, o))
    torch.cuda.synchronize()
    for t, o in outs:
        assert np.array_equal(host(o), K.approx_mod_down(x, q, rq, p, rp, t)), t
