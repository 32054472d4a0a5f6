"""GPU parity: the HIP backend (through the C ABI) against the oracle and the
committed golden vectors.  Bit-exact for every op (integer arithmetic).

Mirrors the reference's own tests: UnitTestTransform (KAT), UnitTestNTT
(round trips), UnitTestMubintvec (vector ModAdd/ModSub/ModMul KATs),
UnitTestDCRTElements (random DCRTPoly + and * against an independent check).
"""
import ctypes

import numpy as np
import pytest
from conftest import load_golden

pytestmark = pytest.mark.gpu

REF = load_golden("reference_fixtures.json")


def dev(x):
    import torch

    return torch.from_numpy(np.ascontiguousarray(x, dtype=np.uint64).view(np.int64)).cuda()


def host(t):
    import torch

    torch.cuda.synchronize()
    return t.cpu().numpy().view(np.uint64)


def stream():
    import torch

    return torch.cuda.current_stream().cuda_stream


def run_all_ops(hip, plan, a, b):
    """Every plan op on device copies of a, b -> dict of host results."""
    import torch

    out = {}
    x = dev(a)
    plan.forward(x.data_ptr(), a.shape[0], stream())
    out["ntt_a"] = host(x)
    x = dev(a)
    plan.inverse(x.data_ptr(), a.shape[0], stream())
    out["intt_a"] = host(x)
    for op in ("mul", "add", "sub"):
        xa, xb = dev(a), dev(b)
        xc = torch.empty_like(xa)
        getattr(plan, "mod_" + op)(xa.data_ptr(), xb.data_ptr(), xc.data_ptr(), a.shape[0], stream())
        out[op] = host(xc)
    xa, xb = dev(a), dev(b)
    xc = torch.empty_like(xa)
    plan.ntt_mul_intt(xa.data_ptr(), xb.data_ptr(), xc.data_ptr(), a.shape[0], stream())
    out["pipeline"] = host(xc)
    return out


def test_kat_transform(hip):
    """UnitTestTransform.cpp:60-94 on the GPU: [1,2,4,1]^2 mod (x^4+1, 113) = [94,109,11,18]."""
    H, ctx = hip
    k = REF["kat_transform"]
    plan = H.NTTPlan(ctx, 2, [k["q"]], [k["root"]])
    a = np.array(k["a"], np.uint64).reshape(1, 1, 4)
    x = dev(a)
    plan.forward(x.data_ptr(), 1, stream())
    y = dev(np.zeros_like(a))
    plan.mod_mul(x.data_ptr(), x.data_ptr(), y.data_ptr(), 1, stream())
    plan.inverse(y.data_ptr(), 1, stream())
    assert host(y).reshape(-1).tolist() == k["expected"]
    # same through the fused pipeline (b = NTT(a))
    c = dev(np.zeros_like(a))
    da = dev(a)  # referenced until the stream has consumed it
    plan.ntt_mul_intt(da.data_ptr(), x.data_ptr(), c.data_ptr(), 1, stream())
    assert host(c).reshape(-1).tolist() == k["expected"]


def test_kat_mubintvec(hip):
    """UnitTestMubintvec.cpp:276-359 (q = 163841) through the element-wise kernels."""
    import torch

    H, ctx = hip
    k = REF["kat_mubintvec"]
    q = k["q"]
    # q = 163841 = 1 mod 2^15: a valid NTT modulus for N = 16; root from the oracle rule
    psi = next(r for r in range(2, q) if pow(r, 16, q) == q - 1)
    psi = min(pow(psi, e, q) for e in range(1, 32, 2))
    plan = H.NTTPlan(ctx, 4, [q], [psi])
    a, b = dev(np.array(k["a"], np.uint64)), dev(np.array(k["b"], np.uint64))
    for op in ("add", "sub", "mul"):
        c = torch.empty_like(a)
        getattr(plan, "mod_" + op)(a.data_ptr(), b.data_ptr(), c.data_ptr(), 1, stream())
        assert host(c).tolist() == k["mod" + op], op


@pytest.mark.parametrize("log_n,batch", [(4, 1), (16, 3)])
def test_kat_mubintvec_2limb(hip, log_n, batch):
    """UnitTestMubintvec.cpp:402-484 (a 52-bit modulus) through the element-wise
    kernels, the 16-element vectors tiled to N = 2^log_n over `batch` entries."""
    import torch

    H, ctx = hip
    k = REF["kat_mubintvec_2limb"]
    q = k["q"]  # = 1 mod 2^20: an NTT modulus up to N = 2^19; root from the oracle rule
    n = 1 << log_n
    g = next(r for r in range(2, 1000) if pow(r, (q - 1) // 2, q) == q - 1)
    psi = pow(g, (q - 1) // (2 * n), q)
    plan = H.NTTPlan(ctx, log_n, [q], [psi])
    reps = n // 16
    tile = lambda v: np.tile(np.array(v, np.uint64), batch * reps).reshape(batch, 1, n)  # noqa: E731
    a, b = dev(tile(k["a"])), dev(tile(k["b"]))
    for op in ("add", "sub", "mul"):
        c = torch.empty_like(a)
        getattr(plan, "mod_" + op)(a.data_ptr(), b.data_ptr(), c.data_ptr(), batch, stream())
        assert np.array_equal(host(c), tile(k["mod" + op])), op
    plan.close()


def test_kat_dcrt_arithmetic(hip):
    """UnitTestDCRTElements.cpp:285-417 (three towers 8353 / 8369 / 8513, N = 4,
    evaluation form) through the C ABI: Plus, Minus, Times, AddILElementOne."""
    import torch

    H, ctx = hip
    k = REF["kat_dcrt_arithmetic"]
    plan = H.NTTPlan(ctx, 2, k["q"], k["root"])
    rep = lambda v: np.stack([np.array(v, np.uint64)] * 3)[None]  # noqa: E731
    a, b = dev(rep(k["a"])), dev(rep(k["b"]))
    for op, key in (("add", "plus"), ("sub", "minus"), ("mul", "times")):
        c = torch.empty_like(a)
        getattr(plan, "mod_" + op)(a.data_ptr(), b.data_ptr(), c.data_ptr(), 1, stream())
        assert np.array_equal(host(c), rep(k[key])), op
    c = torch.empty_like(a)
    plan.mod_add_scalar(a.data_ptr(), [1, 1, 1], c.data_ptr(), 1, stream())
    assert np.array_equal(host(c), rep(k["add_one"]))
    plan.close()


def test_kat_common_elements(hip):
    """UnitTestCommonElements.cpp (q = 73, N = 4) through the C ABI:
    common_binary_ops (240-320) -- evaluation-form Plus / Minus / Times and
    SwitchFormat -> Times -> SwitchFormat, here both as separate transforms and
    as the fused pipeline; common_arithmetic_ops_element (381-446) -- Plus(1)
    in coefficient form at coefficient 0 only, Minus(1) / Times(2) on every
    slot; AddILElementOne (457-483)."""
    import torch

    H, ctx = hip
    k = REF["kat_common_elements"]
    plan = H.NTTPlan(ctx, 2, [k["q"]], [k["root"]])
    vec = lambda v: dev(np.array(v, np.uint64).reshape(1, 1, 4))  # noqa: E731
    flat = lambda t: host(t).reshape(-1).tolist()  # noqa: E731
    bo = k["binary_ops"]
    a, b = vec(bo["a"]), vec(bo["b"])
    for op, key in (("add", "plus_eval"), ("sub", "minus_eval"), ("mul", "times_eval")):
        c = torch.empty_like(a)
        getattr(plan, "mod_" + op)(a.data_ptr(), b.data_ptr(), c.data_ptr(), 1, stream())
        assert flat(c) == bo[key], op
    fa, fb = vec(bo["a"]), vec(bo["b"])
    plan.forward(fa.data_ptr(), 1, stream())
    plan.forward(fb.data_ptr(), 1, stream())
    c = torch.empty_like(fa)
    plan.mod_mul(fa.data_ptr(), fb.data_ptr(), c.data_ptr(), 1, stream())
    plan.inverse(c.data_ptr(), 1, stream())
    assert flat(c) == bo["switchformat_times_switchformat"]
    c2 = torch.empty_like(fa)
    plan.ntt_mul_intt(a.data_ptr(), fb.data_ptr(), c2.data_ptr(), 1, stream())
    assert flat(c2) == bo["switchformat_times_switchformat"]
    so = k["scalar_ops"]
    x = vec(so["coef_x"])
    plan.mod_add_scalar_at(x.data_ptr(), 0, [1], x.data_ptr(), 1, stream())
    assert flat(x) == so["plus_1_coefficient_form"]
    e = vec(so["eval_x"])
    c = torch.empty_like(e)
    plan.mod_sub_scalar(e.data_ptr(), [1], c.data_ptr(), 1, stream())
    assert flat(c) == so["minus_1_eval"]
    plan.mod_mul_scalar(e.data_ptr(), [2], c.data_ptr(), 1, stream())
    assert flat(c) == so["times_2_eval"]
    one = k["add_il_element_one"]
    x = vec(one["x"])
    plan.mod_add_scalar(x.data_ptr(), [1], x.data_ptr(), 1, stream())
    assert flat(x) == one["expected"]
    plan.close()


@pytest.mark.parametrize("case", range(5))
def test_golden_vectors(hip, case):
    H, ctx = hip
    c = load_golden("oracle_vectors.json")["cases"][case]
    n, T, B = 1 << c["log_n"], c["towers"], c["batch"]
    plan = H.NTTPlan(ctx, c["log_n"], c["q"], c["psi"])
    a = np.array(c["a"], np.uint64).reshape(B, T, n)
    b = np.array(c["b"], np.uint64).reshape(B, T, n)
    got = run_all_ops(H, plan, a, b)
    for key in ("ntt_a", "intt_a", "mul", "add", "sub", "pipeline"):
        assert got[key].reshape(-1).tolist() == c[key], key


@pytest.mark.parametrize("idx", range(6))
def test_fingerprints_full_size(hip, O, idx):
    """Benchmark shapes (N = 2^12 .. 2^17): FNV-1a of every output equals the
    committed oracle fingerprint, and the oracle run here agrees element-wise."""
    H, ctx = hip
    f = load_golden("oracle_fingerprints.json")["fingerprints"][idx]
    n, T, B = 1 << f["log_n"], f["towers"], f["batch"]
    plan = H.NTTPlan(ctx, f["log_n"], f["q"], f["psi"])
    a = O.uniform_dcrt(B, T, n, f["q"], f["seed_a"])
    b = O.uniform_dcrt(B, T, n, f["q"], f["seed_b"])
    got = run_all_ops(H, plan, a, b)
    assert O.fnv64(got["ntt_a"]) == f["fnv_ntt_a"]
    assert O.fnv64(got["intt_a"]) == f["fnv_intt_a"]
    assert O.fnv64(got["mul"]) == f["fnv_mul"]
    assert O.fnv64(got["pipeline"]) == f["fnv_pipeline"]


def test_survey_probe_dcrt_pipeline(hip, O):
    """Reference output: DCRTPoly N=2^14, T=8, c[0][0]."""
    import torch

    H, ctx = hip
    pr = REF["survey_probes"]["dcrt_pipeline"]
    n, T = 1 << pr["log_n"], pr["towers"]
    qs, rs = O.moduli_chain(pr["log_n"], T)
    st = O.U([pr["seed"]])
    a = np.zeros((1, T, n), np.uint64)
    b = np.zeros((1, T, n), np.uint64)
    for t in range(T):
        ab = O.splitmix_fill(2 * n, qs[t], st)
        a[0, t], b[0, t] = ab[0::2], ab[1::2]
    plan = H.NTTPlan(ctx, pr["log_n"], qs, rs)
    xa, xb = dev(a), dev(b)
    xc = torch.empty_like(xa)
    plan.ntt_mul_intt(xa.data_ptr(), xb.data_ptr(), xc.data_ptr(), 1, stream())
    c = host(xc)
    assert int(c[0, 0, 0]) == pr["c00"]
    assert np.array_equal(c, O.ntt_mul_intt(a, b, O.Tables(n, qs, rs)))


@pytest.mark.parametrize("log_n,towers,batch", [(1, 1, 3), (2, 3, 2), (5, 2, 4), (9, 4, 3), (11, 2, 2),
                                                (12, 3, 3), (13, 1, 2), (14, 8, 2), (15, 3, 1), (16, 2, 2),
                                                (17, 1, 2)])
def test_random_shapes_vs_oracle(hip, O, log_n, towers, batch):
    """Element-wise equality with the oracle over ragged (batch, tower) shapes."""
    H, ctx = hip
    n = 1 << log_n
    qs, rs = O.moduli_chain(log_n, towers)
    tb = O.Tables(n, qs, rs)
    a = O.uniform_dcrt(batch, towers, n, qs, 100 + log_n)
    b = O.uniform_dcrt(batch, towers, n, qs, 200 + log_n)
    got = run_all_ops(H, H.NTTPlan(ctx, log_n, qs, rs), a, b)
    assert np.array_equal(got["ntt_a"], O.ntt_fwd(a, tb))
    assert np.array_equal(got["intt_a"], O.ntt_inv(a, tb))
    assert np.array_equal(got["mul"], O.eltwise("mul", a, b, qs))
    assert np.array_equal(got["pipeline"], O.ntt_mul_intt(a, b, tb))


@pytest.mark.parametrize("log_n", [14, 16, 17])
def test_edge_values(hip, O, log_n):
    """All-zero, all-(q-1) and alternating extreme inputs (lazy-reduction corners);
    2^16 runs the k_tcols column pass, 2^17 k_cols (k_tcols9: test_split9_n17_vs_oracle)."""
    H, ctx = hip
    T = 3 if log_n == 14 else 1
    n = 1 << log_n
    qs, rs = O.moduli_chain(log_n, T)
    tb = O.Tables(n, qs, rs)
    q = np.array(qs, np.uint64)[None, :, None]
    for a in (np.zeros((1, T, n), np.uint64), np.broadcast_to(q - np.uint64(1), (1, T, n)).copy(),
              np.where(np.arange(n) % 2 == 0, q - np.uint64(1), np.uint64(0)).astype(np.uint64)):
        b = np.broadcast_to(q - np.uint64(1), (1, T, n)).copy()
        got = run_all_ops(H, H.NTTPlan(ctx, log_n, qs, rs), a, b)
        assert np.array_equal(got["ntt_a"], O.ntt_fwd(a, tb))
        assert np.array_equal(got["intt_a"], O.ntt_inv(a, tb))
        assert np.array_equal(got["pipeline"], O.ntt_mul_intt(a, b, tb))


def test_inplace_and_roundtrip_full_size(hip, O):
    """N = 2^16, T = 16: INTT(NTT(x)) = x in place; fused op with c aliasing a;
    linearity NTT(a + b) = NTT(a) + NTT(b)."""
    import torch

    H, ctx = hip
    log_n, T, B = 16, 16, 2
    n = 1 << log_n
    qs, rs = O.moduli_chain(log_n, T)
    plan = H.NTTPlan(ctx, log_n, qs, rs)
    a = O.uniform_dcrt(B, T, n, qs, 77)
    b = O.uniform_dcrt(B, T, n, qs, 78)
    x = dev(a)
    plan.forward(x.data_ptr(), B, stream())
    plan.inverse(x.data_ptr(), B, stream())
    assert np.array_equal(host(x), a)
    xa, xb = dev(a), dev(b)
    plan.ntt_mul_intt(xa.data_ptr(), xb.data_ptr(), xa.data_ptr(), B, stream())
    assert np.array_equal(host(xa), O.ntt_mul_intt(a, b, O.Tables(n, qs, rs)))
    xa, xb, xs = dev(a), dev(b), torch.empty_like(dev(a))
    plan.mod_add(xa.data_ptr(), xb.data_ptr(), xs.data_ptr(), B, stream())
    for t_ in (xa, xb, xs):
        plan.forward(t_.data_ptr(), B, stream())
    s2 = torch.empty_like(xs)
    plan.mod_add(xa.data_ptr(), xb.data_ptr(), s2.data_ptr(), B, stream())
    assert np.array_equal(host(xs), host(s2))


def test_scalar_modmul(hip, O):
    import torch

    H, ctx = hip
    log_n, T, B = 12, 3, 2
    n = 1 << log_n
    qs, rs = O.moduli_chain(log_n, T)
    plan = H.NTTPlan(ctx, log_n, qs, rs)
    a = O.uniform_dcrt(B, T, n, qs, 5)
    sc = [qs[0] - 1, 12345678901234567, 2**63 + 5]  # the last is reduced mod q first
    x = dev(a)
    y = torch.empty_like(x)
    plan.mod_mul_scalar(x.data_ptr(), sc, y.data_ptr(), B, stream())
    assert np.array_equal(host(y), O.mul_scalar(a, [s % q for s, q in zip(sc, qs)], qs))


@pytest.mark.parametrize("case", range(3))
def test_base_conversion_golden(hip, O, case):
    import torch

    H, ctx = hip
    c = load_golden("bconv_vectors.json")["cases"][case]
    n, B, sq, sp = 1 << c["log_n"], c["batch"], len(c["q"]), len(c["p"])
    bc = H.BaseConverter(ctx, c["log_n"], c["q"], c["p"], c["qhat_inv_modq"], c["qhat_modp"])
    x = dev(np.array(c["x"], np.uint64).reshape(B, sq, n))
    out = torch.zeros((B, sp, n), dtype=torch.int64, device="cuda")
    bc.switch(x.data_ptr(), out.data_ptr(), B, stream())
    assert host(out).reshape(-1).tolist() == c["out"]


@pytest.mark.parametrize("log_n", [3, 5, 12, 17])
def test_kat_fast_expand_crt_basis(hip, log_n):
    """UnitTestBFVrnsCRTOperations.cpp:290-376 through the C ABI: the R_l towers
    of FastExpandCRTBasisPloverQ's answer (its ApproxSwitchCRTBasis loop,
    dcrtpoly-impl.h:1419-1441) with the test's constants; the N = 8 vectors
    tiled to N = 2^log_n (the conversion is coefficient-wise) so the small-ring,
    matrix-core and 2^17 kernels all see them; batch entry 1 holds the columns
    reversed."""
    import torch
    from test_oracle import fast_expand_constants

    H, ctx = hip
    k = REF["kat_fast_expand_crt_basis"]
    q, r = k["q"], k["r"]
    c, d = fast_expand_constants(q, r)
    reps = (1 << log_n) // 8
    x0 = np.tile(np.array(k["x"], np.uint64), (1, reps))
    want0 = np.tile(np.array(k["expected_rl"], np.uint64), (1, reps))
    x = np.stack([x0, x0[:, ::-1]])
    want = np.stack([want0, want0[:, ::-1]])
    bc = H.BaseConverter(ctx, log_n, q, r, c, [v for row in d for v in row])
    out = torch.zeros((2, len(r), 1 << log_n), dtype=torch.int64, device="cuda")
    bc.switch(dev(x).data_ptr(), out.data_ptr(), 2, stream())
    assert np.array_equal(host(out), want)


@pytest.mark.parametrize("log_n,towers,batch", [(4, 4096, 1), (11, 700, 1), (13, 300, 2)])
def test_plan_tower_limits(hip, O, log_n, towers, batch):
    """Plans up to the C ABI's 4096 towers (ofhe_hip_plan_create): forward,
    inverse and the fused pipeline against the oracle on every tower; 4097
    is refused."""
    import torch

    H, ctx = hip
    n = 1 << log_n
    qs, rs = O.moduli_chain(log_n, towers)
    plan = H.NTTPlan(ctx, log_n, qs, rs)
    tb = O.Tables(n, qs, rs)
    a = O.uniform_dcrt(batch, towers, n, qs, 51)
    b = O.uniform_dcrt(batch, towers, n, qs, 52)
    x = dev(a)
    plan.forward(x.data_ptr(), batch, stream())
    assert np.array_equal(host(x), O.ntt_fwd(a, tb))
    x = dev(a)
    plan.inverse(x.data_ptr(), batch, stream())
    assert np.array_equal(host(x), O.ntt_inv(a, tb))
    xa, xb = dev(a), dev(b)
    c = torch.empty_like(xa)
    plan.ntt_mul_intt(xa.data_ptr(), xb.data_ptr(), c.data_ptr(), batch, stream())
    assert np.array_equal(host(c), O.ntt_mul_intt(a, b, tb))
    plan.close()
    if towers == 4096:
        q2, r2 = O.moduli_chain(log_n, 4097)
        with pytest.raises(H.MathError):
            H.NTTPlan(ctx, log_n, q2, r2)


@pytest.mark.parametrize("log_n,sq,sp", [(5, 256, 256), (12, 200, 56), (12, 17, 256)])
def test_base_conversion_size_limits(hip, O, log_n, sq, sp):
    """ApproxSwitchCRTBasis at the C ABI's basis limits (256 source or target
    towers, ofhe_hip_bconv_create) against the oracle; 257 is refused."""
    import torch

    H, ctx = hip
    n = 1 << log_n
    chain, _ = O.moduli_chain(log_n, sq + sp)
    q, p = chain[:sq], chain[sq:]
    pre = O.base_conv_precompute(q, p)
    x = O.uniform_dcrt(2, sq, n, q, 41)
    bc = H.BaseConverter(ctx, log_n, q, p, [int(v) for v in pre["qhinv"]], [int(v) for v in pre["qhmodp"]])
    out = torch.zeros((2, sp, n), dtype=torch.int64, device="cuda")
    bc.switch(dev(x).data_ptr(), out.data_ptr(), 2, stream())
    got = host(out)
    for bi in range(2):
        assert np.array_equal(got[bi], O.approx_switch_crt_basis(x[bi], q, p, pre)), bi
    bc.close()
    with pytest.raises(H.MathError):
        H.BaseConverter(ctx, log_n, chain[:1] * 257, p[:1], [1] * 257, [1] * 257)


def test_base_conversion_config5_shape(hip, O):
    """N = 2^17 digit -> complement (16 -> 17 towers), vs the oracle."""
    import torch

    H, ctx = hip
    log_n, sq, sp = 17, 16, 17
    n = 1 << log_n
    chain, _ = O.moduli_chain(log_n, sq + sp)
    q, p = chain[:sq], chain[sq:]
    pre = O.base_conv_precompute(q, p)
    x = O.uniform_dcrt(1, sq, n, q, 31)
    bc = H.BaseConverter(ctx, log_n, q, p, [int(v) for v in pre["qhinv"]], [int(v) for v in pre["qhmodp"]])
    out = torch.zeros((1, sp, n), dtype=torch.int64, device="cuda")
    dx = dev(x)
    bc.switch(dx.data_ptr(), out.data_ptr(), 1, stream())
    assert np.array_equal(host(out)[0], O.approx_switch_crt_basis(x[0], q, p, pre))


def test_errors_raise(hip, O):
    """Invalid parameters fail loudly (math_error analogue), as OPENFHE_THROW does."""
    H, ctx = hip
    qs, rs = O.moduli_chain(10, 1)
    with pytest.raises(H.MathError):
        H.NTTPlan(ctx, 10, [qs[0]], [1])               # root 1 is not primitive
    with pytest.raises(H.MathError):
        H.NTTPlan(ctx, 10, [qs[0] + 2], [rs[0]])       # not 1 mod 2N
    with pytest.raises(H.MathError):
        H.NTTPlan(ctx, 18, qs, rs)                     # ring too large
    plan = H.NTTPlan(ctx, 10, qs, rs)
    with pytest.raises(H.MathError):
        plan.forward(0, 1, stream())                   # NULL data
    with pytest.raises(H.MathError):
        plan.forward(1 << 20, 0, stream())             # empty batch


def test_creation_options_refused(hip, O):
    """Creation options outside their domain are refused with OFHE_ERR_ARG
    (ofhe_hip_plan_create_ex / _bconv_create_ex / _ks_create_ex), never
    silently replaced by a default kernel: every split names the log_n it
    applies to, and flags are 0 or 1."""
    H, ctx = hip
    bad_splits = [(10, H.SPLIT_COLS), (10, H.SPLIT_8_8), (17, H.SPLIT_8_8), (16, H.SPLIT_9_8),
                  (16, H.SPLIT_8_9), (14, H.SPLIT_8_9), (16, 5), (17, 99)]
    for log_n, split in bad_splits:
        qs, rs = O.moduli_chain(log_n, 1)
        with pytest.raises(H.MathError):
            H.NTTPlan(ctx, log_n, qs, rs, split=split)
    qs, rs = O.moduli_chain(16, 1)
    o = H.PlanOptions(H.SPLIT_AUTO, 2)                  # generic_moduli is a flag
    h = H._vp()
    assert H.lib().ofhe_hip_plan_create_ex(ctx.handle, 16, 1, H._arr(qs), H._arr(rs), H._opt_ptr(o),
                                           ctypes.byref(h)) != 0
    for log_n, split in ((13, H.SPLIT_COLS), (16, H.SPLIT_8_8), (17, H.SPLIT_9_8), (17, H.SPLIT_8_9)):
        qs, rs = O.moduli_chain(log_n, 1)
        H.NTTPlan(ctx, log_n, qs, rs, split=split).close()  # the accepted combinations
    q, _ = O.moduli_chain(10, 3)
    p = [int(v) for v in O.moduli_chain(10, 5)[0][3:5]]
    pre = O.base_conv_precompute(q, p)
    args = (ctx, 10, q, p, [int(v) for v in pre["qhinv"]], [int(v) for v in pre["qhmodp"]])
    with pytest.raises(H.MathError):
        H.BaseConverter(*args, kernel=3)
    H.BaseConverter(*args, kernel=H.BCONV_KERNEL_WIDE).close()
    qs, rs = O.moduli_chain(12, 6)
    for opt in (H.KsOptions(H.PlanOptions(H.SPLIT_8_8, 0), 0, 0, 0, 0),  # a 2^16-only split at 2^12
                H.KsOptions(H.PlanOptions(0, 0), 2, 0, 0, 0), H.KsOptions(H.PlanOptions(0, 0), 0, 3, 0, 0),
                H.KsOptions(H.PlanOptions(0, 0), 0, 0, 0, 7)):
        with pytest.raises(H.MathError):
            H.KeySwitch(ctx, 12, qs[:4], rs[:4], qs[4:], rs[4:], 2, opt)


def _generic_moduli(O, log_n, towers, bits=58):
    """NTT primes q = 1 mod 2N in the middle of [2^bits, 2^(bits+1)): NOT of the
    special form 2^L - d (d < 2^32), so the generic Shoup kernels run."""
    m = 2 << log_n
    qs, rs = [], []
    cand = ((3 << (bits - 1)) // m) * m + 1  # ~1.5 * 2^bits
    while len(qs) < towers:
        if O.lib().oracle_is_prime(cand):
            qs.append(cand)
            rs.append(O.root_of_unity(m, cand))
        cand += m
    return qs, rs


@pytest.mark.parametrize("log_n,towers,batch", [(11, 2, 2), (12, 2, 2), (13, 3, 1), (16, 2, 2), (17, 1, 1)])
def test_generic_moduli_vs_oracle(hip, O, log_n, towers, batch):
    """Moduli that are not 2^L - d: exercises the generic (non special-prime) kernels."""
    H, ctx = hip
    n = 1 << log_n
    qs, rs = _generic_moduli(O, log_n, towers)
    assert all((q >> 32) != (1 << (q.bit_length() - 32)) - 1 for q in qs)
    tb = O.Tables(n, qs, rs)
    a = O.uniform_dcrt(batch, towers, n, qs, 300 + log_n)
    b = O.uniform_dcrt(batch, towers, n, qs, 400 + log_n)
    got = run_all_ops(H, H.NTTPlan(ctx, log_n, qs, rs), a, b)
    assert np.array_equal(got["ntt_a"], O.ntt_fwd(a, tb))
    assert np.array_equal(got["intt_a"], O.ntt_inv(a, tb))
    assert np.array_equal(got["pipeline"], O.ntt_mul_intt(a, b, tb))


def test_special_prime_switch_identical(hip, O):
    """Special-prime and generic kernels give identical results on the same
    (special-form) moduli; the plan option generic_moduli forces the generic
    instantiation."""
    import torch

    H, ctx = hip
    log_n, T, B = 16, 4, 2
    n = 1 << log_n
    qs, rs = O.moduli_chain(log_n, T)
    a = O.uniform_dcrt(B, T, n, qs, 5)
    b = O.uniform_dcrt(B, T, n, qs, 6)
    outs = []
    for generic in (False, True):
        plan = H.NTTPlan(ctx, log_n, qs, rs, generic_moduli=generic)
        xa, xb = dev(a), dev(b)
        xc = torch.empty_like(xa)
        plan.ntt_mul_intt(xa.data_ptr(), xb.data_ptr(), xc.data_ptr(), B, stream())
        outs.append(host(xc))
    assert np.array_equal(outs[0], outs[1])
    assert np.array_equal(outs[0], O.ntt_mul_intt(a, b, O.Tables(n, qs, rs)))


@pytest.mark.parametrize("split", ["SPLIT_9_8", "SPLIT_8_9"])
@pytest.mark.parametrize("edge", [False, True])
def test_split9_n17_vs_oracle(hip, O, edge, split):
    """N = 2^17 under OFHE_SPLIT_9_8 (k_tcols9: 9 column stages + the 8-stage
    block pass) and OFHE_SPLIT_8_9 (k_tcols' 8 column stages on 512 columns +
    the 9-stage block pass) gives the oracle's forward, inverse and pipeline
    outputs; edge = all-(q-1) inputs (lazy-reduction corners of the split)."""
    import torch

    H, ctx = hip
    log_n, T, B = 17, 2, 2
    n = 1 << log_n
    qs, rs = O.moduli_chain(log_n, T)
    tb = O.Tables(n, qs, rs)
    if edge:
        a = np.broadcast_to(np.array(qs, np.uint64)[None, :, None] - np.uint64(1), (B, T, n)).copy()
    else:
        a = O.uniform_dcrt(B, T, n, qs, 17)
    b = O.uniform_dcrt(B, T, n, qs, 18)
    plan = H.NTTPlan(ctx, log_n, qs, rs, split=getattr(H, split))
    xa, xb = dev(a), dev(b)
    xc = torch.empty_like(xa)
    plan.ntt_mul_intt(xa.data_ptr(), xb.data_ptr(), xc.data_ptr(), B, stream())
    xf, xi = dev(a), dev(a)
    plan.forward(xf.data_ptr(), B, stream())
    plan.inverse(xi.data_ptr(), B, stream())
    assert np.array_equal(host(xf), O.ntt_fwd(a, tb))
    assert np.array_equal(host(xi), O.ntt_inv(a, tb))
    assert np.array_equal(host(xc), O.ntt_mul_intt(a, b, tb))


def test_split4_identical(hip, O):
    """N = 2^16 under OFHE_SPLIT_COLS (4 column stages + a 12-stage block pass, so
    the inverse block twist covers groups of 4096 instead of 256) gives the
    same canonical results as the default 8 | 8 split."""
    import torch

    H, ctx = hip
    log_n, T, B = 16, 3, 2
    n = 1 << log_n
    qs, rs = O.moduli_chain(log_n, T)
    tb = O.Tables(n, qs, rs)
    a = O.uniform_dcrt(B, T, n, qs, 7)
    b = O.uniform_dcrt(B, T, n, qs, 8)
    want_pipe, want_inv = O.ntt_mul_intt(a, b, tb), O.ntt_inv(a, tb)
    for split in (H.SPLIT_AUTO, H.SPLIT_COLS):
        plan = H.NTTPlan(ctx, log_n, qs, rs, split=split)
        xa, xb = dev(a), dev(b)
        xc = torch.empty_like(xa)
        plan.ntt_mul_intt(xa.data_ptr(), xb.data_ptr(), xc.data_ptr(), B, stream())
        xi = dev(a)
        plan.inverse(xi.data_ptr(), B, stream())
        assert np.array_equal(host(xc), want_pipe), split
        assert np.array_equal(host(xi), want_inv), split


def test_stream_ordered_alloc_and_zero(hip):
    """ofhe_hip_alloc_async / free_async / zero on a caller stream."""
    import torch

    H, ctx = hip
    s = torch.cuda.Stream()
    n = 1 << 20
    with torch.cuda.stream(s):
        p = ctx.alloc_async(n * 8, s.cuda_stream)
        src = torch.arange(n, dtype=torch.int64, device="cuda")
        ctx.copy_device(p, src.data_ptr(), n * 8, s.cuda_stream)
        ctx.zero(p, n * 4, s.cuda_stream)  # first half
        out = torch.empty(n, dtype=torch.int64, device="cuda")
        ctx.copy_device(out.data_ptr(), p, n * 8, s.cuda_stream)
        ctx.free_async(p, s.cuda_stream)
    s.synchronize()
    h = out.cpu().numpy()
    assert not h[: n // 2].any() and np.array_equal(h[n // 2:], np.arange(n // 2, n))


def test_chunked_pipeline_matches(hip, O):
    """ofhe_hip_plan_tune chunking (opt-in A/B settings): chunks of 3 and 4
    polynomials (a ragged last chunk) on one and two streams, out of place and
    in place, against the oracle's pipeline."""
    import torch

    H, ctx = hip
    log_n, T, B = 16, 3, 7
    n = 1 << log_n
    qs, rs = O.moduli_chain(log_n, T)
    plan = H.NTTPlan(ctx, log_n, qs, rs)
    a = O.uniform_dcrt(B, T, n, qs, 71)
    b = O.uniform_dcrt(B, T, n, qs, 72)
    want = O.ntt_mul_intt(a, b, O.Tables(n, qs, rs))
    for cb, ns in ((3, 1), (4, 2), (3, 2)):
        plan.tune(cb, ns)
        xa, xb = dev(a), dev(b)
        xc = torch.empty_like(xa)
        plan.ntt_mul_intt(xa.data_ptr(), xb.data_ptr(), xc.data_ptr(), B, stream())
        assert np.array_equal(host(xc), want), (cb, ns)
        plan.ntt_mul_intt(xa.data_ptr(), xb.data_ptr(), xa.data_ptr(), B, stream())
        assert np.array_equal(host(xa), want), ("in place", cb, ns)
    plan.tune(0, 1)
