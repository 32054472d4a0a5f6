"""GPU parity of the persistent one-launch pipeline (k_pipe, pipe_kernels.hpp;
ofhe_hip_plan_pipeline): c = INTT(NTT(a) (.) b) -- DCRTPoly SwitchFormat ->
Times -> SwitchFormat, dcrtpoly-impl.h:2518-2524, dcrtpoly.h:185-200 -- against
the oracle at small shapes (fewer towers than XCD queues, ragged queue loads,
lags 1..7, in place, generic moduli) and against the three-launch pipeline
over configs[2]'s whole batch of 1024, with no given-up waits."""
import numpy as np
import pytest

import oracle as O
from test_gpu_parity import dev, host, stream

pytestmark = pytest.mark.gpu


# knob settings read by ofhe_hip_plan_pipeline: hand-off by acquire + plain
# loads or by sc1 loads; dynamic queue or static item assignment; pieces per item
CFGS = {
    "acq": {"OFHE_PIPE_HM": "0"},
    "sc1": {"OFHE_PIPE_HM": "1"},
    "static_p4_nt": {"OFHE_PIPE_HM": "2", "OFHE_PIPE_STATIC": "1", "OFHE_PIPE_PIECES": "4"},
    "dyn_p2_acq_nt": {"OFHE_PIPE_HM": "3", "OFHE_PIPE_PIECES": "2"},
}


def _cfg(monkeypatch, name):
    for k in ("OFHE_PIPE_HM", "OFHE_PIPE_STATIC", "OFHE_PIPE_PIECES"):
        monkeypatch.delenv(k, raising=False)
    for k, v in CFGS[name].items():
        monkeypatch.setenv(k, v)


@pytest.mark.parametrize("cfg", sorted(CFGS))
@pytest.mark.parametrize("T,B", [(1, 1), (1, 5), (3, 7), (16, 2), (5, 13)])
def test_pipe_vs_oracle(hip, T, B, cfg, monkeypatch):
    """Every knob setting of the persistent pipeline against the oracle."""
    import torch

    H, ctx = hip
    _cfg(monkeypatch, cfg)
    log_n = 16
    n = 1 << log_n
    qs, rs = O.moduli_chain(log_n, T)
    plan = H.NTTPlan(ctx, log_n, qs, rs)
    a = O.uniform_dcrt(B, T, n, qs, 100 + T)
    b = O.uniform_dcrt(B, T, n, qs, 200 + B)
    want = O.ntt_mul_intt(a, b, O.Tables(n, qs, rs))
    for lag in (1, 4, 7):
        plan.pipeline(True, lag)
        xa, xb = dev(a), dev(b)
        xc = torch.empty_like(xa)
        plan.ntt_mul_intt(xa.data_ptr(), xb.data_ptr(), xc.data_ptr(), B, stream())
        got = host(xc)
        bad = np.argwhere(got != want)
        assert bad.size == 0, (lag, len(bad), bad[:5].tolist())
        # in place (c = a)
        plan.ntt_mul_intt(xa.data_ptr(), xb.data_ptr(), xa.data_ptr(), B, stream())
        assert np.array_equal(host(xa), want), ("in place", lag)
    assert plan.pipeline_status() == (True, 0)
    plan.pipeline(False)
    assert plan.pipeline_status()[0] is False
    plan.close()


def test_pipe_edge_values_generic_moduli(hip, monkeypatch):
    """Residues q - 1, 0, 1 and the generic-modulus kernel (OFHE_NO_SPQ)."""
    import torch

    H, ctx = hip
    log_n, T, B = 16, 2, 3
    n = 1 << log_n
    qs, rs = O.moduli_chain(log_n, T)
    monkeypatch.setenv("OFHE_NO_SPQ", "1")
    plan = H.NTTPlan(ctx, log_n, qs, rs)
    monkeypatch.delenv("OFHE_NO_SPQ")
    a = O.uniform_dcrt(B, T, n, qs, 5)
    b = O.uniform_dcrt(B, T, n, qs, 6)
    for t, q in enumerate(qs):
        a[0, t, : n // 2] = q - 1
        b[0, t, n // 2 :] = q - 1
        a[1, t, ::3] = 0
        b[2, t, ::5] = 1
    want = O.ntt_mul_intt(a, b, O.Tables(n, qs, rs))
    plan.pipeline(True)
    xa, xb = dev(a), dev(b)
    xc = torch.empty_like(xa)
    plan.ntt_mul_intt(xa.data_ptr(), xb.data_ptr(), xc.data_ptr(), B, stream())
    assert np.array_equal(host(xc), want)
    assert plan.pipeline_status() == (True, 0)
    plan.close()


@pytest.mark.parametrize("cfg", sorted(CFGS))
def test_pipe_full_batch_matches_three_launches(hip, cfg, monkeypatch):
    """configs[2] (N = 2^16, 16 towers, batch 1024, 8 GiB per operand): the
    persistent pipeline's c equals the three-launch pipeline's, every word, and
    sampled rows equal the oracle."""
    import torch

    H, ctx = hip
    _cfg(monkeypatch, cfg)
    log_n, T, B = 16, 16, 1024
    n = 1 << log_n
    qs, rs = O.moduli_chain(log_n, T)
    plan = H.NTTPlan(ctx, log_n, qs, rs)
    sp = stream()
    a = torch.empty((B, T, n), dtype=torch.int64, device="cuda")
    b = torch.empty_like(a)
    plan.fill_uniform(a.data_ptr(), B, 1, 0, sp)
    plan.fill_uniform(b.data_ptr(), B, 2, 0, sp)
    c3 = torch.empty_like(a)
    plan.ntt_mul_intt(a.data_ptr(), b.data_ptr(), c3.data_ptr(), B, sp)
    plan.pipeline(True)
    cp = torch.empty_like(a)
    plan.ntt_mul_intt(a.data_ptr(), b.data_ptr(), cp.data_ptr(), B, sp)
    torch.cuda.synchronize()
    assert torch.equal(cp, c3)
    for bi, ti in ((0, 0), (1023, 15), (517, 8)):
        aa = a[bi, ti].cpu().numpy().view(np.uint64).reshape(1, 1, n)
        bb = b[bi, ti].cpu().numpy().view(np.uint64).reshape(1, 1, n)
        want = O.ntt_mul_intt(aa, bb, O.Tables(n, [qs[ti]], [rs[ti]]))
        assert np.array_equal(cp[bi, ti].cpu().numpy().view(np.uint64), want.reshape(-1)), (bi, ti)
    assert plan.pipeline_status() == (True, 0)
    del a, b, c3, cp
    plan.close()
    torch.cuda.empty_cache()


def test_pipe_refused_where_it_does_not_apply(hip):
    H, ctx = hip
    log_n, T = 14, 2
    qs, rs = O.moduli_chain(log_n, T)
    plan = H.NTTPlan(ctx, log_n, qs, rs)
    with pytest.raises(H.MathError):
        plan.pipeline(True)
    plan.pipeline(False)  # always allowed
    assert plan.pipeline_status() == (False, 0)
    plan.close()
