"""CPU restatement of ApproxModUp / ApproxModDown, HYBRID key switching,
SwitchModulus and AutomorphismTransform (numpy on top of the C oracle).

TEST INFRASTRUCTURE ONLY: imported by tests/, never by the product path.

Each function follows the reference loop structure step by step and cites it
(paths relative to the reference root).  The CRT tables are computed as the
reference computes them -- BigInteger quotients such as Q/q_i and modular
inverses of those -- here with Python's exact integers
(CryptoParametersRNS::PrecomputeCRTTables, pke/lib/schemerns/
rns-cryptoparameters.cpp:72-345).  The product path derives the same residues
from products of the moduli (csrc/keyswitch.hip), so this is an independent
computation of every table entry.
"""
from __future__ import annotations

import math
from functools import lru_cache

import numpy as np

import oracle as O

U = O.U


def _prod(xs):
    r = 1
    for x in xs:
        r *= int(x)
    return r


@lru_cache(maxsize=None)
def _tables(n: int, moduli: tuple, roots: tuple) -> O.Tables:
    return O.Tables(n, list(moduli), list(roots))


def set_format(x: np.ndarray, moduli, roots, to_eval: bool) -> np.ndarray:
    """DCRTPolyImpl::SetFormat over towers (dcrtpoly-impl.h:2518-2524): x [B][T][N]."""
    x = np.ascontiguousarray(x, dtype=np.uint64)
    tb = _tables(x.shape[2], tuple(int(m) for m in moduli), tuple(int(r) for r in roots))
    return O.ntt_fwd(x, tb) if to_eval else O.ntt_inv(x, tb)


def _switch_basis(x: np.ndarray, q, p, qhinv, qhmodp) -> np.ndarray:
    """ApproxSwitchCRTBasis (dcrtpoly-impl.h:1034-1063) on every batch entry,
    with tables given as Python ints: qhinv[i], qhmodp[i][j]."""
    sq, sp = len(q), len(p)
    pre = dict(
        qhinv=U([int(v) for v in qhinv]),
        qhinv_pre=U([(int(v) << 64) // int(q[i]) for i, v in enumerate(qhinv)]),
        qhmodp=U([int(qhmodp[i][j]) for i in range(sq) for j in range(sp)]),
        mu_lo=U([((1 << 128) // int(pj)) & ((1 << 64) - 1) for pj in p]),
        mu_hi=U([((1 << 128) // int(pj)) >> 64 for pj in p]),
    )
    out = np.empty((x.shape[0], sp, x.shape[2]), np.uint64)
    for b in range(x.shape[0]):
        out[b] = O.approx_switch_crt_basis(x[b], q, p, pre)
    return out


def switch_tables(q, p):
    """QHatInvModq / QHatModp as rns-cryptoparameters.cpp:235-271 builds them."""
    Q = _prod(q)
    qhat = [Q // int(qi) for qi in q]
    qhinv = [pow(qh % int(qi), -1, int(qi)) for qh, qi in zip(qhat, q)]
    qhmodp = [[qh % int(pj) for pj in p] for qh in qhat]
    return qhinv, qhmodp


def _scale(x: np.ndarray, scalars, moduli) -> np.ndarray:
    return O.mul_scalar(x, [int(s) % int(m) for s, m in zip(scalars, moduli)], moduli)


# ---------------------------------------------------------------------------
# Element maps
# ---------------------------------------------------------------------------
def switch_modulus(v: np.ndarray, om: int, nm: int) -> np.ndarray:
    """NativeVectorT::SwitchModulus, mubintvecnat.cpp:111-136."""
    v = np.asarray(v, dtype=np.uint64).copy()
    half = om >> 1
    if nm > om:
        diff = np.uint64(nm - om)
        m = v > np.uint64(half)
        v[m] += diff
    else:
        diff = np.uint64(nm - (om % nm))
        m = v > np.uint64(half)
        v[m] += diff
        big = v >= np.uint64(nm)
        v[big] %= np.uint64(nm)
    return v


def _rev(x: int, bits: int) -> int:
    return int(format(x, f"0{bits}b")[::-1], 2) if bits else 0


def automorphism(x: np.ndarray, k: int, eval_form: bool, q: int) -> np.ndarray:
    """PolyImpl::AutomorphismTransform(k), poly-impl.h:312-365, one tower of n."""
    n = x.shape[-1]
    logn = n.bit_length() - 1
    mask = n - 1
    if k % 2 == 0:
        raise ValueError("Automorphism index not odd")
    out = np.zeros_like(x)
    if eval_form:
        jk = k
        for j in range(n):
            jrev = _rev(j, logn)
            idxrev = _rev(((jk & 0xFFFFFFFF) >> 1) & mask, logn)
            out[..., jrev] = x[..., idxrev]
            jk += 2 * k
        return out
    jk = 0
    for j in range(n):
        v = x[..., j]
        neg = ((jk & 0xFFFFFFFF) >> logn) & 1
        out[..., jk & mask] = (np.uint64(q) - v) if neg else v
        jk += k
    return out


# ---------------------------------------------------------------------------
# ApproxModUp / ApproxModDown
# ---------------------------------------------------------------------------
def approx_mod_up(x, q, rq, p, rp, eval_form: bool) -> np.ndarray:
    """DCRTPolyImpl::ApproxModUp, dcrtpoly-impl.h:1085-1131.  x [B][Q][N] ->
    [B][Q+P][N] evaluation form."""
    x = np.ascontiguousarray(x, dtype=np.uint64)
    saved = x if eval_form else None
    coeff = set_format(x, q, rq, False) if eval_form else x
    qhinv, qhmodp = switch_tables(q, p)
    part_p = _switch_basis(coeff, q, p, qhinv, qhmodp)
    part_p = set_format(part_p, p, rp, True)
    part_q = saved if saved is not None else set_format(x, q, rq, True)
    return np.concatenate([part_q, part_p], axis=1)


def moddown_tables(q, p, t: int = 0):
    P = _prod(p)
    pinv_modq = [pow(P % int(qi), -1, int(qi)) for qi in q]
    phat = [P // int(pj) for pj in p]
    phinv = [pow(ph % int(pj), -1, int(pj)) for ph, pj in zip(phat, p)]
    phmodq = [[ph % int(qi) for qi in q] for ph in phat]
    tinv_modp = [pow(t % int(pj), -1, int(pj)) for pj in p] if t else None
    return dict(pinv_modq=pinv_modq, phinv=phinv, phmodq=phmodq, tinv_modp=tinv_modp)


def approx_mod_down(x, q, rq, p, rp, t: int = 0, tables=None) -> np.ndarray:
    """DCRTPolyImpl::ApproxModDown, dcrtpoly-impl.h:1134-1175.  x [B][Q+P][N]
    evaluation form -> [B][Q][N] evaluation form."""
    x = np.ascontiguousarray(x, dtype=np.uint64)
    sq = len(q)
    T = tables or moddown_tables(q, p, t)
    part_p = set_format(x[:, sq:], p, rp, False)
    if t > 0:
        part_p = _scale(part_p, T["tinv_modp"], p)
    switched = _switch_basis(part_p, p, q, T["phinv"], T["phmodq"])
    if t > 0:
        switched = _scale(switched, [t] * sq, q)
    switched = set_format(switched, q, rq, True)
    diff = O.eltwise("sub", x[:, :sq].copy(), switched, q)
    return _scale(diff, T["pinv_modq"], q)


# ---------------------------------------------------------------------------
# HYBRID key switching (pke/lib/keyswitch/keyswitch-hybrid.cpp)
# ---------------------------------------------------------------------------
class KeySwitchParams:
    """The HYBRID part of CryptoParametersRNS::PrecomputeCRTTables
    (rns-cryptoparameters.cpp:72-345) for given Q, P and dnum."""

    def __init__(self, n, q, rq, p, rp, num_part_q):
        self.n = n
        self.q, self.rq = [int(v) for v in q], [int(v) for v in rq]
        self.p, self.rp = [int(v) for v in p], [int(v) for v in rp]
        sq = len(q)
        self.num_part_q = num_part_q
        self.alpha = math.ceil(sq / num_part_q)
        if sq - self.alpha * (num_part_q - 1) <= 0:
            raise ValueError("can't distribute towers into digits")

    def beta(self, size_ql):
        # keyswitch-hybrid.cpp:341-345
        return min(math.ceil(size_ql / self.alpha), self.num_part_q)

    def digit(self, size_ql, j):
        st = self.alpha * j
        return st, min(self.alpha, size_ql - st)

    def complement(self, size_ql, j):
        """m_paramsComplPartQ[l][j] (rns-cryptoparameters.cpp:238-287): the Ql
        towers outside digit j, in order, then P."""
        st, n = self.digit(size_ql, j)
        idx = [i for i in range(size_ql) if i < st or i >= st + n]
        return ([self.q[i] for i in idx] + self.p, [self.rq[i] for i in idx] + self.rp)

    def part_tables(self, size_ql, j):
        """m_PartQlHatInvModq[j][n-1] and m_PartQlHatModp[l][j] (289-341)."""
        st, n = self.digit(size_ql, j)
        dq = self.q[st:st + n]
        part_q = _prod(dq)
        cm, _ = self.complement(size_ql, j)
        hinv = [pow((part_q // qi) % qi, -1, qi) for qi in dq]
        hmod = [[(part_q // qi) % c for c in cm] for qi in dq]
        return hinv, hmod


def ks_precompute(kp: KeySwitchParams, c: np.ndarray) -> np.ndarray:
    """EvalKeySwitchPrecomputeCore, keyswitch-hybrid.cpp:330-412.
    c [B][Ql][N] evaluation form -> [B][beta][Ql+P][N]."""
    c = np.ascontiguousarray(c, dtype=np.uint64)
    B, l, n = c.shape
    beta = kp.beta(l)
    out = np.empty((B, beta, l + len(kp.p), n), np.uint64)
    for j in range(beta):
        st, cnt = kp.digit(l, j)
        dq, dr = kp.q[st:st + cnt], kp.rq[st:st + cnt]
        part = c[:, st:st + cnt]
        coeff = set_format(part, dq, dr, False)                       # 384-385
        cm, cr = kp.complement(l, j)
        hinv, hmod = kp.part_tables(l, j)
        compl = _switch_basis(coeff, dq, cm, hinv, hmod)             # 388-394
        compl = set_format(compl, cm, cr, True)
        ext = out[:, j]
        ext[:, :st] = compl[:, :st]                                   # 400-409
        ext[:, st:st + cnt] = part
        ext[:, st + cnt:] = compl[:, st:]
    return out


def ks_key_index(kp: KeySwitchParams, size_ql: int):
    """Tower of the QP key used for tower i of Ql|P (keyswitch-hybrid.cpp:459-476)."""
    sq = len(kp.q)
    return list(range(size_ql)) + [sq + k for k in range(len(kp.p))]


def ks_fast_core_ext(kp: KeySwitchParams, digits: np.ndarray, key_b: np.ndarray, key_a: np.ndarray):
    """EvalFastKeySwitchCoreExt, keyswitch-hybrid.cpp:438-482.  key_*:
    [num_part_q][Q+P][N].  Returns ct0, ct1: [B][Ql+P][N]."""
    B, beta, lp, n = digits.shape
    l = lp - len(kp.p)
    moduli = kp.q[:l] + kp.p
    kidx = ks_key_index(kp, l)
    ct0 = np.zeros((B, lp, n), np.uint64)
    ct1 = np.zeros((B, lp, n), np.uint64)
    for j in range(beta):
        bj = np.ascontiguousarray(np.broadcast_to(key_b[j][kidx], (B, lp, n)))
        aj = np.ascontiguousarray(np.broadcast_to(key_a[j][kidx], (B, lp, n)))
        cj = np.ascontiguousarray(digits[:, j])
        ct0 = O.eltwise("add", ct0, O.eltwise("mul", cj, bj, moduli), moduli)
        ct1 = O.eltwise("add", ct1, O.eltwise("mul", cj, aj, moduli), moduli)
    return ct0, ct1


def ks_mod_down(kp: KeySwitchParams, x: np.ndarray, t: int = 0) -> np.ndarray:
    """ApproxModDown with paramsQl and the P tables (keyswitch-hybrid.cpp:423-435)."""
    l = x.shape[1] - len(kp.p)
    return approx_mod_down(x, kp.q[:l], kp.rq[:l], kp.p, kp.rp, t)


def ks_core(kp: KeySwitchParams, c, key_b, key_a, t: int = 0):
    """KeySwitchCore (keyswitch-hybrid.cpp:325-328)."""
    d = ks_precompute(kp, c)
    ct0, ct1 = ks_fast_core_ext(kp, d, key_b, key_a)
    return ks_mod_down(kp, ct0, t), ks_mod_down(kp, ct1, t)


# ---------------------------------------------------------------------------
# Key generation for semantic tests: KeySwitchGenInternal,
# keyswitch-hybrid.cpp:53-128 (uniform a, small error e, P*s_old on the digit).
# ---------------------------------------------------------------------------
def ternary(n, rng):
    return rng.integers(-1, 2, size=n)


def small_poly_eval(coeffs, moduli, roots):
    """signed small coefficients -> [1][T][N] evaluation form."""
    n = len(coeffs)
    c = np.asarray(coeffs, dtype=np.int64)  # |coeffs| small; every modulus < 2^60 fits int64
    x = np.empty((1, len(moduli), n), np.uint64)
    for t, m in enumerate(moduli):
        x[0, t] = (c % np.int64(int(m))).astype(np.uint64)  # numpy %: the divisor's sign, as Python's
    return set_format(x, moduli, roots, True)


def keyswitch_gen(kp: KeySwitchParams, s_old, s_new, rng, err_bound=3):
    qp, rqp = kp.q + kp.p, kp.rq + kp.rp
    n = kp.n
    so = small_poly_eval(s_old, kp.q, kp.rq)[0]
    sn = small_poly_eval(s_new, qp, rqp)[0]
    P = _prod(kp.p)
    sq = len(kp.q)
    kb = np.empty((kp.num_part_q, sq + len(kp.p), n), np.uint64)
    ka = np.empty_like(kb)
    for part in range(kp.num_part_q):
        a = np.stack([rng.integers(0, m, size=n, dtype=np.uint64) for m in qp])
        e = small_poly_eval(rng.integers(-err_bound, err_bound + 1, size=n), qp, rqp)[0]
        st = kp.alpha * part
        en = min(st + kp.alpha, sq)
        for i, m in enumerate(qp):
            mm = [m]
            v = O.eltwise("mul", a[i][None, None], sn[i][None, None], mm)[0, 0]
            v = O.eltwise("sub", np.zeros((1, 1, n), np.uint64), v[None, None], mm)[0, 0]
            if st <= i < en:
                ps = O.mul_scalar(so[i][None, None], [P % m], mm)[0, 0]
                v = O.eltwise("add", v[None, None], ps[None, None], mm)[0, 0]
            v = O.eltwise("add", v[None, None], e[i][None, None], mm)[0, 0]
            kb[part, i] = v
            ka[part, i] = a[i]
    return kb, ka


def crt_centered(x_coeff: np.ndarray, moduli):
    """[T][N] residues -> list of centred big integers."""
    M = _prod(moduli)
    out = []
    for c in range(x_coeff.shape[1]):
        v = 0
        for t, m in enumerate(moduli):
            m = int(m)
            Mi = M // m
            v += int(x_coeff[t, c]) * Mi * pow(Mi % m, -1, m)
        v %= M
        out.append(v - M if v > M // 2 else v)
    return out


# ---------------------------------------------------------------------------
# Rescaling: the callers that drop the last tower
# ---------------------------------------------------------------------------
def rescale_tables(q):
    """QlQlInvModqlDivqlModq / qlInvModq for dropping the last of the towers q,
    as ckksrns-cryptoparameters.cpp:65-86 (and bfvrns-cryptoparameters.cpp:
    639-657) build them: Ql = prod(q[:-1]); result = (Ql^-1 mod ql) Ql / ql."""
    ql, Ql = int(q[-1]), _prod(q[:-1])
    result = (pow(Ql % ql, -1, ql) * Ql) // ql
    return [result % int(qi) for qi in q[:-1]], [pow(ql, -1, int(qi)) for qi in q[:-1]]


def drop_last_and_scale(x: np.ndarray, q, rq, eval_form: bool, c, a) -> np.ndarray:
    """DCRTPolyImpl::DropLastElementAndScale, dcrtpoly-impl.h:746-768, on every
    batch entry: x [B][L+1][N] -> [B][L][N]."""
    L = len(q) - 1
    x = np.ascontiguousarray(x, dtype=np.uint64)
    last = x[:, L:L + 1]
    if eval_form:  # lastPoly.SetFormat(Format::COEFFICIENT)
        last = set_format(last, [q[L]], [rq[L]], False)
    out = np.empty((x.shape[0], L, x.shape[2]), np.uint64)
    for i in range(L):
        qi = int(q[i])
        tmp = switch_modulus(last[:, 0], int(q[L]), qi)[:, None]     # tmp.SwitchModulus
        tmp = _scale(tmp, [c[i]], [qi])                             # tmp *= QlQlInvModqlDivqlModq[i]
        if eval_form:
            tmp = set_format(tmp, [qi], [rq[i]], True)              # tmp.SwitchFormat()
        m = _scale(x[:, i:i + 1], [a[i]], [qi])                     # m_vectors[i] *= qlInvModq[i]
        m = O.eltwise("add", m, tmp, [qi])                          # m_vectors[i] += tmp
        if not eval_form:
            m = set_format(m, [qi], [rq[i]], True)                  # m_vectors[i].SwitchFormat()
        out[:, i:i + 1] = m
    return out


def mod_reduce(x: np.ndarray, q, rq, eval_form: bool, t: int, neg_t_inv_modq: int, a) -> np.ndarray:
    """DCRTPolyImpl::ModReduce, dcrtpoly-impl.h:792-812: x [B][L+1][N] -> [B][L][N]."""
    L = len(q) - 1
    x = np.ascontiguousarray(x, dtype=np.uint64)
    delta = x[:, L:L + 1]
    if eval_form:  # delta.SetFormat(Format::COEFFICIENT)
        delta = set_format(delta, [q[L]], [rq[L]], False)
    delta = _scale(delta, [neg_t_inv_modq], [q[L]])                 # delta *= negtInvModq
    out = np.empty((x.shape[0], L, x.shape[2]), np.uint64)
    for i in range(L):
        qi = int(q[i])
        tmp = switch_modulus(delta[:, 0], int(q[L]), qi)[:, None]    # tmp.SwitchModulus
        if eval_form:
            tmp = set_format(tmp, [qi], [rq[i]], True)              # tmp.SwitchFormat()
        tmp = _scale(tmp, [t], [qi])                                # tmp *= t
        m = O.eltwise("add", np.ascontiguousarray(x[:, i:i + 1]), tmp, [qi])  # m_vectors[i] += tmp
        out[:, i:i + 1] = _scale(m, [a[i]], [qi])                   # m_vectors[i] *= qlInvModq[i]
    return out


# ---------------------------------------------------------------------------
# BV key switching, digitSize = 0
# ---------------------------------------------------------------------------
def crt_decompose0(c: np.ndarray, q, rq) -> np.ndarray:
    """DCRTPolyImpl::CRTDecompose(0), dcrtpoly-impl.h:266-288, for c [B][T][N]
    in evaluation form: digit i = a copy of c (evaluation form) whose towers
    k != i are tower i of the coefficient form, SwitchModulus'd to q_k and
    transformed.  -> [B][T (digit)][T][N]."""
    B, T, n = c.shape
    coef = set_format(c, q, rq, False)                       # cp.SwitchFormat()
    out = np.empty((B, T, T, n), np.uint64)
    for i in range(T):
        out[:, i] = c                                        # result[i] = *eval
        for k in range(T):
            if k != i:
                tmp = switch_modulus(coef[:, i], int(q[i]), int(q[k]))[:, None]
                out[:, i, k:k + 1] = set_format(tmp, [q[k]], [rq[k]], True)
    return out


def bv_fast_core(digits: np.ndarray, kb: np.ndarray, ka: np.ndarray, q):
    """KeySwitchBV::EvalFastKeySwitchCore, keyswitch-bv.cpp:314-340: keys
    [T][Tk][N] (the first T towers used, DropLastElements); digits [B][T][T][N]."""
    B, T = digits.shape[0], digits.shape[1]
    out0 = np.empty((B, T, digits.shape[3]), np.uint64)
    out1 = np.empty_like(out0)
    for b in range(B):
        ct1 = O.eltwise("mul", ka[0:1, :T], digits[b, 0:1], q)            # av[0] *= digits[0]
        ct0 = O.eltwise("mul", kb[0:1, :T], digits[b, 0:1], q)            # bv[0] *= digits[0]
        for i in range(1, T):
            ct0 = O.eltwise("add", ct0, O.eltwise("mul", kb[i:i + 1, :T], digits[b, i:i + 1], q), q)
            ct1 = O.eltwise("add", ct1, O.eltwise("mul", ka[i:i + 1, :T], digits[b, i:i + 1], q), q)
        out0[b], out1[b] = ct0[0], ct1[0]
    return out0, out1


def bv_keygen(q, rq, s_old, s_new, rng, err_bound=3):
    """KeySwitchBV::KeySwitchGenInternal with digitSize = 0 (keyswitch-bv.cpp:
    99-111): bv[i] = filtered_i - (a_i s_new + e_i), filtered_i = s_old in tower
    i only; s_old, s_new in evaluation form [T][N].  Returns (kb, ka, e) with the
    errors e [T][T][N] in evaluation form (noise scale 1)."""
    T, n = len(q), s_old.shape[1]
    kb = np.empty((T, T, n), np.uint64)
    ka = np.empty_like(kb)
    es = np.empty_like(kb)
    for i in range(T):
        a = np.stack([rng.integers(0, int(qk), size=n, dtype=np.uint64) for qk in q])
        e = small_poly_eval(rng.integers(-err_bound, err_bound + 1, size=n), q, rq)[0]
        filt = np.zeros((T, n), np.uint64)
        filt[i] = s_old[i]
        ase = O.eltwise("add", O.eltwise("mul", a[None], s_new[None], q), e[None], q)
        kb[i] = O.eltwise("sub", filt[None], ase, q)[0]
        ka[i] = a
        es[i] = e
    return kb, ka, es
