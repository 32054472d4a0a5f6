"""CPU tests: the oracle (oracle/ofhe_oracle.c) against the reference's own
known-answer tests and recorded reference outputs, plus algebraic properties.
These pin the checker the GPU parity tests rely on."""
import numpy as np
import pytest
from conftest import load_golden

REF = load_golden("reference_fixtures.json")


def test_kat_transform(O):
    """UnitTestTransform.cpp:60-94 CRT_polynomial_mult."""
    k = REF["kat_transform"]
    q = k["q"]
    assert O.root_of_unity(k["m"], q) == k["root"]
    tb = O.Tables(k["m"] // 2, [q], [k["root"]])
    a = O.U(k["a"]).reshape(1, 1, -1)
    A = O.ntt_fwd(a, tb)
    AB = O.eltwise("mul", A, A, [q])
    assert O.ntt_inv(AB, tb).reshape(-1).tolist() == k["expected"]


def test_forward_is_evaluation_at_odd_powers(O):
    """The identity tests/test_gpu_definition.py checks the GPU against at
    full size: the forward transform leaves a(psi^(2 rev(i) + 1)) at slot i.
    On the reference's own KAT (UnitTestTransform.cpp:60-94, N = 4, q = 113)
    and on the oracle at N = 2^5 .. 2^10 (the oracle pinned by that KAT), with
    exact Python integers."""
    import random

    def rev(x, bits):
        return int(format(x, f"0{bits}b")[::-1], 2) if bits else 0

    def evaluate(a, x, q):
        v = 0
        for c in reversed(a):
            v = (v * x + c) % q
        return v

    k = REF["kat_transform"]
    q, psi, n = k["q"], k["root"], k["m"] // 2
    A = O.ntt_fwd(O.U(k["a"]).reshape(1, 1, -1), O.Tables(n, [q], [psi])).reshape(-1)
    assert [evaluate(k["a"], pow(psi, 2 * rev(i, 2) + 1, q), q) for i in range(n)] == [int(v) for v in A]
    rng = random.Random(3)
    for log_n in (5, 7, 10):
        n = 1 << log_n
        qs, rs = O.moduli_chain(log_n, 1)
        a = [rng.randrange(qs[0]) for _ in range(n)]
        y = O.ntt_fwd(O.U(a).reshape(1, 1, -1), O.Tables(n, qs, rs)).reshape(-1)
        for i in range(0, n, max(1, n // 64)):
            assert int(y[i]) == evaluate(a, pow(rs[0], 2 * rev(i, log_n) + 1, qs[0]), qs[0])


def test_kat_mubintvec(O):
    """UnitTestMubintvec.cpp:276-359 basic_vector_vector_mod_math_1_limb."""
    k = REF["kat_mubintvec"]
    a = O.U(k["a"]).reshape(1, 1, -1)
    b = O.U(k["b"]).reshape(1, 1, -1)
    for op in ("add", "sub", "mul"):
        assert O.eltwise(op, a, b, [k["q"]]).reshape(-1).tolist() == k["mod" + op]


def test_kat_mubintvec_2limb(O):
    """UnitTestMubintvec.cpp:402-484 basic_vector_vector_mod_math_2_limb (q < 2^52)."""
    k = REF["kat_mubintvec_2limb"]
    a = O.U(k["a"]).reshape(1, 1, -1)
    b = O.U(k["b"]).reshape(1, 1, -1)
    for op in ("add", "sub", "mul"):
        assert O.eltwise(op, a, b, [k["q"]]).reshape(-1).tolist() == k["mod" + op]


@pytest.mark.parametrize("bits,towers", [(22, 1), (28, 2)])
def test_ntt_roundtrip_reference_inputs(O, bits, towers):
    """UnitTestNTT.cpp:53-133: SwitchFormat twice is the identity."""
    k = REF["roundtrip_ntt"]
    m = k["m"]
    q = O.first_prime(bits, m)
    qs = [q]
    for _ in range(towers - 1):
        qs.append(O.next_prime(qs[-1], m))
    rs = [O.root_of_unity(m, x) for x in qs]
    tb = O.Tables(m // 2, qs, rs)
    for key in ("x1", "x2"):
        x = np.stack([O.U(k[key]) % np.uint64(q) for q in qs])[None]
        assert np.array_equal(O.ntt_inv(O.ntt_fwd(x, tb), tb), x)


def test_survey_probe_ntt(O):
    """Reference outputs recorded in SURVEY.md §8(c): modulus chain, minimal
    root, and forward NTT samples for N = 2^14 and 2^16."""
    for pr in REF["survey_probes"]["ntt"]:
        qs, rs = O.moduli_chain(pr["log_n"], pr["tower"] + 1)
        assert qs[pr["tower"]] == pr["q"]
        assert rs[pr["tower"]] == pr["psi"]
        if "y0" not in pr:
            continue
        n = 1 << pr["log_n"]
        x = O.splitmix_fill(n, pr["q"], O.U([pr["seed"]]))
        y = O.ntt_fwd(x.reshape(1, 1, -1), O.Tables(n, [pr["q"]], [pr["psi"]])).reshape(-1)
        assert int(y[0]) == pr["y0"]
        if "y1" in pr:
            assert int(y[1]) == pr["y1"]


def test_survey_probe_dcrt_pipeline(O):
    """DCRTPoly N=2^14, T=8, c = INTT(NTT(a) (.) b), c[0][0]."""
    pr = REF["survey_probes"]["dcrt_pipeline"]
    n, T = 1 << pr["log_n"], pr["towers"]
    qs, rs = O.moduli_chain(pr["log_n"], T)
    st = O.U([pr["seed"]])
    a = np.zeros((T, n), np.uint64)
    b = np.zeros((T, n), np.uint64)
    for t in range(T):  # interleaved draws per coefficient, tower-major
        ab = O.splitmix_fill(2 * n, qs[t], st)
        # the stream draws a then b for every i: re-draw with the true modulus each time
        a[t] = ab[0::2]
        b[t] = ab[1::2]
    c = O.ntt_mul_intt(a[None], b[None], O.Tables(n, qs, rs))
    assert int(c[0, 0, 0]) == pr["c00"]


def test_barrett_and_shoup_exact(O):
    """ModMulFastEq (Barrett) and ModMulFastConst (Shoup) return the exact
    canonical residue (so bit-exact parity = mathematical correctness)."""
    L = O.lib()
    rng = np.random.default_rng(7)
    for q in [113, 163841, O.moduli_chain(16, 1)[0][0], O.moduli_chain(14, 3)[0][2], (1 << 59) + 21]:
        mu = L.oracle_compute_mu(q)
        for _ in range(300):
            a, b = (int(v) % q for v in rng.integers(0, 2**63, 2, dtype=np.uint64))
            assert L.oracle_modmul_barrett(a, b, q, mu) == a * b % q
            assert L.oracle_modmul_shoup(a, b, q, L.oracle_shoup_prep(b, q)) == a * b % q
        # worst cases
        for a, b in ((q - 1, q - 1), (0, q - 1), (q - 1, 1)):
            assert L.oracle_modmul_barrett(a, b, q, mu) == a * b % q


def test_primes_and_roots(O):
    qs, rs = O.moduli_chain(16, 16)
    m = 1 << 17
    assert all(q < 2**60 and q % m == 1 for q in qs)
    assert qs == sorted(qs, reverse=True) and len(set(qs)) == 16
    for q, r in zip(qs, rs):
        assert pow(r, m // 2, q) == q - 1          # primitive 2N-th root
        # minimality: no smaller odd power of r is a primitive root smaller than r
        assert all(pow(r, k, q) >= r for k in range(3, 4001, 2))
    # FirstPrime(22,16) / NextPrime as in UnitTestNTT
    q = O.first_prime(22, 16)
    assert q > 2**22 and q % 16 == 1 and all(q % d for d in range(2, 2100))


def test_ntt_properties(O):
    """INTT(NTT(x)) = x; NTT-domain product = negacyclic convolution."""
    n = 64
    qs, rs = O.moduli_chain(6, 2)
    tb = O.Tables(n, qs, rs)
    a = O.uniform_dcrt(1, 2, n, qs, 3)
    b = O.uniform_dcrt(1, 2, n, qs, 4)
    assert np.array_equal(O.ntt_inv(O.ntt_fwd(a, tb), tb), a)
    c = O.ntt_inv(O.eltwise("mul", O.ntt_fwd(a, tb), O.ntt_fwd(b, tb), qs), tb)
    for t, q in enumerate(qs):
        A = [int(v) for v in a[0, t]]
        B = [int(v) for v in b[0, t]]
        ref = [0] * n
        for i in range(n):
            for j in range(n):
                k = i + j
                if k < n:
                    ref[k] = (ref[k] + A[i] * B[j]) % q
                else:
                    ref[k - n] = (ref[k - n] - A[i] * B[j]) % q
        assert [int(v) for v in c[0, t]] == ref


def test_base_conversion_exact(O):
    """ApproxSwitchCRTBasis = sum_i [x_i Qhat_i^-1]_{q_i} Qhat_i mod p_j (exact big-int check)."""
    chain, _ = O.moduli_chain(5, 7)
    q, p = chain[:4], chain[4:]
    pre = O.base_conv_precompute(q, p)
    x = O.uniform_dcrt(1, 4, 32, q, 9)[0]
    out = O.approx_switch_crt_basis(x, q, p, pre)
    Q = 1
    for v in q:
        Q *= v
    for ri in range(32):
        s = 0
        for i, qi in enumerate(q):
            Qh = Q // qi
            y = int(x[i, ri]) * pow(Qh, -1, qi) % qi
            s += y * Qh
        for j, pj in enumerate(p):
            assert int(out[j, ri]) == s % pj


def test_golden_vectors_regenerate(O):
    """The committed oracle vectors are reproduced by the current oracle."""
    g = load_golden("oracle_vectors.json")
    for c in g["cases"]:
        n, T, B = 1 << c["log_n"], c["towers"], c["batch"]
        tb = O.Tables(n, c["q"], c["psi"])
        a = O.U(c["a"]).reshape(B, T, n)
        b = O.U(c["b"]).reshape(B, T, n)
        assert O.ntt_fwd(a, tb).reshape(-1).tolist() == c["ntt_a"]
        assert O.ntt_mul_intt(a, b, tb).reshape(-1).tolist() == c["pipeline"]


def fast_expand_constants(q, r):
    """The BFVrns precomputations FastExpandCRTBasisPloverQ reads
    (bfvrns-cryptoparameters.cpp:501-523), with Python big integers:
    c_i = q_i - [R QHat_i^-1]_{q_i} (m_negRlQHatInvModq) and
    d_ij = q_i^-1 mod r_j (m_qInvModr); Q and R are the products of q and r."""
    Q = R = 1
    for v in q:
        Q *= v
    for v in r:
        R *= v
    c = [qi - R * pow(Q // qi, -1, qi) % qi for qi in q]
    d = [[pow(qi, -1, rj) for rj in r] for qi in q]
    return c, d


def test_kat_fast_expand_crt_basis(O):
    """UnitTestBFVrnsCRTOperations.cpp:290-376: the R_l towers of
    FastExpandCRTBasisPloverQ's answer are the base conversion of
    dcrtpoly-impl.h:1419-1441 -- y_i = [x_i c_i]_{q_i} (Shoup), the 128-bit sum
    of y_i d_ij, BarrettUint128ModUint64 -- i.e. ApproxSwitchCRTBasis with the
    caller's constants in place of QHatInv / QHatModp."""
    k = REF["kat_fast_expand_crt_basis"]
    q, r = k["q"], k["r"]
    c, d = fast_expand_constants(q, r)
    pre = O.base_conv_precompute(q, r)
    pre["qhinv"] = O.U(c)
    pre["qhinv_pre"] = O.U([(ci << 64) // qi for ci, qi in zip(c, q)])  # PrepModMulConst
    pre["qhmodp"] = O.U([v for row in d for v in row])
    out = O.approx_switch_crt_basis(O.U(k["x"]), q, r, pre)
    assert out.tolist() == k["expected_rl"]


def test_kat_common_elements(O):
    """UnitTestCommonElements.cpp: common_binary_ops (240-320: evaluation-form
    Plus / Minus / Times, and SwitchFormat -> Times -> SwitchFormat, i.e. the
    negacyclic product), common_arithmetic_ops_element (381-446: Plus(1) in
    coefficient form touches coefficient 0 only, Minus(1) / Times(2) every
    slot) and AddILElementOne (457-483)."""
    k = REF["kat_common_elements"]
    q = [k["q"]]
    vec = lambda v: O.U(v).reshape(1, 1, -1)  # noqa: E731
    bo = k["binary_ops"]
    a, b = vec(bo["a"]), vec(bo["b"])
    assert O.eltwise("add", a, b, q).reshape(-1).tolist() == bo["plus_eval"]
    assert O.eltwise("sub", a, b, q).reshape(-1).tolist() == bo["minus_eval"]
    assert O.eltwise("mul", a, b, q).reshape(-1).tolist() == bo["times_eval"]
    tb = O.Tables(k["m"] // 2, q, [k["root"]])
    got = O.ntt_mul_intt(a, O.ntt_fwd(b, tb), tb)
    assert got.reshape(-1).tolist() == bo["switchformat_times_switchformat"]
    so = k["scalar_ops"]
    assert O.add_scalar_at(vec(so["coef_x"]), 0, [1], q).reshape(-1).tolist() == so["plus_1_coefficient_form"]
    assert O.sub_scalar(vec(so["eval_x"]), [1], q).reshape(-1).tolist() == so["minus_1_eval"]
    assert O.mul_scalar(vec(so["eval_x"]), [2], q).reshape(-1).tolist() == so["times_2_eval"]
    one = k["add_il_element_one"]
    assert O.add_scalar(vec(one["x"]), [1], q).reshape(-1).tolist() == one["expected"]


def test_kat_nbtheory(O):
    """UnitTestNbTheory.cpp:165-186 (FirstPrime) and 381-394 (NextPrime chain):
    the prime search behind the moduli chains, in the oracle and in bench.py's
    own product-side chain (FirstPrime then PreviousPrime, poly-benchmark-16k.cpp:89-96)."""
    import bench

    k = REF["kat_nbtheory"]
    for c in k["first_prime"]:
        assert O.first_prime(c["bits"], c["m"]) == c["expected"]
    ch = k["next_prime_chain"]
    q = O.first_prime(ch["bits"], ch["m"])
    got = []
    for _ in ch["expected"]:
        q = O.next_prime(q, ch["m"])
        got.append(q)
    assert got == ch["expected"]
    for log_n, towers in ((14, 8), (16, 16), (17, 4)):
        assert bench.moduli_chain(log_n, towers) == O.moduli_chain(log_n, towers)


def test_kat_dcrt_arithmetic(O):
    """UnitTestDCRTElements.cpp:285-417: a three-tower DCRTPoly (moduli 8353,
    8369, 8513) in evaluation form, the same small values in every tower:
    Plus / Minus / Times / AddILElementOne, tower by tower."""
    k = REF["kat_dcrt_arithmetic"]
    q = k["q"]
    rep = lambda v: np.stack([O.U(v)] * len(q))[None]  # noqa: E731
    a, b = rep(k["a"]), rep(k["b"])
    for op, key in (("add", "plus"), ("sub", "minus"), ("mul", "times")):
        assert np.array_equal(O.eltwise(op, a, b, q), rep(k[key])), op
    assert np.array_equal(O.add_scalar(a, [1, 1, 1], q), rep(k["add_one"]))
