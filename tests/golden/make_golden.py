"""Generates tests/golden/*.json.

Two kinds of fixture live here:

1. Vectors copied as DATA from the reference's own unit tests and from the
   reference-run probe results recorded in SURVEY.md §8(c) (the reference's
   native code, compiled during the survey, run on the inputs described
   there).  These pin the oracle:
     - UnitTestTransform.cpp:60-94  CRT_polynomial_mult KAT (q=113, m=8)
     - UnitTestMubintvec.cpp:276-359 1-limb and 402-484 2-limb (a 52-bit
       modulus, one native word here) vector ModAdd/ModSub/ModMul KATs
     - UnitTestNTT.cpp:53-133 round-trip inputs
     - UnitTestPolyElements.cpp:265-305 SwitchModulus KAT, 500-523
       AutomorphismTransform KAT and 535-571 transposition (q=73, m=8)
     - UnitTestCommonElements.cpp:240-320 common_binary_ops and 381-446
       common_arithmetic_ops_element (q=73, m=8): Plus / Minus / Times in
       evaluation form, SwitchFormat -> Times -> SwitchFormat, scalar ops;
       457-483 AddILElementOne
     - UnitTestDCRTElements.cpp:285-417 three-tower Plus / Minus / Times /
       AddILElementOne in evaluation form
     - UnitTestNbTheory.cpp:165-186 FirstPrime KATs and 381-394 the NextPrime
       chain (the moduli generation behind every plan)
     - UnitTestBFVrnsCRTOperations.cpp:290-376 FastExpandCRTBasisPloverQ KAT
       (N = 8, two 60-bit towers): its P_l part is the ApproxSwitchCRTBasis
       sum of dcrtpoly-impl.h:1419-1441 with the constants of
       bfvrns-cryptoparameters.cpp:501-523
     - SURVEY.md §8(c) probe outputs (moduli, minimal roots, y[0], y[1], c[0][0])
2. Oracle outputs (oracle/ofhe_oracle.c) at small sizes, used as committed
   golden vectors for the GPU parity tests (regenerate with this script; the
   oracle is itself checked against the fixtures of kind 1 in
   tests/test_oracle.py).

Run:  python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402


def reference_fixtures():
    return {
        "source": "reference unit tests + SURVEY.md §8(c) probe outputs",
        "kat_transform": {
            "ref": "src/core/unittest/UnitTestTransform.cpp:60-94",
            "q": 113, "m": 8, "a": [1, 2, 4, 1], "expected": [94, 109, 11, 18], "root": 18,
        },
        "kat_mubintvec": {
            "ref": "src/core/unittest/UnitTestMubintvec.cpp:276-359",
            "q": 163841,
            "a": [127753, 77706, 17133, 22582, 112132, 27625, 126773, 8924,
                  125972, 2551, 113837, 112045, 100953, 77352, 132013, 57029],
            "b": [66773, 69572, 142134, 141115, 123182, 155822, 128147, 94818,
                  135782, 30844, 88634, 99407, 53647, 111689, 28502, 26401],
            "modadd": [30685, 147278, 159267, 163697, 71473, 19606, 91079, 103742,
                       97913, 33395, 38630, 47611, 154600, 25200, 160515, 83430],
            "modsub": [60980, 8134, 38840, 45308, 152791, 35644, 162467, 77947,
                       154031, 135548, 25203, 12638, 47306, 129504, 103511, 30628],
            "modmul": [69404, 64196, 13039, 115321, 28519, 151998, 89117, 80908,
                       57386, 39364, 8355, 146135, 61336, 31598, 25961, 87680],
        },
        "kat_mubintvec_2limb": {
            "ref": "src/core/unittest/UnitTestMubintvec.cpp:402-484 (values < 2^52: one native word here)",
            "q": 4057816419532801,
            "a": [185225172798255, 98879665709163, 3497410031351258, 4012431933509255,
                  1543020758028581, 135094568432141, 3976954337141739, 4030348521557120,
                  175940803531155, 435236277692967, 3304652649070144, 2032520019613814,
                  375749152798379, 3933203511673255, 2293434116159938, 1201413067178193],
            "b": [698898215124963, 39832572186149, 1835473200214782, 1041547470449968,
                  1076152419903743, 433588874877196, 2336100673132075, 2990190360138614,
                  754647536064726, 702097990733190, 2102063768035483, 119786389165930,
                  3976652902630043, 3238750424196678, 2978742255253796, 2124827461185795],
            "modadd": [884123387923218, 138712237895312, 1275066812033239, 996162984426422,
                       2619173177932324, 568683443309337, 2255238590741013, 2962722462162933,
                       930588339595881, 1137334268426157, 1348899997572826, 2152306408779744,
                       294585635895621, 3114137516337132, 1214359951880933, 3326240528363988],
            "modsub": [3544143377206093, 59047093523014, 1661936831136476, 2970884463059287,
                       466868338124838, 3759322113087746, 1640853664009664, 1040158161418506,
                       3479109686999230, 3790954706492578, 1202588881034661, 1912733630447884,
                       456912669701137, 694453087476577, 3372508280438943, 3134402025525199],
            "modmul": [585473140075497, 3637571624495703, 1216097920193708, 1363577444007558,
                       694070384788800, 2378590980295187, 903406520872185, 559510929662332,
                       322863634303789, 1685429502680940, 1715852907773825, 2521152917532260,
                       781959737898673, 2334258943108700, 2573793300043944, 1273980645866111],
        },
        "roundtrip_ntt": {
            "ref": "src/core/unittest/UnitTestNTT.cpp:53-133",
            "m": 16,
            "x1": [431, 3414, 1234, 7845, 2145, 7415, 5471, 8452],
            "x2": [4127, 9647, 1987, 5410, 6541, 7014, 9741, 1256],
            "single_crt_bits": 22, "double_crt_bits": 28,
        },
        "kat_switch_modulus": {
            "ref": "src/core/unittest/UnitTestPolyElements.cpp:265-305",
            "q": 73, "m": 8, "root": 22,
            "cases": [
                {"x": [56, 1, 37, 2], "new_q": 17, "new_root": 15, "expected": [0, 1, 15, 2]},
                {"x": [56, 43, 35, 28], "new_q": 193, "new_root": 150, "expected": [176, 163, 35, 28]},
            ],
        },
        "kat_automorphism": {
            "ref": "src/core/unittest/UnitTestPolyElements.cpp:500-523",
            "q": 73, "m": 8, "root": 22, "format": "coefficient",
            "x": [56, 1, 37, 2], "k": 3, "expected": [56, 2, 36, 1],
            # UnitTestPolyElements.cpp:535-571: Transpose() = AutomorphismTransform(m - 1)
            # in evaluation form (poly-interface.h:443-450): SwitchFormat, Transpose, SwitchFormat
            "transpose": {"ref": "src/core/unittest/UnitTestPolyElements.cpp:535-571",
                          "x": [31, 21, 15, 34], "k": 7, "expected": [31, 39, 58, 52]},
        },
        "kat_common_elements": {
            "ref": "src/core/unittest/UnitTestCommonElements.cpp:240-320, 381-446, 457-483",
            "q": 73, "m": 8, "root": 22,
            "binary_ops": {
                "a": [2, 1, 1, 1], "b": [1, 0, 1, 1],
                "plus_eval": [3, 1, 2, 2], "minus_eval": [1, 1, 0, 0], "times_eval": [2, 0, 1, 1],
                "switchformat_times_switchformat": [0, 72, 2, 4],
            },
            "scalar_ops": {
                "coef_x": [1, 3, 4, 1], "plus_1_coefficient_form": [2, 3, 4, 1],
                "eval_x": [2, 1, 4, 1], "minus_1_eval": [1, 0, 3, 0], "times_2_eval": [4, 2, 8, 2],
            },
            "add_il_element_one": {"x": [2, 1, 3, 2], "expected": [3, 2, 4, 3]},
        },
        "kat_dcrt_arithmetic": {
            "ref": "src/core/unittest/UnitTestDCRTElements.cpp:285-417",
            "m": 8, "q": [8353, 8369, 8513], "root": [8163, 6677, 156],
            "a": [2, 4, 3, 2], "b": [2, 1, 2, 0],
            "plus": [4, 5, 5, 2], "minus": [0, 3, 1, 2], "times": [4, 4, 6, 0], "add_one": [3, 5, 4, 3],
        },
        "kat_nbtheory": {
            "ref": "src/core/unittest/UnitTestNbTheory.cpp:165-186, 381-394",
            "first_prime": [{"bits": 30, "m": 2048, "expected": 1073750017},
                            {"bits": 49, "m": 4096, "expected": 562949953548289}],
            "next_prime_chain": {"bits": 22, "m": 2048,
                                 "expected": [4208641, 4263937, 4270081, 4274177, 4294657,
                                              4300801, 4304897, 4319233, 4323329, 4360193]},
        },
        "kat_fast_expand_crt_basis": {
            "ref": "src/pke/unittest/utbfvrns/UnitTestBFVrnsCRTOperations.cpp:290-376",
            "op": "DCRTPolyImpl::FastExpandCRTBasisPloverQ (dcrtpoly-impl.h:1413-1466); its first loop "
                  "(1419-1441) is ApproxSwitchCRTBasis from Q to R_l with x_i * (-R_l QHat_i^-1 mod q_i) "
                  "(m_negRlQHatInvModq, bfvrns-cryptoparameters.cpp:501-515) and q_i^-1 mod r_j "
                  "(m_qInvModr, 517-523)",
            "m": 16,
            "q": [1152921504606846577, 1152921504606846097],
            "r": [1152921504606845777, 1152921504606845473],
            "x": [[242947838436205858, 458804958636264704, 813208723994158017, 738376275125875131,
                   269337450701982501, 633721177525656427, 406635995163024073, 763204304316606329],
                  [1024863409567898083, 845721255474383902, 537504300724180111, 1018489837930110795,
                   112800627588840746, 1119710169440476902, 77894506676832730, 34149187620514595]],
            "expected_rl": [[955839852875274614, 186398073668078476, 710455872402389881, 1065981546244475424,
                             1049296073052489283, 578396240339812092, 26954876970280156, 1019223053257416912],
                            [874592295621923164, 585167928946466637, 612704504638527027, 551633899923050545,
                             758002500979691774, 694035684451390662, 625796987487151016, 96319544173820807]],
            "expected_ql_note": "towers 0-1 of the test's answer (ans0, ans1) come from the exact HPS "
                                "SwitchCRTBasis (dcrtpoly-impl.h:1445-1447, floating-point alpha), not on the path",
            "expected_ql": [[805568738929329616, 1078766251747424582, 785656076316475932, 599125608237504784,
                             541576441836927290, 152721755350883626, 574857357780891061, 1081393409810468825],
                            [434562805454153184, 312761043978375123, 509951653046700586, 879239171041671808,
                             385039618723450975, 638710747265582661, 246115869294473638, 352338293114574371]],
        },
        "survey_probes": {
            "ref": "SURVEY.md §8(c) (reference native code run in the survey container)",
            "rng": "splitmix64, state += 0x9E3779B97F4A7C15; x_i = sm() % q in index order",
            "ntt": [
                {"log_n": 14, "tower": 0, "seed": 42, "q": 1152921504606748673, "psi": 62213374832584,
                 "y0": 698053391994828643, "y1": 668512656094057990},
                {"log_n": 14, "tower": 1, "seed": 43, "q": 1152921504606683137, "psi": 212089012217363},
                {"log_n": 16, "tower": 0, "seed": 42, "q": 1152921504606584833, "psi": 18043022392882,
                 "y0": 1114074043317201401},
                {"log_n": 16, "tower": 1, "seed": 43, "q": 1152921504598720513, "psi": 800790938143},
            ],
            "dcrt_pipeline": {
                "log_n": 14, "towers": 8, "seed": 1,
                "draw": "one stream; for t: for i: a[t][i] = sm() % q_t; b[t][i] = sm() % q_t",
                "op": "c = INTT(NTT(a) (.) b)", "c00": 866544996928583785,
            },
        },
    }


def fx(a):
    return [int(v) for v in np.asarray(a).reshape(-1)]


def oracle_vectors():
    """Small full vectors from the oracle for GPU parity (N <= 2^12)."""
    cases = []
    for log_n, towers, batch in ((1, 2, 2), (3, 2, 2), (6, 3, 1), (10, 2, 2), (11, 1, 1)):
        n = 1 << log_n
        qs, rs = O.moduli_chain(log_n, towers)
        tb = O.Tables(n, qs, rs)
        a = O.uniform_dcrt(batch, towers, n, qs, seed=1)
        b = O.uniform_dcrt(batch, towers, n, qs, seed=2)
        cases.append({
            "log_n": log_n, "towers": towers, "batch": batch, "q": qs, "psi": rs,
            "a": fx(a), "b": fx(b),
            "ntt_a": fx(O.ntt_fwd(a, tb)),
            "intt_a": fx(O.ntt_inv(a, tb)),
            "mul": fx(O.eltwise("mul", a, b, qs)),
            "add": fx(O.eltwise("add", a, b, qs)),
            "sub": fx(O.eltwise("sub", a, b, qs)),
            "pipeline": fx(O.ntt_mul_intt(a, b, tb)),
        })
    return {"source": "oracle/ofhe_oracle.c via tests/golden/make_golden.py", "cases": cases}


def oracle_fingerprints():
    """FNV-1a fingerprints of oracle outputs at the benchmark shapes (GPU parity
    at full size without shipping megabytes of vectors)."""
    out = []
    for log_n, towers, batch in ((12, 2, 2), (13, 3, 2), (14, 8, 1), (15, 2, 1), (16, 4, 1), (17, 2, 1)):
        n = 1 << log_n
        qs, rs = O.moduli_chain(log_n, towers)
        tb = O.Tables(n, qs, rs)
        a = O.uniform_dcrt(batch, towers, n, qs, seed=11)
        b = O.uniform_dcrt(batch, towers, n, qs, seed=12)
        out.append({
            "log_n": log_n, "towers": towers, "batch": batch, "q": qs, "psi": rs,
            "seed_a": 11, "seed_b": 12,
            "fnv_ntt_a": O.fnv64(O.ntt_fwd(a, tb)),
            "fnv_intt_a": O.fnv64(O.ntt_inv(a, tb)),
            "fnv_mul": O.fnv64(O.eltwise("mul", a, b, qs)),
            "fnv_pipeline": O.fnv64(O.ntt_mul_intt(a, b, tb)),
        })
    return {"source": "oracle/ofhe_oracle.c via tests/golden/make_golden.py", "fingerprints": out}


def bconv_vectors():
    out = []
    for log_n, sq, sp, batch in ((4, 3, 2, 2), (9, 5, 4, 1), (10, 2, 11, 1)):
        n = 1 << log_n
        chain, _ = O.moduli_chain(log_n, sq + sp)
        q, p = chain[:sq], chain[sq:]
        pre = O.base_conv_precompute(q, p)
        x = O.uniform_dcrt(batch, sq, n, q, seed=5)
        y = np.stack([O.approx_switch_crt_basis(x[bi], q, p, pre) for bi in range(batch)])
        out.append({"log_n": log_n, "batch": batch, "q": q, "p": p, "qhat_inv_modq": fx(pre["qhinv"]),
                    "qhat_modp": fx(pre["qhmodp"]), "x": fx(x), "out": fx(y)})
    return {"source": "oracle/ofhe_oracle.c via tests/golden/make_golden.py", "cases": out}


def main():
    for name, obj in (("reference_fixtures.json", reference_fixtures()),
                      ("oracle_vectors.json", oracle_vectors()),
                      ("oracle_fingerprints.json", oracle_fingerprints()),
                      ("bconv_vectors.json", bconv_vectors())):
        with open(os.path.join(HERE, name), "w") as f:
            json.dump(obj, f, separators=(",", ":"))
        print("wrote", name, os.path.getsize(os.path.join(HERE, name)), "bytes")


if __name__ == "__main__":
    main()
