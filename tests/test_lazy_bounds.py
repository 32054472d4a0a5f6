"""Worst-case range checks of the lazy reductions in the column passes (CPU).

The GPU kernels keep residues in redundant ranges between butterfly stages
(csrc/ntt_kernels.hpp: gs_bfly_b / inv_stage16_b, OFHE_LAZY_GS; ct_bfly_cs,
OFHE_LAZY_FWD).  These tests replay the exact compile-time schedule of those
kernels on the largest representative of every residue each step may produce
and check (1) no intermediate reaches 2^64 and (2) the final canonicalisation
returns the residue.  Parity of the kernels themselves is checked on the GPU
(tests/test_gpu_parity.py); this pins the range argument at q just below 2^60,
the largest modulus the reference allows (basicint.h:44-45, MAX_MODULUS_SIZE 60).
"""
import random

import pytest

TWO64 = 1 << 64


def _worst(res, q, bound):
    """largest value < bound congruent to res mod q"""
    v = res + ((bound - 1 - res) // q) * q
    assert v < bound and v % q == res
    return v


def _csub(x, m):
    return x - m if x >= m else x


def _gs_round(v, b8, q, rng):
    """inv_round16_b: stages half = 8, 4, 2, 1; sum < 8q, Shoup output < 4q"""
    for half in (8, 4, 2, 1):
        for base in range(0, 16, 2 * half):
            for k in range(base, base + half):
                x, y = v[k], v[k + half]
                in8 = b8[k] or b8[k + half]
                B = 8 * q if in8 else 4 * q
                assert x < B and y < B
                s = x + y
                d = x + B - y
                assert 0 < d < TWO64 and s < TWO64
                w = rng.randrange(1, q)
                v[k] = _csub(s, 8 * q) if in8 else s
                # shoup_lazy: any 64-bit input, result in [0, 4q)
                v[k + half] = _worst(d * w % q, q, 4 * q)
                b8[k], b8[k + half] = True, False
                assert v[k] < 8 * q
    return v, b8


def _canon8(x, q):
    return _csub(_csub(_csub(x, 4 * q), 2 * q), q)


def _canon4(x, q):
    return _csub(_csub(x, 2 * q), q)


@pytest.mark.parametrize("q", [(1 << 60) - (1 << 17) + 1, 1152921504606584833, (1 << 59) + 1])
def test_lazy_gs_two_rounds(q):
    rng = random.Random(q)
    for _ in range(200):
        # round 1 input: the block pass's lazy twist, [0, 4q)
        res = [rng.randrange(q) for _ in range(16)]
        v = [_worst(r, q, 4 * q) for r in res]
        b8 = [False] * 16
        v, b8 = _gs_round(v, b8, q, rng)
        # round 2 registers all come from one round-1 position: taken as < 8q
        res2 = [x % q for x in v]
        v = [_worst(r, q, 8 * q) for r in res2]
        assert max(v) < 8 * q
        b8 = [True] * 16
        v, b8 = _gs_round(v, b8, q, rng)
        want = [x % q for x in v]
        got = [_canon8(x, q) if b else _canon4(x, q) for x, b in zip(v, b8)]
        assert got == want
        assert b8 == [k % 2 == 0 for k in range(16)]


@pytest.mark.parametrize("q", [(1 << 60) - (1 << 17) + 1, (1 << 59) + 1])
def test_lazy_ct_alternating(q):
    """ct_bfly_cs with OFHE_LAZY_FWD: CS stages subtract 8q, outputs stay < 16q"""
    rng = random.Random(q ^ 1)
    for _ in range(200):
        v = [_worst(rng.randrange(q), q, 12 * q) for _ in range(16)]  # column-pass output < 12q
        for s in range(8):  # two radix-16 rounds of the block pass
            cs = s % 2 == 1
            half = 8 >> (s % 4)
            for base in range(0, 16, 2 * half):
                for k in range(base, base + half):
                    x, y = v[k], v[k + half]
                    assert x < 16 * q and y < TWO64
                    t = _worst(y * rng.randrange(1, q) % q, q, 4 * q)
                    a = _csub(x, 8 * q) if cs else x
                    assert a < (8 if cs else 12) * q
                    v[k], v[k + half] = a + t, a + 4 * q - t
                    assert v[k] < TWO64 and v[k + half] < TWO64
            assert max(v) < (12 if cs else 16) * q


@pytest.mark.parametrize("q", [(1 << 60) - (1 << 17) + 1, (1 << 59) + 1])
def test_fwd_first_round_canonical_input(q):
    """fwd_round16_canon (OFHE_FWD_CANON): inputs < 4q, no conditional subtract
    before the round's last stage, output < 12q like every other round"""
    rng = random.Random(q ^ 2)
    for _ in range(200):
        v = [_worst(rng.randrange(q), q, 4 * q) for _ in range(16)]
        for s in range(4):
            cs = s == 3
            half = 8 >> s
            for base in range(0, 16, 2 * half):
                for k in range(base, base + half):
                    x, y = v[k], v[k + half]
                    assert x < 16 * q and y < TWO64
                    t = _worst(y * rng.randrange(1, q) % q, q, 4 * q)
                    a = _csub(x, 8 * q) if cs else x
                    v[k], v[k + half] = a + t, a + 4 * q - t
        assert max(v) < 12 * q
