"""CPU check of k_bconv_cols' in-kernel inverse column pass schedule
(bconv_cols.hpp, bcc_icol_source), restated from the kernel: one wave per
source tower, lane (qq, col) holding rows 8 qq .. 8 qq + 7, distances 1 / 2 / 4
in the lane and 8 / 16 across lanes with the half swap -- against the
reference's Gentleman-Sande order on the 32-row column
(transformnat-impl.h:492-552 as cols_inv_b runs it), over exact integers mod a
prime.

No GPU: the schedule is index arithmetic."""
import random

import pytest

Q = 1152921504606584833  # a 60-bit NTT prime of the headline chain


def gs_reference(v, itw):
    """cols_inv_b<32> on one column: s = 4 .. 0, half = 32 >> (s + 1)."""
    v = list(v)
    for s in range(4, -1, -1):
        half = 32 >> (s + 1)
        for j in range(1 << s):
            w = itw[(1 << s) + j]
            for k in range(j * 2 * half, j * 2 * half + half):
                x, y = v[k], v[k + half]
                v[k], v[k + half] = (x + y) % Q, (x - y) * w % Q
    return v


def gs_icol(v, itw):
    """bcc_icol_source's lane layout, four lanes of one column."""
    lanes = [[v[8 * qq + k] for k in range(8)] for qq in range(4)]

    def bf(lv, i, j, w):
        x, y = lv[i], lv[j]
        lv[i], lv[j] = (x + y) % Q, (x - y) * w % Q

    for qq in range(4):
        lv = lanes[qq]
        for j in range(4):
            bf(lv, 2 * j, 2 * j + 1, itw[16 + 4 * qq + j])
        for j in range(2):
            for i in range(2):
                bf(lv, 4 * j + i, 4 * j + i + 2, itw[8 + 2 * qq + j])
        for i in range(4):
            bf(lv, i, i + 4, itw[4 + qq])

    def cross(xmask, wsel, upper_of):
        new = [list(lv) for lv in lanes]
        for qq in range(4):
            partner = qq ^ (xmask // 16)
            upper = upper_of(qq)
            w = itw[wsel(qq)]
            for m in range(4):
                snd_partner = lanes[partner][m] if upper_of(partner) else lanes[partner][4 + m]
                rcv = snd_partner
                xv = rcv if upper else lanes[qq][m]
                yv = lanes[qq][4 + m] if upper else rcv
                new[qq][m], new[qq][4 + m] = (xv + yv) % Q, (xv - yv) * w % Q
        return new

    lanes = cross(16, lambda qq: 2 + (qq >> 1), lambda qq: qq & 1)
    lanes = cross(32, lambda qq: 1, lambda qq: (qq >> 1) & 1)
    out = [None] * 32
    for qq in range(4):
        r0 = 4 * (qq & 1) + 8 * (qq >> 1)
        for m in range(8):
            out[r0 + (m & 3) + (16 if m >= 4 else 0)] = lanes[qq][m]
    return out


@pytest.mark.parametrize("seed", range(4))
def test_icol_lane_layout_equals_gs_order(seed):
    rng = random.Random(seed)
    v = [rng.randrange(Q) for _ in range(32)]
    itw = [rng.randrange(1, Q) for _ in range(32)]
    assert gs_icol(v, itw) == gs_reference(v, itw)
