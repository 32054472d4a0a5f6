"""CPU checks of two round-4 index schedules, restated from their kernels:

* k_bconv_cols' in-kernel inverse column pass (bconv_cols.hpp,
  bcc_icol_source): one wave per source tower, lane (qq, col) holding rows
  8 qq .. 8 qq + 7, distances 1 / 2 / 4 in the lane and 8 / 16 across lanes
  with the half swap -- against the reference's Gentleman-Sande order on the
  32-row column (transformnat-impl.h:492-552 as cols_inv_b runs it), over
  exact integers mod a prime;
* k_pipe's work-item schedule (pipe_kernels.hpp): every (pass, tower, tile)
  item handed out exactly once per XCD queue, and every dependency (forward
  column tiles before the tower's block pass, block pass before the inverse
  column tiles) handed out earlier in the same queue, for the dynamic queue
  and the static assignment, across lags and tiles per item.

No GPU: the schedules are index arithmetic."""
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


def pipe_items(units, nq, lag, pieces, wpq=0, grid_per_q=None):
    """Decode k_pipe's items per queue: list of (queue, item index, phase, unit, piece)."""
    ipp = 16 // pieces
    out = []
    for q in range(nq):
        nu = (units - q + nq - 1) // nq if units > q else 0
        total = (nu + 2 * lag) * 3 * ipp if nu else 0
        # dynamic: items in hand-out order; static (wpq): workgroup r runs
        # r, r + wpq, ... in increasing order -- either way the lowest unfinished
        # item waits on nothing unfinished when every dependency has a lower index
        for item in range(total):
            if wpq and item % wpq >= (grid_per_q or wpq):
                continue
            step, slot = divmod(item, 3 * ipp)
            ph, grp = divmod(slot, ipp)
            if step >= ph * lag and step - ph * lag < nu:
                u = q + nq * (step - ph * lag)
                for k in range(pieces):
                    out.append((q, item, ph, u, grp * pieces + k))
    return out


@pytest.mark.parametrize("units,lag,pieces,static", [
    (1, 1, 1, False), (5, 4, 1, False), (16 * 3, 12, 1, False), (21, 2, 2, False),
    (64, 8, 4, False), (13, 2048, 16, False), (40, 3, 1, True), (64, 12, 4, True),
])
def test_pipe_schedule_covers_and_orders(units, lag, pieces, static):
    nq = 8
    items = pipe_items(units, nq, lag, pieces, wpq=128 if static else 0)
    seen = {}
    for q, pos, ph, u, piece in items:
        key = (ph, u, piece)
        assert key not in seen, key
        assert u % nq == q  # a tower's three passes share one queue (one XCD)
        seen[key] = pos
    assert len(seen) == 3 * 16 * units
    for (ph, u, piece), pos in seen.items():
        if ph:  # every tile of the previous pass was handed out before this item
            assert all(seen[(ph - 1, u, k)] < pos for k in range(16)), (ph, u, piece)
