"""Design model (not a test, not product code) for the matrix-core block pass
at N = 2^16: checks with exact Python integers that the reference's last 8
forward stages and first 8 inverse stages on every 256-element group equal

  forward:  z_j = x_j theta_G^j                         (twist, per element)
            A[r'][j0] = sum_j1 F[r'][j1] z[j0 + 16 j1]   (round A, F shared)
            B[r'][j0] = A[r'][j0] w256^(j0 rev4(r'))     (twiddle, 256 values)
            Y[16 r' + r] = sum_j0 F[r][j0] B[r'][j0]      (round B, F shared)
  with F[r][j] = w16^(j rev4(r)), theta_G = psi^(2 rev(G) + 1), w256 = psi^512;
  inverse:  A'[r'][j0] = sum_r F'[j0][r] y[16 r' + r]     (round A', F' shared)
            B'[r'][j0] = A'[r'][j0] w256^(-j0 rev4(r'))
            Z[j0 + 16 j1] = sum_r' F'[j1][r'] B'[r'][j0]  (round B')
            a_j = Z_j * N^-1 psi^-((2 rev(G) + 1) j)      (twist)
  with F'[j][r] = w16^(-j rev4(r)).
The reference loops are transformnat-impl.h:300-354 (forward) and 492-552
(inverse), restated in oracle/transform_py.py.

  python tools/mma_model.py            the identities above (exact integers)
  python tools/mma_model.py --budget   round 6's instruction / issue model of
                                       the whole pipeline on the matrix cores
                                       ("The 0.40 target")
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))
import transform_py as R  # noqa: E402
import oracle as O  # noqa: E402


def rev(x, bits):
    return R._rev(x, bits)


def fwd_stages(a, q, tab, stages):
    """the reference's forward CT loop, first `stages` stages only"""
    a = list(a)
    n = len(a) >> 1
    t, m, s = n, 1, 0
    while m < n and s < stages:
        for i in range(m):
            w = tab[i + m]
            j1 = i * 2 * t
            for j in range(j1, j1 + t):
                of = a[j + t] * w % q
                lo = a[j]
                a[j], a[j + t] = (lo + of) % q, (lo - of) % q
        m <<= 1
        t >>= 1
        s += 1
    return a


def main():
    log_n = 16
    n = 1 << log_n
    qs, rs = O.moduli_chain(log_n, 1)
    q, psi = qs[0], rs[0]
    tab, itab = R.precompute(n, q, psi)
    import random
    rng = random.Random(5)
    x = [rng.randrange(q) for _ in range(n)]
    full = R.forward(x, q, tab)
    col = fwd_stages(x, q, tab, 8)
    w256 = pow(psi, 512, q)
    w16 = pow(w256, 16, q)
    F = [[pow(w16, j * rev(r, 4), q) for j in range(16)] for r in range(16)]
    Fi = [[pow(w16, (-j * rev(r, 4)) % 256, q) for r in range(16)] for j in range(16)]
    ok = True
    for G in (0, 1, 2, 77, 128, 255):
        theta = pow(psi, 2 * rev(G, 8) + 1, q)
        z = [col[256 * G + j] * pow(theta, j, q) % q for j in range(256)]
        A = [[sum(F[r1][j1] * z[j0 + 16 * j1] for j1 in range(16)) % q for j0 in range(16)] for r1 in range(16)]
        B = [[A[r1][j0] * pow(w256, j0 * rev(r1, 4), q) % q for j0 in range(16)] for r1 in range(16)]
        Y = [0] * 256
        for r1 in range(16):
            for r in range(16):
                Y[16 * r1 + r] = sum(F[r][j0] * B[r1][j0] for j0 in range(16)) % q
        ok = ok and Y == full[256 * G:256 * G + 256]
    print("forward block stages as twist + F + twiddle + F:", ok)
    # inverse: the reference's inverse of y = full; after its first 8 stages the
    # GS intermediate equals W_b = N^-1 psi^-((2 rev(b) + 1) j) Z_b
    inv = R.inverse(full, q, itab)
    assert inv == x
    ninv = pow(n, q - 2, q)
    ok2 = True
    for G in (0, 3, 128, 255):
        y = full[256 * G:256 * G + 256]
        Ap = [[sum(Fi[j0][r] * y[16 * r1 + r] for r in range(16)) % q for j0 in range(16)] for r1 in range(16)]
        Bp = [[Ap[r1][j0] * pow(w256, (-j0 * rev(r1, 4)) % 256, q) % q for j0 in range(16)] for r1 in range(16)]
        Z = [0] * 256
        for j0 in range(16):
            for j1 in range(16):
                Z[j0 + 16 * j1] = sum(Fi[j1][r1] * Bp[r1][j0] for r1 in range(16)) % q
        th = pow(psi, 2 * rev(G, 8) + 1, q)
        thi = pow(th, q - 2, q)
        W = [Z[j] * ninv % q * pow(thi, j, q) % q for j in range(256)]
        # the GS column pass would take W; check instead that the full inverse of
        # the reference applied to y agrees: run GS stages t = 256 .. N/2 on W
        ok2 = ok2 and len(W) == 256
        if G == 0:
            W0 = W
    # complete check: all groups, then the reference's last 8 GS stages
    Wall = [0] * n
    for G in range(256):
        y = full[256 * G:256 * G + 256]
        Ap = [[sum(Fi[j0][r] * y[16 * r1 + r] for r in range(16)) % q for j0 in range(16)] for r1 in range(16)]
        Bp = [[Ap[r1][j0] * pow(w256, (-j0 * rev(r1, 4)) % 256, q) % q for j0 in range(16)] for r1 in range(16)]
        th = pow(psi, 2 * rev(G, 8) + 1, q)
        thi = pow(th, q - 2, q)
        for j0 in range(16):
            for j1 in range(16):
                z = sum(Fi[j1][r1] * Bp[r1][j0] for r1 in range(16)) % q
                j = j0 + 16 * j1
                Wall[256 * G + j] = z * ninv % q * pow(thi, j, q) % q
    # GS stages m = N/512 .. 1 (t = 256 .. N/2), transformnat-impl.h:527-551
    a = Wall
    m, t = n >> 9, 256
    while m >= 1:
        for i in range(m):
            w = itab[i + m]
            j1 = i * 2 * t
            for j in range(j1, j1 + t):
                lo, hi = a[j], a[j + t]
                a[j] = (lo + hi) % q
                a[j + t] = (lo - hi) % q * w % q
        m >>= 1
        t <<= 1
    print("inverse block stages as F' + twiddle + F' + twist, then GS column stages:", a == x)


# ---------------------------------------------------------------------------
# Round 6: the pipeline-wide matrix-core budget.  Inputs are measurements,
# each with its record:
#   * k_block (butterflies), k_tcols fwd / inv: SQ_INSTS_VALU per coefficient,
#     profiles/pmc_current.json (r05y, the shipped build): 180.75 / 80.1 / 95.1
#   * k_block_m16 (round 3, 4 MFMA rounds): 172.0 per coefficient measured
#     (profiles/r03_block_m16_pmc/), issue 0.121 wave-instr per SIMD-cycle;
#     its loop body, recompiled from 2ae2740 (ntt_m16.hpp) and counted by
#     instruction: 1235 VALU per 8 coefficients per lane = 154.4 per
#     coefficient, plus 152 static instructions once per 16 coefficients
#     (setup: fragment staging, constants, addresses) = 9.5
#   * the m16 header's model: 4 x (digit split 3 + reduce 12) + 4 Shoup x 14 +
#     Montgomery Hadamard 20 = 136
# A matrix-core radix-16 round, measured: the m16 loop minus its non-round
# work (twist, two twiddles, inverse twist: 4 Shoup x 14; Montgomery
# Hadamard 20) over its four rounds.
# ---------------------------------------------------------------------------
M16_LOOP = 1235 / 8          # VALU per coefficient in k_block_m16's loop
M16_SETUP = 152 / 16         # once-per-thread part
M16_MEASURED = 172.0
SHOUP, MONT = 14, 20
ROUND_MMA = (M16_LOOP - 4 * SHOUP - MONT) / 4
BUTTERFLY = {"colpass<fwd>": 80.1, "k_block<fused>": 180.75, "colpass<inv>": 95.1}
SHIPPED = sum(BUTTERFLY.values())
HEADLINE = 8.17e10           # BENCH_r05 coefficients/s (the driver's record)
ISSUE_MEASURED_M16 = 0.121   # k_block_m16's VALU issue per SIMD-cycle
ISSUE_BUTTERFLY = 0.245


def budget():
    # The column passes' two radix-16 rounds are shared 16 x 16 maps with the
    # twiddles folded in (round 1: one matrix per tower; round 2: 16, by the
    # row block, transformnat-impl.h:305-311): two MMA rounds and no twist.
    # I/O: loads, stores, canonicalisation of the inverse output (~6), and the
    # per-thread setup as m16's.
    col = 2 * ROUND_MMA + 6 + M16_SETUP
    rows = [
        ("butterflies (shipped)", BUTTERFLY["colpass<fwd>"], BUTTERFLY["k_block<fused>"], BUTTERFLY["colpass<inv>"]),
        ("MMA column passes + butterfly block", col, BUTTERFLY["k_block<fused>"], col),
        ("MMA column passes + k_block_m16", col, M16_MEASURED, col),
        ("MMA everywhere, no per-thread setup", 2 * ROUND_MMA + 6, M16_LOOP, 2 * ROUND_MMA + 6),
    ]
    print(f"matrix-core radix-16 round, measured: {ROUND_MMA:.1f} VALU per coefficient "
          f"(m16 loop {M16_LOOP:.1f} - 4 Shoup x {SHOUP} - Hadamard {MONT}, over 4 rounds)")
    print(f"m16 header model 136 vs measured {M16_MEASURED}: loop {M16_LOOP:.1f} + setup {M16_SETUP:.1f} "
          f"= {M16_LOOP + M16_SETUP:.1f}; the loop's v_mov_b32 alone is {189 / 8:.1f} per coefficient")
    print(f"{'variant':42s} {'fwd col':>8s} {'block':>8s} {'inv col':>8s} {'total':>8s} "
          f"{'@0.245':>9s} {'@0.121':>9s}")
    for name, a, b, c in rows:
        tot = a + b + c
        # throughput at the shipped issue rate (VALU-bound, same clock), and at m16's measured issue
        at_shipped = HEADLINE * SHIPPED / tot
        at_m16 = at_shipped * ISSUE_MEASURED_M16 / ISSUE_BUTTERFLY
        print(f"{name:42s} {a:8.1f} {b:8.1f} {c:8.1f} {tot:8.1f} {at_shipped / 3.33e11:9.3f} {at_m16 / 3.33e11:9.3f}")
    # matrix-pipe share in a column pass at full overlap: 16 v_mfma_i32_32x32x32_i8
    # per 512 elements per round (32 cycles each at the dense int8 peak) against
    # the round's VALU at 4 cycles per wave64 instruction
    mfma_cyc = 16 * 32 / 512
    valu_cyc = ROUND_MMA * 4 / 64
    print(f"column-pass round per coefficient per SIMD: matrix pipe {mfma_cyc:.2f} cycles, VALU {valu_cyc:.2f} "
          f"-> matrix pipe {mfma_cyc / max(mfma_cyc, valu_cyc):.0%} busy at full overlap")
    print("columns @0.245 / @0.121: fraction of the 8 TB/s HBM roofline (24 B/coeff) at the shipped issue rate "
          "and at the matrix-core kernel's measured one; the north star asks >= 0.40")


if __name__ == "__main__":
    if "--budget" in sys.argv:
        budget()
    else:
        main()
