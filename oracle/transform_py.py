"""Pure-Python, big-integer transcription of the reference's NTT loops.

TEST INFRASTRUCTURE ONLY (tests/ import it; nothing in the product path does).
An independent second restatement of the reference's forward and inverse
negacyclic NTT and of its table precomputation, written with Python integers
(no 64-bit wraparound, no Shoup approximation: every product is reduced with
`%`), so that it pins the C oracle (oracle/ofhe_oracle.c) over full vectors.

  precompute  ChineseRemainderTransformFTTNat::PreCompute, transformnat-impl.h:708-763
  forward     NumberTheoreticTransformNat::ForwardTransformToBitReverseInPlace,
              transformnat-impl.h:300-354 (natural order in, bit-reversed out)
  inverse     NumberTheoreticTransformNat::InverseTransformFromBitReverseInPlace,
              transformnat-impl.h:492-552 (n^-1 fused into the first stage)
  n^-1        TableCOI[msb(N-1)], transformnat-impl.h:661-665

The reference's ModMulFastConstEq (ubintnat.h:1491-1497) returns the canonical
residue of x * w mod q, and its butterflies keep every value in [0, q), so
exact `%` arithmetic gives the same integers.
"""


def _rev(x: int, bits: int) -> int:
    r = 0
    for _ in range(bits):
        r = (r << 1) | (x & 1)
        x >>= 1
    return r


def precompute(n: int, q: int, psi: int):
    """Table[rev(i)] = psi^i, TableI[rev(i)] = psi^-i (transformnat-impl.h:724-729)."""
    lg = n.bit_length() - 1
    psi_inv = pow(psi, q - 2, q)
    tab, itab = [0] * n, [0] * n
    x = xi = 1
    for i in range(n):
        r = _rev(i, lg)
        tab[r], itab[r] = x, xi
        x, xi = x * psi % q, xi * psi_inv % q
    return tab, itab


def forward(x, q: int, tab):
    """transformnat-impl.h:300-354: for m = 1, 2, ..., N/2 (t = N/2m), pairs
    (j1, j1 + t) of group i use omega = Table[i + m]: (lo + w hi, lo - w hi)."""
    a = [int(v) for v in x]
    n = len(a) >> 1
    t, m = n, 1
    while m < n:
        for i in range(m):
            w = tab[i + m]
            j1 = i * 2 * t
            for j in range(j1, j1 + t):
                of = a[j + t] * w % q
                lo = a[j]
                a[j], a[j + t] = (lo + of) % q, (lo - of) % q
        m <<= 1
        t >>= 1
    # the split-out last stage (332-353): pairs (i, i + 1), omega = Table[i/2 + n]
    for i in range(0, n << 1, 2):
        of = a[i + 1] * tab[(i >> 1) + n] % q
        lo = a[i]
        a[i], a[i + 1] = (lo + of) % q, (lo - of) % q
    return a


def inverse(y, q: int, itab):
    """transformnat-impl.h:492-552: first stage (t = 1) with omega = TableI[(i + n)/2]
    and both outputs times n^-1; then m = N/4 ... 1 (t = 2 ... N/2) GS
    butterflies (lo + hi, (lo - hi) * TableI[i + m])."""
    a = [int(v) for v in y]
    n = len(a)
    ninv = pow(n, q - 2, q)  # TableCOI[msb(n - 1)] = (2^log n)^-1
    for i in range(0, n, 2):
        w = itab[(i + n) >> 1]
        lo, hi = a[i], a[i + 1]
        a[i] = (lo + hi) % q * ninv % q
        a[i + 1] = (lo - hi) % q * w % q * ninv % q
    m, t = n >> 2, 2
    while m >= 1:
        for i in range(m):
            w = itab[i + m]
            j1 = i * 2 * t
            for j in range(j1, j1 + t):
                lo, hi = a[j], a[j + t]
                a[j], a[j + t] = (lo + hi) % q, (lo - hi) % q * w % q
        m >>= 1
        t <<= 1
    return a
