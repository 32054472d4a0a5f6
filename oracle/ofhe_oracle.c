/*
 * ofhe_oracle.c -- CPU restatement of the reference's RNS hot path.
 *
 * *** TEST INFRASTRUCTURE ONLY. ***
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library, and only as the checker / the timed CPU baseline.  The
 * product path (upmem--openfhe_amd/csrc) never links or calls it.
 *
 * Every function restates an algorithm of the reference snapshot
 * (MpokiAbel/UPMEM--OpenFHE = OpenFHE v1.1.1 + PIM layer) and cites the
 * file:line it follows (paths relative to the reference root).  Nothing here
 * is copied; it is written from the algorithm description in SURVEY.md §8(a).
 *
 * Parity pinning (see DESIGN.md "Oracle"):
 *   - KAT  src/core/unittest/UnitTestTransform.cpp:60-94     (q=113, m=8)
 *   - KATs src/core/unittest/UnitTestMubintvec.cpp:276-359   (q=163841)
 *   - round trips src/core/unittest/UnitTestNTT.cpp:53-133
 *   - outputs of the reference's own native code recorded in SURVEY.md
 *     §8(c) (N=2^14 / 2^16 forward NTT fingerprints, DCRTPoly pipeline).
 *   The reference cannot be compiled here without stand-in headers
 *   (<dpu.h>, cereal), so there is no oracle/_ref build.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef unsigned __int128 u128;
typedef uint64_t u64;

/* ---------------------------------------------------------------------------
 * Scalar arithmetic (src/core/include/math/hal/intnat/ubintnat.h)
 * ------------------------------------------------------------------------- */

/* lbcrypto::GetMSB: 1-based index of the most significant set bit, 0 for 0. */
unsigned oracle_msb(u64 x) { return x ? 64u - (unsigned)__builtin_clzll(x) : 0u; }

/* ComputeMu, ubintnat.h:651-656: floor(2^(2*msb(q)+3) / q), truncated to 64 bits. */
u64 oracle_compute_mu(u64 q) {
    unsigned s = 2u * oracle_msb(q) + 3u;
    u128 num = (s >= 128) ? 0 : ((u128)1 << s);
    return (u64)(num / q);
}

/* ModMulFastEq(b, q, mu), ubintnat.h:1399-1413 (Barrett, NATIVEINT_BARRET_MOD). */
u64 oracle_modmul_barrett(u64 a, u64 b, u64 q, u64 mu) {
    u128 prod = (u128)a * b;
    int n = (int)oracle_msb(q) - 2;
    u128 t = (u128)(u64)(prod >> n) * mu;
    u128 r = prod - (u128)q * (t >> (n + 7));
    u64 v = (u64)r;
    if (v >= q) v -= q;
    return v;
}

/* PrepModMulConst, ubintnat.h:1448-1455: floor(w * 2^64 / q). */
u64 oracle_shoup_prep(u64 w, u64 q) { return (u64)(((u128)w << 64) / q); }

/* ModMulFastConst(Eq), ubintnat.h:1478-1497 (Shoup / Harvey). */
u64 oracle_modmul_shoup(u64 a, u64 w, u64 q, u64 wp) {
    u64 qh = (u64)(((u128)a * wp) >> 64) + 1;
    int64_t y = (int64_t)(a * w - qh * q);
    return (u64)(y >= 0 ? y : y + (int64_t)q);
}

/* ModAddFastEq ubintnat.h:760-767; ModSubFastEq ubintnat.h:934-938. */
u64 oracle_modadd(u64 a, u64 b, u64 q) { u64 r = a + b; return r >= q ? r - q : r; }
u64 oracle_modsub(u64 a, u64 b, u64 q) { return a < b ? a + q - b : a - b; }

static u64 modmul_exact(u64 a, u64 b, u64 q) { return (u64)(((u128)a * b) % q); }

u64 oracle_modexp(u64 b, u64 e, u64 q) {
    u64 r = 1 % q;
    b %= q;
    while (e) {
        if (e & 1) r = modmul_exact(r, b, q);
        b = modmul_exact(b, b, q);
        e >>= 1;
    }
    return r;
}

/* ModInverse via Fermat (q prime). */
u64 oracle_modinv(u64 a, u64 q) { return oracle_modexp(a, q - 2, q); }

/* ---------------------------------------------------------------------------
 * Number theory (src/core/include/math/nbtheory-impl.h)
 * ------------------------------------------------------------------------- */

/* MillerRabinPrimalityTest, nbtheory-impl.h:261-286.  The reference draws 100
 * random witnesses; we use the fixed base set that is deterministic for all
 * n < 3.3e24, so every 64-bit answer coincides with the reference's (whose
 * false-positive probability is 4^-100). */
int oracle_is_prime(u64 n) {
    static const u64 bases[] = {2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37};
    if (n < 2) return 0;
    for (unsigned i = 0; i < 12; i++) {
        if (n == bases[i]) return 1;
        if (n % bases[i] == 0) return 0;
    }
    u64 d = n - 1;
    unsigned s = 0;
    while ((d & 1) == 0) { d >>= 1; s++; }
    for (unsigned i = 0; i < 12; i++) {
        u64 x = oracle_modexp(bases[i], d, n);
        if (x == 1 || x == n - 1) continue;
        int comp = 1;
        for (unsigned r = 1; r < s; r++) {
            x = modmul_exact(x, x, n);
            if (x == n - 1) { comp = 0; break; }
        }
        if (comp) return 0;
    }
    return 1;
}

/* FirstPrime(nBits, m), nbtheory-impl.h:334-359: smallest prime p > 2^nBits,
 * p = 1 mod m. Returns 0 on overflow. */
u64 oracle_first_prime(unsigned nbits, u64 m) {
    if (nbits >= 64) return 0;
    u64 q = (u64)1 << nbits;
    u64 r = q % m;
    u64 cand = q + 1;
    if (r > 0) cand += m - r;
    while (!oracle_is_prime(cand)) {
        u64 nx = cand + m;
        if (nx < cand) return 0;
        cand = nx;
    }
    return cand;
}

/* PreviousPrime(q, m), nbtheory-impl.h:372-379. */
u64 oracle_previous_prime(u64 q, u64 m) {
    u64 cand = q - m;
    while (!oracle_is_prime(cand)) {
        u64 nx = cand - m;
        if (nx > cand) return 0;
        cand = nx;
    }
    return cand;
}

/* NextPrime(q, m), nbtheory-impl.h:362-369. */
u64 oracle_next_prime(u64 q, u64 m) {
    u64 cand = q + m;
    while (!oracle_is_prime(cand)) {
        u64 nx = cand + m;
        if (nx < cand) return 0;
        cand = nx;
    }
    return cand;
}

/* RootOfUnity(m, q), nbtheory-impl.h:183-231: the SMALLEST primitive m-th root
 * of unity (m a power of two).  The reference starts from a random generator
 * and scans its odd powers; the set of odd powers of any primitive root is the
 * set of all primitive roots, so the minimum is generator-independent. */
u64 oracle_root_of_unity(u64 m, u64 q) {
    if (m < 2 || (q - 1) % m) return 0;
    u64 e = (q - 1) / m, psi = 0;
    for (u64 c = 2; c < q; c++) {
        u64 x = oracle_modexp(c, e, q);
        if (oracle_modexp(x, m / 2, q) == q - 1) { psi = x; break; }
    }
    if (!psi) return 0;
    u64 psi2 = modmul_exact(psi, psi, q), x = psi, best = psi;
    for (u64 k = 3; k < m; k += 2) {
        x = modmul_exact(x, psi2, q);
        if (x < best && x != 1) best = x;
    }
    return best;
}

/* Modulus chain of the poly benchmarks, benchmark/src/poly-benchmark-16k.cpp:89-96:
 * q0 = PreviousPrime(FirstPrime(bits, 2N), 2N), q_{i+1} = PreviousPrime(q_i, 2N). */
int oracle_moduli_chain(unsigned bits, u64 cyclo_order, unsigned count, u64* q_out, u64* psi_out) {
    u64 q = oracle_first_prime(bits, cyclo_order);
    if (!q) return -1;
    for (unsigned i = 0; i < count; i++) {
        q = oracle_previous_prime(q, cyclo_order);
        if (!q) return -1;
        q_out[i] = q;
        if (psi_out) psi_out[i] = oracle_root_of_unity(cyclo_order, q);
    }
    return 0;
}

/* ---------------------------------------------------------------------------
 * NTT tables: ChineseRemainderTransformFTTNat::PreCompute,
 * src/core/include/math/hal/intnat/transformnat-impl.h:708-763.
 *   Table[rev(i)] = psi^i, TableI[rev(i)] = psi^-i (rev over log2 N bits),
 *   COI[i] = (2^i)^-1 mod q, i = 0..log2 N, and the Shoup precons of each.
 * ------------------------------------------------------------------------- */
static u64 rev_bits(u64 x, unsigned bits) {
    u64 r = 0;
    for (unsigned i = 0; i < bits; i++) { r = (r << 1) | (x & 1); x >>= 1; }
    return r;
}

int oracle_ntt_tables(u64 n, u64 q, u64 psi, u64* tab, u64* tab_pre, u64* itab, u64* itab_pre,
                      u64* coi, u64* coi_pre) {
    if (n < 2 || (n & (n - 1))) return -1;
    unsigned lg = oracle_msb(n - 1);
    u64 mu = oracle_compute_mu(q);
    u64 psi_inv = oracle_modinv(psi, q);
    u64 x = 1, xi = 1;
    for (u64 i = 0; i < n; i++) {
        u64 r = rev_bits(i, lg);
        tab[r] = x;
        itab[r] = xi;
        x = oracle_modmul_barrett(x, psi, q, mu);
        xi = oracle_modmul_barrett(xi, psi_inv, q, mu);
    }
    for (u64 i = 0; i < n; i++) {
        tab_pre[i] = oracle_shoup_prep(tab[i], q);
        itab_pre[i] = oracle_shoup_prep(itab[i], q);
    }
    if (coi) {
        for (unsigned i = 0; i <= lg; i++) {
            coi[i] = oracle_modinv(((u64)1 << i) % q, q);
            if (coi_pre) coi_pre[i] = oracle_shoup_prep(coi[i], q);
        }
    }
    return 0;
}

/* NumberTheoreticTransformNat::ForwardTransformToBitReverseInPlace(table, precon, x),
 * transformnat-impl.h:300-354 (GCC branch).  Natural order in, bit-reversed out. */
void oracle_ntt_fwd(u64* x, u64 len, u64 q, const u64* tab, const u64* tab_pre) {
    u64 n = len >> 1, t = n;
    unsigned logt = oracle_msb(t);
    for (u64 m = 1; m < n; m <<= 1, t >>= 1, --logt) {
        for (u64 i = 0; i < m; ++i) {
            u64 w = tab[i + m], wp = tab_pre[i + m];
            for (u64 j1 = i << logt, j2 = j1 + t; j1 < j2; ++j1) {
                u64 of = oracle_modmul_shoup(x[j1 + t], w, q, wp);
                u64 lo = x[j1];
                u64 hi = lo + of;
                if (hi >= q) hi -= q;
                if (lo < of) lo += q;
                lo -= of;
                x[j1] = hi;
                x[j1 + t] = lo;
            }
        }
    }
    for (u64 i = 0; i < (n << 1); i += 2) {
        u64 of = oracle_modmul_shoup(x[i + 1], tab[(i >> 1) + n], q, tab_pre[(i >> 1) + n]);
        u64 lo = x[i];
        u64 hi = lo + of;
        if (hi >= q) hi -= q;
        if (lo < of) lo += q;
        lo -= of;
        x[i] = hi;
        x[i + 1] = lo;
    }
}

/* NumberTheoreticTransformNat::InverseTransformFromBitReverseInPlace(tableI, preconI, nInv,
 * nInvPrecon, x), transformnat-impl.h:492-552 (GCC branch).  First GS stage fused with n^-1. */
void oracle_ntt_inv(u64* x, u64 n, u64 q, const u64* itab, const u64* itab_pre, u64 ninv,
                    u64 ninv_pre) {
    for (u64 i = 0; i < n; i += 2) {
        u64 w = itab[(i + n) >> 1], wp = itab_pre[(i + n) >> 1];
        u64 hi = x[i + 1], lo = x[i];
        u64 of = lo;
        if (of < hi) of += q;
        of -= hi;
        lo += hi;
        if (lo >= q) lo -= q;
        lo = oracle_modmul_shoup(lo, ninv, q, ninv_pre);
        of = oracle_modmul_shoup(of, w, q, wp);
        of = oracle_modmul_shoup(of, ninv, q, ninv_pre);
        x[i] = lo;
        x[i + 1] = of;
    }
    for (u64 m = n >> 2, t = 2, logt = 2; m >= 1; m >>= 1, t <<= 1, ++logt) {
        for (u64 i = 0; i < m; ++i) {
            u64 w = itab[i + m], wp = itab_pre[i + m];
            for (u64 j1 = i << logt, j2 = j1 + t; j1 < j2; ++j1) {
                u64 hi = x[j1 + t], lo = x[j1];
                u64 of = lo;
                if (of < hi) of += q;
                of -= hi;
                lo += hi;
                if (lo >= q) lo -= q;
                of = oracle_modmul_shoup(of, w, q, wp);
                x[j1] = lo;
                x[j1 + t] = of;
            }
        }
    }
}

/* ---------------------------------------------------------------------------
 * Vector ops, src/core/include/math/hal/intnat/mubintvecnat.h:426-432,501-513 and
 * src/core/lib/math/hal/intnat/mubintvecnat.cpp:245-367.
 * ------------------------------------------------------------------------- */
void oracle_vec_modmul(const u64* a, const u64* b, u64* c, u64 n, u64 q) {
    u64 mu = oracle_compute_mu(q);
    for (u64 i = 0; i < n; i++) c[i] = oracle_modmul_barrett(a[i], b[i], q, mu);
}
void oracle_vec_modadd(const u64* a, const u64* b, u64* c, u64 n, u64 q) {
    for (u64 i = 0; i < n; i++) c[i] = oracle_modadd(a[i], b[i], q);
}
void oracle_vec_modsub(const u64* a, const u64* b, u64* c, u64 n, u64 q) {
    for (u64 i = 0; i < n; i++) c[i] = oracle_modsub(a[i], b[i], q);
}
/* scalar ModMul(Eq), mubintvecnat.cpp:310-332 (Shoup with precomputed constant). */
void oracle_vec_modmul_scalar(const u64* a, u64 s, u64* c, u64 n, u64 q) {
    if (s >= q) s %= q;
    u64 sp = oracle_shoup_prep(s, q);
    for (u64 i = 0; i < n; i++) c[i] = oracle_modmul_shoup(a[i], s, q, sp);
}
/* scalar ModAdd(Eq) / ModSub(Eq), mubintvecnat.cpp:198-219, 267-288: the scalar is
 * reduced (ModEq) when >= q, then ModAddFast / ModSubFastEq per element. */
void oracle_vec_modadd_scalar(const u64* a, u64 s, u64* c, u64 n, u64 q) {
    if (s >= q) s %= q;
    for (u64 i = 0; i < n; i++) c[i] = oracle_modadd(a[i], s, q);
}
void oracle_vec_modsub_scalar(const u64* a, u64 s, u64* c, u64 n, u64 q) {
    if (s >= q) s %= q;
    for (u64 i = 0; i < n; i++) c[i] = oracle_modsub(a[i], s, q);
}

/* ---------------------------------------------------------------------------
 * DCRT (towers) level, [B][T][N] contiguous, OpenMP over (batch, tower) as the
 * reference's DCRTPolyImpl::SwitchFormat / Times do over towers
 * (src/core/include/lattice/hal/default/dcrtpoly-impl.h:2518-2524,
 *  dcrtpoly.h:185-200).  tables: [T][N] each; coi: [T] = n^-1 and its precon.
 * ------------------------------------------------------------------------- */
void oracle_dcrt_ntt_fwd(u64* x, u64 batch, u64 n, unsigned towers, const u64* q, const u64* tab,
                         const u64* tab_pre) {
    long long total = (long long)(batch * towers);
#pragma omp parallel for schedule(static)
    for (long long bt = 0; bt < total; bt++) {
        unsigned t = (unsigned)(bt % towers);
        oracle_ntt_fwd(x + (u64)bt * n, n, q[t], tab + (u64)t * n, tab_pre + (u64)t * n);
    }
}

void oracle_dcrt_ntt_inv(u64* x, u64 batch, u64 n, unsigned towers, const u64* q, const u64* itab,
                         const u64* itab_pre, const u64* ninv, const u64* ninv_pre) {
    long long total = (long long)(batch * towers);
#pragma omp parallel for schedule(static)
    for (long long bt = 0; bt < total; bt++) {
        unsigned t = (unsigned)(bt % towers);
        oracle_ntt_inv(x + (u64)bt * n, n, q[t], itab + (u64)t * n, itab_pre + (u64)t * n, ninv[t],
                       ninv_pre[t]);
    }
}

/* The metric op: c = INTT(NTT(a) (.) b) per (batch, tower); a in coefficient
 * form, b in evaluation form (poly-benchmark semantics). */
void oracle_dcrt_ntt_mul_intt(const u64* a, const u64* b, u64* c, u64 batch, u64 n, unsigned towers,
                              const u64* q, const u64* tab, const u64* tab_pre, const u64* itab,
                              const u64* itab_pre, const u64* ninv, const u64* ninv_pre) {
    long long total = (long long)(batch * towers);
#pragma omp parallel for schedule(static)
    for (long long bt = 0; bt < total; bt++) {
        unsigned t = (unsigned)(bt % towers);
        u64* x = c + (u64)bt * n;
        if (x != a + (u64)bt * n) memcpy(x, a + (u64)bt * n, n * sizeof(u64));
        oracle_ntt_fwd(x, n, q[t], tab + (u64)t * n, tab_pre + (u64)t * n);
        oracle_vec_modmul(x, b + (u64)bt * n, x, n, q[t]);
        oracle_ntt_inv(x, n, q[t], itab + (u64)t * n, itab_pre + (u64)t * n, ninv[t], ninv_pre[t]);
    }
}

/* op: 0 modmul (Barrett), 1 modadd, 2 modsub; [B][T][N]. */
void oracle_dcrt_eltwise(int op, const u64* a, const u64* b, u64* c, u64 batch, u64 n,
                         unsigned towers, const u64* q) {
    long long total = (long long)(batch * towers);
#pragma omp parallel for schedule(static)
    for (long long bt = 0; bt < total; bt++) {
        unsigned t = (unsigned)(bt % towers);
        u64 off = (u64)bt * n;
        if (op == 0) oracle_vec_modmul(a + off, b + off, c + off, n, q[t]);
        else if (op == 1) oracle_vec_modadd(a + off, b + off, c + off, n, q[t]);
        else oracle_vec_modsub(a + off, b + off, c + off, n, q[t]);
    }
}

/* ---------------------------------------------------------------------------
 * RNS base conversion: DCRTPolyImpl::ApproxSwitchCRTBasis,
 * src/core/include/lattice/hal/default/dcrtpoly-impl.h:1034-1063, with Mul128 and
 * BarrettUint128ModUint64 from src/core/include/utils/utilities-int.h:47-103.
 * x: [sizeQ][N] (coefficient form), out: [sizeP][N].
 * qhat_modp: [sizeQ][sizeP] row-major; mu_lo/mu_hi: floor(2^128 / p_j).
 * ------------------------------------------------------------------------- */
static u64 barrett_u128_mod_u64(u128 a, u64 m, u128 mu) {
    /* (a * mu) >> 128, keeping only the low word, as the reference does */
    u64 a_lo = (u64)a, a_hi = (u64)(a >> 64), mu_lo = (u64)mu, mu_hi = (u64)(mu >> 64);
    u64 left_hi = (u64)(((u128)a_lo * mu_lo) >> 64);
    u128 mid = (u128)a_lo * mu_hi;
    u64 mid_lo = (u64)mid, mid_hi = (u64)(mid >> 64);
    u64 tmp1 = mid_lo + left_hi;
    u64 carry = tmp1 < mid_lo;
    u64 tmp2 = mid_hi + carry;
    mid = (u128)a_hi * mu_lo;
    mid_lo = (u64)mid;
    mid_hi = (u64)(mid >> 64);
    u64 s = mid_lo + tmp1;
    carry = s < mid_lo;
    left_hi = mid_hi + carry;
    tmp1 = a_hi * mu_hi + tmp2 + left_hi;
    u64 r = a_lo - tmp1 * m;
    while (r >= m) r -= m;
    return r;
}

void oracle_approx_switch_crt_basis(const u64* x, u64* out, u64 n, unsigned sizeQ, unsigned sizeP,
                                    const u64* q, const u64* p, const u64* qhatinv_modq,
                                    const u64* qhatinv_modq_pre, const u64* qhat_modp,
                                    const u64* mu_lo, const u64* mu_hi) {
#pragma omp parallel
    {
        u128* sum = (u128*)malloc(sizeof(u128) * (sizeP ? sizeP : 1));
#pragma omp for schedule(static)
        for (long long ri = 0; ri < (long long)n; ri++) {
            for (unsigned j = 0; j < sizeP; j++) sum[j] = 0;
            for (unsigned i = 0; i < sizeQ; i++) {
                u64 y = oracle_modmul_shoup(x[(u64)i * n + ri], qhatinv_modq[i], q[i],
                                            qhatinv_modq_pre[i]);
                for (unsigned j = 0; j < sizeP; j++) sum[j] += (u128)y * qhat_modp[(u64)i * sizeP + j];
            }
            for (unsigned j = 0; j < sizeP; j++) {
                u128 mu = ((u128)mu_hi[j] << 64) | mu_lo[j];
                out[(u64)j * n + ri] = barrett_u128_mod_u64(sum[j], p[j], mu);
            }
        }
        free(sum);
    }
}

/* Precomputations for ApproxSwitchCRTBasis as the pke layer builds them
 * (src/pke/lib/schemerns/rns-cryptoparameters.cpp:273-337):
 *   QHatInvModq[i] = (Q/q_i)^-1 mod q_i, QHatModp[i][j] = (Q/q_i) mod p_j,
 *   mu_j = floor(2^128 / p_j). */
void oracle_base_conv_precompute(unsigned sizeQ, unsigned sizeP, const u64* q, const u64* p,
                                 u64* qhatinv_modq, u64* qhatinv_modq_pre, u64* qhat_modp,
                                 u64* mu_lo, u64* mu_hi) {
    for (unsigned i = 0; i < sizeQ; i++) {
        u64 prod = 1 % q[i];
        for (unsigned k = 0; k < sizeQ; k++)
            if (k != i) prod = modmul_exact(prod, q[k] % q[i], q[i]);
        qhatinv_modq[i] = oracle_modinv(prod, q[i]);
        qhatinv_modq_pre[i] = oracle_shoup_prep(qhatinv_modq[i], q[i]);
        for (unsigned j = 0; j < sizeP; j++) {
            u64 pr = 1 % p[j];
            for (unsigned k = 0; k < sizeQ; k++)
                if (k != i) pr = modmul_exact(pr, q[k] % p[j], p[j]);
            qhat_modp[(u64)i * sizeP + j] = pr;
        }
    }
    for (unsigned j = 0; j < sizeP; j++) {
        u128 mu = (~(u128)0) / p[j]; /* == floor(2^128/p) for odd p > 1 */
        mu_lo[j] = (u64)mu;
        mu_hi[j] = (u64)(mu >> 64);
    }
}

/* PolyImpl::AutomorphismTransform(k), X -> X^k for odd k, one tower of n
 * words (src/core/include/lattice/hal/default/poly-impl.h:312-365):
 * evaluation form permutes the bit-reversed slots, out[rev(j)] =
 * x[rev(((j*2k + k) mod 2^32 >> 1) & (n-1))]; coefficient form maps
 * coefficient j to (j*k) mod n, negated (q - x, so a zero becomes q as in the
 * reference) when bit log n of the 32-bit j*k is set.  k must be odd. */
void oracle_automorphism(const u64* x, u64* out, u64 n, uint32_t k, int eval_form, u64 q) {
    const unsigned logn = oracle_msb(n) - 1;
    const uint32_t mask = (uint32_t)n - 1;
    if (eval_form) {
        uint32_t jk = k;
        for (uint32_t j = 0; j < (uint32_t)n; j++, jk += 2 * k)
            out[rev_bits(j, logn)] = x[rev_bits((jk >> 1) & mask, logn)];
        return;
    }
    uint32_t jk = 0;
    for (uint32_t j = 0; j < (uint32_t)n; j++, jk += k)
        out[jk & mask] = ((jk >> logn) & 1u) ? q - x[j] : x[j];
}

/* ---------------------------------------------------------------------------
 * Deterministic synthetic inputs and fingerprints.
 * ------------------------------------------------------------------------- */
/* splitmix64: s += 0x9E3779B97F4A7C15; z = mix(s). */
u64 oracle_splitmix64(u64* s) {
    u64 z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* x_i = sm() % q, i = 0..n-1, continuing the stream in *state. */
void oracle_fill_uniform(u64* x, u64 n, u64 q, u64* state) {
    for (u64 i = 0; i < n; i++) x[i] = oracle_splitmix64(state) % q;
}

/* word-wise FNV-1a over 64-bit words */
u64 oracle_fnv64(const u64* x, u64 n) {
    u64 h = 0xcbf29ce484222325ull;
    for (u64 i = 0; i < n; i++) { h ^= x[i]; h *= 0x100000001b3ull; }
    return h;
}

void oracle_set_threads(int n) {
#ifdef _OPENMP
    omp_set_num_threads(n > 0 ? n : 1);
#else
    (void)n;
#endif
}

int oracle_num_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}
