// ntt_kernels.hpp -- negacyclic NTT / INTT / fused pipeline kernels for gfx950.
//
// Algorithm (the reference's, restated; transformnat-impl.h:300-354, 492-552):
//   forward, Cooley-Tukey, natural -> bit-reversed: for m = 1, 2, ..., N/2 with
//   t = N/(2m), every pair (j, j+t) in group i = j/(2t) becomes
//   (x_j + w x_{j+t}, x_j - w x_{j+t}) with w = Table[m + i];
//   inverse, Gentleman-Sande: m = N/2 ... 1 (t = 1 ... N/2),
//   (x_j + x_{j+t}, (x_j - x_{j+t}) * TableI[m + i]), with n^-1 fused into the
//   first (t = 1) stage.  Here the inverse's first stages (those inside the
//   block pass) run as a cyclic decimation-in-time transform plus a twist --
//   the same values, see dit_round3() below -- and its column-pass stages as
//   the reference's GS.
// Values stay lazily reduced between stages (forward and DIT in [0, 16q),
// GS in [0, 8q) with compile-time bounds per register, OFHE_LAZY_GS) and are
// made canonical on output, so results equal the
// reference bit for bit (its outputs are the canonical residues).
//
// Decomposition for N = 2^logN >= 2^12 (one tower = 512 KiB at 2^16, more
// than a CU's 160 KiB LDS):
//   column pass: the first logN-12 stages (k_cols: each thread owns one or
//             two "columns" {c + 4096 k}, all butterflies in registers), or at
//             N = 2^16 the first 8 stages on 16-column x 256-row tiles
//             (k_tcols);
//   k_block : the last 12 (8 at N = 2^16) stages on contiguous 4096-element
//             blocks (34 KiB of LDS per workgroup): rounds of 4 radix-2
//             stages held in registers (16 values per thread), padded LDS
//             exchanges between rounds (see lds_pad()).
//   The metric pipeline runs column pass (fwd) -> k_block (fwd + Hadamard +
//   inverse) -> column pass (inv): the Hadamard and the block stages of both
//   directions share one residency.
// N <= 2^11 uses k_small (whole tower in LDS, one stage per step).
// Every kernel is instantiated for generic moduli (SPQ = false) and for
// moduli q = 2^L - d, d < 2^32 (SPQ = true, one fewer multiply per Shoup).
#pragma once
#include "arith.hpp"

namespace ofhe {

struct TowerConst {
    u64 q;
    u64 ninv;      // N^-1 mod q
    u64 ninv_pre;  // Shoup precon of ninv
    u64 mu;        // ComputeMu() for Barrett (ubintnat.h:651-656)
    u64 nq;        // 2^64 - q   (loaded, not derived: keeps LLVM from turning
    u64 nq4;       // 2^64 - 4q   the lazy adds back into carry-chain subtractions)
    u32 nshift;    // msb(q) - 2
    u32 spq_sh;    // msb(q) - 32 when q = 2^msb - d with d < 2^32, else 0
    u64 qinv;      // q^-1 mod 2^64 (Montgomery Hadamard)
    u32 one;       // 1, loaded so LLVM cannot fold it (Mod::one, mulhi_approx)
    u32 pad_;
};
// Shoup quotient form per kernel (Mod<SPQ, QA>, arith.hpp): add_co/addc into
// the accumulator pair (1) or zero-extending moves and a 64-bit add (0).
// Same-process A/B (tools/exp_variants.py) decides each default.
#ifndef OFHE_QA_TCF
#define OFHE_QA_TCF 0  // k_tcols forward
#endif
#ifndef OFHE_QA_TCI
#define OFHE_QA_TCI 0  // k_tcols inverse
#endif
#ifndef OFHE_QA_BLK
#define OFHE_QA_BLK 0  // k_block
#endif
#ifndef OFHE_QA_CF
#define OFHE_QA_CF 0  // k_cols forward
#endif
#ifndef OFHE_QA_CI
#define OFHE_QA_CI 0  // k_cols inverse
#endif
#ifndef OFHE_QA_BCC
#define OFHE_QA_BCC 0  // k_bconv_cols
#endif
template <bool SPQ, bool QA = false>
__device__ __forceinline__ Mod<SPQ, QA> load_mod(const TowerConst& tc) {
    return Mod<SPQ, QA>{tc.q, 4 * tc.q, 8 * tc.q, tc.nq, tc.nq4, 0 - 8 * tc.q, tc.spq_sh, tc.one};
}

// Device view of a plan. Twiddles are interleaved (w, w') pairs so one
// 16-byte load fetches a twiddle and its Shoup precon.
struct PlanArgs {
    const TowerConst* tc;  // [T]
    const u64* tw;         // [T][N][2]   forward Table (bit-reversed powers of psi)
    const u64* itw;        // [T][N][2]   inverse TableI (GS column passes)
    const u64* tw3;        // [T][15N/16][2] round-3 forward twiddles, lane-contiguous (log_n >= 12)
    u64 sstride;           // words between batch entries of src (towers * N when dense)
    u64 dstride;           // words between batch entries of dst (and of the Hadamard operand)
    u64 bstride;           // words between batch entries of the second operand (bdat)
    const u64* scal;       // MODE_FWD_SUB: [towers][3] = (q, s, s') per tower of the range
    const u64* dtw;        // [T][N][2]   DIT inverse twiddles: dtw[t + k] = psi^(-k N / t), k < t
    const u64* twist;      // [T][N][2]   output twist N^-1 psi^-j (times 2^64 mod q for the fused pipeline)
    u32 log_n;
    u32 towers;            // towers in this launch (a plan range starts at tc[0])
};

// MODE_FWD_SUB: forward transform whose output is (x - NTT(y)) * s_t mod q,
// the last step of ApproxModDown (dcrtpoly-impl.h:1167-1173) fused into the
// block pass (x = bdat with batch stride bstride, (s, s') per tower in scal).
enum { MODE_FWD = 0, MODE_INV = 1, MODE_FUSED = 2, MODE_FWD_SUB = 3 };

// Bijective XCD-aware block remap (cdna_hip_programming.md T1): consecutive
// work items land on the same XCD.
__device__ __forceinline__ u32 xcd_remap(u32 bid, u32 nwg) {
    u32 q = nwg >> 3, r = nwg & 7, xcd = bid & 7, loc = bid >> 3;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
}

struct Tw {
    u64 w, wp;
};

// Streaming (non-temporal) access for polynomial data, so that the data
// streaming through L2 does not evict the twiddles every block re-reads
// (OFHE_NT, A/B switch).
#ifndef OFHE_NT
#define OFHE_NT 1
#endif
typedef u64 u64x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u64 ld_s(const u64* p) { return OFHE_NT ? __builtin_nontemporal_load(p) : *p; }
__device__ __forceinline__ void st_s(u64* p, u64 v) {
    if (OFHE_NT)
        __builtin_nontemporal_store(v, p);
    else
        *p = v;
}
__device__ __forceinline__ u64x2 ld2_s(const u64* p) {
    const u64x2* q = reinterpret_cast<const u64x2*>(p);
    return OFHE_NT ? __builtin_nontemporal_load(q) : *q;
}
__device__ __forceinline__ void st2_s(u64* p, u64x2 v) {
    u64x2* q = reinterpret_cast<u64x2*>(p);
    if (OFHE_NT)
        __builtin_nontemporal_store(v, q);
    else
        *q = v;
}
// OFHE_ABL_NOTW (ablation builds only, wrong results): twiddles from
// registers instead of memory, to measure what the loads cost.
__device__ __forceinline__ Tw ldtw(const u64* base, u32 idx) {
#ifdef OFHE_ABL_NOTW
    const u64 f = (u64)(uintptr_t)base ^ idx;
    return Tw{f & 0x0fffffffffffffffull, f * 0x9E3779B97F4A7C15ull};
#else
    const ulonglong2 v = *reinterpret_cast<const ulonglong2*>(base + 2 * (u64)idx);
    return Tw{v.x, v.y};
#endif
}

// Cooley-Tukey butterfly.  Two lazy-reduction schemes (OFHE_LAZY_FWD):
//  0: every stage subtracts 4q from x when x >= 4q; values stay in [0, 8q).
//  1: stages alternate.  A "CS" stage (odd stage of a radix-16 round, the
//     last stage of a column pass) subtracts 8q when x >= 8q and maps
//     [0, 16q) -> [0, 12q); the other stages skip the conditional subtract and
//     map [0, 12q) -> [0, 16q).  16q <= 2^64 because q < 2^60, and shoup_lazy
//     accepts any 64-bit input, so half of the butterflies save the compare,
//     two selects and the 64-bit subtract.
#ifndef OFHE_LAZY_FWD
#define OFHE_LAZY_FWD 1
#endif
// OFHE_THR (special primes q = 2^L - d only): the CS stages subtract 8q when
// bit L+3 of x is set instead of comparing with 8q: one bit-field extract and
// two ANDs build the mask, one 64-bit add applies it -- no compare, no VCC,
// no selects.  2^(L+3) > 8q, so the invariant becomes [0, 2^(L+3) + 8q)
// (< 2^(L+4) <= 2^64, where the bit test is exact); canon_fwd takes one more
// conditional subtract.  Measured 3 % slower in the block pass despite the
// shorter instruction stream (tools/exp_variants.py), so it is off.
#ifndef OFHE_THR
#define OFHE_THR 0
#endif
template <bool SPQ, bool QA>
__device__ __forceinline__ u64 csub_thr8(u64 x, const Mod<SPQ, QA>& M) {
    const u32 m = (u32)__builtin_amdgcn_sbfe((int)hi32(x), M.sh + 3, 1);
    return x + pack(m & lo32(M.nq8), m & hi32(M.nq8));
}
// OFHE_FOLD (special primes): the lazy reductions [0, 16q) -> [0, 8q) (CS
// stages, GS sums) use fold_spq (3 instructions, result < 2q) instead of the
// conditional subtract (4).  OFHE_BFLY_ACC: the butterfly's x + w y is the
// Shoup product with x as the addend of its first multiply-add, and
// x - w y = (2x + 4q) - (x + w y): one 64-bit add fewer per butterfly.
#ifndef OFHE_FOLD
#define OFHE_FOLD 1
#endif
#ifndef OFHE_BFLY_ACC
#define OFHE_BFLY_ACC 1
#endif
// [0, 16q) -> [0, 8q) ([0, 2q) by the fold)
template <bool SPQ, bool QA>
__device__ __forceinline__ u64 red16(u64 x, const Mod<SPQ, QA>& M) {
    if (SPQ && OFHE_FOLD) return fold_spq(x, M);
    return csub_s(x, M.q8);
}
// The Gentleman-Sande sums keep the conditional subtract by default
// (OFHE_FOLD_GS=0): same-process A/B, the inverse column pass was 1 % slower
// with the fold there (profiles/r04a_fold_acc_ab.txt, r04b_qh2_ab.txt).
#ifndef OFHE_FOLD_GS
#define OFHE_FOLD_GS 0
#endif
// [0, 8q) -> [0, 4q) ([0, 2q) by the fold)
template <bool SPQ, bool QA>
__device__ __forceinline__ u64 red8(u64 x, const Mod<SPQ, QA>& M) {
    if (SPQ && OFHE_FOLD && OFHE_FOLD_GS) return fold_spq(x, M);
    return csub_s(x, M.q4);
}
// GS sums [0, 16q) -> [0, 8q)
template <bool SPQ, bool QA>
__device__ __forceinline__ u64 red16_gs(u64 x, const Mod<SPQ, QA>& M) {
    if (SPQ && OFHE_FOLD && OFHE_FOLD_GS) return fold_spq(x, M);
    return csub_s(x, M.q8);
}
template <bool SPQ, bool QA>
__device__ __forceinline__ void ct_bfly_cs(u64& x, u64& y, Tw w, const Mod<SPQ, QA>& M, bool cs) {
    u64 a;
    if (OFHE_LAZY_FWD)
        a = cs ? ((SPQ && OFHE_THR) ? csub_thr8(x, M) : red16(x, M)) : x;
    else
        a = csub_s(x, M.q4);
    if (OFHE_BFLY_ACC == 2) {
        const u64 c2 = (a << 1) + M.q4;          // computed first: a dies in the mad chain
        x = shoup_lazy_acc(y, w.w, w.wp, M, a);  // a + [0, 4q)
        y = c2 - x;                              // a + 4q - [0, 4q)
    } else if (OFHE_BFLY_ACC) {
        x = shoup_lazy_acc(y, w.w, w.wp, M, a);  // a + [0, 4q)
        y = (a << 1) + M.q4 - x;                 // a + 4q - [0, 4q)
    } else {
        const u64 t = shoup_lazy(y, w.w, w.wp, M);  // [0, 4q)
        x = a + t;
        y = a + M.q4 - t;
    }
}
template <int CS, class M_>
__device__ __forceinline__ void ct_bfly(u64& x, u64& y, Tw w, const M_& M) {
    ct_bfly_cs(x, y, w, M, CS != 0);
}

// Gentleman-Sande butterfly, inputs in [0, 4q), outputs in [0, 4q).
template <class M_>
__device__ __forceinline__ void gs_bfly(u64& x, u64& y, Tw w, const M_& M) {
    const u64 s = x + y;          // [0, 8q)
    const u64 d = x + M.q4 - y;   // (0, 8q)
    x = red8(s, M);
    y = shoup_lazy(d, w.w, w.wp, M);  // [0, 4q)
}

__device__ __forceinline__ u64 canon8(u64 x, u64 q) {  // [0, 8q) -> [0, q)
    x = csub_s(x, 4 * q);
    x = csub_s(x, 2 * q);
    return csub_s(x, q);
}
__device__ __forceinline__ u64 canon4(u64 x, u64 q) {  // [0, 4q) -> [0, q)
    x = csub_s(x, 2 * q);
    return csub_s(x, q);
}
// Special prime q = 2^L - d (plan condition: d < 2^32 and 16 d < q): any
// x < 2^(L+4) -> [0, q) with one quotient by shift.  qh = x >> L < 16,
// r = (x mod 2^L) + qh d = x - qh q < 2^L + 15 d = q + 16 d < 2q, one
// conditional subtract: 3 + 4 instructions against 12 (canon8) or 16 (canon_fwd).
#ifndef OFHE_SPQ_CANON
#define OFHE_SPQ_CANON 1
#endif
template <bool SPQ, bool QA>
__device__ __forceinline__ u64 canon_spq(u64 x, const Mod<SPQ, QA>& M) {
    const u32 qh = hi32(x) >> M.sh;
    const u64 d = (1ull << (M.sh + 32)) - M.q;  // wave-uniform (scalar unit)
    const u64 xm = pack(lo32(x), hi32(x) & ((1u << M.sh) - 1));
    return csub_s(mad32(qh, lo32(d), xm), M.q);
}
template <bool SPQ, bool QA>
__device__ __forceinline__ u64 canon8m(u64 x, const Mod<SPQ, QA>& M) {  // [0, 8q) -> [0, q)
    return (SPQ && OFHE_SPQ_CANON) ? canon_spq(x, M) : canon8(x, M.q);
}
template <bool SPQ, bool QA>
__device__ __forceinline__ u64 canon4m(u64 x, const Mod<SPQ, QA>& M) {  // [0, 4q) -> [0, q)
    return (SPQ && OFHE_SPQ_CANON) ? canon_spq(x, M) : canon4(x, M.q);
}
// forward-transform output (any stage pattern) -> [0, q)
template <bool SPQ, bool QA>
__device__ __forceinline__ u64 canon_fwd(u64 x, const Mod<SPQ, QA>& M) {
    if (SPQ && OFHE_SPQ_CANON && !OFHE_THR) return canon_spq(x, M);  // < 16q < 2^(L+4)
    const u64 q = M.q;
    if (SPQ && OFHE_THR) x = csub_s(x, 8 * q);  // [0, 2^(L+3) + 8q) -> [0, 8q + 8d)
    if (OFHE_LAZY_FWD) x = csub_s(x, 8 * q);    // [0, 16q) -> [0, 8q)
    return canon8(x, q);
}

// ---------------------------------------------------------------------------
// Inverse transform as a cyclic decimation-in-time NTT plus an output twist
// The reference's inverse (GS, transformnat-impl.h:492-552) is
//   a_j = N^-1 psi^-j sum_k Y[k] omega^-kj,   omega = psi^2, Y[k] = y[rev(k)],
// and the sum over the bit-reversed input y is the textbook iterative
// Cooley-Tukey DIT: stages t = 1, 2, ..., N/2 pair (e, e + t) as
// (x + w y, x - w y) with w = psi^(-(e mod t) N / t) = dtw[t + e mod t].
// Compared with the merged-twist GS form this
//   * uses the cheaper CT butterfly (lazy, alternating reduction as forward);
//   * has trivial twiddles (w = 1) at e mod t = 0: every butterfly of stage
//     t = 1, half of t = 2, ... -- and in the block pass's last round (t <= 8)
//     they sit at fixed register positions, so they cost two adds;
//   * gives that round wave-uniform twiddles (11 scalars per tower);
// The block pass runs the DIT stages inside its groups of G = 2^lb elements
// (lb = block_stages(plan split), internal.hpp); the GS column pass (unchanged)
// runs the rest.  They meet because the GS intermediate after its first lb
// stages is, for group b and position j0 (checked numerically),
//   W_b[j0] = psi^-((2 rev(b) + 1) j0) * Z_b[j0],
// Z_b = the group's cyclic DIT output, rev over logN - lb bits; so the block
// pass ends with the per-element twist N^-1 psi^-((2 rev(b) + 1) j0) (N^-1
// moves here from GS's first stage; for G = N it is N^-1 psi^-j).  Same
// canonical outputs, bit for bit.
// ---------------------------------------------------------------------------
static_assert(OFHE_LAZY_FWD, "the DIT inverse uses the alternating lazy CT butterflies");

// x + y and x + B q - y for y < B q (B q passed as bq): the w = 1 butterfly
__device__ __forceinline__ void triv_bfly(u64& x, u64& y, u64 bq) {
    const u64 s = x + y;
    y = x + bq - y;
    x = s;
}

// DIT stage of a radix-16 register round with element stride st: the thread
// holds v[k] = x[p0 + k st], r = p0 mod st; half = 2^H pairs (k, k + half),
// twiddle index st half + r + st (k mod half) -- base points at entry
// st half + r.  CS: conditional-subtract stage (inputs < 16q, else < 12q).
template <int H, int CS, class M_>
__device__ __forceinline__ void dit_stage16(u64 (&v)[16], const u64* base, u32 st, const M_& M) {
    constexpr int half = 1 << H;
#pragma unroll
    for (int j = 0; j < half; j++) {
        const Tw w = ldtw(base, st * j);
#pragma unroll
        for (int g = 0; g < 16; g += 2 * half) ct_bfly<CS>(v[g + j], v[g + j + half], w, M);
    }
}
template <class M_>
__device__ __forceinline__ void dit_round16(u64 (&v)[16], const u64* dtw, u32 st, u32 r, const M_& M) {
    dit_stage16<0, 1>(v, dtw + 2 * ((u64)st + r), st, M);
    dit_stage16<1, 0>(v, dtw + 2 * ((u64)2 * st + r), st, M);
    dit_stage16<2, 1>(v, dtw + 2 * ((u64)4 * st + r), st, M);
    dit_stage16<3, 0>(v, dtw + 2 * ((u64)8 * st + r), st, M);
}

// The first four DIT stages (t = 1, 2, 4, 8) on 16 consecutive elements, inputs
// < 2q (the Montgomery Hadamard's (0, 2q) or canonical data): twiddles
// dtw[t + j] are the same for every thread, j = 0 is w = 1.
//   t = 1: all trivial, -> < 4q;  t = 2: -> < 8q;  t = 4: -> < 16q (trivial)
//   / < 12q;  t = 8: conditional subtract first, -> < 16q.
template <bool SPQ, bool QA>
__device__ __forceinline__ void dit_round3(u64 (&v)[16], const u64* dtw, const Mod<SPQ, QA>& M) {
#pragma unroll
    for (int g = 0; g < 16; g += 2) triv_bfly(v[g], v[g + 1], 2 * M.q);
#pragma unroll
    for (int g = 0; g < 16; g += 4) triv_bfly(v[g], v[g + 2], M.q4);
    {
        const Tw w = ldtw(dtw, 3);
#pragma unroll
        for (int g = 0; g < 16; g += 4) ct_bfly<0>(v[g + 1], v[g + 3], w, M);
    }
#pragma unroll
    for (int g = 0; g < 16; g += 8) triv_bfly(v[g], v[g + 4], M.q8);
#pragma unroll
    for (int j = 1; j < 4; j++) {
        const Tw w = ldtw(dtw, 4 + j);
#pragma unroll
        for (int g = 0; g < 16; g += 8) ct_bfly<0>(v[g + j], v[g + j + 4], w, M);
    }
    {
        const u64 a = red16(v[0], M), b = red16(v[8], M);
        v[0] = a;
        v[8] = b;
        triv_bfly(v[0], v[8], M.q8);
    }
#pragma unroll
    for (int j = 1; j < 8; j++) ct_bfly<1>(v[j], v[j + 8], ldtw(dtw, 8 + j), M);
}

// last step of every inverse: x * N^-1 psi^-j (the twist entry f) -> [0, q)
template <bool SPQ, bool QA>
__device__ __forceinline__ u64 twist_out(u64 x, Tw f, const Mod<SPQ, QA>& M) {
    return canon4m(shoup_lazy(x, f.w, f.wp, M), M);
}

// ---------------------------------------------------------------------------
// Register radix-16 rounds.  A thread holds v[k] = x[p0 + k*st], k < 16, where
// p0 = hb*16*st + r (r < st).  Stage s (s = 0..3, t = st * 2^(3-s)) pairs
// (k, k + 2^(3-s)); its twiddle index is 2^s * M0 + (k >> (4 - s)) with
// M0 = N/(16 st) + (global index of the 16*st super-group).
// ---------------------------------------------------------------------------
template <int S, class M_, int CS = S & 1>
__device__ __forceinline__ void fwd_stage16(u64 (&v)[16], const u64* tw, u32 M0, const M_& M) {
    constexpr int half = 8 >> S;
    const u64* base = tw + 2 * ((u64)M0 << S);  // one address per stage, j as immediate offsets
#pragma unroll
    for (int j = 0; j < (1 << S); j++) {
        Tw w = ldtw(base, j);
#pragma unroll
        for (int k = j * 2 * half; k < j * 2 * half + half; k++) ct_bfly<CS>(v[k], v[k + half], w, M);
    }
}

template <int S, class M_>
__device__ __forceinline__ void inv_stage16(u64 (&v)[16], const u64* itw, u32 M0, const M_& M) {
    constexpr int half = 8 >> S;
    const u64* base = itw + 2 * ((u64)M0 << S);
#pragma unroll
    for (int j = 0; j < (1 << S); j++) {
        Tw w = ldtw(base, j);
#pragma unroll
        for (int k = j * 2 * half; k < j * 2 * half + half; k++) gs_bfly(v[k], v[k + half], w, M);
    }
}

// Lazy GS radix-16 round for the inverse column pass (OFHE_LAZY_GS).  The
// bound of every register is known at compile time (b8[k]: < 8q, else < 4q):
// a GS butterfly's sum output is < 8q and its Shoup output < 4q whatever the
// inputs, so only butterflies with an 8q input take the conditional subtract
// (12 of 32 in a round fed with < 4q, 20 of 32 fed with < 8q) and the rest
// add straight through.  d = x + Bq - y < 16q <= 2^64 (q < 2^60).
#ifndef OFHE_LAZY_GS
#define OFHE_LAZY_GS 1
#endif
template <class M_>
__device__ __forceinline__ void gs_bfly_b(u64& x, u64& y, Tw w, const M_& M, bool in8) {
    const u64 s = x + y;
    const u64 d = x + (in8 ? M.q8 : M.q4) - y;
    x = in8 ? red16_gs(s, M) : s;
    y = shoup_lazy(d, w.w, w.wp, M);
}
template <int S, class M_>
__device__ __forceinline__ void inv_stage16_b(u64 (&v)[16], bool (&b8)[16], const u64* itw, u32 M0, const M_& M) {
    constexpr int half = 8 >> S;
    const u64* base = itw + 2 * ((u64)M0 << S);
#pragma unroll
    for (int j = 0; j < (1 << S); j++) {
        Tw w = ldtw(base, j);
#pragma unroll
        for (int k = j * 2 * half; k < j * 2 * half + half; k++) {
            gs_bfly_b(v[k], v[k + half], w, M, b8[k] || b8[k + half]);
            b8[k] = true;
            b8[k + half] = false;
        }
    }
}
template <class M_>
__device__ __forceinline__ void inv_round16_b(u64 (&v)[16], bool (&b8)[16], const u64* itw, u32 M0, const M_& M) {
    inv_stage16_b<3>(v, b8, itw, M0, M);
    inv_stage16_b<2>(v, b8, itw, M0, M);
    inv_stage16_b<1>(v, b8, itw, M0, M);
    inv_stage16_b<0>(v, b8, itw, M0, M);
}

template <class M_>
__device__ __forceinline__ void fwd_round16(u64 (&v)[16], const u64* tw, u32 M0, const M_& M) {
    fwd_stage16<0>(v, tw, M0, M);
    fwd_stage16<1>(v, tw, M0, M);
    fwd_stage16<2>(v, tw, M0, M);
    fwd_stage16<3>(v, tw, M0, M);
}
// First round of a forward transform on canonical input (OFHE_FWD_CANON):
// [0, q) -> 5q -> 9q -> 13q without a conditional subtract, then the CS stage
// -> [0, 12q), the bound the alternating schedule leaves after any round.
// Needs inputs < 4q (canonical, per the C ABI contract).
#ifndef OFHE_FWD_CANON
#define OFHE_FWD_CANON 1
#endif
template <class M_>
__device__ __forceinline__ void fwd_round16_canon(u64 (&v)[16], const u64* tw, u32 M0, const M_& M) {
    fwd_stage16<0>(v, tw, M0, M);
    fwd_stage16<1, M_, OFHE_FWD_CANON ? 0 : 1>(v, tw, M0, M);
    fwd_stage16<2>(v, tw, M0, M);
    fwd_stage16<3>(v, tw, M0, M);
}
template <class M_>
__device__ __forceinline__ void inv_round16(u64 (&v)[16], const u64* itw, u32 M0, const M_& M) {
    inv_stage16<3>(v, itw, M0, M);
    inv_stage16<2>(v, itw, M0, M);
    inv_stage16<1>(v, itw, M0, M);
    inv_stage16<0>(v, itw, M0, M);
}

// ---------------------------------------------------------------------------
// Round 3 of k_block (st = 1) gives every thread its own twiddles: thread u
// of the block's 256 (global u = 256 g + tid, M0 = N/16 + u) needs
// Table[(M0 << S) + j], j < 2^S.  Read from Table directly, lanes are 2^S
// entries apart and one wave-wide 16-byte load touches 64 cache lines.  The
// plan therefore also stores these twiddles transposed, tw3[S][j][u] at
// ((2^S - 1) U + j U + u) with U = N/16, so a wave reads 1 KiB contiguous per
// load, from a uniform (scalar) base plus the lane offset.
// ---------------------------------------------------------------------------
#ifndef OFHE_TW3
#define OFHE_TW3 1
#endif
// OFHE_MONT: the fused pipeline's Hadamard is a Montgomery product on the lazy
// forward output (no canonicalisation, no Barrett), and the 2^-64 it
// introduces is cancelled by 2^64 folded into the inverse's N^-1 twist
// (PlanArgs::twist = the plan's twist_r table).  Intermediate values differ in representation only;
// the canonical output is the same integer.
#ifndef OFHE_MONT
#define OFHE_MONT 1
#endif
// k_block's round-3 layout gives each thread 16 consecutive words, so direct
// global access is one 128-byte line per lane per instruction.  With
// OFHE_COAL (inverse input, forward output) and OFHE_COAL_B (the Hadamard
// operand) these go through the wave's own LDS slots instead (wave_stage_*).
#ifndef OFHE_COAL
#define OFHE_COAL 1
#endif
#ifndef OFHE_COAL_B
#define OFHE_COAL_B 1
#endif
constexpr bool kMontFused = OFHE_MONT && OFHE_COAL_B;
// mont_mul takes a < 12q: the forward output after a CS stage (OFHE_THR widens it)
static_assert(!(kMontFused && OFHE_THR), "Montgomery Hadamard needs the forward output < 12q");
template <int S, class M_>
__device__ __forceinline__ void fwd_stage16_t3(u64 (&v)[16], const u64* tw3, u32 U, u32 u, const M_& M) {
    constexpr int half = 8 >> S;
    const u64* base = tw3 + 2 * (u64)(((1u << S) - 1) * U);
#pragma unroll
    for (int j = 0; j < (1 << S); j++) {
        Tw w = ldtw(base + 2 * (u64)j * U, u);
#pragma unroll
        for (int k = j * 2 * half; k < j * 2 * half + half; k++) ct_bfly<S & 1>(v[k], v[k + half], w, M);
    }
}
// LDS placement of block element p: one u64 of padding per 16 elements.  It is
// additive, so every round addresses its 16 values as one base register plus
// immediate offsets, and it is bank-conflict free for the round-2/3 patterns
// and 2-way on one half-wave for round 1 (tools/lds_banks.py).
__device__ __forceinline__ u32 lds_pad(u32 p) { return p + (p >> 4); }
constexpr u32 LDS_WORDS = 4096 + 4096 / 16;

// Wave-private staging through the round-3 LDS slots.  In round 3 thread t
// owns block elements 16t + k at lds_pad = 17t + k, so wave w's 64 threads own
// the 1024 consecutive elements [1024w, 1024w + 1024).  From a thread's
// round-3 LDS reads until the next block barrier no other wave touches that
// region, so a wave can turn its lane-strided (128 B per lane) global accesses
// into contiguous ones through it without a block barrier: instruction k,
// lane i moves elements 128k + 2i and 128k + 2i + 1 of the wave's range.
// LDS processes one wave's operations in order; wave_barrier keeps the
// compiler from reordering them across lanes.
__device__ __forceinline__ void wave_stage_in(const u64* wsrc, u64* lds, u32 tid, u64 (&out)[16]) {
    const u32 lane = tid & 63, base = (tid >> 6) * 1024;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const u64x2 v = ld2_s(wsrc + 128 * k + 2 * lane);
        const u32 p = base + 128 * k + 2 * lane;  // even: p, p + 1 share a 16-group
        lds[lds_pad(p)] = v.x;
        lds[lds_pad(p) + 1] = v.y;
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < 16; k++) out[k] = lds[tid * 17 + k];
    __builtin_amdgcn_wave_barrier();
}
// wave_stage_in whose first NPRE 16-byte loads were issued earlier (pre[]),
// so their HBM latency overlaps the caller's compute
template <int NPRE>
__device__ __forceinline__ void wave_stage_in_pre(const u64* wsrc, u64* lds, u32 tid, const u64x2 (&pre)[NPRE > 0 ? NPRE : 1],
                                                  u64 (&out)[16]) {
    const u32 lane = tid & 63, base = (tid >> 6) * 1024;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const u64x2 v = k < NPRE ? pre[k < NPRE ? k : 0] : ld2_s(wsrc + 128 * k + 2 * lane);
        const u32 p = base + 128 * k + 2 * lane;
        lds[lds_pad(p)] = v.x;
        lds[lds_pad(p) + 1] = v.y;
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < 16; k++) out[k] = lds[tid * 17 + k];
    __builtin_amdgcn_wave_barrier();
}
__device__ __forceinline__ void wave_stage_out(const u64 (&v)[16], u64* lds, u32 tid, u64* wdst) {
    const u32 lane = tid & 63, base = (tid >> 6) * 1024;
#pragma unroll
    for (int k = 0; k < 16; k++) lds[tid * 17 + k] = v[k];
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const u32 p = base + 128 * k + 2 * lane;
        u64x2 w;
        w.x = lds[lds_pad(p)];
        w.y = lds[lds_pad(p) + 1];
        st2_s(wdst + 128 * k + 2 * lane, w);
    }
}

// ---------------------------------------------------------------------------
// k_block: the last 12 stages on a 4096-element block; MODE selects
// forward (canonical out), inverse (first 12 inverse stages), or the fused
// forward -> Hadamard -> inverse pipeline.
// ---------------------------------------------------------------------------
#ifndef OFHE_B_PF
#define OFHE_B_PF 8  // early second-operand loads in the fused / forward-subtract block pass (0..8)
#endif
#ifndef OFHE_KB_WAVES
#define OFHE_KB_WAVES 4
#endif
// SK = 3 (NR = 3 only, SPLIT_T8B9): the column pass ran the first three
// stages of round 1 (strides 2048, 1024, 512), so the forward round 1 keeps
// its last stage (stride 256) and the inverse round 1' its first (t = 256);
// the inverse twist is the one of 512-element groups.
// The body of k_block for work item wid (block g = wid % G of polynomial
// tower pb = wid / G), on the caller's LDS (LDS_WORDS words).
template <int MODE, bool SPQ, int NR, int SK = 0>
__device__ __forceinline__ void block_body(const PlanArgs& P, const u64* src, u64* dst, const u64* __restrict__ bdat,
                                           u32 batch, u32 wid, u64* lds, u32 tid) {
    static_assert(NR == 2 || NR == 3, "k_block covers the last 8 (NR=2) or 12 (NR=3) stages");
    static_assert(SK == 0 || (SK == 3 && NR == 3), "k_block: SK = 3 needs NR = 3");
    const u32 logn = P.log_n;
    const u32 N = 1u << logn;
    const u32 G = N >> 12;  // blocks per polynomial
    const u32 g = wid % G;
    const u32 pb = wid / G;
    const u32 t = pb / batch, b = pb % batch;
    const u64 inner = (u64)t * N + ((u64)g << 12);
    const u64 off = (u64)b * P.dstride + inner;
    const u64 boff = (u64)b * P.bstride + inner;
    const u64* blk = src + (u64)b * P.sstride + inner;
    u64* oblk = dst + off;
    const TowerConst tc = P.tc[t];
    const u64 q = tc.q;
    const auto M = load_mod<SPQ, (bool)OFHE_QA_BLK>(tc);
    const u64* tw = P.tw + (u64)t * N * 2;
    const u32 h = tid >> 4, r = tid & 15;
    // padded LDS bases (lds_pad(p) = p + p/16) of the three round layouts
    const u32 L1 = tid + h;      // lds_pad(tid + 256 k)      = L1 + 272 k
    const u32 L2 = h * 272 + r;  // lds_pad(256 h + r + 16 k) = L2 + 17 k
    const u32 L3 = tid * 17;     // lds_pad(16 tid + k)       = L3 + k
    u64 v[16];

    if (MODE == MODE_FWD || MODE == MODE_FUSED || MODE == MODE_FWD_SUB) {
        if (NR == 3) {
            // round 1: st = 256, p = tid + 256k
#pragma unroll
            for (int k = 0; k < 16; k++) v[k] = ld_s(blk + tid + 256 * k);
            if (SK == 3)
                fwd_stage16<3>(v, tw, (N >> 12) + g, M);  // input < 12q (k_tcols) -> < 12q
            else
                fwd_round16(v, tw, (N >> 12) + g, M);
#pragma unroll
            for (int k = 0; k < 16; k++) lds[L1 + 272 * k] = v[k];
            __syncthreads();
            // round 2: st = 16, p = h*256 + r + 16k
#pragma unroll
            for (int k = 0; k < 16; k++) v[k] = lds[L2 + 17 * k];
        } else {
#pragma unroll
            for (int k = 0; k < 16; k++) v[k] = ld_s(blk + h * 256 + r + 16 * k);
        }
        fwd_round16(v, tw, (N >> 8) + g * 16 + h, M);
#pragma unroll
        for (int k = 0; k < 16; k++) lds[L2 + 17 * k] = v[k];
        __syncthreads();
        // round 3: st = 1, p = 16 tid + k
#pragma unroll
        for (int k = 0; k < 16; k++) v[k] = lds[L3 + k];
        // the second operand (the fused pipeline's Hadamard b, ModDown's x):
        // the first OFHE_B_PF of its 8 wave-coalesced 16-byte loads go out
        // now, so their HBM latency hides under round 3 (same-process A/B,
        // batch 256: fused block pass 1.740 -> 1.673 ms, VGPRs unchanged)
        constexpr int BPF = ((MODE == MODE_FUSED && OFHE_COAL_B) || MODE == MODE_FWD_SUB) ? OFHE_B_PF : 0;
        u64x2 bpre[BPF > 0 ? BPF : 1];
#pragma unroll
        for (int k = 0; k < BPF; k++) bpre[k] = ld2_s(bdat + boff + (tid >> 6) * 1024 + 128 * k + 2 * (tid & 63));
        if (OFHE_TW3) {
            const u64* tw3 = P.tw3 + (u64)t * (N / 16) * 30;
            const u32 U = N >> 4, u = g * 256 + tid;
            fwd_stage16_t3<0>(v, tw3, U, u, M);
            fwd_stage16_t3<1>(v, tw3, U, u, M);
            fwd_stage16_t3<2>(v, tw3, U, u, M);
            fwd_stage16_t3<3>(v, tw3, U, u, M);
        } else {
            fwd_round16(v, tw, (N >> 4) + g * 256 + tid, M);
        }
        if (!(MODE == MODE_FUSED && kMontFused) && MODE != MODE_FWD_SUB) {
#pragma unroll
            for (int k = 0; k < 16; k++) v[k] = canon_fwd<SPQ>(v[k], M);
        }
        if (MODE == MODE_FWD_SUB) {
            // x + 12q - v needs the forward output v < 12q; OFHE_THR's bit-test
            // reduction leaves it below 2^(L+3) + 8q (up to 16q), which could wrap
            static_assert(!OFHE_THR, "the lazy forward-subtract needs the forward output < 12q (OFHE_THR widens it)");
            // (x - NTT(y)) s mod q without canonicalising NTT(y) first: v < 12q
            // (round 3 ends with a CS stage), so d = x + 12q - v is in (0, 13q)
            // < 2^64, the lazy Shoup takes any 64-bit input to [0, 4q), and one
            // canonicalisation gives the same residue as ModSubFastEq followed
            // by ModMulFastConstEq (~10 instructions per coefficient fewer)
            u64 xx[16];
            wave_stage_in_pre<BPF>(bdat + boff + (tid >> 6) * 1024, lds, tid, bpre, xx);
            const u64 sc = P.scal[3 * t + 1], scp = P.scal[3 * t + 2];
            const u64 q12 = M.q8 + M.q4;
#pragma unroll
            for (int k = 0; k < 16; k++) v[k] = canon4m(shoup_lazy(xx[k] + q12 - v[k], sc, scp, M), M);
            wave_stage_out(v, lds, tid, oblk + (tid >> 6) * 1024);
            return;
        }
        if (MODE == MODE_FWD) {
            if (OFHE_COAL) {
                wave_stage_out(v, lds, tid, oblk + (tid >> 6) * 1024);
            } else {
                ulonglong2* o = reinterpret_cast<ulonglong2*>(oblk + tid * 16);
#pragma unroll
                for (int k = 0; k < 8; k++) o[k] = make_ulonglong2(v[2 * k], v[2 * k + 1]);
            }
            return;
        }
        // Hadamard with b (evaluation form), NativeVectorT::ModMulNoCheckEq
        if (OFHE_COAL_B) {
            u64 bb[16];
            wave_stage_in_pre<BPF>(bdat + boff + (tid >> 6) * 1024, lds, tid, bpre, bb);
            if (kMontFused) {
#pragma unroll
                for (int k = 0; k < 16; k++) v[k] = mont_mul(v[k], bb[k], q, tc.qinv);  // (0, 2q)
            } else {
#pragma unroll
                for (int k = 0; k < 16; k++) v[k] = barrett_ref(v[k], bb[k], q, tc.mu, tc.nshift);
            }
        } else {
            const ulonglong2* bp = reinterpret_cast<const ulonglong2*>(bdat + boff + tid * 16);
#pragma unroll
            for (int k = 0; k < 8; k++) {
#ifdef OFHE_ABL_NOB
                ulonglong2 bb = make_ulonglong2(v[k] ^ off, v[k + 8] ^ tid);
#else
                ulonglong2 bb = bp[k];
#endif
                v[2 * k] = barrett_ref(v[2 * k], bb.x, q, tc.mu, tc.nshift);
                v[2 * k + 1] = barrett_ref(v[2 * k + 1], bb.y, q, tc.mu, tc.nshift);
            }
        }
        // no barrier: round 3' below rewrites only this thread's own LDS slots
    } else {
        if (OFHE_COAL) {
            wave_stage_in(blk + (tid >> 6) * 1024, lds, tid, v);
        } else {
            const ulonglong2* ip = reinterpret_cast<const ulonglong2*>(blk + tid * 16);
#pragma unroll
            for (int k = 0; k < 8; k++) {
                ulonglong2 a = ip[k];
                v[2 * k] = a.x;
                v[2 * k + 1] = a.y;
            }
        }
    }
    // inverse as DIT inside the block's groups: round 3' (t = 1..8, uniform
    // twiddles), round 2' (t = 16..128, st = 16, r = tid & 15), round 1'
    // (NR = 3: t = 256..2048, st = 256, r = tid), then the twist (group b =
    // position / G): canonical when the block ran every stage (N = 2^12),
    // else lazy [0, 4q) for the GS column pass
    const u64* dtw = P.dtw + (u64)t * N * 2;
    dit_round3(v, dtw, M);
#pragma unroll
    for (int k = 0; k < 16; k++) lds[L3 + k] = v[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 16; k++) v[k] = lds[L2 + 17 * k];
    dit_round16(v, dtw, 16, r, M);
    const u64* tw_ = P.twist + (u64)t * N * 2 + 2 * ((u64)g << 12);
    if (NR == 2) {
        // twist into the GS column pass's input, lazy [0, 4q)
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const u32 p = h * 256 + r + 16 * k;
            const Tw f = ldtw(tw_, p);
            st_s(oblk + p, shoup_lazy(v[k], f.w, f.wp, M));
        }
        return;
    }
#pragma unroll
    for (int k = 0; k < 16; k++) lds[L2 + 17 * k] = v[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 16; k++) v[k] = lds[L1 + 272 * k];
    if (SK == 3)
        dit_stage16<0, 1>(v, dtw + 2 * ((u64)256 + tid), 256, M);  // t = 256 only: < 16q -> < 12q
    else
        dit_round16(v, dtw, 256, tid, M);
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const Tw f = ldtw(tw_, tid + 256 * k);
        v[k] = logn == 12 ? twist_out(v[k], f, M) : shoup_lazy(v[k], f.w, f.wp, M);
    }
#pragma unroll
    for (int k = 0; k < 16; k++) st_s(oblk + tid + 256 * k, v[k]);
}
template <int MODE, bool SPQ, int NR, int SK = 0>
__global__ __launch_bounds__(256, OFHE_KB_WAVES) void k_block(PlanArgs P, const u64* src, u64* dst,
                                                              const u64* __restrict__ bdat, u32 batch, u32 nwg) {
    OFHE_VGPR_FLOOR();
    __shared__ u64 lds[LDS_WORDS];
    block_body<MODE, SPQ, NR, SK>(P, src, dst, bdat, batch, xcd_remap(blockIdx.x, nwg), lds, threadIdx.x);
}

// Rescaling source of the forward column pass (k_cols / k_tcols <.., SWS = true>):
// element (b, t, pos) is SwitchModulus(last[b][pos]) from ql to q_t, times w_t
// (tab[6 t + 1], Shoup constant at + 2; skipped when w_t = 1), so the lifted
// towers are never written to HBM before their transform (keyswitch.hip,
// DropLastElementAndScale / ModReduce in evaluation form).
struct SwSrc {
    const u64* last;
    u64 lstride;
    u64 ql;
    const u64* tab;
    u64 pre, pre_p;  // scalar on last mod ql before the lift (ModReduce's negtInvModq), 1: none
};
// ---------------------------------------------------------------------------
// k_tcols: the first 8 forward stages (or the last 8 inverse stages) of an
// N = 2^16 transform.  Element j = row * 256 + col; for a fixed col the 256
// rows form one sub-transform.  A workgroup owns a tile of 16 columns x 256
// rows (tile element p = row * 16 + col_in_tile) and runs the same two
// radix-16 register rounds and padded LDS exchange as k_block's rounds 1-2:
// twiddle indices depend on the row only (j / (2t) = row / (256/m)).  Global
// accesses are 128-byte row segments.  With 8 column stages the pass has as
// much multiply work as HBM time, instead of k_cols' 4 stages that leave the
// VALU idle behind HBM.
// ---------------------------------------------------------------------------
#ifndef OFHE_TCOLS_W
#define OFHE_TCOLS_W 16  // tile width in columns: 16 (128-byte row segments) or 32 (256-byte)
#endif
constexpr u32 TCOLS_W = OFHE_TCOLS_W;
#ifndef OFHE_TCOLS_PADF
#define OFHE_TCOLS_PADF 1
#endif
static_assert(TCOLS_W == 16 || TCOLS_W == 32, "column tile width");
// LOGN = 17 (the 8 | 9 split, SPLIT_T8B9): element j = row * 512 + col, the
// same 256-row sub-transforms on 512 columns (the twiddle index of stage m is
// m + row / (256 / m) whatever the row length).
constexpr u32 TCOLS_LDS_WORDS = 16 * 16 * TCOLS_W + 16 * 16;
// OFHE_TCOLS_HALF: the inverse column pass transposes through half the LDS in
// two passes (A/B knob), its kernel sized for OFHE_TCOLS_HALF_WAVES waves per SIMD
#ifndef OFHE_TCOLS_HALF
#define OFHE_TCOLS_HALF 0
#endif
#ifndef OFHE_TCOLS_HALF_WAVES
#define OFHE_TCOLS_HALF_WAVES 5
#endif
constexpr u32 TCOLS_LDS_INV_WORDS = OFHE_TCOLS_HALF ? 8 * 16 * TCOLS_W : TCOLS_LDS_WORDS;
// The body of k_tcols for work item wid (column tile cb = wid % (S / W) of
// polynomial tower pb = wid / (S / W)) on the caller's LDS (TCOLS_LDS_WORDS).
template <bool INV, bool SPQ, bool SWS = false, int LOGN = 16>
__device__ __forceinline__ void tcols_body(const PlanArgs& P, const u64* src, u64* dst, u32 batch, u32 wid,
                                           const SwSrc& SWA, u64* lds, u32 tid) {
    static_assert(LOGN == 16 || LOGN == 17, "k_tcols: N = 2^16 or 2^17");
    constexpr u32 N = 1u << LOGN, S = N / 256, W = TCOLS_W;
    // Exchange patterns p = tid + 16W k (round 1) and p = 16W h + W k + r
    // (round 2).  The inverse writes the second and reads the first: unpadded,
    // both conflict free (SQ_LDS_BANK_CONFLICT = 0; a p + p/16 padding made its
    // 32-lane ds_read_b64 groups 2-way conflicted).  The forward READS the
    // second pattern, where a half-wave's two rows h, h + 1 hit the same 32
    // banks (2-way, measured 0.56 conflict cycles per active LDS cycle); with
    // OFHE_TCOLS_PADF it shifts row h by 16 words per 16W-word row
    // (lds index p + 16 (p / 16W)), so rows h and h + 1 cover all 64 banks.
    const u32 cb = wid % (S / W);
    const u32 pb = wid / (S / W);
    const u32 t = pb / batch, b = pb % batch;
    const u64 inner = (u64)t * N + cb * W;
    const u64* x = src + (u64)b * P.sstride + inner;
    u64* y = dst + (u64)b * P.dstride + inner;
    const TowerConst tc = P.tc[t];
    const auto M = load_mod<SPQ, INV ? (bool)OFHE_QA_TCI : (bool)OFHE_QA_TCF>(tc);
    const u32 h = tid / W, r = tid % W;
    const u32 L1 = tid, L2 = h * 16 * W + r;
    u64 v[16];
    if (!INV) {
        const u64* tw = P.tw + (u64)t * N * 2;
        constexpr u32 RP = OFHE_TCOLS_PADF ? 16 * W + 16 : 16 * W;  // padded row pitch
        // round 1: rows h + 16k (p = tid + 16W k), stages m = 1..8
        if (SWS) {
            const u64 w = SWA.tab[6 * t + 1], wp = SWA.tab[6 * t + 2];
            const SwMod sm = sw_mod(SWA.ql, tc.q);
            const u64* lp = SWA.last + (u64)b * SWA.lstride + cb * W;
#pragma unroll
            for (int k = 0; k < 16; k++) {
                u64 e = lp[(u64)(h + 16 * k) * S + r];
                if (SWA.pre != 1) e = shoup_canon(e, SWA.pre, SWA.pre_p, SWA.ql);
                e = switch_mod1(e, sm);
                v[k] = w != 1 ? shoup_canon(e, w, wp, tc.q) : e;
            }
        } else {
#pragma unroll
            for (int k = 0; k < 16; k++) v[k] = ld_s(x + (u64)(h + 16 * k) * S + r);
        }
        fwd_round16_canon(v, tw, 1, M);
#pragma unroll
        for (int k = 0; k < 16; k++) lds[L1 + RP * k] = v[k];
        __syncthreads();
        // round 2: rows 16h + k (p = 16W h + W k + r), stages m = 16..128
#pragma unroll
        for (int k = 0; k < 16; k++) v[k] = lds[h * RP + r + W * k];
        fwd_round16(v, tw, 16 + h, M);
#pragma unroll
        for (int k = 0; k < 16; k++) st_s(y + (u64)(16 * h + k) * S + r, v[k]);
    } else {
        const u64* itw = P.itw + (u64)t * N * 2;
#pragma unroll
        for (int k = 0; k < 16; k++) v[k] = ld_s(x + (u64)(16 * h + k) * S + r);
        if (OFHE_LAZY_GS) {
            // input < 4q (the block pass's lazy twist); round 2's registers all
            // come from one round-1 position, taken as < 8q
            bool b8[16];
#pragma unroll
            for (int k = 0; k < 16; k++) b8[k] = false;
            inv_round16_b(v, b8, itw, 16 + h, M);
            if (OFHE_TCOLS_HALF) {
                // the transpose through half the LDS (8 W x 16 words) in two
                // passes: writers h < 8, then h >= 8 (wave-uniform), every
                // thread reading 8 values per pass; 16 KiB per workgroup lets
                // more workgroups share a CU (A/B knob)
                u64 o[16];
                if (h < 8) {
#pragma unroll
                    for (int k = 0; k < 16; k++) lds[L2 + W * k] = v[k];
                }
                __syncthreads();
#pragma unroll
                for (int k = 0; k < 8; k++) o[k] = lds[L1 + 16 * W * k];
                __syncthreads();
                if (h >= 8) {
#pragma unroll
                    for (int k = 0; k < 16; k++) lds[L2 - 8 * 16 * W + W * k] = v[k];
                }
                __syncthreads();
#pragma unroll
                for (int k = 8; k < 16; k++) o[k] = lds[L1 + 16 * W * (k - 8)];
#pragma unroll
                for (int k = 0; k < 16; k++) {
                    v[k] = o[k];
                    b8[k] = true;
                }
            } else {
#pragma unroll
                for (int k = 0; k < 16; k++) lds[L2 + W * k] = v[k];
                __syncthreads();
#pragma unroll
                for (int k = 0; k < 16; k++) {
                    v[k] = lds[L1 + 16 * W * k];
                    b8[k] = true;
                }
            }
            inv_round16_b(v, b8, itw, 1, M);
#pragma unroll
            for (int k = 0; k < 16; k++)
                st_s(y + (u64)(h + 16 * k) * S + r, b8[k] ? canon8m(v[k], M) : canon4m(v[k], M));
        } else {
            inv_round16(v, itw, 16 + h, M);
#pragma unroll
            for (int k = 0; k < 16; k++) lds[L2 + W * k] = v[k];
            __syncthreads();
#pragma unroll
            for (int k = 0; k < 16; k++) v[k] = lds[L1 + 16 * W * k];
            inv_round16(v, itw, 1, M);
#pragma unroll
            for (int k = 0; k < 16; k++) st_s(y + (u64)(h + 16 * k) * S + r, canon4m(v[k], M));
        }
    }
}

template <bool INV, bool SPQ, bool SWS = false, int LOGN = 16>
__global__ __launch_bounds__(16 * TCOLS_W, (INV && OFHE_TCOLS_HALF) ? OFHE_TCOLS_HALF_WAVES : OFHE_KB_WAVES) void k_tcols(
    PlanArgs P, const u64* src, u64* dst, u32 batch, u32 nwg, SwSrc SWA) {
    OFHE_VGPR_FLOOR();
    __shared__ u64 lds[INV ? TCOLS_LDS_INV_WORDS : TCOLS_LDS_WORDS];
    tcols_body<INV, SPQ, SWS, LOGN>(P, src, dst, batch, xcd_remap(blockIdx.x, nwg), SWA, lds, threadIdx.x);
}

// ---------------------------------------------------------------------------
// k_tcols9: the first 9 forward stages (or the last 9 inverse stages) of an
// N = 2^17 transform, so that the block pass keeps its 8 stages (k_block
// NR = 2) and the two passes split the multiply work 9 | 8 instead of k_cols'
// 5 | 12 (whose column pass sits idle behind HBM while the 12-stage block
// pass is VALU-bound).  Element j = row * 256 + col, 512 rows.  A workgroup of
// 512 threads owns 16 columns x 512 rows; half hf = tid / 256 holds rows
// [256 hf, 256 hf + 256) in k_tcols' layout.  Forward: stage m = 1 pairs row
// rho with rho + 256 (twiddle Table[1]) through one LDS exchange -- the half
// holding y computes w y, so no product is computed twice -- then each half
// runs k_tcols' two radix-16 rounds as the independent sub-transform it now
// is (twiddle bases 2 + hf and 32 + 16 hf + h: index m + rho / (512 / m)).
// Inverse: the mirror, ending in the GS stage across the halves.  Lazy bounds
// as k_tcols: the extra forward stage maps [0, q) to [0, 5q).
// ---------------------------------------------------------------------------
template <bool INV, bool SPQ>
__global__ __launch_bounds__(512) void k_tcols9(PlanArgs P, const u64* src, u64* dst, u32 batch, u32 nwg) {
    OFHE_VGPR_FLOOR();
    constexpr u32 N = 1u << 17, S = 256, W = 16, HALF = 16 * 16 * W;  // words per half tile
    __shared__ u64 lds[2 * HALF];
    const u32 tid = threadIdx.x;
    const u32 hf = tid >> 8, tl = tid & 255;
    const u32 wid = xcd_remap(blockIdx.x, nwg);
    const u32 cb = wid % (S / W);
    const u32 pb = wid / (S / W);
    const u32 t = pb / batch, b = pb % batch;
    const u64 inner = (u64)t * N + (u64)hf * 256 * S + cb * W;  // row 256 hf of this tile
    const u64* x = src + (u64)b * P.sstride + inner;
    u64* y = dst + (u64)b * P.dstride + inner;
    const TowerConst tc = P.tc[t];
    const Mod<SPQ> M = load_mod<SPQ>(tc);
    const u32 h = tl / W, r = tl % W;
    u64* my = lds + hf * HALF;
    const u64* other = lds + (hf ^ 1) * HALF;
    const u32 L1 = tl, L2 = h * 16 * W + r;
    u64 v[16];
    if (!INV) {
        const u64* tw = P.tw + (u64)t * N * 2;
#pragma unroll
        for (int k = 0; k < 16; k++) v[k] = ld_s(x + (u64)(h + 16 * k) * S + r);
        // stage m = 1: (x, y) = rows (rho, rho + 256) -> (x + w y, x + 4q - w y)
        const Tw w1 = ldtw(tw, 1);
        if (hf) {
#pragma unroll
            for (int k = 0; k < 16; k++) v[k] = shoup_lazy(v[k], w1.w, w1.wp, M);  // w y, [0, 4q)
        }
#pragma unroll
        for (int k = 0; k < 16; k++) my[L1 + 16 * W * k] = v[k];
        __syncthreads();
        if (hf) {
#pragma unroll
            for (int k = 0; k < 16; k++) v[k] = other[L1 + 16 * W * k] + M.q4 - v[k];
        } else {
#pragma unroll
            for (int k = 0; k < 16; k++) v[k] += other[L1 + 16 * W * k];
        }
        __syncthreads();  // the partner has read this half's slots
        fwd_round16(v, tw, 2 + hf, M);
#pragma unroll
        for (int k = 0; k < 16; k++) my[L1 + 16 * W * k] = v[k];
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 16; k++) v[k] = my[L2 + W * k];
        fwd_round16(v, tw, 32 + 16 * hf + h, M);
#pragma unroll
        for (int k = 0; k < 16; k++) st_s(y + (u64)(16 * h + k) * S + r, v[k]);
    } else {
        const u64* itw = P.itw + (u64)t * N * 2;
#pragma unroll
        for (int k = 0; k < 16; k++) v[k] = ld_s(x + (u64)(16 * h + k) * S + r);
        inv_round16(v, itw, 32 + 16 * hf + h, M);
#pragma unroll
        for (int k = 0; k < 16; k++) my[L2 + W * k] = v[k];
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 16; k++) v[k] = my[L1 + 16 * W * k];
        inv_round16(v, itw, 2 + hf, M);
        // each thread rewrites only the round-1 slots it read itself
#pragma unroll
        for (int k = 0; k < 16; k++) my[L1 + 16 * W * k] = v[k];
        __syncthreads();
        // stage m = 1 (GS): rows (rho, rho + 256) -> (x + y, (x - y) w), inputs [0, 4q)
        if (hf) {
            const Tw w1 = ldtw(itw, 1);
#pragma unroll
            for (int k = 0; k < 16; k++)
                v[k] = canon4m(shoup_lazy(other[L1 + 16 * W * k] + M.q4 - v[k], w1.w, w1.wp, M), M);
        } else {
#pragma unroll
            for (int k = 0; k < 16; k++) v[k] = canon4m(csub_s(v[k] + other[L1 + 16 * W * k], M.q4), M);
        }
#pragma unroll
        for (int k = 0; k < 16; k++) st_s(y + (u64)(h + 16 * k) * S + r, v[k]);
    }
}

// ---------------------------------------------------------------------------
// k_cols: the first KA = logN - 12 forward stages (or the last KA inverse
// stages) on columns {c + 4096 k}, k < 2^KA, entirely in registers.  CPT
// adjacent columns per thread make every global access 8*CPT bytes wide.
// ---------------------------------------------------------------------------
template <int E, int CPT, class M_>
__device__ __forceinline__ void cols_fwd(u64 (&v)[CPT][E], const u64* tw, const M_& M) {
    constexpr int KA = __builtin_ctz(E);
#pragma unroll
    for (int s = 0; s < KA; s++) {
        const int half = E >> (s + 1);
#pragma unroll
        for (int j = 0; j < (1 << s); j++) {
            Tw w = ldtw(tw, (1u << s) + j);
#pragma unroll
            for (int k = j * 2 * half; k < j * 2 * half + half; k++)
#pragma unroll
                for (int c = 0; c < CPT; c++) ct_bfly_cs(v[c][k], v[c][k + half], w, M, ((KA - 1 - s) & 1) == 0);
        }
    }
}
template <int E, int CPT, class M_>
__device__ __forceinline__ void cols_inv(u64 (&v)[CPT][E], const u64* itw, const M_& M) {
    constexpr int KA = __builtin_ctz(E);
#pragma unroll
    for (int s = KA - 1; s >= 0; s--) {
        const int half = E >> (s + 1);
#pragma unroll
        for (int j = 0; j < (1 << s); j++) {
            Tw w = ldtw(itw, (1u << s) + j);
#pragma unroll
            for (int k = j * 2 * half; k < j * 2 * half + half; k++)
#pragma unroll
                for (int c = 0; c < CPT; c++) gs_bfly(v[c][k], v[c][k + half], w, M);
        }
    }
}
// lazy form (OFHE_LAZY_GS): compile-time bounds b8 as in inv_stage16_b, inputs < 4q
template <int E, int CPT, class M_>
__device__ __forceinline__ void cols_inv_b(u64 (&v)[CPT][E], bool (&b8)[E], const u64* itw, const M_& M) {
    constexpr int KA = __builtin_ctz(E);
#pragma unroll
    for (int k = 0; k < E; k++) b8[k] = false;
#pragma unroll
    for (int s = KA - 1; s >= 0; s--) {
        const int half = E >> (s + 1);
#pragma unroll
        for (int j = 0; j < (1 << s); j++) {
            Tw w = ldtw(itw, (1u << s) + j);
#pragma unroll
            for (int k = j * 2 * half; k < j * 2 * half + half; k++) {
                const bool in8 = b8[k] || b8[k + half];
#pragma unroll
                for (int c = 0; c < CPT; c++) gs_bfly_b(v[c][k], v[c][k + half], w, M, in8);
                b8[k] = true;
                b8[k + half] = false;
            }
        }
    }
}

template <int KA, bool INV, int CPT, bool SPQ, bool SWS = false>
__global__ __launch_bounds__(256) void k_cols(PlanArgs P, const u64* src, u64* dst, u32 batch, u32 nwg, SwSrc S) {
    OFHE_VGPR_FLOOR();
    constexpr int E = 1 << KA;
    constexpr u32 N = 1u << (KA + 12);
    constexpr u32 CB = 16 / CPT;  // column blocks per polynomial
    const u32 wid = xcd_remap(blockIdx.x, nwg);
    const u32 cb = wid % CB;
    const u32 pb = wid / CB;
    const u32 t = pb / batch, b = pb % batch;
    const u64 inner = (u64)t * N + cb * (256 * CPT) + threadIdx.x * CPT;
    const u64* x = src + (u64)b * P.sstride + inner;
    u64* y = dst + (u64)b * P.dstride + inner;
    const TowerConst tc = P.tc[t];
    const auto M = load_mod<SPQ, INV ? (bool)OFHE_QA_CI : (bool)OFHE_QA_CF>(tc);
    u64 v[CPT][E];
    if (SWS) {
        const u64 w = S.tab[6 * t + 1], wp = S.tab[6 * t + 2];
        const SwMod sm = sw_mod(S.ql, tc.q);
        const u64* lp = S.last + (u64)b * S.lstride + (inner - (u64)t * N);
#pragma unroll
        for (int k = 0; k < E; k++) {
            u64 lv[2];
            if (CPT == 2) {
                const u64x2 p = *reinterpret_cast<const u64x2*>(lp + (u64)k * 4096);
                lv[0] = p.x;
                lv[1] = p.y;
            } else {
                lv[0] = lp[(u64)k * 4096];
            }
#pragma unroll
            for (int c = 0; c < CPT; c++) {
                u64 e = lv[c];
                if (S.pre != 1) e = shoup_canon(e, S.pre, S.pre_p, S.ql);
                e = switch_mod1(e, sm);
                if (w != 1) e = shoup_canon(e, w, wp, tc.q);
                v[c][k] = e;
            }
        }
    }
#pragma unroll
    for (int k = 0; k < E && !SWS; k++) {
        if (CPT == 2) {
            const u64x2 p = ld2_s(x + (u64)k * 4096);
            v[0][k] = p.x;
            v[CPT - 1][k] = p.y;
        } else {
            v[0][k] = ld_s(x + (u64)k * 4096);
        }
    }
    if (!INV) {
        cols_fwd<E, CPT>(v, P.tw + (u64)t * N * 2, M);
    } else {
        if (OFHE_LAZY_GS) {
            bool b8[E];
            cols_inv_b<E, CPT>(v, b8, P.itw + (u64)t * N * 2, M);
#pragma unroll
            for (int k = 0; k < E; k++)
#pragma unroll
                for (int c = 0; c < CPT; c++) v[c][k] = b8[k] ? canon8m(v[c][k], M) : canon4m(v[c][k], M);
        } else {
            cols_inv<E, CPT>(v, P.itw + (u64)t * N * 2, M);
#pragma unroll
            for (int k = 0; k < E; k++)
#pragma unroll
                for (int c = 0; c < CPT; c++) v[c][k] = canon4m(v[c][k], M);
        }
    }
#pragma unroll
    for (int k = 0; k < E; k++) {
        if (CPT == 2) {
            u64x2 w;
            w.x = v[0][k];
            w.y = v[CPT - 1][k];
            st2_s(y + (u64)k * 4096, w);
        } else {
            st_s(y + (u64)k * 4096, v[0][k]);
        }
    }
}

// ---------------------------------------------------------------------------
// k_small: N <= 2^11, one workgroup per polynomial, whole tower in LDS.
// ---------------------------------------------------------------------------
template <int MODE, bool SPQ>
__global__ __launch_bounds__(256) void k_small(PlanArgs P, const u64* src, u64* dst, const u64* __restrict__ bdat,
                                               u32 batch) {
    OFHE_VGPR_FLOOR();
    __shared__ u64 lds[2048];
    const u32 logn = P.log_n, N = 1u << logn, half = N >> 1;
    const u32 pb = blockIdx.x;
    const u32 t = pb % P.towers, b = pb / P.towers;
    const u64 soff = (u64)b * P.sstride + (u64)t * N;
    const u64 off = (u64)b * P.dstride + (u64)t * N;
    const TowerConst tc = P.tc[t];
    const u64 q = tc.q;
    const Mod<SPQ> M = load_mod<SPQ>(tc);
    const u64* tw = P.tw + (u64)t * N * 2;
    (void)batch;
    for (u32 i = threadIdx.x; i < N; i += blockDim.x) lds[i] = src[soff + i];
    __syncthreads();
    if (MODE == MODE_FWD || MODE == MODE_FUSED) {
        for (u32 m = 1, lt = logn - 1; m < N; m <<= 1, lt--) {
            const u32 tt = 1u << lt;
            for (u32 k = threadIdx.x; k < half; k += blockDim.x) {
                const u32 i = k >> lt, j = (i << (lt + 1)) + (k & (tt - 1));
                u64 x = lds[j], y = lds[j + tt];
                ct_bfly<1>(x, y, ldtw(tw, m + i), M);
                lds[j] = x;
                lds[j + tt] = y;
            }
            __syncthreads();
        }
        for (u32 i = threadIdx.x; i < N; i += blockDim.x) {
            u64 x = canon_fwd<SPQ>(lds[i], M);
            if (MODE == MODE_FUSED) x = barrett_ref(x, bdat[off + i], q, tc.mu, tc.nshift);
            lds[i] = x;
        }
        __syncthreads();
        if (MODE == MODE_FWD) {
            for (u32 i = threadIdx.x; i < N; i += blockDim.x) dst[off + i] = lds[i];
            return;
        }
    }
    const u64* dtw = P.dtw + (u64)t * N * 2;
    for (u32 lt = 0; lt < logn; lt++) {
        const u32 tt = 1u << lt;
        for (u32 k = threadIdx.x; k < half; k += blockDim.x) {
            const u32 i = k >> lt, e = k & (tt - 1), j = (i << (lt + 1)) + e;
            u64 x = lds[j], y = lds[j + tt];
            ct_bfly<1>(x, y, ldtw(dtw, tt + e), M);
            lds[j] = x;
            lds[j + tt] = y;
        }
        __syncthreads();
    }
    const u64* tw_ = P.twist + (u64)t * N * 2;
    for (u32 i = threadIdx.x; i < N; i += blockDim.x) dst[off + i] = twist_out(lds[i], ldtw(tw_, i), M);
}

}  // namespace ofhe
