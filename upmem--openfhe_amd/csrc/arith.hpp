// arith.hpp -- 64-bit modular arithmetic for gfx950 (device side).
//
// gfx950 has no 64x64 integer multiplier: a u64 product is built from
// v_mad_u64_u32 / v_mul_lo_u32 / v_mul_hi_u32, each a multi-cycle VALU op
// (tools/microbench/*.hip; the block kernel runs at ~100 % of the VALU issue
// capacity by SQ counters, profiles/).  The NTT is therefore bound by integer
// multiplies, and these helpers minimise them:
//   * mulhi_approx: floor(a*b/2^64) - {0,1,2} with 3 multiplies (drops the
//     a0*b0 term and one carry; lazy reduction absorbs the slack);
//   * shoup_lazy: a*w mod q in [0, 4q) (Shoup/Harvey, "Faster arithmetic for
//     number-theoretic transforms"; the reference's canonical form is
//     NativeIntegerT::ModMulFastConstEq, ubintnat.h:1491-1497) -- 9 multiplies,
//     8 when q = 2^L - d with d < 2^32 (Mod<true>, see below);
//   * barrett_ref: bit-exact restatement of NativeIntegerT::ModMulFastEq
//     (ubintnat.h:1399-1413) for the vector x vector Hadamard product.
// All moduli satisfy q < 2^60 (OpenFHE MAX_MODULUS_SIZE = 60, basicint.h:44),
// so lazy values up to 8q < 2^63 never overflow.
//
// Alternatives measured and rejected (tools/exp_variants.py):
// VCC-free sign-mask conditional subtract, add_co/addc-chained 64-bit adds,
// splitting the fused multiply-adds into v_mul_lo_u32 + adds.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ofhe {

typedef uint64_t u64;
typedef uint32_t u32;

// VGPR allocation floor for every kernel of the library.  Round 2's
// grid-stride EvalMultCore, compiled to 56 VGPRs, returned wrong words
// whenever two or more of its workgroups shared a CU; the SAME machine code
// with its allocation raised to 64 (or 72) VGPRs is exact at every shape
// (tools/diag, DESIGN.md "The round-2 EvalMultCore failure").  A clobber of
// v63 makes every kernel allocate at least 64 VGPRs; at 64 a SIMD still holds
// its maximum of 8 waves, so occupancy is unchanged.
// The clobber sits in a guard's destructor, i.e. at every exit of the kernel
// where nothing is live any more, so it does not perturb the scheduling or
// the register assignment of the kernel body (at the kernel's entry it did:
// the column passes lost 10-19 %, same-process A/B).
struct VgprFloor {
    __device__ __forceinline__ ~VgprFloor() { asm volatile("" ::: "v63"); }
};
#define OFHE_VGPR_FLOOR() const VgprFloor ofhe_vgpr_floor_guard_

__device__ __forceinline__ u32 lo32(u64 x) { return (u32)x; }
__device__ __forceinline__ u32 hi32(u64 x) { return (u32)(x >> 32); }
__device__ __forceinline__ u64 pack(u32 lo, u32 hi) { return ((u64)hi << 32) | lo; }

// v_mad_u64_u32: a*b + c, exact in 64 bits for 32-bit a, b, c < 2^64 - (2^32-1)^2
__device__ __forceinline__ u64 mad32(u32 a, u32 b, u64 c) { return (u64)a * (u64)b + c; }

__device__ __forceinline__ u64 csub(u64 x, u64 m) { return x >= m ? x - m : x; }

// the general remainder of switch_mod1 (old modulus more than twice the new
// one): out of line, so the unrolled callers carry one copy of the division
__device__ __noinline__ u64 umod64(u64 v, u64 m) { return v % m; }
// NativeVectorT::SwitchModulus (mubintvecnat.cpp:111-136) of one value, with
// the per-modulus-pair constants computed once (sw_mod) outside the loops
struct SwMod {
    u64 half, nm, diff;
    bool down, small;  // nm <= om; om <= 2 nm (v < om + nm < 3 nm: two csubs)
};
__device__ __forceinline__ SwMod sw_mod(u64 om, u64 nm) {
    const bool down = nm <= om;
    return SwMod{om >> 1, nm, down ? nm - (om % nm) : nm - om, down, om <= 2 * nm};
}
__device__ __forceinline__ u64 switch_mod1(u64 v, const SwMod& m) {
    if (v > m.half) v += m.diff;
    if (m.down && v >= m.nm) v = m.small ? csub(csub(v, m.nm), m.nm) : umod64(v, m.nm);
    return v;
}

// csub for a wave-uniform m (held in SGPRs: the NTT kernels' per-tower
// moduli).  The compiler emits v_cmp_u64 + 2 cndmask + sub/subb (5 VALU ops)
// for csub; this selects on the borrow of the subtraction itself (sub_co,
// subb_co, 2 cndmask on that vcc: 4 ops, no 64-bit compare, fewer VCC
// hazard nops).  m MUST be uniform across the wave: an "s" operand of a
// divergent value would be read from lane 0.
#ifndef OFHE_CSUB_ASM
#define OFHE_CSUB_ASM 1
#endif
__device__ __forceinline__ u64 csub_s(u64 x, u64 m) {
#if OFHE_CSUB_ASM
    u32 lo, hi;
    asm("v_subrev_co_u32 %0, vcc, %4, %2\n\t"
        "v_subbrev_co_u32 %1, vcc, %5, %3, vcc\n\t"
        "v_cndmask_b32 %0, %0, %2, vcc\n\t"
        "v_cndmask_b32 %1, %1, %3, vcc"
        : "=&v"(lo), "=&v"(hi)
        : "v"(lo32(x)), "v"(hi32(x)), "s"(lo32(m)), "v"(hi32(m))
        : "vcc");
    return pack(lo, hi);
#else
    return csub(x, m);
#endif
}

// floor(a*b / 2^64) - e, e in {0, 1, 2}: drops a0*b0 and the carry of the
// middle sum.
#ifndef OFHE_QH_ADDC
#define OFHE_QH_ADDC 0  // measured: more instructions (add_co + cndmask), kept for reference
#endif
#ifndef OFHE_QH_MAD1
#define OFHE_QH_MAD1 0  // 1: the quotient's second middle word added by a multiply-add by an opaque 1 (A/B: no gain)
#endif
// `one` is 1 held in an SGPR the compiler cannot see through (Mod::one, loaded
// from the tower constants by the kernels' load_mod): then hi32(m2) * one + acc is ONE v_mad_u64_u32,
// where the plain 64-bit add of two zero-extended words costs a v_mov_b32 (the
// zero high word) plus a v_lshl_add_u64.  With a literal 1 LLVM folds the
// multiply away and the add comes back.
template <bool QA = false>
__device__ __forceinline__ u64 mulhi_approx(u64 a, u64 b, u32 one = 1) {
    if (QA) {
        // the two middle high words summed by add_co / addc_co straight into
        // an aligned (sum, carry) pair: the 64-bit accumulator of the final
        // mad without zero-extending moves or a 64-bit add
        const u32 h1 = __umulhi(lo32(a), hi32(b));
        const u32 h2 = __umulhi(hi32(a), lo32(b));
        u32 s, c;
        asm("v_add_co_u32 %0, vcc, %2, %3\n\t"
            "v_addc_co_u32 %1, vcc, 0, 0, vcc"
            : "=&v"(s), "=v"(c)
            : "v"(h1), "v"(h2)
            : "vcc");
        u64 sc = pack(s, c);
        asm("" : "+v"(sc));
        return mad32(hi32(a), hi32(b), sc);
    }
    if (OFHE_QH_ADDC) {
        // the two middle high words summed with an explicit carry word, so the
        // 64-bit accumulator is built by add/carry instead of zero-extending
        // moves plus a 64-bit add
        const u32 h1 = __umulhi(lo32(a), hi32(b));
        const u32 h2 = __umulhi(hi32(a), lo32(b));
        const u32 s = h1 + h2;
        return mad32(hi32(a), hi32(b), pack(s, s < h1));
    }
    const u64 m1 = mad32(lo32(a), hi32(b), 0);
    const u64 m2 = mad32(hi32(a), lo32(b), 0);
    if (OFHE_QH_MAD1) return mad32(hi32(m2), one, mad32(hi32(a), hi32(b), m1 >> 32));
    return mad32(hi32(a), hi32(b), (m1 >> 32) + (m2 >> 32));
}

// exact floor(a*b / 2^64)
__device__ __forceinline__ u64 mulhi_exact(u64 a, u64 b) {
    u64 p00 = mad32(lo32(a), lo32(b), 0);
    u64 m1 = mad32(lo32(a), hi32(b), (u64)hi32(p00));
    u64 m2 = mad32(hi32(a), lo32(b), (u64)lo32(m1));
    u64 h = mad32(hi32(a), hi32(b), (u64)hi32(m1));
    return h + (u64)hi32(m2);
}

// Modulus constants for the lazy butterflies.  SPQ ("special prime") marks a
// modulus q = 2^L - d with 33 <= L <= 60 and d < 2^32, i.e. hi32(q) is all
// ones below bit L-32.  Then 2^64 - q has high word 2^32 - 2^(L-32), and the
// cross product lo32(qh) * hi32(2^64-q) is -(lo32(qh) << (L-32)): a shift
// instead of a multiply.  Every modulus chain OpenFHE builds with
// FirstPrime/PreviousPrime near 2^L (nbtheory-impl.h:334-379) has this form.
// QA: the Shoup quotient's two middle words summed by add_co/addc into the
// final mad's accumulator pair (mulhi_approx<true>); chosen per kernel where a
// same-process A/B measured it faster (OFHE_QA_* in ntt_kernels.hpp)
template <bool SPQ, bool QA = false>
struct Mod {
    u64 q;    // modulus, q < 2^60
    u64 q4;   // 4q
    u64 q8;   // 8q
    u64 nq;   // 2^64 - q   (loaded, not derived, so LLVM keeps the adds)
    u64 nq4;  // 2^64 - 4q
    u64 nq8;  // 2^64 - 8q
    u32 sh;   // L - 32 (SPQ only)
    u32 one = 1;  // 1; loaded from TowerConst (opaque to LLVM) in the NTT kernels, see mulhi_approx
};

// Shoup with precomputed wp = floor(w*2^64/q): a*w mod q in [0, 4q) for any
// a < 2^64.  Harvey's bound gives [0, 2q) with the exact quotient; the
// approximate quotient is at most 2 short.  The remainder is formed as
// lo64(a*w) + lo64(qh*(2^64-q)), so there is no 64-bit subtraction.
template <bool SPQ, bool QA>
__device__ __forceinline__ u64 shoup_lazy(u64 a, u64 w, u64 wp, const Mod<SPQ, QA>& M) {
    const u64 qh = mulhi_approx<QA>(a, wp, M.one);
    u64 s = mad32(lo32(a), lo32(w), 0);
    s = mad32(lo32(qh), lo32(M.nq), s);
    u32 hi;
    if (SPQ)
        hi = hi32(s) + lo32(a) * hi32(w) + hi32(a) * lo32(w) - (lo32(qh) << M.sh) + hi32(qh) * lo32(M.nq);
    else
        hi = hi32(s) + lo32(a) * hi32(w) + hi32(a) * lo32(w) + lo32(qh) * hi32(M.nq) + hi32(qh) * lo32(M.nq);
    return pack(lo32(s), hi);
}

#ifndef OFHE_ACC_PIN
#define OFHE_ACC_PIN 1
#endif
// acc + shoup_lazy(a, w, wp) mod 2^64 with acc folded into the first
// multiply-add of the remainder: the Cooley-Tukey butterfly's x + w y costs no
// separate 64-bit add (the true value acc + [0, 4q) is below 2^64 at every
// call site, so the wrap-around arithmetic returns it exactly).
template <bool SPQ, bool QA>
__device__ __forceinline__ u64 shoup_lazy_acc(u64 a, u64 w, u64 wp, const Mod<SPQ, QA>& M, u64 acc) {
    const u64 qh = mulhi_approx<QA>(a, wp, M.one);
    u64 s = mad32(lo32(a), lo32(w), acc);
#if OFHE_ACC_PIN
    asm("" : "+v"(s));  // keeps LLVM from re-associating acc out of the mad chain
#endif
    s = mad32(lo32(qh), lo32(M.nq), s);
    u32 hi;
    if (SPQ)
        hi = hi32(s) + lo32(a) * hi32(w) + hi32(a) * lo32(w) - (lo32(qh) << M.sh) + hi32(qh) * lo32(M.nq);
    else
        hi = hi32(s) + lo32(a) * hi32(w) + hi32(a) * lo32(w) + lo32(qh) * hi32(M.nq) + hi32(qh) * lo32(M.nq);
    return pack(lo32(s), hi);
}

// Special-prime fold (q = 2^L - d, d < 2^32, 16 d < q; L - 32 = M.sh): any
// x < 2^(L+4) to r = (x mod 2^L) + (x >> L) d = x - (x >> L) q, r < 2^L + 15 d
// = q + 16 d < 2q.  Three instructions (shift, mask, one v_mad_u64_u32)
// against four for a conditional subtract, and a tighter result.
template <bool SPQ, bool QA>
__device__ __forceinline__ u64 fold_spq(u64 x, const Mod<SPQ, QA>& M) {
    const u32 xh = hi32(x) >> M.sh;
    const u32 d = lo32((1ull << (M.sh + 32)) - M.q);  // wave-uniform (scalar unit)
    return mad32(xh, d, pack(lo32(x), hi32(x) & ((1u << M.sh) - 1)));
}

// canonical Shoup: ModMulFastConstEq semantics (result in [0, q)), generic q.
__device__ __forceinline__ u64 shoup_canon(u64 a, u64 w, u64 wp, u64 q) {
    const Mod<false> M{q, 4 * q, 8 * q, 0 - q, 0 - 4 * q, 0 - 8 * q, 0};
    u64 r = shoup_lazy(a, w, wp, M);
    r = csub(r, 2 * q);
    return csub(r, q);
}

// NativeIntegerT::ModMulFastEq(b, q, mu), ubintnat.h:1399-1413, bit for bit:
//   prod = a*b (128-bit); n = msb(q) - 2;
//   est  = ((prod >> n) * mu) >> (n + 7);   r = lo64(prod - q*est); r -= q if r >= q.
// n_shift = msb(q) - 2 is passed in (per tower constant).
__device__ __forceinline__ u64 barrett_ref(u64 a, u64 b, u64 q, u64 mu, u32 n_shift) {
    // 128-bit product
    u64 p00 = mad32(lo32(a), lo32(b), 0);
    u64 m1 = mad32(lo32(a), hi32(b), (u64)hi32(p00));
    u64 m2 = mad32(hi32(a), lo32(b), (u64)lo32(m1));
    u64 hi = mad32(hi32(a), hi32(b), (u64)hi32(m1)) + (u64)hi32(m2);
    u64 lo = ((u64)lo32(m2) << 32) | lo32(p00);
    // (prod >> n) truncated to 64 bits (n in [0, 62])
    u64 sh = n_shift ? ((lo >> n_shift) | (hi << (64 - n_shift))) : lo;
    // (sh * mu) >> (n + 7): 128-bit product then shift
    u64 q00 = mad32(lo32(sh), lo32(mu), 0);
    u64 r1 = mad32(lo32(sh), hi32(mu), (u64)hi32(q00));
    u64 r2 = mad32(hi32(sh), lo32(mu), (u64)lo32(r1));
    u64 th = mad32(hi32(sh), hi32(mu), (u64)hi32(r1)) + (u64)hi32(r2);
    u64 tl = ((u64)lo32(r2) << 32) | lo32(q00);
    u32 s = n_shift + 7;  // in [7, 69]
    u64 est = s >= 64 ? (th >> (s - 64)) : ((tl >> s) | (th << (64 - s)));
    u64 r = lo - est * q;
    return r >= q ? r - q : r;
}

// Montgomery product a*b*2^-64 mod q in (0, 2q) for a < 12q (the lazy
// forward output after a CS stage), b < q canonical, q < 2^60.
//   t = a*b: with a < 1.5*2^63 and b1 = hi32(b) < 2^28 the two middle
//     products and the carry word sum to < 2^64, so they chain through one
//     64-bit accumulator (no zero-extended halves, no carry word);
//   m = lo64(t) * q^-1 mod 2^64, so lo64(m*q) = lo64(t) and
//   (t - m*q) / 2^64 = hi64(t) - hi64(m*q) exactly, in (-q, q): adding q
//   gives (0, 2q) with no carry/borrow test on the low word.
// qinv = q^-1 mod 2^64.
//
// OFHE_MONT2: the same value with the carries taken by add_co/addc instead
// of zero-extended 64-bit adds (LLVM emitted 9 register moves per product for
// the form below):
//   u = a1 b0 + a0 b1 (< 2^64 under the same bounds), t1 = x1 + u0 with
//   carry c, hi64(t) = a1 b1 + (u1 + c);
//   hi64(m q) = m1 q1 + hi32(S1) + L1 + carry(lo32(S1) + L0) with
//   S1 = m1 q0 + hi32(m0 q0) < 2^64 and L = m0 q1 < 2^60 (q < 2^60).
#ifndef OFHE_MONT2
#define OFHE_MONT2 0
#endif
__device__ __forceinline__ u64 mont_mul2(u64 a, u64 b, u64 q, u64 qinv) {
    const u64 x = mad32(lo32(a), lo32(b), 0);
    const u64 u = mad32(hi32(a), lo32(b), mad32(lo32(a), hi32(b), 0));
    u32 t1, e;
    asm("v_add_co_u32 %0, vcc, %2, %3\n\t"
        "v_addc_co_u32 %1, vcc, %4, 0, vcc"
        : "=&v"(t1), "=v"(e)
        : "v"(hi32(x)), "v"(lo32(u)), "v"(hi32(u))
        : "vcc");
    const u32 t0 = lo32(x);
    const u64 m0w = mad32(t0, lo32(qinv), 0);
    const u32 m0 = lo32(m0w), m1 = hi32(m0w) + t0 * hi32(qinv) + t1 * lo32(qinv);
    const u64 s1 = mad32(m1, lo32(q), (u64)__umulhi(m0, lo32(q)));
    const u64 l = mad32(m0, hi32(q), 0);
    u32 k, k2, junk;
    asm("v_add_co_u32 %2, vcc, %3, %5\n\t"
        "v_addc_co_u32 %0, vcc, %4, %6, vcc\n\t"
        "v_addc_co_u32 %1, vcc, 0, 0, vcc"
        : "=&v"(k), "=&v"(k2), "=&v"(junk)
        : "v"(lo32(s1)), "v"(hi32(s1)), "v"(lo32(l)), "v"(hi32(l))
        : "vcc");
    u64 kk = pack(k, k2);
    asm("" : "+v"(kk));
    const u64 h = mad32(m1, hi32(q), kk);               // hi64(m q)
    const u64 tq = mad32(hi32(a), hi32(b), q);          // a1 b1 + q
    return tq - h + (u64)e;
}
__device__ __forceinline__ u64 mont_mul(u64 a, u64 b, u64 q, u64 qinv) {
    if (OFHE_MONT2) return mont_mul2(a, b, q, qinv);
    const u64 x = mad32(lo32(a), lo32(b), 0);
    const u64 y = mad32(hi32(a), lo32(b), x >> 32);  // < 1.5*2^63 + 2^32
    const u64 z = mad32(lo32(a), hi32(b), y);        // + < 2^60: no wrap
    const u64 th = mad32(hi32(a), hi32(b), z >> 32);
    const u32 t0 = lo32(x), t1 = lo32(z);
    const u64 m0 = mad32(t0, lo32(qinv), 0);
    const u64 m = pack(lo32(m0), hi32(m0) + t0 * hi32(qinv) + t1 * lo32(qinv));
    return th + q - mulhi_exact(m, q);
}

// Exact 64x64 -> 128 product (for base conversion accumulation).
__device__ __forceinline__ void mul128(u64 a, u64 b, u64& lo, u64& hi) {
    u64 p00 = mad32(lo32(a), lo32(b), 0);
    u64 m1 = mad32(lo32(a), hi32(b), (u64)hi32(p00));
    u64 m2 = mad32(hi32(a), lo32(b), (u64)lo32(m1));
    hi = mad32(hi32(a), hi32(b), (u64)hi32(m1)) + (u64)hi32(m2);
    lo = ((u64)lo32(m2) << 32) | lo32(p00);
}

// BarrettUint128ModUint64, utils/utilities-int.h:61-103 (exact value; the
// final while-loop makes it canonical).  mu = floor(2^128 / m).
__device__ __forceinline__ u64 barrett128(u64 a_lo, u64 a_hi, u64 m, u64 mu_lo, u64 mu_hi) {
    u64 left_hi = mulhi_exact(a_lo, mu_lo);
    u64 mid_lo, mid_hi;
    mul128(a_lo, mu_hi, mid_lo, mid_hi);
    u64 tmp1 = mid_lo + left_hi;
    u64 carry = tmp1 < mid_lo;
    u64 tmp2 = mid_hi + carry;
    mul128(a_hi, mu_lo, mid_lo, mid_hi);
    u64 s = mid_lo + tmp1;
    carry = s < mid_lo;
    left_hi = mid_hi + carry;
    tmp1 = a_hi * mu_hi + tmp2 + left_hi;
    u64 r = a_lo - tmp1 * m;
    while (r >= m) r -= m;
    return r;
}

}  // namespace ofhe
