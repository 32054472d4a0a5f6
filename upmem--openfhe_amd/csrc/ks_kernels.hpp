// ks_kernels.hpp -- element kernels of ApproxModUp / ApproxModDown, the
// HYBRID key-switching inner product, SwitchModulus and automorphisms.
//
// All are HBM streams over [batch][towers][N] data with explicit batch
// strides (words), so they can address a tower range of a wider polynomial
// (the Q part of a Q|P polynomial, one digit slot of the key-switch digits)
// without copies.  Each thread handles two adjacent coefficients (16-byte
// accesses); N >= 2 keeps pairs inside one tower.
#pragma once
#include "eltwise_kernels.hpp"

namespace ofhe {

// one scalar per tower: s and its Shoup precon for modulus q
struct TowerScalar {
    u64 q, s, sp;
};
static_assert(sizeof(TowerScalar) == 24, "PlanArgs::scal reads TowerScalar as [towers][3] words");

// (pair index) -> (batch entry, tower, coefficient) for `towers` towers of N
struct PairIndex {
    u32 b, t, c;
};
__device__ __forceinline__ PairIndex pair_index(u64 i, u32 log_n, u32 towers) {
    const u64 e = 2 * i;
    const u32 row = (u32)(e >> log_n);  // batch * towers < 2^32 for any buffer that fits in HBM: 32-bit divide
    return PairIndex{row / towers, row % towers, (u32)(e & ((1ull << log_n) - 1))};
}

// out = x * s_t mod q_t (NativeVectorT::ModMulEq(scalar), mubintvecnat.cpp:310-332)
__global__ __launch_bounds__(256) void k_scale_towers(const TowerScalar* __restrict__ ts, const u64* x, u64* out,
                                                      u64 xstride, u64 ostride, u64 npairs, u32 log_n,
                                                      u32 towers) {
    OFHE_VGPR_FLOOR();
    const u64 step = (u64)gridDim.x * blockDim.x;
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < npairs; i += step) {
        const PairIndex p = pair_index(i, log_n, towers);
        const TowerScalar c = ts[p.t];
        const u64 inner = ((u64)p.t << log_n) + p.c;
        const ulonglong2 v = *reinterpret_cast<const ulonglong2*>(x + p.b * xstride + inner);
        *reinterpret_cast<ulonglong2*>(out + p.b * ostride + inner) =
            make_ulonglong2(shoup_canon(v.x, c.s, c.sp, c.q), shoup_canon(v.y, c.s, c.sp, c.q));
    }
}

// out = (x - y mod q_t) * s_t mod q_t: the last step of ApproxModDown,
// (m_vectors[i] - partPSwitchedToQ[i]) * PInvModq[i] (dcrtpoly-impl.h:1172).
__global__ __launch_bounds__(256) void k_sub_scale(const TowerScalar* __restrict__ ts, const u64* x, const u64* y,
                                                   u64* out, u64 xstride, u64 ystride, u64 ostride, u64 npairs,
                                                   u32 log_n, u32 towers) {
    OFHE_VGPR_FLOOR();
    const u64 step = (u64)gridDim.x * blockDim.x;
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < npairs; i += step) {
        const PairIndex p = pair_index(i, log_n, towers);
        const TowerScalar c = ts[p.t];
        const u64 inner = ((u64)p.t << log_n) + p.c;
        const ulonglong2 a = *reinterpret_cast<const ulonglong2*>(x + p.b * xstride + inner);
        const ulonglong2 b = *reinterpret_cast<const ulonglong2*>(y + p.b * ystride + inner);
        const u64 d0 = a.x < b.x ? a.x + c.q - b.x : a.x - b.x;  // ModSubFastEq
        const u64 d1 = a.y < b.y ? a.y + c.q - b.y : a.y - b.y;
        *reinterpret_cast<ulonglong2*>(out + p.b * ostride + inner) =
            make_ulonglong2(shoup_canon(d0, c.s, c.sp, c.q), shoup_canon(d1, c.s, c.sp, c.q));
    }
}

// Tower of the extended basis Ql|P for the key-switch inner product.
struct KsTower {
    u64 m;                // modulus
    u64 mu_lo, mu_hi;     // floor(2^128 / m)
    u64 key_off;          // word offset of this tower inside one key polynomial (QP layout)
    u64 r60, r60p, mu1;   // limb_reduce constants
};

// EvalFastKeySwitchCoreExt (keyswitch-hybrid.cpp:452-478):
//   ct0[i] = sum_j digits_j[i] * b_j[key(i)],  ct1[i] = sum_j digits_j[i] * a_j[key(i)]
// The reference accumulates canonical ModMul / ModAdd terms; the sum of exact
// 128-bit products reduced once by BarrettUint128ModUint64 is the same
// canonical residue (beta <= 2^8 terms below 2^120 cannot overflow 128 bits).
__global__ __launch_bounds__(256) void k_ks_inner(const KsTower* __restrict__ tw, const u64* __restrict__ digits,
                                                  const u64* __restrict__ kb, const u64* __restrict__ ka,
                                                  u64* __restrict__ ct0, u64* __restrict__ ct1, u64 key_stride,
                                                  u32 beta, u64 npairs, u32 log_n, u32 towers) {
    OFHE_VGPR_FLOOR();
    const u64 step = (u64)gridDim.x * blockDim.x;
    const u64 poly = (u64)towers << log_n;
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < npairs; i += step) {
        const PairIndex p = pair_index(i, log_n, towers);
        const KsTower T = tw[p.t];
        const u64 inner = ((u64)p.t << log_n) + p.c;
        const u64* d = digits + (u64)p.b * beta * poly + inner;
        const u64* pb = kb + T.key_off + p.c;
        const u64* pa = ka + T.key_off + p.c;
        u64 b0l = 0, b0h = 0, b1l = 0, b1h = 0, a0l = 0, a0h = 0, a1l = 0, a1h = 0;
        for (u32 j = 0; j < beta; j++) {
            const ulonglong2 x = *reinterpret_cast<const ulonglong2*>(d + (u64)j * poly);
            const ulonglong2 vb = *reinterpret_cast<const ulonglong2*>(pb + (u64)j * key_stride);
            const ulonglong2 va = *reinterpret_cast<const ulonglong2*>(pa + (u64)j * key_stride);
            u64 l, h;
            mul128(x.x, vb.x, l, h);
            b0l += l;
            b0h += h + (b0l < l);
            mul128(x.y, vb.y, l, h);
            b1l += l;
            b1h += h + (b1l < l);
            mul128(x.x, va.x, l, h);
            a0l += l;
            a0h += h + (a0l < l);
            mul128(x.y, va.y, l, h);
            a1l += l;
            a1h += h + (a1l < l);
        }
        const u64 o = (u64)p.b * poly + inner;
        *reinterpret_cast<ulonglong2*>(ct0 + o) = make_ulonglong2(barrett128(b0l, b0h, T.m, T.mu_lo, T.mu_hi),
                                                                  barrett128(b1l, b1h, T.m, T.mu_lo, T.mu_hi));
        *reinterpret_cast<ulonglong2*>(ct1 + o) = make_ulonglong2(barrett128(a0l, a0h, T.m, T.mu_lo, T.mu_hi),
                                                                  barrett128(a1l, a1h, T.m, T.mu_lo, T.mu_hi));
    }
}

// Same product, batch-stationary keys: a thread owns (tower, C coefficients)
// and walks the batch, so each key word is read once per launch instead of
// once per ciphertext.  Sums use the 30-bit limb split and limb_reduce of
// k_bconv_limb (beta <= 16 terms below 2^60 per limb sum).  BETA is the exact
// digit count (no masked slots), and the next ciphertext's digits are loaded
// before the current one is reduced, so one load latency hides behind a
// whole iteration of arithmetic.  C = 1 halves the per-thread state of C = 2
// (more waves in flight).  SQ counters (configs[4]): 149 VALU instructions per
// ciphertext per thread, two thirds of them limb_reduce, at ~66 % of the VALU
// issue peak; a two-deep prefetch (6 loads in flight) measured no gain.
#ifndef OFHE_KS_CPT
#define OFHE_KS_CPT 1
#endif
template <int C>
struct Words {
    u64 v[C];
};
template <int C>
__device__ __forceinline__ Words<C> ldw(const u64* p) {
    Words<C> w;
    if constexpr (C == 2) {
        const u64x2 t = ld2_s(p);
        w.v[0] = t.x;
        w.v[1] = t.y;
    } else {
        w.v[0] = ld_s(p);
    }
    return w;
}
template <int C>
__device__ __forceinline__ void stw(u64* p, const u64* v) {
    if constexpr (C == 2) {
        u64x2 t;
        t.x = v[0];
        t.y = v[1];
        st2_s(p, t);
    } else {
        st_s(p, v[0]);
    }
}

// Digit j's own towers [own.start[j], own.start[j] + own.cnt[j]) are the
// ciphertext's evaluation-form towers unchanged (keyswitch-hybrid.cpp:402-404);
// when `c` is given they are read from it (c: [batch][size_ql][N], stride
// c_stride) instead of from a copy in the digit slot, so KeySwitchCore skips
// writing and re-reading that copy.
struct KsOwn {
    u32 start[4], cnt[4];
};
template <int BETA, int C>
__global__ __launch_bounds__(256) void k_ks_inner_bs(const KsTower* __restrict__ tw, const u64* __restrict__ digits,
                                                     const u64* __restrict__ kb, const u64* __restrict__ ka,
                                                     u64* __restrict__ ct0, u64* __restrict__ ct1, u64 key_stride,
                                                     u32 batch, u64 nthreads, u32 log_n, u32 towers,
                                                     const u64* __restrict__ c_in, u64 c_stride, KsOwn own) {
    OFHE_VGPR_FLOOR();
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nthreads) return;
    const u64 e = C * i;
    const u32 t = (u32)(e >> log_n), c = (u32)(e & ((1ull << log_n) - 1));
    const KsTower T = tw[t];
    const LimbRed R{T.m, T.r60, T.r60p, T.mu1};
    const u64 poly = (u64)towers << log_n;
    const u64 inner = ((u64)t << log_n) + c;
    u64 kl[BETA][2 * C];  // (b[0..C), a[0..C)) as (lo30 | hi30 << 32)
#pragma unroll
    for (int j = 0; j < BETA; j++) {
        const u64 off = T.key_off + c + (u64)j * key_stride;
        const Words<C> vb = ldw<C>(kb + off), va = ldw<C>(ka + off);
#pragma unroll
        for (int k = 0; k < C; k++) {
            kl[j][k] = (vb.v[k] & LIMB_MASK) | ((vb.v[k] >> LIMB) << 32);
            kl[j][C + k] = (va.v[k] & LIMB_MASK) | ((va.v[k] >> LIMB) << 32);
        }
    }
    // one ciphertext: BETA digit words -> ct0/ct1 words of batch entry b
    auto one = [&](const Words<C> (&x)[BETA], u32 b) {
        u64 acc[2 * C][4];  // k < C: ct0 coefficient k; k >= C: ct1 coefficient k - C
#pragma unroll
        for (int k = 0; k < 2 * C; k++) acc[k][0] = acc[k][1] = acc[k][2] = acc[k][3] = 0;
#pragma unroll
        for (int j = 0; j < BETA; j++) {
#pragma unroll
            for (int k = 0; k < 2 * C; k++) {
                const u64 xv = x[j].v[k % C];
                const u32 x0 = (u32)(xv & LIMB_MASK), x1 = (u32)(xv >> LIMB);
                const u64 kw = kl[j][k];
                acc[k][0] = mad32(x0, lo32(kw), acc[k][0]);
                acc[k][1] = mad32(x0, hi32(kw), acc[k][1]);
                acc[k][2] = mad32(x1, lo32(kw), acc[k][2]);
                acc[k][3] = mad32(x1, hi32(kw), acc[k][3]);
            }
        }
        u64 r[2 * C];
#pragma unroll
        for (int k = 0; k < 2 * C; k++) r[k] = limb_reduce<false>(acc[k][0], acc[k][1], acc[k][2], acc[k][3], R);
        const u64 o = (u64)b * poly + inner;
        stw<C>(ct0 + o, r);
        stw<C>(ct1 + o, r + C);
    };
    auto load = [&](Words<C> (&x)[BETA], u32 b) {
        const u64* d = digits + (u64)b * BETA * poly + inner;
#pragma unroll
        for (int j = 0; j < BETA; j++) {
            const bool mine = c_in && t - own.start[j] < own.cnt[j];  // wave-uniform for N >= 64 C
            x[j] = ldw<C>(mine ? c_in + (u64)b * c_stride + inner : d + (u64)j * poly);
        }
    };
    Words<C> xn[BETA];
    load(xn, 0);
    for (u32 b = 0; b < batch; b++) {
        Words<C> x[BETA];
#pragma unroll
        for (int j = 0; j < BETA; j++) x[j] = xn[j];
        if (b + 1 < batch) load(xn, b + 1);
        one(x, b);
    }
}

// NativeVectorT::SwitchModulus (mubintvecnat.cpp:111-136), value for value.
__global__ __launch_bounds__(256) void k_switch_modulus(const u64* src, u64* dst, u64 n, u64 om, u64 nm) {
    OFHE_VGPR_FLOOR();
    const u64 step = (u64)gridDim.x * blockDim.x;
    const u64 half = om >> 1;
    const bool up = nm > om;
    const u64 diff = up ? nm - om : nm - (om % nm);
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += step) {
        u64 v = src[i];
        if (v > half) v += diff;
        if (!up && v >= nm) v %= nm;
        dst[i] = v;
    }
}

// Rescaling callers of SwitchModulus (dcrtpoly-impl.h:746-768 and 792-812):
// the dropped tower's coefficients v (canonical mod ql), optionally scaled
// first by pre (ModReduce's delta *= negtInvModq), are lifted into every
// remaining q_i and combined per tower with the scalars of tab[i] =
// (q_i, w_i, w_i', a_i, a_i', 0):
//   SW_SCALE  y = sw(v) w                   (evaluation form; the NTT and the
//                                            x a / (x - .) a step follow in
//                                            the fused forward-subtract pass)
//   SW_AXPY   y = x a + sw(v) w             (DropLastElementAndScale, coefficient form)
//   SW_XPYA   y = (x + sw(v) w) a           (ModReduce, coefficient form)
// one thread per (batch entry, tower, coefficient); canonical outputs.
enum { SW_SCALE = 0, SW_AXPY = 1, SW_XPYA = 2 };
struct SwArgs {
    const u64* last;  // [batch] rows of N (stride lstride)
    u64 lstride;
    const u64* x;     // [batch][towers][N] (stride xstride), SW_AXPY / SW_XPYA
    u64 xstride;
    u64* y;           // [batch][towers][N] (stride ystride)
    u64 ystride;
    const u64* tab;   // [towers][6]
    u64 ql, pre, pre_p;  // pre: scalar on v mod ql first (1: none)
    u32 log_n, towers;
};
// two coefficients per thread (16-byte accesses); w = 1 (DropLastElementAndScale
// with the reference's constants, where QlQlInvModqlDivqlModq = -qlInvModq)
// skips the multiply
template <int MODE>
__global__ __launch_bounds__(256) void k_switch_scale(SwArgs A, u32 bpr) {
    OFHE_VGPR_FLOOR();
    const u32 row = blockIdx.x / bpr, b = row / A.towers, t = row % A.towers;  // bpr blocks per row
    const u64 N = 1ull << A.log_n;
    const u64 j = 2 * ((u64)(blockIdx.x % bpr) * blockDim.x + threadIdx.x);
    if (j >= N) return;
    const u64* T = A.tab + 6 * (u64)t;
    const u64 q = T[0], w = T[1], wp = T[2], a = T[3], ap = T[4];
    const SwMod sm = sw_mod(A.ql, q);
    const ulonglong2 lv = *reinterpret_cast<const ulonglong2*>(A.last + b * A.lstride + j);
    u64 r[2] = {lv.x, lv.y};
    ulonglong2 xv = make_ulonglong2(0, 0);
    if (MODE != SW_SCALE) xv = *reinterpret_cast<const ulonglong2*>(A.x + b * A.xstride + (u64)t * N + j);
    const u64 xs[2] = {xv.x, xv.y};
#pragma unroll
    for (int k = 0; k < 2; k++) {
        u64 v = r[k];
        if (A.pre != 1) v = shoup_canon(v, A.pre, A.pre_p, A.ql);
        v = switch_mod1(v, sm);
        if (w != 1) v = shoup_canon(v, w, wp, q);
        if (MODE == SW_AXPY) v = csub(shoup_canon(xs[k], a, ap, q) + v, q);
        if (MODE == SW_XPYA) v = shoup_canon(csub(xs[k] + v, q), a, ap, q);
        r[k] = v;
    }
    st2_s(A.y + b * A.ystride + (u64)t * N + j, u64x2{r[0], r[1]});
}

// KeySwitchBV::EvalFastKeySwitchCore (keyswitch-bv.cpp:314-340):
//   ct0 = sum_i bv[i] . d_i,  ct1 = sum_i av[i] . d_i   (per tower, mod q_t)
// over `nd` digits.  One thread per (batch entry, tower, coefficient): the
// products are summed exactly in 128 bits (nd <= 256 terms below 2^120) and
// reduced once (BarrettUint128ModUint64, utilities-int.h:61-103) -- the
// canonical residue the reference's per-term ModMul / ModAdd chain ends on.
struct BvArgs {
    const u64* d;     // [batch][nd][towers][N]
    const u64* kb;    // [nd][key_towers][N]
    const u64* ka;
    u64* o0;          // [batch][towers][N]
    u64* o1;
    const u64* mu;    // [towers][3]: q, floor(2^128 / q) lo, hi
    u32 nd, towers, key_towers, log_n;
};
__global__ __launch_bounds__(256) void k_bv_inner(BvArgs A, u32 bpr) {
    OFHE_VGPR_FLOOR();
    const u32 row = blockIdx.x / bpr, b = row / A.towers, t = row % A.towers;
    const u64 N = 1ull << A.log_n;
    const u64 j = (u64)(blockIdx.x % bpr) * blockDim.x + threadIdx.x;
    if (j >= N) return;
    const u64 dstep = (u64)A.towers * N, kstep = (u64)A.key_towers * N;
    const u64* dp = A.d + (u64)b * A.nd * dstep + (u64)t * N + j;
    const u64* bp = A.kb + (u64)t * N + j;
    const u64* ap = A.ka + (u64)t * N + j;
    u64 l0 = 0, h0 = 0, l1 = 0, h1 = 0;
    for (u32 i = 0; i < A.nd; i++) {
        const u64 dv = ld_s(dp + i * dstep);
        u64 lo, hi;
        mul128(bp[i * kstep], dv, lo, hi);
        l0 += lo;
        h0 += hi + (l0 < lo);
        mul128(ap[i * kstep], dv, lo, hi);
        l1 += lo;
        h1 += hi + (l1 < lo);
    }
    const u64 q = A.mu[3 * t], ml = A.mu[3 * t + 1], mh = A.mu[3 * t + 2];
    const u64 o = (u64)b * A.towers * N + (u64)t * N + j;
    st_s(A.o0 + o, barrett128(l0, h0, q, ml, mh));
    st_s(A.o1 + o, barrett128(l1, h1, q, ml, mh));
}

// PolyImpl::AutomorphismTransform(k) (poly-impl.h:338-364).  One thread per
// index j of one (batch, tower) row:
//   evaluation form:  dst[rev(j)] = src[rev(((k (2j+1)) >> 1) mod n)]
//   coefficient form: dst[(j k) mod n] = bit_logn(j k) ? q - src[j] : src[j]
// (products taken mod 2n, which is what the reference's wrapping uint32
// arithmetic keeps, 2n dividing 2^32).
template <bool EVAL>
__global__ __launch_bounds__(256) void k_automorphism(const TowerConst* __restrict__ tcs, const u64* src, u64* dst,
                                                      u32 k, u64 total, u32 log_n, u32 towers) {
    OFHE_VGPR_FLOOR();
    const u64 step = (u64)gridDim.x * blockDim.x;
    const u64 n = 1ull << log_n, mask = n - 1, m2 = 2 * n - 1;
    for (u64 e = (u64)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += step) {
        const u64 row = e >> log_n;
        const u64 j = e & mask;
        const u64 base = row << log_n;
        if (EVAL) {
            const u64 jk = ((u64)k * (2 * j + 1)) & m2;
            const u32 jrev = __builtin_bitreverse32((u32)j) >> (32 - log_n);
            const u32 irev = __builtin_bitreverse32((u32)((jk >> 1) & mask)) >> (32 - log_n);
            dst[base + jrev] = src[base + irev];
        } else {
            const u64 q = tcs[(u32)row % towers].q;
            const u64 jk = ((u64)k * j) & m2;
            const u64 v = src[base + j];
            dst[base + (jk & mask)] = ((jk >> log_n) & 1) ? q - v : v;
        }
    }
}

}  // namespace ofhe
