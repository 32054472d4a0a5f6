// eltwise_kernels.hpp -- coefficient-wise RNS ops and base conversion (gfx950).
//
// Element-wise kernels are pure HBM streams (24 B per coefficient for a
// vector-vector op): 16-byte loads/stores, grid-stride, one tower constant
// set per polynomial.  They replace the DPU VECTOR/VECTOR_EQ kernels of
// src/core/pim/dpu/element-wise/{add-mod,sub-mod,mult-mod}.c and the CPU loops
// of NativeVectorT (mubintvecnat.cpp:245-367).
#pragma once
#include "ntt_kernels.hpp"

namespace ofhe {

enum { ELT_MUL = 0, ELT_ADD = 1, ELT_SUB = 2, ELT_MULS = 3, ELT_ADDS = 4, ELT_SUBS = 5 };

// ModAddFastEq (ubintnat.h:760-767) and ModSubFastEq (934-938) on canonical operands
__device__ __forceinline__ u64 modadd_fast(u64 a, u64 b, u64 q) { return csub(a + b, q); }
__device__ __forceinline__ u64 modsub_fast(u64 a, u64 b, u64 q) { return a < b ? a + q - b : a - b; }

// a, b, c: [batch][towers][N], vector (.) vector.  Each thread moves
// elt_unroll(OP) independent 16-byte pairs, all loads issued before any
// arithmetic, streaming hints on data.  The host launches one thread per
// elt_unroll(OP) pairs (no grid-stride at the sizes used): measured at N=2^16,
// 16 towers, batch 256 on MI355X, a 4096-block grid-stride launch moved
// 4.5-4.7 TB/s, the full grid 6.0-6.3 TB/s (ModMul best with 2 pairs per
// thread, the add/sub/scalar ops with 1; DESIGN.md "Element-wise bandwidth").
#ifdef OFHE_ELT_UNROLL
__host__ __device__ constexpr int elt_unroll(int) { return OFHE_ELT_UNROLL; }
#else
__host__ __device__ constexpr int elt_unroll(int op) { return op == ELT_MUL ? 2 : 1; }
#endif
// LeveledSHEBase::EvalMultCore for two 2-element ciphertexts
// (base-leveledshe.cpp:667-672): o2 = c1 d1, o1 = c1 d0 + c0 d1, o0 = d0 c0,
// each product NativeVectorT::ModMul (Barrett, ubintnat.h:1399-1413) and the
// sum ModAdd, in one pass: 32 B read and 24 B written per coefficient against
// 120 B for the four products and the sum as separate vector ops.
// One (batch, tower) row per bpr blocks, so the tower constants are
// wave-uniform (scalar loads); two coefficients per thread.
template <int V = 0>  // a template: this header is included by several translation units
__global__ __launch_bounds__(256) void k_tensor2(const TowerConst* __restrict__ tcs, const u64* c0, const u64* c1,
                                                 const u64* d0, const u64* d1, u64* o0, u64* o1, u64* o2, u32 bpr,
                                                 u32 log_n, u32 towers) {
    OFHE_VGPR_FLOOR();
    const u32 row = blockIdx.x / bpr;
    const u64 j = 2 * ((u64)(blockIdx.x % bpr) * blockDim.x + threadIdx.x);
    if (j >= (1ull << log_n)) return;
    const u64 e = ((u64)row << log_n) + j;
    const TowerConst tc = tcs[row % towers];
    const u64x2 a0 = ld2_s(c0 + e), a1 = ld2_s(c1 + e), b0 = ld2_s(d0 + e), b1 = ld2_s(d1 + e);
    u64x2 r0, r1, r2;
    r2.x = barrett_ref(a1.x, b1.x, tc.q, tc.mu, tc.nshift);
    r2.y = barrett_ref(a1.y, b1.y, tc.q, tc.mu, tc.nshift);
    r1.x = modadd_fast(barrett_ref(a1.x, b0.x, tc.q, tc.mu, tc.nshift), barrett_ref(a0.x, b1.x, tc.q, tc.mu, tc.nshift), tc.q);
    r1.y = modadd_fast(barrett_ref(a1.y, b0.y, tc.q, tc.mu, tc.nshift), barrett_ref(a0.y, b1.y, tc.q, tc.mu, tc.nshift), tc.q);
    r0.x = barrett_ref(b0.x, a0.x, tc.q, tc.mu, tc.nshift);
    r0.y = barrett_ref(b0.y, a0.y, tc.q, tc.mu, tc.nshift);
    st2_s(o0 + e, r0);
    st2_s(o1 + e, r1);
    st2_s(o2 + e, r2);
}

template <int OP>
__global__ __launch_bounds__(256) void k_eltwise(const TowerConst* __restrict__ tcs,
                                                 const u64* a, const u64* b, u64* c, u64 npairs,
                                                 u32 log_n, u32 towers) {
    OFHE_VGPR_FLOOR();
    constexpr int ELT_U = elt_unroll(OP);
    const u64 stride = (u64)gridDim.x * blockDim.x;
    for (u64 i0 = (u64)blockIdx.x * blockDim.x + threadIdx.x; i0 < npairs; i0 += stride * ELT_U) {
        u64x2 x[ELT_U], y[ELT_U];
#pragma unroll
        for (int u = 0; u < ELT_U; u++) {
            const u64 i = i0 + u * stride;
            if (i < npairs) {
                x[u] = ld2_s(a + 2 * i);
                y[u] = ld2_s(b + 2 * i);
            }
        }
#pragma unroll
        for (int u = 0; u < ELT_U; u++) {
            const u64 i = i0 + u * stride;
            if (i >= npairs) break;
            const u32 t = (u32)((2 * i) >> log_n) % towers;  // row < 2^32: 32-bit modulo
            u64x2 r;
            if (OP == ELT_MUL) {
                const TowerConst tc = tcs[t];
                r.x = barrett_ref(x[u].x, y[u].x, tc.q, tc.mu, tc.nshift);
                r.y = barrett_ref(x[u].y, y[u].y, tc.q, tc.mu, tc.nshift);
            } else if (OP == ELT_ADD) {
                const u64 q = tcs[t].q;
                r.x = modadd_fast(x[u].x, y[u].x, q);
                r.y = modadd_fast(x[u].y, y[u].y, q);
            } else {
                const u64 q = tcs[t].q;
                r.x = modsub_fast(x[u].x, y[u].x, q);
                r.y = modsub_fast(x[u].y, y[u].y, q);
            }
            st2_s(c + 2 * i, r);
        }
    }
}

// Vector (.) scalar with one scalar per tower, the scalars passed by value in
// the kernel arguments (no device table, so no upload to order against other
// launches): ModMul(const IntegerType&) (Shoup, mubintvecnat.cpp:310-332),
// ModAdd(Eq) / ModSub(Eq)(const IntegerType&) (mubintvecnat.cpp:198-219, 267-288), the
// DPU SCALAR kernels of src/core/pim/dpu/element-wise/{add,sub,mult}-mod.c.
// One launch covers towers [t0, t0 + cnt) of every batch entry (cnt <=
// SCALAR_MAX); the host splits wider plans into several launches.
constexpr u32 SCALAR_MAX = 96;  // 96 x 24 B = 2304 B of kernel arguments
struct ScalarPack {
    u64 v[3 * SCALAR_MAX];  // per tower of the range: q, s (reduced mod q), Shoup precon of s
};
template <int OP>
__global__ __launch_bounds__(256) void k_scalar(ScalarPack S, const u64* a, u64* c, u64 npairs, u32 log_n,
                                                u32 cnt, u32 t0, u32 towers) {
    OFHE_VGPR_FLOOR();
    const u64 stride = (u64)gridDim.x * blockDim.x;
    const u64 mask = (1ull << log_n) - 1;
    constexpr int ELT_U = elt_unroll(OP);
    for (u64 i0 = (u64)blockIdx.x * blockDim.x + threadIdx.x; i0 < npairs; i0 += stride * ELT_U) {
        u64x2 x[ELT_U];
        u64 at[ELT_U];
#pragma unroll
        for (int u = 0; u < ELT_U; u++) {
            const u64 i = i0 + u * stride;
            const u64 e = 2 * i;
            const u32 row = (u32)(e >> log_n);  // b * cnt + tl (< 2^32: batch * towers fits a launch)
            at[u] = (((u64)(row / cnt) * towers + t0 + row % cnt) << log_n) | (e & mask);
            if (i < npairs) x[u] = ld2_s(a + at[u]);
        }
#pragma unroll
        for (int u = 0; u < ELT_U; u++) {
            const u64 i = i0 + u * stride;
            if (i >= npairs) break;
            const u32 tl = (u32)((2 * i) >> log_n) % cnt;
            const u64 q = S.v[3 * tl], s = S.v[3 * tl + 1];
            u64x2 r;
            if (OP == ELT_MULS) {
                const u64 sp = S.v[3 * tl + 2];
                r.x = shoup_canon(x[u].x, s, sp, q);
                r.y = shoup_canon(x[u].y, s, sp, q);
            } else if (OP == ELT_ADDS) {
                r.x = modadd_fast(x[u].x, s, q);
                r.y = modadd_fast(x[u].y, s, q);
            } else {
                r.x = modsub_fast(x[u].x, s, q);
                r.y = modsub_fast(x[u].y, s, q);
            }
            st2_s(c + at[u], r);
        }
    }
}

// NativeVectorT::ModAddAtIndex(Eq)(i, b) (mubintvecnat.cpp:221-231): c[idx] of every
// (batch, tower) = a[idx] + s_t mod q_t -- what PolyImpl::Plus(Integer) does in
// coefficient form (poly-impl.h:213-220).  One thread per (batch, tower) of the
// range; the other words are the caller's (in place, or copied beforehand).
static __global__ __launch_bounds__(256) void k_scalar_at(ScalarPack S, const u64* a, u64* c, u32 batch, u32 log_n,
                                                   u32 cnt, u32 t0, u32 towers, u64 idx) {
    OFHE_VGPR_FLOOR();
    const u64 r = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= (u64)batch * cnt) return;
    const u32 tl = (u32)(r % cnt);
    const u64 b = r / cnt;
    const u64 at = ((b * towers + t0 + tl) << log_n) + idx;
    c[at] = modadd_fast(a[at], S.v[3 * tl + 1], S.v[3 * tl]);
}

// Synthetic uniform residues (bench / tests): word i of tower
// t of batch entry b is splitmix64 draw i + 1 of the stream seeded
// 0x5EED ^ (b << 20) ^ (t << 8) ^ seed, mod q_t -- the same numbers as the
// oracle's sequential generator (splitmix64 is counter-based: draw k mixes
// seed + k * 0x9E3779B97F4A7C15).
static __global__ __launch_bounds__(256) void k_fill_uniform(const TowerConst* __restrict__ tcs, u64* dst, u64 words,
                                                      u32 log_n, u32 towers, u32 b0, u64 seed) {
    OFHE_VGPR_FLOOR();
    const u64 stride = (u64)gridDim.x * blockDim.x;
    for (u64 e = (u64)blockIdx.x * blockDim.x + threadIdx.x; e < words; e += stride) {
        const u32 row = (u32)(e >> log_n);
        const u32 t = row % towers;
        const u64 b = (u64)(row / towers) + b0;
        const u64 i = e & ((1ull << log_n) - 1);
        u64 z = (0x5EEDull ^ (b << 20) ^ ((u64)t << 8) ^ seed) + (i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        dst[e] = z % tcs[t].q;
    }
}

// ---------------------------------------------------------------------------
// ApproxSwitchCRTBasis (dcrtpoly-impl.h:1034-1063): per coefficient ri,
//   y_i   = [x_i * QHatInvModq_i]_{q_i}                 (Shoup, canonical)
//   s_j   = sum_i y_i * QHatModp_{i,j}                  (128-bit accumulate)
//   out_j = BarrettUint128ModUint64(s_j, p_j, mu_j)     (canonical)
// One thread per (batch, ri); the P side is processed in tiles of PT towers
// so the 128-bit accumulators stay in registers.
// ---------------------------------------------------------------------------
struct BconvArgs {
    const u64* qv;        // [sizeQ]
    const u64* qhinv;     // [sizeQ][2]  (QHatInvModq, Shoup precon)
    const u64* qhmodp;    // [sizeQ][sizeP]
    const u64* qhlimb;    // [sizeQ][sizeP rounded up to BCONV_PT], (c mod 2^30) | (c >> 30) << 32, zero padded
    const u64* pv;        // [sizeP]
    const u64* pmu;       // [sizeP][2]  (mu_lo, mu_hi) = floor(2^128 / p)
    const u64* pred;      // [sizeP][3]  (2^60 mod p, its Shoup precon, floor(2^64 / p)): limb_reduce
    u64 in_stride;        // words between batch entries of x   (sizeQ * N when dense)
    u64 out_stride;       // words between batch entries of out (sizeP * N when dense)
    u32 log_n, size_q, size_p;
    u32 gap_at, gap;      // output tower j >= gap_at is written at j + gap (key-switch digit slot)
    const void* mm_tab;   // k_bconv_mma fragment table + constants (bconv_mma.hpp), or null
    u32 mm_tiles, mm_ks;  // its target tiles (4 towers) and K-steps (4 source towers)
    u32 mm_tpc;           // target tiles per block (blockIdx.y chunk) that fit the LDS budget
    u32 lazy_out;         // internal callers: outputs in [0, 4p) (a forward NTT follows)
    u32 mm_spq;           // k_bconv_mma: every target a special prime (bm_reduce's shift fold)
    u32 kernel;           // OFHE_BCONV_KERNEL_* (host-side choice in bconv_run)
};

template <int PT>
__global__ __launch_bounds__(256) void k_bconv(BconvArgs A, const u64* __restrict__ x,
                                               u64* __restrict__ out, u32 batch) {
    OFHE_VGPR_FLOOR();
    const u32 N = 1u << A.log_n;
    const u64 gid = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= (u64)batch * N) return;
    const u32 b = (u32)(gid >> A.log_n), ri = (u32)(gid & (N - 1));
    const u64* xb = x + (u64)b * A.in_stride + ri;
    u64* ob = out + (u64)b * A.out_stride + ri;
    for (u32 j0 = 0; j0 < A.size_p; j0 += PT) {
        u64 lo[PT], hi[PT];
#pragma unroll
        for (int j = 0; j < PT; j++) lo[j] = hi[j] = 0;
        const u32 jn = min((u32)PT, A.size_p - j0);
        for (u32 i = 0; i < A.size_q; i++) {
            const u64 y = shoup_canon(ld_s(xb + (u64)i * N), A.qhinv[2 * i], A.qhinv[2 * i + 1], A.qv[i]);
            const u64* qm = A.qhmodp + (u64)i * A.size_p + j0;
#pragma unroll
            for (int j = 0; j < PT; j++) {
                if (j < (int)jn) {
                    u64 pl, ph;
                    mul128(y, qm[j], pl, ph);
                    const u64 s = lo[j] + pl;
                    hi[j] += ph + (s < pl);
                    lo[j] = s;
                }
            }
        }
#pragma unroll
        for (int j = 0; j < PT; j++) {
            if (j < (int)jn) {
                const u32 jj = j0 + j;
                const u32 jo = jj >= A.gap_at ? jj + A.gap : jj;
                ob[(u64)jo * N] = barrett128(lo[j], hi[j], A.pv[jj], A.pmu[2 * jj], A.pmu[2 * jj + 1]);
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Limb variant (any size_q <= 16).  y_i is split into two 30-bit limbs and
// every QHatModp entry c < 2^60 is pre-split the same way, so
//   sum_i y_i c_ij = A0 + (A1 + A2) 2^30 + A3 2^60,
//   A0 = sum y0 c0, A1 = sum y0 c1, A2 = sum y1 c0, A3 = sum y1 c1,
// where every A is a sum of at most 16 products below 2^60: four
// v_mad_u64_u32 per term and no carry handling (mul128 plus a 128-bit add
// needs the same four multiplies and the carries).  The total is reduced by
// limb_reduce to the canonical value BarrettUint128ModUint64 gives.  The limb table is zero-padded to a multiple of PT
// columns so the inner loop has no branches.
// ---------------------------------------------------------------------------
constexpr u32 LIMB = 30;
constexpr u64 LIMB_MASK = (1ull << LIMB) - 1;
#ifndef OFHE_BCONV_PT
#define OFHE_BCONV_PT 8
#endif
constexpr u32 BCONV_PT = OFHE_BCONV_PT;  // output towers per tile
constexpr u32 BCONV_LIMB_QMAX = 16;

// S mod m for S = A0 + (A1 + A2) 2^30 + A3 2^60 < 2^124 (every limb sum below
// 2^64; m < 2^60), canonical: the value BarrettUint128ModUint64 returns for
// the same S, with about half its instructions.  Write S = H 2^60 + L,
// L < 2^60 (H < 2^64 by the bound on S); then
//   r1 = H * (2^60 mod m) mod m in [0, 4m)       (Shoup, shoup_lazy)
//   T  = r1 + L < 4m + 2^60 < 2^63
//   r2 = T - floor~(T * floor(2^64/m) / 2^64) m  in [0, 4m)
// (the quotient estimate is at most 3 short: 1 from the truncated reciprocal,
// 2 from mulhi_approx), and two conditional subtractions.  R carries
// (m, 2^60 mod m, its Shoup precon, floor(2^64 / m)); UNI: m is wave-uniform.
struct LimbRed {
    u64 m, r60, r60p, mu1;
};
template <bool UNI>
__device__ __forceinline__ u64 limb_reduce(u64 a0, u64 a1, u64 a2, u64 a3, const LimbRed& R) {
    constexpr u64 M60 = (1ull << 60) - 1;
    const u64 mid = a1 + a2;
    const u64 mh = (mid >> LIMB) | ((u64)(mid < a1) << (64 - LIMB));  // (A1 + A2) >> 30, 65-bit sum
    const u64 low = (a0 & M60) + ((mid & LIMB_MASK) << LIMB);          // < 2^61
    const u64 H = a3 + mh + (a0 >> 60) + (low >> 60);
    const Mod<false> M{R.m, 0, 0, 0 - R.m, 0, 0, 0};
    const u64 t = shoup_lazy(H, R.r60, R.r60p, M) + (low & M60);
    const u64 qh = mulhi_approx(t, R.mu1);
    const u64 nq = 0 - R.m;
    const u64 s = mad32(lo32(qh), lo32(nq), t);  // t - qh m, low 64 bits
    u64 r = pack(lo32(s), hi32(s) + lo32(qh) * hi32(nq) + hi32(qh) * lo32(nq));
    if (UNI) {
        r = csub_s(r, 2 * R.m);
        return csub_s(r, R.m);
    }
    r = csub(r, 2 * R.m);
    return csub(r, R.m);
}

template <int PT>
__global__ __launch_bounds__(256) void k_bconv_limb(BconvArgs A, const u64* __restrict__ x, u64* __restrict__ out,
                                                    u32 batch) {
    OFHE_VGPR_FLOOR();
    // y limbs of every source tower, computed once per coefficient and kept
    // in this thread's own LDS column across the P tiles (no barrier needed)
    __shared__ u64 ys[BCONV_LIMB_QMAX][256];
    const u32 N = 1u << A.log_n;
    const u64 gid = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= (u64)batch * N) return;
    const u32 b = (u32)(gid >> A.log_n), ri = (u32)(gid & (N - 1));
    const u64* xb = x + (u64)b * A.in_stride + ri;
    u64* ob = out + (u64)b * A.out_stride + ri;
    const u32 ppad = (A.size_p + PT - 1) / PT * PT;
    const u32 tid = threadIdx.x;
    for (u32 i = 0; i < A.size_q; i++) {
        const u64 y = shoup_canon(ld_s(xb + (u64)i * N), A.qhinv[2 * i], A.qhinv[2 * i + 1], A.qv[i]);
        ys[i][tid] = (y & LIMB_MASK) | ((y >> LIMB) << 32);
    }
    for (u32 j0 = 0; j0 < A.size_p; j0 += PT) {
        u64 a0[PT], a1[PT], a2[PT], a3[PT];
#pragma unroll
        for (int j = 0; j < PT; j++) a0[j] = a1[j] = a2[j] = a3[j] = 0;
        // unrolled so that one s_waitcnt covers several towers' constant loads
        // (scalar loads return out of order: each wait is lgkmcnt(0))
#ifndef OFHE_BCONV_UNROLL
#define OFHE_BCONV_UNROLL 4
#endif
#pragma unroll OFHE_BCONV_UNROLL
        for (u32 i = 0; i < A.size_q; i++) {
            const u64 yy = ys[i][tid];
            const u32 y0 = lo32(yy), y1 = hi32(yy);
            const u64* cl = A.qhlimb + (u64)i * ppad + j0;
#pragma unroll
            for (int j = 0; j < PT; j++) {
                const u64 c = cl[j];
                a0[j] = mad32(y0, lo32(c), a0[j]);
                a1[j] = mad32(y0, hi32(c), a1[j]);
                a2[j] = mad32(y1, lo32(c), a2[j]);
                a3[j] = mad32(y1, hi32(c), a3[j]);
            }
        }
#pragma unroll
        for (int j = 0; j < PT; j++) {
            const u32 jj = j0 + j;
            if (jj < A.size_p) {
                const u32 jo = jj >= A.gap_at ? jj + A.gap : jj;
                const LimbRed R{A.pv[jj], A.pred[3 * jj], A.pred[3 * jj + 1], A.pred[3 * jj + 2]};
                st_s(ob + (u64)jo * N, limb_reduce<true>(a0[j], a1[j], a2[j], a3[j], R));
            }
        }
    }
}

}  // namespace ofhe
