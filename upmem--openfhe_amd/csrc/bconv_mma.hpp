// bconv_mma.hpp -- ApproxSwitchCRTBasis (dcrtpoly-impl.h:1034-1063) on the
// matrix cores: the sum over source towers is an integer GEMM, done with
// v_mfma_i32_32x32x32_i8 on signed 8-bit digits, and only the reduction mod
// p_j stays on the VALU.
//
// Per coefficient, y_i = [x_i * QHatInvModq_i]_{q_i} (canonical, < 2^60) and
//   out_j = sum_i y_i * QHatModp_{i,j}  mod p_j.
// Write y_i = sum_a d_{i,a} 2^(8a) with signed digits d in [-128, 127]
// (a = 0..7), and fold the digit weight into the constant:
//   h_{(i,a),j} = 2^(8a) * QHatModp_{i,j} mod p_j = sum_b e_{(i,a),j,b} 2^(8b)
// (signed digits again).  Then
//   out_j == sum_b 2^(8b) C_{j,b}  (mod p_j),   C_{j,b} = sum_{(i,a)} d_{i,a} e_{(i,a),j,b},
// an exact int32 GEMM with K = 8 * size_q (|C| <= 8 size_q 2^14 <= 2^22 for
// size_q <= 32) and 8 columns per target.  The reduction of the 8 partial
// sums costs ~45 VALU instructions per output against ~130 for the 64
// v_mad_u64_u32 of the limb kernel plus its reduction (k_bconv_limb).
//
// Signed digits of v < 2^63: z = v + 0x8080808080808080, d_a = byte_a(z) - 128
// = byte_a(z) ^ 0x80 read as int8 (sum_a (byte_a(z) - 128) 2^(8a) = z - 0x80..80 = v).
// So a 64-bit word of 8 packed digits is ((v + C) ^ C), three instructions,
// and is directly one half of a lane's 16-byte MFMA operand.
//
// MFMA orientation: D[(j,b)][coef] = sum_k H[(j,b)][k] * Y[k][coef], A = H
// (constant, pre-swizzled on the host into per-lane fragments), B = Y.
// 32x32x32 i8, lane l = c + 32h (c = l & 31, h = l >> 5):
//   B: lane l holds 16 k's of column c; we label them k = (source 4s + 2h +
//      (e >> 3), digit e & 7) for byte e of the fragment (K-step s);
//   A: lane l holds the same 16 k labels of row c;
//   D: lane l holds column c, rows (reg & 3) + 8 (reg >> 2) + 4h, reg 0..15.
// The host orders A's rows so that register reg of lane half h is
// (target 4t + 2h + (reg >> 3), digit b = reg & 7): every lane ends a tile
// with all 8 partial sums of 2 outputs of its coefficient, no lane exchange.
// The k labelling only has to agree between A and B, which it does by
// construction; tests/test_gpu_keyswitch.py checks the kernel against the
// oracle at every tile / K-step count the key switch uses.
#pragma once
#include "eltwise_kernels.hpp"

namespace ofhe {

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));

constexpr u64 DIGIT_BIAS = 0x8080808080808080ull;
constexpr u32 BCONV_MMA_QMAX = 64;            // size_q <= 64: |C| <= 2^23 (K-steps up to 16)
constexpr u32 BCONV_MMA_LDS_MAX = 64 * 1024;  // one target chunk's fragments + constants (dynamic LDS)
constexpr u32 BCONV_MMA_THREADS = 512;
#ifndef OFHE_BCONV_MMA
#define OFHE_BCONV_MMA 1  // 0: the limb / 128-bit kernels only (A/B builds)
#endif
#ifndef OFHE_BCONV_MMA_SPQ
#define OFHE_BCONV_MMA_SPQ 1  // special-prime reduction when every target allows it
#endif
#ifndef OFHE_BCONV_MMA_PF
#define OFHE_BCONV_MMA_PF 1  // prefetch the next group's x (K-steps <= 8)
#endif
#ifndef OFHE_BCONV_MMA_WAVES
#define OFHE_BCONV_MMA_WAVES 0  // __launch_bounds__ min waves per SIMD (0: compiler's choice)
#endif
#ifndef OFHE_BCONV_MMA_BPC
#define OFHE_BCONV_MMA_BPC 3
#endif
constexpr u32 BCONV_MMA_BLOCKS_PER_CU = OFHE_BCONV_MMA_BPC;  // grid cap: 256 CUs x this

// per-target reduction constants (64 B, one LDS row)
struct BmRed {
    u64 p, np;        // p, 2^64 - p
    u64 r60, r60p;    // 2^60 mod p, floor(r60 * 2^64 / p)   (SPQ: d, (L - 32) | mask << 32)
    u64 mu1;          // floor(2^64 / p)
    u64 blo, bhi;     // bias: blo + bhi * 2^32 = k p >= 2^80, blo in [2^48, 2^48 + 2^32), bhi >= 2^48 - 2^16
    u64 p2;           // 2p
};
// per-source constants
struct BmSrc {
    u64 q, w, wp, pad;  // q_i, QHatInvModq_i, its Shoup precon
};

// 8 signed digits of v (< 2^63), packed
__device__ __forceinline__ u64 digits8(u64 v) { return (v + DIGIT_BIAS) ^ DIGIT_BIAS; }

// The digit weights arrive in SGPRs the compiler cannot see through (1, 2^8,
// 2^16, 2^24), so each 64-bit term is one v_mad_i64_i32; with literal powers
// of two LLVM emits sign-extension, a 64-bit shift and an add per term instead.
struct BmW {
    int w0, w8, w16, w24;
};
__device__ __forceinline__ BmW bm_weights() {
    BmW W;
    asm volatile("s_mov_b32 %0, 1\n\ts_mov_b32 %1, 0x100\n\ts_mov_b32 %2, 0x10000\n\ts_mov_b32 %3, 0x1000000"
                 : "=s"(W.w0), "=s"(W.w8), "=s"(W.w16), "=s"(W.w24));
    return W;
}
__device__ __forceinline__ long long mad_i64(int a, int b, long long c) { return (long long)a * (long long)b + c; }

// sum_b C_b 2^(8b) mod p for |C_b| <= 2^23: canonical, or in [0, 4p) when
// LAZY (internal callers whose next step is a forward NTT, which takes < 4p).
//   lo_u = blo + sum_{b<4} C_b 2^(8b),  hi_u = bhi + sum_{b>=4} C_b 2^(8(b-4))   (both in (0, 2^49))
//     WIDE (|C| up to 2^23): four v_mad_i64_i32 per half; else (|C| <= 2^22)
//     x01 = C0 + C1 2^8 (int32, |x| < 2^30.01) and two v_mad_i64_i32 per half
//   T' = lo_u + hi_u 2^32 = T + k p = H 2^60 + L',  H = hi_u >> 28 < 2^21,
//        L' = lo_u + (hi_u mod 2^28) 2^32 < 2^60 + 2^49
//   t  = H (2^60 mod p) - qh p + L'   with qh = single-word Shoup quotient
//        (<= 1 short: H (2^60 mod p) - qh p in [0, 3p)), so t < 2^62.01
//   r  = t - mulhi~(t, floor(2^64/p)) p in [0, 4p)   (as limb_reduce), then two csubs.
//
// SPQ (every target p = 2^L - d, d < 2^32, with (2^(81-L) + 1) d + 2^49 + 2d
// < 2^L, checked by the host): T' = H 2^L + L'' with H = hi_u >> (L - 32)
// < 2^(81-L) and L'' < 2^L + 2^49, and T' == L'' + H d (mod p) with
// L'' + H d < 2p: one v_mad_u64_u32 and at most one conditional subtract.
template <bool LAZY, bool SPQ, bool WIDE>
__device__ __forceinline__ u64 bm_reduce(const int* C, const BmRed& R, const BmW& W) {
    u64 lo_u, hi_u;
    if (WIDE) {
        lo_u = (u64)mad_i64(C[3], W.w24, mad_i64(C[2], W.w16, mad_i64(C[1], W.w8, mad_i64(C[0], W.w0, (long long)R.blo))));
        hi_u = (u64)mad_i64(C[7], W.w24, mad_i64(C[6], W.w16, mad_i64(C[5], W.w8, mad_i64(C[4], W.w0, (long long)R.bhi))));
    } else {
        const int x01 = C[0] + C[1] * 256, x23 = C[2] + C[3] * 256;
        const int x45 = C[4] + C[5] * 256, x67 = C[6] + C[7] * 256;
        lo_u = (u64)mad_i64(x23, W.w16, mad_i64(x01, W.w0, (long long)R.blo));
        hi_u = (u64)mad_i64(x67, W.w16, mad_i64(x45, W.w0, (long long)R.bhi));
    }
    if (SPQ) {
        const u32 sh = lo32(R.r60p), mask = hi32(R.r60p);
        const u32 H = (u32)(hi_u >> sh);
        const u64 l2 = pack(lo32(lo_u), hi32(lo_u) + (lo32(hi_u) & mask));
        const u64 r = mad32(H, lo32(R.r60), l2);  // < 2p
        return LAZY ? r : csub(r, R.p);
    }
    const u32 H = (u32)(hi_u >> 28);
    const u32 qh = hi32(mad32(H, hi32(R.r60p), (u64)__umulhi(H, lo32(R.r60p))));
    const u32 lh = hi32(lo_u) + (lo32(hi_u) & 0x0FFFFFFFu) + H * hi32(R.r60) + qh * hi32(R.np);
    u64 t = mad32(qh, lo32(R.np), pack(lo32(lo_u), lh));
    t = mad32(H, lo32(R.r60), t);
    const u64 q2 = mulhi_approx(t, R.mu1);
    const u64 s = mad32(lo32(q2), lo32(R.np), t);
    u64 r = pack(lo32(s), hi32(s) + lo32(q2) * hi32(R.np) + hi32(q2) * lo32(R.np));
    if (LAZY) return r;
    r = csub(r, R.p2);
    return csub(r, R.p);
}

// One wave = 32 coefficients (a group of one batch entry, N >= 32); the
// block's waves walk the groups grid-stride and share one target chunk's
// fragment table in LDS: blockIdx.y selects tiles [y*tpc, y*tpc + tpc) of the
// targets (mm_tpc tiles per chunk, sized so a chunk fits 64 KiB), so any
// number of targets converts on the matrix cores; each chunk recomputes the
// sources' digits for its coefficients.  KS = K-steps of 4 source towers
// (size_q <= 4 KS); above 8 the partial sums need the WIDE combine.
template <int KS, bool LAZY, bool SPQ>
__global__ __launch_bounds__(BCONV_MMA_THREADS, OFHE_BCONV_MMA_WAVES) void k_bconv_mma(
    BconvArgs A, const u64* __restrict__ x, u64* __restrict__ out, u32 batch) {
    OFHE_VGPR_FLOOR();
    constexpr bool WIDE = KS > 8;
    constexpr bool PF = OFHE_BCONV_MMA_PF && KS <= 8;  // registers: the prefetch holds 2 KS words
    extern __shared__ __attribute__((aligned(16))) unsigned char bm_lds[];
    const u32 tiles = A.mm_tiles, tpc = A.mm_tpc;
    const u32 t0 = blockIdx.y * tpc;
    const u32 nt = min(tpc, tiles - t0);
    i32x4* frag = reinterpret_cast<i32x4*>(bm_lds);                       // [nt][KS][64]
    BmRed* red = reinterpret_cast<BmRed*>(bm_lds + (size_t)nt * KS * 1024);  // [4 nt]
    BmSrc* src = reinterpret_cast<BmSrc*>(red + 4 * nt);                  // [4 KS]
    {
        // global image: fragments [tiles][KS][64], BmRed [4 tiles], BmSrc [4 KS]
        const i32x4* gf = reinterpret_cast<const i32x4*>(A.mm_tab) + (size_t)t0 * KS * 64;
        const i32x4* gr = reinterpret_cast<const i32x4*>(A.mm_tab) + (size_t)tiles * KS * 64 + (size_t)t0 * 16;
        const i32x4* gs = reinterpret_cast<const i32x4*>(A.mm_tab) + (size_t)tiles * KS * 64 + (size_t)tiles * 16;
        i32x4* lf = frag;
        i32x4* lr = reinterpret_cast<i32x4*>(red);
        i32x4* ls = reinterpret_cast<i32x4*>(src);
        for (u32 k = threadIdx.x; k < nt * KS * 64; k += blockDim.x) lf[k] = gf[k];
        for (u32 k = threadIdx.x; k < nt * 16; k += blockDim.x) lr[k] = gr[k];
        for (u32 k = threadIdx.x; k < KS * 8; k += blockDim.x) ls[k] = gs[k];
    }
    __syncthreads();
    const BmW W = bm_weights();
    const u32 lane = threadIdx.x & 63, c = lane & 31, h = lane >> 5;
    const u32 N = 1u << A.log_n;
    const u64 groups = ((u64)batch << A.log_n) >> 5;
    const u32 wpb = blockDim.x >> 6;
    const u64 gstep = (u64)gridDim.x * wpb;
    // x of the wave's next group is loaded before the current group's tiles
    // (PF), so the HBM latency hides under the MFMA / VALU work
    u64 xv[KS][2];
    auto load_x = [&](u64 gg) {
        const u64 e = (gg << 5) + c;
        const u64* xb = x + (e >> A.log_n) * A.in_stride + (e & (N - 1));
#pragma unroll
        for (int s = 0; s < KS; s++)
#pragma unroll
            for (int u = 0; u < 2; u++) {
                const u32 i = 4 * s + 2 * h + u;
                xv[s][u] = i < A.size_q ? ld_s(xb + (u64)i * N) : 0;
            }
    };
    u64 g = (u64)blockIdx.x * wpb + (threadIdx.x >> 6);
    if (PF && g < groups) load_x(g);
    for (; g < groups; g += gstep) {
        const u64 e = (g << 5) + c;
        const u64 b = e >> A.log_n;
        const u32 ri = (u32)(e & (N - 1));
        u64* ob = out + b * A.out_stride + ri;
        if (!PF) load_x(g);
        i32x4 bf[KS];
#pragma unroll
        for (int s = 0; s < KS; s++) {
            u64 d[2];
#pragma unroll
            for (int u = 0; u < 2; u++) {
                const u32 i = 4 * s + 2 * h + u;
                u64 y = 0;
                if (i < A.size_q) {
                    const BmSrc S = src[i];
                    y = shoup_canon(xv[s][u], S.w, S.wp, S.q);
                }
                d[u] = digits8(y);
            }
            bf[s] = i32x4{(int)lo32(d[0]), (int)hi32(d[0]), (int)lo32(d[1]), (int)hi32(d[1])};
        }
        if (PF && g + gstep < groups) load_x(g + gstep);
        for (u32 t = 0; t < nt; t++) {
            i32x16 acc = {};
#pragma unroll
            for (int s = 0; s < KS; s++)
                acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(frag[(t * KS + s) * 64 + lane], bf[s], acc, 0, 0, 0);
#pragma unroll
            for (int u = 0; u < 2; u++) {
                const u32 j = 4 * (t0 + t) + 2 * h + u;
                if (j < A.size_p) {
                    int C[8];
#pragma unroll
                    for (int k = 0; k < 8; k++) C[k] = acc[8 * u + k];
                    const u32 jo = j >= A.gap_at ? j + A.gap : j;
                    st_s(ob + (u64)jo * N, bm_reduce<LAZY, SPQ, WIDE>(C, red[4 * t + 2 * h + u], W));
                }
            }
        }
    }
}

}  // namespace ofhe
