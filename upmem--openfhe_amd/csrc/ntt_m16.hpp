// ntt_m16.hpp -- the fused pipeline's block pass at N = 2^16 with all four of
// its radix-16 rounds on the matrix cores, every round one SHARED 16 x 16 map
// (k_block_m16).
//
// After the column pass (stages 1-8), group G of 256 elements holds the
// coefficients of a(X) mod (X^256 - theta_G^256), theta_G = psi^(2 rev8(G) + 1)
// (transformnat-impl.h:300-354 run to stage 8).  The reference's remaining
// forward stages evaluate it at theta_G w256^rev8(i), w256 = psi^512, i.e. a
// twist followed by a cyclic 256-point DFT in bit-reversed order, which splits
// 16 x 16 with one shared matrix F[r][j] = w16^(j rev4(r)) (w16 = w256^16):
//   z_j = x_j theta_G^j                               (twist, per element)
//   A[r'][j0] = sum_j1 F[r'][j1] z[j0 + 16 j1]       (round A, columns (j0, G))
//   B[r'][j0] = A[r'][j0] w256^(j0 rev4(r'))         (twiddle, 256 values)
//   Y[16 r' + r] = sum_j0 F[r][j0] B[r'][j0]          (round B, columns (r', G))
// and the inverse (the DIT form of ntt_kernels.hpp, transformnat-impl.h:492-552)
// mirrors it with F'[j][r] = w16^(-j rev4(r)):
//   A'[r'][j0] = sum_r F'[j0][r] y[16 r' + r]          (round A', columns (r', G))
//   B'[r'][j0] = A'[r'][j0] w256^(-j0 rev4(r'))
//   Z[j0 + 16 j1] = sum_r' F'[j1][r'] B'[r'][j0]      (round B', columns (j0, G))
//   out_j = Z_j N^-1 2^64 theta_G^-j                  (twist_r, as k_block)
// tools/mma_model.py checks these identities with exact integers against the
// reference's loops.  Between round B and round A' sits the Montgomery
// Hadamard; it needs no data movement because an MFMA tile's output layout
// (lane (c, h) holds rows 4 mt + 2 h + u of column c) is the next tile's
// B-operand layout (inputs 4 s + 2 h + u).  Rounds A -> B and A' -> B'
// transpose through a wave-private LDS region (the two groups of the tile).
//
// Each round is the k_bconv_mma digit GEMM (bconv_mma.hpp): K = 16 inputs x 8
// signed digits, M = 16 outputs x 8 constant digits, 16 v_mfma_i32_32x32x32_i8
// per 32 columns, and bm_reduce<lazy, SPQ> (< 2q) on the VALU; F and F'
// fragments sit in LDS (32 KiB, shared by the workgroup's 8 waves).  VALU work
// per coefficient: 4 x (digit split 3 + reduce ~12) + twist, two twiddles and
// the inverse twist (4 Shoup products, ~14 each) + Montgomery Hadamard (~20),
// against k_block's 8 butterfly stages per direction (block pass).
// Special-prime plans only (bm_reduce<.., SPQ>), checked by the host.
#pragma once
#include "ntt_mma.hpp"

namespace ofhe {

constexpr u32 M16_WAVES = 8;
constexpr u32 M16_THREADS = 64 * M16_WAVES;
constexpr u32 M16_XW = 2 * 272;  // words of a wave's exchange region: 2 groups x 16 rows x 17
#ifndef OFHE_M16_WAVES
#define OFHE_M16_WAVES 4  // __launch_bounds__ waves per SIMD (<= 128 VGPRs)
#endif

struct M16Args {
    const i32x4* frag;  // [towers][2][1024]: F then F' (A-operand fragments)
    const BmRed* red;   // [towers]
    const u64* twf;     // [towers][N][2]: theta_G^j, Shoup pairs (forward twist)
    const u64* w16;     // [towers][2][256][2]: w256^(j0 rev4(r')), then w256^(-j0 rev4(r')), at [r'][j0]
};

// exchange placement of (group gs of the tile, row, column), rows padded to 17
__device__ __forceinline__ u32 m16_x(u32 gs, u32 row, u32 col) { return gs * 272 + row * 17 + col; }

// src: column-pass output (any u64; the twist takes it to [0, 4q)), dst: the
// inverse column pass's input (< 4q), bdat: the Hadamard operand (canonical)
__global__ __launch_bounds__(M16_THREADS, OFHE_M16_WAVES) void k_block_m16(PlanArgs P, M16Args Q, const u64* src,
                                                                           u64* dst, const u64* __restrict__ bdat,
                                                                           u32 batch, u32 nwg) {
    OFHE_VGPR_FLOOR();
    constexpr u32 N = 1u << 16;
    __shared__ i32x4 fr[2 * 1024];          // F, F' (32 KiB)
    __shared__ u64 xb[M16_WAVES * M16_XW];  // wave-private exchange regions (34 KiB)
    const u32 tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const u32 wid = xcd_remap(blockIdx.x, nwg);
    const u32 bp = wid & 7;  // groups 32 bp .. 32 bp + 31 (two 4096-element blocks)
    const u32 pb = wid >> 3;
    const u32 t = pb / batch, b = pb % batch;
    {
        const i32x4* g = Q.frag + (size_t)t * 2048;
#pragma unroll
        for (u32 k = 0; k < 2048 / M16_THREADS; k++) fr[tid + k * M16_THREADS] = g[tid + k * M16_THREADS];
    }
    const TowerConst tc = P.tc[t];
    const Mod<true> M = load_mod<true>(tc);
    const BmRed R = Q.red[t];
    const BmW W = bm_weights();
    const u32 c = lane & 31, h = lane >> 5, col = c & 15, gs = c >> 4;
    const u64 inner = (u64)t * N;
    const u64* xs = src + (u64)b * P.sstride + inner;
    u64* ys = dst + (u64)b * P.dstride + inner;
    const u64* bs = bdat + (u64)b * P.bstride + inner;
    const u64* twf = Q.twf + inner * 2;
    const u64* twi = P.twist + inner * 2;
    const u64* w16f = Q.w16 + (size_t)t * 1024;
    const u64* w16i = w16f + 512;
    u64* xw = xb + w * M16_XW;
    __syncthreads();
#pragma unroll 1
    for (u32 it = 0; it < 2; it++) {
        const u32 tau = w + M16_WAVES * it;  // tile: the workgroup's groups 2 tau, 2 tau + 1
        const u32 gbase = (32 * bp + 2 * tau + gs) * 256;
        u64 xv[8];
        // round A: column (j0 = col, G), inputs z[j0 + 16 j1], j1 = 4 s + 2 h + u
#pragma unroll
        for (int s = 0; s < 4; s++)
#pragma unroll
            for (int u = 0; u < 2; u++) {
                const u32 e = gbase + col + 16 * (4 * s + 2 * h + u);
                const Tw f = ldtw(twf, e);
                xv[2 * s + u] = shoup_lazy(ld_s(xs + e), f.w, f.wp, M);  // [0, 4q)
            }
        nm_gemm(xv, fr, lane, h, R, W, [&](u32 k, u64 v) {  // k = r'
            const Tw f = ldtw(w16f, k * 16 + col);
            xw[m16_x(gs, k, col)] = shoup_lazy(v, f.w, f.wp, M);
        });
        __builtin_amdgcn_wave_barrier();
        // round B: column (r' = col, G), inputs B[r'][j0], j0 = 4 s + 2 h + u
#pragma unroll
        for (int s = 0; s < 4; s++)
#pragma unroll
            for (int u = 0; u < 2; u++) xv[2 * s + u] = xw[m16_x(gs, col, 4 * s + 2 * h + u)];
        __builtin_amdgcn_wave_barrier();
        u64 yv[8];
        nm_gemm(xv, fr, lane, h, R, W, [&](u32 k, u64 v) { yv[2 * (k >> 2) + (k & 1)] = v; });  // k = r, < 2q
        // Hadamard with b at position 16 r' + r (Montgomery; twist_r carries 2^64)
#pragma unroll
        for (int mt = 0; mt < 4; mt++) {
            const u64x2 bb = ld2_s(bs + gbase + 16 * col + 4 * mt + 2 * h);
            yv[2 * mt] = mont_mul(yv[2 * mt], bb.x, tc.q, tc.qinv);  // (0, 2q)
            yv[2 * mt + 1] = mont_mul(yv[2 * mt + 1], bb.y, tc.q, tc.qinv);
        }
        // round A': the same column (r' = col, G), inputs y[16 r' + r] in yv's order
        nm_gemm(yv, fr + 1024, lane, h, R, W, [&](u32 k, u64 v) {  // k = j0
            const Tw f = ldtw(w16i, col * 16 + k);
            xw[m16_x(gs, col, k)] = shoup_lazy(v, f.w, f.wp, M);
        });
        __builtin_amdgcn_wave_barrier();
        // round B': column (j0 = col, G), inputs B'[r'][j0], r' = 4 s + 2 h + u
#pragma unroll
        for (int s = 0; s < 4; s++)
#pragma unroll
            for (int u = 0; u < 2; u++) xv[2 * s + u] = xw[m16_x(gs, 4 * s + 2 * h + u, col)];
        __builtin_amdgcn_wave_barrier();
        nm_gemm(xv, fr + 1024, lane, h, R, W, [&](u32 k, u64 v) {  // k = j1
            const u32 e = gbase + col + 16 * k;
            const Tw f = ldtw(twi, e);
            st_s(ys + e, shoup_lazy(v, f.w, f.wp, M));  // [0, 4q) for the inverse column pass
        });
    }
}

}  // namespace ofhe
