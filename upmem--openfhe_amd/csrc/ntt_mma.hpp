// ntt_mma.hpp -- the fused pipeline's block pass at N = 2^16 with two of its
// four radix-16 rounds on the matrix cores (k_block_mma).
//
// The block pass of c = INTT(NTT(a) . b) runs, on every 256-element group i of
// a tower (transformnat-impl.h:300-354 and 492-552, stages in the reference's
// order):
//   level 3  forward CT stages m = 256 .. 2048 (t = 128 .. 16): for each
//            column cc < 16 the 16 elements cc + 16 j mix through one 16 x 16
//            map F_i -- the same for every column and every polynomial;
//   level 4  forward stages m = 4096 .. 32768 on contiguous 16-element blocks
//            (twiddles per block);
//   Hadamard with b (Montgomery, as k_block);
//   inverse  GS stages t = 1 .. 8 on the contiguous blocks, then GS stages
//            t = 16 .. 128 on the columns: again one map per group, V_i, with
//            N^-1 and the Montgomery 2^64 folded in.
// The k_block pass runs all four rounds as butterflies (~36 VALU instructions
// per coefficient per round, plus a 14-instruction twist); here F_i and V_i
// are exact int32 GEMMs on signed base-256 digits
// (v_mfma_i32_32x32x32_i8, the k_bconv_mma scheme of bconv_mma.hpp: K = 16
// inputs x 8 digits, M = 16 outputs x 8 constant digits, |partial sum| <=
// 128 * 2^14 = 2^21), and only the digit split (SPQ fold + 4 instructions)
// and the special-prime reduction of the 8 partial sums (~12 instructions)
// stay on the VALU.  The inverse keeps the reference's GS form, so there is no
// output twist.
//
// F_i and V_i differ per group, so their reuse comes from the batch: a
// workgroup owns one (tower, group) and walks a chunk of the batch, 16
// polynomials per iteration, with both matrices' A fragments (32 KiB) in LDS,
// loaded once.  Each iteration:
//   A  waves: 2 polynomials x 16 columns = the 32 MFMA columns; 4 M-tiles x
//      4 K-steps; reduce (lazy, < 2q) into the exchange buffer;
//   B  threads (polynomial, block r): level 4, Hadamard, inverse GS t = 1..8;
//   C  waves: V_i like A, canonical-lazy (< 2q) output to the inverse column
//      pass (k_tcols<inv>, which takes < 4q).
// Special-prime plans only (bm_reduce<.., SPQ>); the host checks the
// reduction's admissibility per tower.
#pragma once
#include "ntt_kernels.hpp"
#include "bconv_mma.hpp"

namespace ofhe {

constexpr u32 NM_POLYS = 16;    // polynomials per iteration
constexpr u32 NM_THREADS = 256;
constexpr u32 NM_FRAG = 16 * 64;  // i32x4 fragments per matrix (4 M-tiles x 4 K-steps x 64 lanes)

struct NmArgs {
    const i32x4* frag;  // [towers][256 groups][2 matrices][NM_FRAG]
    const BmRed* red;   // [towers]
    u32 chunk;          // polynomials per workgroup (multiple of NM_POLYS)
    u32 nchunks;
};

// Exchange buffer placement of element pos of local polynomial pl.  Blocks r =
// pos / 16 of odd polynomials swap halves (r ^ 1) and a block's words are
// XOR-rotated by r, so both access patterns are conflict free over 32 lanes:
// (polynomial pair, column c of one block r) in A / C, (polynomial pair, block
// r, fixed c) in B.
__device__ __forceinline__ u32 nm_x(u32 pl, u32 pos) {
    const u32 r = pos >> 4;
    return pl * 256 + ((r ^ (pl & 1)) << 4) + ((pos ^ r) & 15);
}

// x < 2^(L+4) -> (x mod 2^L) + (x >> L) d < 2^L + 16 d: same residue, small
// enough for the signed digit split (< 2^63)
template <bool SPQ, bool QA>
__device__ __forceinline__ u64 spq_fold(u64 x, const Mod<SPQ, QA>& M) {
    const u32 qh = hi32(x) >> M.sh;
    const u64 d = (1ull << (M.sh + 32)) - M.q;
    return mad32(qh, lo32(d), pack(lo32(x), hi32(x) & ((1u << M.sh) - 1)));
}

// one 16 x 16 map on 2 polynomials x 16 columns: B operand from xv (8 inputs
// per lane: j = 4 s + 2 h + u), A fragments from LDS; out(k, value) for the
// lane's 8 outputs k = 4 mt + 2 h + u
template <class OUT>
__device__ __forceinline__ void nm_gemm(const u64 (&xv)[8], const i32x4* fr, u32 lane, u32 h, const BmRed& R,
                                        const BmW& W, OUT out) {
    i32x4 bf[4];
#pragma unroll
    for (int s = 0; s < 4; s++) {
        const u64 d0 = digits8(xv[2 * s]), d1 = digits8(xv[2 * s + 1]);
        bf[s] = i32x4{(int)lo32(d0), (int)hi32(d0), (int)lo32(d1), (int)hi32(d1)};
    }
#pragma unroll
    for (int mt = 0; mt < 4; mt++) {
        i32x16 acc = {};
#pragma unroll
        for (int s = 0; s < 4; s++) acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(fr[(mt * 4 + s) * 64 + lane], bf[s], acc, 0, 0, 0);
#pragma unroll
        for (int u = 0; u < 2; u++) {
            int C[8];
#pragma unroll
            for (int b = 0; b < 8; b++) C[b] = acc[8 * u + b];
            out(4 * mt + 2 * h + u, bm_reduce<true, true, false>(C, R, W));
        }
    }
}

__global__ __launch_bounds__(NM_THREADS, 2) void k_block_mma(PlanArgs P, NmArgs Q, const u64* src, u64* dst,
                                                              const u64* __restrict__ bdat, u32 batch, u32 nwg) {
    OFHE_VGPR_FLOOR();
    constexpr u32 N = 1u << 16;
    __shared__ i32x4 fr[2 * NM_FRAG];          // F_i, V_i (32 KiB)
    __shared__ u64 xb[NM_POLYS * 256];         // exchange buffer (32 KiB)
    const u32 tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const u32 wid = xcd_remap(blockIdx.x, nwg);  // the chunks of one group land on one XCD
    const u32 ch = wid % Q.nchunks, gi = wid / Q.nchunks;
    const u32 i = gi & 255, t = gi >> 8;
    {
        const i32x4* g = Q.frag + ((size_t)gi) * 2 * NM_FRAG;
        for (u32 k = tid; k < 2 * NM_FRAG; k += NM_THREADS) fr[k] = g[k];
    }
    const TowerConst tc = P.tc[t];
    const Mod<true> M = load_mod<true>(tc);
    const BmRed R = Q.red[t];
    const BmW W = bm_weights();
    const u64* tw = P.tw + (u64)t * N * 2;
    const u64* itw = P.itw + (u64)t * N * 2;
    const u64 inner = (u64)t * N + (u64)i * 256;
    const u32 n = lane & 31, h = lane >> 5, cc = n & 15;
    const u32 pr = tid >> 4, r = tid & 15;  // phase B: polynomial, block
    const u32 M0 = N / 16 + 16 * i + r;
    const u32 b_lo = ch * Q.chunk, b_hi = min(batch, b_lo + Q.chunk);
    __syncthreads();
    // software pipeline: the next iteration's level-3 input is loaded during
    // phase B, the Hadamard operand at the end of phase A, so their HBM
    // latency hides under compute (2 workgroups per CU, too few to hide it
    // by occupancy alone)
    u64 xr[2][8];
    auto load_a = [&](u32 c0) {
#pragma unroll
        for (int ps = 0; ps < 2; ps++) {
            const u32 pl = 4 * w + 2 * ps + (n >> 4);
            const bool ok = c0 + pl < b_hi;
            const u64* xs = src + (u64)(c0 + pl) * P.sstride + inner + cc;
#pragma unroll
            for (int s = 0; s < 4; s++)
#pragma unroll
                for (int u = 0; u < 2; u++) xr[ps][2 * s + u] = ok ? ld_s(xs + 16 * (4 * s + 2 * h + u)) : 0;
        }
    };
    load_a(b_lo);
    for (u32 b0 = b_lo; b0 < b_hi; b0 += NM_POLYS) {
        // A: level 3 (F_i); wave w owns polynomials 4w .. 4w + 3, two per pass
#pragma unroll
        for (int ps = 0; ps < 2; ps++) {
            const u32 pl = 4 * w + 2 * ps + (n >> 4);
            u64 xv[8];
#pragma unroll
            for (int k = 0; k < 8; k++) xv[k] = spq_fold(xr[ps][k], M);
            nm_gemm(xv, fr, lane, h, R, W, [&](u32 k, u64 v) { xb[nm_x(pl, cc + 16 * k)] = v; });
        }
        const bool okb = b0 + pr < b_hi;
        const u64* bp = bdat + (u64)(b0 + pr) * P.bstride + inner + 16 * r;
        u64x2 bb[8];
#pragma unroll
        for (int k = 0; k < 8; k++) bb[k] = okb ? ld2_s(bp + 2 * k) : u64x2{0, 0};
        __syncthreads();
        // B: level 4, Hadamard, inverse GS t = 1..8 on block r of polynomial pr
        {
            u64 v[16];
#pragma unroll
            for (int k = 0; k < 16; k++) v[k] = xb[nm_x(pr, 16 * r + k)];
            if (b0 + NM_POLYS < b_hi) load_a(b0 + NM_POLYS);
            fwd_round16(v, tw, M0, M);  // < 2q in, < 12q out
#pragma unroll
            for (int k = 0; k < 8; k++) {
                v[2 * k] = mont_mul(v[2 * k], bb[k].x, tc.q, tc.qinv);  // (0, 2q)
                v[2 * k + 1] = mont_mul(v[2 * k + 1], bb[k].y, tc.q, tc.qinv);
            }
            bool b8[16];
#pragma unroll
            for (int k = 0; k < 16; k++) b8[k] = false;
            inv_round16_b(v, b8, itw, M0, M);  // < 8q
#pragma unroll
            for (int k = 0; k < 16; k++) xb[nm_x(pr, 16 * r + k)] = v[k];
        }
        __syncthreads();
        // C: inverse GS t = 16..128 (V_i, N^-1 2^64 folded in), output < 2q
#pragma unroll
        for (int ps = 0; ps < 2; ps++) {
            const u32 pl = 4 * w + 2 * ps + (n >> 4);
            const bool ok = b0 + pl < b_hi;
            u64 xv[8];
#pragma unroll
            for (int s = 0; s < 4; s++)
#pragma unroll
                for (int u = 0; u < 2; u++) xv[2 * s + u] = spq_fold(xb[nm_x(pl, cc + 16 * (4 * s + 2 * h + u))], M);
            u64* ys = dst + (u64)(b0 + pl) * P.dstride + inner + cc;
            nm_gemm(xv, fr + NM_FRAG, lane, h, R, W, [&](u32 k, u64 v) {
                if (ok) st_s(ys + 16 * k, v);
            });
        }
        __syncthreads();
    }
}

}  // namespace ofhe
