// bconv_cols.hpp -- ApproxSwitchCRTBasis (dcrtpoly-impl.h:1034-1063) fused with
// the forward column pass of the targets' NTT at N = 2^17 (k_bconv_cols).
//
// Key switching converts a digit to its complement (ApproxModUp,
// keyswitch-hybrid.cpp:388-394) and P back to Q (ApproxModDown,
// dcrtpoly-impl.h:1156-1165), and both send every converted tower straight
// into a forward NTT.  Run apart, k_bconv_mma writes the converted towers to
// HBM and the column pass (k_cols<5>, stages 1-5 on columns {c + 4096 k})
// reads them back: 2 x 8 B per target coefficient of pure traffic, and the
// column pass is HBM-bound while the conversion is VALU / MFMA-bound.  Here one
// workgroup owns 16 columns x 32 rows (512 coefficients) of one batch entry:
//   1. the sources' digits (y_i = [x_i QHatInv_i]_{q_i} as 8 signed bytes, the
//      B operand of bconv_mma.hpp) go to LDS once, [source pair][position];
//   2. each wave takes target tiles (4 targets) and, for 16 MFMA groups of 32
//      positions, runs k_bconv_mma's digit GEMM and bm_reduce; a group is the
//      16 columns x rows {2g, 2g + 1}, so lane (c, h) ends with rows
//      2g + (c >> 4), g = 0..15, of column c & 15 for its two targets;
//   3. the column pass's 5 stages run on those registers: stages 1-4 pair
//      rows of the same parity (inside the lane), stage 5 pairs rows 2g and
//      2g + 1 across lanes c and c ^ 16, which first swap halves so that each
//      computes 8 whole butterflies;
//   4. the stage-5 outputs go to HBM as the block pass's input (< 12q).
// Same twiddle order, stage schedule and lazy bounds as k_cols<5, fwd>, so the
// block pass that follows is unchanged and the result is the same residue.
#pragma once
#include "bconv_mma.hpp"

namespace ofhe {

#ifndef OFHE_BCC_STAGE_BAR
#define OFHE_BCC_STAGE_BAR 1  // scheduling barrier between the column stages (A/B)
#endif
#ifndef OFHE_BCC_MINW
#define OFHE_BCC_MINW 3  // waves per SIMD the register budget is sized for
#endif
#ifndef OFHE_BCC_WAVES
#define OFHE_BCC_WAVES 12  // one target tile per wave at 48 targets (A/B: 12 > 6 > 4 waves per workgroup)
#endif
constexpr u32 BC_WAVES = OFHE_BCC_WAVES;
constexpr u32 BC_THREADS = 64 * BC_WAVES;
constexpr u32 BC_COLS = 16, BC_ROWS = 32, BC_POS = BC_COLS * BC_ROWS;

// ICOL: the sources arrive as the inverse block pass's output (the first 12
// of the 17 inverse stages, lazy [0, 4q)), and the workgroup runs the last 5
// -- the inverse column pass, GS on the columns {c + 4096 k} it owns -- before
// the conversion, so the INTT's column pass (k_cols<5, inverse>) and its HBM
// round trip disappear.  One wave per source tower (its modulus wave-uniform):
// lane (qq, col) holds rows 8 qq .. 8 qq + 7 of column col; stages with row
// distance 1, 2, 4 are in-lane, 8 and 16 cross lanes (xor 16, xor 32), each
// partner computing 4 whole butterflies as in the target column pass below.
// Values stay below 8q (the lazy-GS bounds of cols_inv_b), and the
// conversion's Shoup product takes the lazy value: the same residue.
// src_rel: plan tower of source 0 relative to P's first tower.
template <bool SPQ>
__device__ __forceinline__ void bcc_icol_source(const PlanArgs& P, const BmSrc* srcc, const u64* __restrict__ xb,
                                                u32 src, u32 src_rel, u32 lane, u64* dg64) {
    constexpr u32 N = 1u << 17, COLS = N / BC_ROWS;
    const u32 col = lane & 15, qq = lane >> 4;
    const u32 ts = src_rel + src;
    const auto M = load_mod<SPQ, (bool)OFHE_QA_CI>(P.tc[ts]);
    const u64* itw = P.itw + (u64)ts * N * 2;
    const u64* xs = xb + (u64)src * N + col;
    u64 v[8];
#pragma unroll
    for (int k = 0; k < 8; k++) v[k] = ld_s(xs + (u64)(8 * qq + k) * COLS);
    // compile-time bounds per register as in cols_inv_b (b8: < 8q, else < 4q;
    // a GS sum leaves < 8q, a Shoup difference < 4q): inputs < 4q
    bool b8[8];
#pragma unroll
    for (int k = 0; k < 8; k++) b8[k] = false;
    auto bf = [&](int i, int j, const Tw w) {
        gs_bfly_b(v[i], v[j], w, M, b8[i] || b8[j]);
        b8[i] = true;
        b8[j] = false;
    };
    // stage row distance 1: pairs (2j, 2j + 1), twiddle 16 + 4 qq + j
#pragma unroll
    for (int j = 0; j < 4; j++) bf(2 * j, 2 * j + 1, ldtw(itw, 16 + 4 * qq + j));
    // distance 2: pairs (4j + i, 4j + i + 2), twiddle 8 + 2 qq + j
#pragma unroll
    for (int j = 0; j < 2; j++) {
        const Tw w = ldtw(itw, 8 + 2 * qq + j);
#pragma unroll
        for (int i = 0; i < 2; i++) bf(4 * j + i, 4 * j + i + 2, w);
    }
    // distance 4: pairs (i, i + 4), twiddle 4 + qq
    {
        const Tw w = ldtw(itw, 4 + qq);
#pragma unroll
        for (int i = 0; i < 4; i++) bf(i, i + 4, w);
    }
    // distance 8 (lanes qq, qq ^ 1) then 16 (qq, qq ^ 2): the lower lane keeps
    // butterflies 0..3, the upper 4..7; afterwards v[m] / v[4 + m] hold rows
    // base + m / base + step + m
    auto cross = [&](u32 xmask, const Tw w, bool upper) {
#pragma unroll
        for (int m = 0; m < 4; m++) {
            const u64 snd = upper ? v[m] : v[4 + m];
            const u64 rcv = pack((u32)__shfl_xor((int)lo32(snd), (int)xmask), (u32)__shfl_xor((int)hi32(snd), (int)xmask));
            u64 xv = upper ? rcv : v[m];
            u64 yv = upper ? v[4 + m] : rcv;
            // either partner's slot: the union of both bounds (partners share b8)
            gs_bfly_b(xv, yv, w, M, b8[m] || b8[4 + m]);
            v[m] = xv;
            v[4 + m] = yv;
            b8[m] = true;
            b8[4 + m] = false;
        }
    };
    cross(16, ldtw(itw, 2 + (qq >> 1)), qq & 1);
    cross(32, ldtw(itw, 1), (qq >> 1) & 1);
    // rows: v[m] -> 4 (qq & 1) + 8 (qq >> 1) + m, v[4 + m] -> that + 16
    const BmSrc S = srcc[src];
    const u32 r0 = 4 * (qq & 1) + 8 * (qq >> 1);
    const u32 pr = src >> 1, hv = src & 1;
#pragma unroll
    for (int m = 0; m < 8; m++) {
        const u32 row = r0 + (m & 3) + (m >= 4 ? 16 : 0);
        const u64 y = shoup_canon(v[m], S.w, S.wp, S.q);
        dg64[2 * ((u64)pr * BC_POS + row * BC_COLS + col) + hv] = digits8(y);
    }
}

template <int KS, bool SPQ, bool ICOL = false>
__global__ __launch_bounds__(BC_THREADS, OFHE_BCC_MINW) void k_bconv_cols(BconvArgs A, PlanArgs P, const u64* __restrict__ x,
                                                           u64* __restrict__ out, u32 batch, u32 nwg, u32 src_rel) {
    OFHE_VGPR_FLOOR();
    static_assert(KS >= 1 && KS <= 4, "k_bconv_cols: up to 16 source towers (64 KiB of digits)");
    constexpr u32 N = 1u << 17, COLS = N / BC_ROWS;
    __shared__ i32x4 dg[2 * KS * BC_POS];  // [source pair][position], position = row * 16 + column
    const u32 tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const u32 wid = xcd_remap(blockIdx.x, nwg);
    const u32 cb = wid % (COLS / BC_COLS), b = wid / (COLS / BC_COLS);
    const u32 c0 = cb * BC_COLS;
    const u32 tiles = A.mm_tiles;
    const unsigned char* tab = reinterpret_cast<const unsigned char*>(A.mm_tab);
    const i32x4* frag = reinterpret_cast<const i32x4*>(tab);                                    // [tiles][KS][64]
    const BmRed* red = reinterpret_cast<const BmRed*>(tab + (size_t)tiles * KS * 1024);        // [4 tiles]
    const BmSrc* srcc = reinterpret_cast<const BmSrc*>(red + 4 * tiles);                       // [4 KS]
    if (ICOL) {
        // 1'. the sources' inverse column pass and digits, one wave per source
        u64* dg64 = reinterpret_cast<u64*>(dg);
        const u64* xb = x + (u64)b * A.in_stride + c0;
#pragma unroll 1
        for (u32 src = w; src < 4 * KS; src += BC_WAVES) {
            if (src < A.size_q) {
                bcc_icol_source<SPQ>(P, srcc, xb, src, src_rel, lane, dg64);
            } else {
#pragma unroll
                for (int m = 0; m < 8; m++) {
                    const u32 row = 8 * (lane >> 4) + m;
                    dg64[2 * ((u64)(src >> 1) * BC_POS + row * BC_COLS + (lane & 15)) + (src & 1)] = 0;
                }
            }
        }
    } else {
        // 1. digits of the sources, two per 16-byte slot (the lane's B operand);
        // every load of the thread goes out before the first product
        constexpr u32 ITEMS = 2 * KS * BC_POS, PER = (ITEMS + BC_THREADS - 1) / BC_THREADS;
        const u64* xb = x + (u64)b * A.in_stride + c0;
        u64 xr[PER][2];
#pragma unroll
        for (u32 k = 0; k < PER; k++) {
            const u32 it = tid + k * BC_THREADS, pr = it / BC_POS, pos = it % BC_POS;
            const u64 off = (u64)(pos >> 4) * COLS + (pos & 15);
#pragma unroll
            for (int u = 0; u < 2; u++) {
                const u32 i = 2 * pr + u;
                xr[k][u] = (it < ITEMS && i < A.size_q) ? ld_s(xb + (u64)i * N + off) : 0;
            }
        }
#pragma unroll
        for (u32 k = 0; k < PER; k++) {
            const u32 it = tid + k * BC_THREADS, pr = it / BC_POS;
            if (it >= ITEMS) break;
            u64 d[2];
#pragma unroll
            for (int u = 0; u < 2; u++) {
                const u32 i = 2 * pr + u;
                u64 y = 0;
                if (i < A.size_q) {
                    const BmSrc S = srcc[i];
                    y = shoup_canon(xr[k][u], S.w, S.wp, S.q);
                }
                d[u] = digits8(y);
            }
            dg[it] = i32x4{(int)lo32(d[0]), (int)hi32(d[0]), (int)lo32(d[1]), (int)hi32(d[1])};
        }
    }
    __syncthreads();
    const BmW W = bm_weights();
    const u32 c = lane & 31, h = lane >> 5, col = c & 15, par = c >> 4;
    u64* ob = out + (u64)b * A.out_stride + c0 + col;
    // 3. (below) the column pass on the lane's rows 2g + par of column col
    auto colpass = [&](u64(&vv)[16], u32 j) {
        if (j >= A.size_p) return;  // the partner lane (c ^ 16) has the same h
        const u32 jo = j >= A.gap_at ? j + A.gap : j;
        const auto M = load_mod<SPQ, (bool)OFHE_QA_BCC>(P.tc[jo]);
        const u64* tw = P.tw + (u64)jo * N * 2;
        // stages s = 0..3 (row distance 16 >> s, g distance 8 >> s); CS at s = 0, 2
#pragma unroll
        for (int s = 0; s < 4; s++) {
            const int hg = 8 >> s;
#pragma unroll
            for (int jb = 0; jb < (1 << s); jb++) {
                const Tw tw_ = ldtw(tw, (1u << s) + jb);
#pragma unroll
                for (int g = jb * 2 * hg; g < jb * 2 * hg + hg; g++) ct_bfly_cs(vv[g], vv[g + hg], tw_, M, (s & 1) == 0);
            }
            if (OFHE_BCC_STAGE_BAR) __builtin_amdgcn_sched_barrier(0);  // one stage's twiddles in flight
        }
        // stage s = 4: rows (2g, 2g + 1) = lanes (c, c ^ 16); par 0 keeps g < 8, par 1 g >= 8
        u64* oj = ob + (u64)jo * N;
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const u64 snd = par ? vv[k] : vv[8 + k];
            const u64 rcv = pack((u32)__shfl_xor((int)lo32(snd), 16), (u32)__shfl_xor((int)hi32(snd), 16));
            u64 xv = par ? rcv : vv[k];
            u64 yv = par ? vv[8 + k] : rcv;
            const u32 g = k + 8 * par;
            ct_bfly_cs(xv, yv, ldtw(tw, 16 + g), M, true);  // -> [0, 12q)
            st_s(oj + (u64)(2 * g) * COLS, xv);
            st_s(oj + (u64)(2 * g + 1) * COLS, yv);
        }
    };
#pragma unroll 1
    for (u32 T = w; T < tiles; T += BC_WAVES) {
        i32x4 fa[KS];
#pragma unroll
        for (int s = 0; s < KS; s++) fa[s] = frag[(T * KS + s) * 64 + lane];
        const BmRed R0 = red[4 * T + 2 * h], R1 = red[4 * T + 2 * h + 1];
        // 2. the conversion, 16 groups of 32 positions; group g + 1's MFMA chain
        // is issued before group g's reduction so the two overlap
        u64 v0[16], v1[16];
        auto mma = [&](int g) {
            i32x16 acc = {};
#pragma unroll
            for (int s = 0; s < KS; s++)
                acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[s], dg[(2 * s + h) * BC_POS + 32 * g + c], acc, 0, 0,
                                                             0);
            return acc;
        };
        i32x16 accn = mma(0);
#pragma unroll
        for (int g = 0; g < 16; g++) {
            const i32x16 acc = accn;
            if (g + 1 < 16) accn = mma(g + 1);
            int C0[8], C1[8];
#pragma unroll
            for (int k = 0; k < 8; k++) {
                C0[k] = acc[k];
                C1[k] = acc[8 + k];
            }
            v0[g] = bm_reduce<true, SPQ, false>(C0, R0, W);  // lazy: [0, 4p) (SPQ: < 2p)
            v1[g] = bm_reduce<true, SPQ, false>(C1, R1, W);
            // reduce here: left alone, LLVM sinks every group's reduction to its
            // use in the column pass and keeps 16 accumulator tiles (256 VGPRs)
            // live; the barrier keeps later groups' LDS reads below it
            asm volatile("" : "+v"(v0[g]), "+v"(v1[g]));
            __builtin_amdgcn_sched_barrier(0);
        }
        colpass(v0, 4 * T + 2 * h);
        colpass(v1, 4 * T + 2 * h + 1);
    }
}

}  // namespace ofhe
