// ntt_kernels.hpp -- negacyclic NTT / INTT / fused pipeline kernels for gfx950.
//
// Algorithm (the reference's, restated; transformnat-impl.h:300-354, 492-552):
//   forward, Cooley-Tukey, natural -> bit-reversed: for m = 1, 2, ..., N/2 with
//   t = N/(2m), every pair (j, j+t) in group i = j/(2t) becomes
//   (x_j + w x_{j+t}, x_j - w x_{j+t}) with w = Table[m + i];
//   inverse, Gentleman-Sande: m = N/2 ... 1 (t = 1 ... N/2),
//   (x_j + x_{j+t}, (x_j - x_{j+t}) * TableI[m + i]), with n^-1 fused into the
//   first (t = 1) stage.
// Values stay lazily reduced between stages (forward in [0, 8q), inverse in
// [0, 4q)) and are made canonical on output, so results equal the reference
// bit for bit (its outputs are the canonical residues).
//
// Decomposition for N = 2^logN >= 2^12 (one tower = 512 KiB at 2^16, more
// than a CU's 160 KiB LDS):
//   k_cols  : the first logN-12 stages. Each thread owns one "column"
//             {c + 4096 k}; all its butterflies are in registers.
//   k_block : the last 12 stages on contiguous 4096-element blocks (32 KiB of
//             LDS per workgroup): 3 rounds of 4 radix-2 stages held in
//             registers (16 values per thread), two XOR-swizzled LDS
//             exchanges between rounds (bank-conflict free for all three
//             access patterns, checked by tools/lds_banks.py).
//   The metric pipeline runs k_cols(fwd) -> k_block(fwd + Hadamard + inverse)
//   -> k_cols(inv): the Hadamard and the 24 block stages share one residency.
// N <= 2^11 uses k_small (whole tower in LDS, one stage per step).
#pragma once
#include "arith.hpp"

namespace ofhe {

struct TowerConst {
    u64 q;
    u64 ninv;      // N^-1 mod q
    u64 ninv_pre;  // Shoup precon of ninv
    u64 mu;        // ComputeMu() for Barrett (ubintnat.h:651-656)
    u32 nshift;    // msb(q) - 2
    u32 pad;
};

// Device view of a plan. Twiddles are interleaved (w, w') pairs so one
// 16-byte load fetches a twiddle and its Shoup precon.
struct PlanArgs {
    const TowerConst* tc;  // [T]
    const u64* tw;         // [T][N][2]   forward Table (bit-reversed powers of psi)
    const u64* itw;        // [T][N][2]   inverse TableI
    const u64* itwn;       // [T][N/2][2] TableI[N/2 + i] * N^-1 (first inverse stage)
    u32 log_n;
    u32 towers;
};

enum { MODE_FWD = 0, MODE_INV = 1, MODE_FUSED = 2 };

// Bijective XCD-aware block remap (cdna_hip_programming.md T1): consecutive
// work items land on the same XCD, so workgroups of one tower share its
// twiddles in that XCD's L2.
__device__ __forceinline__ u32 xcd_remap(u32 bid, u32 nwg) {
    u32 q = nwg >> 3, r = nwg & 7, xcd = bid & 7, loc = bid >> 3;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
}

struct Tw {
    u64 w, wp;
};
__device__ __forceinline__ Tw ldtw(const u64* base, u32 idx) {
    const ulonglong2 v = *reinterpret_cast<const ulonglong2*>(base + 2 * (u64)idx);
    return Tw{v.x, v.y};
}

// Cooley-Tukey butterfly, inputs in [0, 8q), outputs in [0, 7q).
__device__ __forceinline__ void ct_bfly(u64& x, u64& y, Tw w, u64 q, u64 q3, u64 q4) {
    u64 t = shoup_lazy(y, w.w, w.wp, q);  // [0, 3q)
    u64 a = csub(x, q4);                  // [0, 4q)
    x = a + t;
    y = a + (q3 - t);
}

// Gentleman-Sande butterfly, inputs in [0, 4q), outputs in [0, 4q).
__device__ __forceinline__ void gs_bfly(u64& x, u64& y, Tw w, u64 q, u64 q4) {
    u64 s = x + y;                                    // [0, 8q)
    u64 d = x + (q4 - y);                             // (0, 8q)
    x = csub(s, q4);
    y = shoup_lazy(d, w.w, w.wp, q);                  // [0, 3q)
}

// First inverse stage (t = 1) with N^-1 folded in: both outputs scaled.
__device__ __forceinline__ void gs_bfly_ninv(u64& x, u64& y, Tw wn, u64 ninv, u64 ninv_pre, u64 q,
                                             u64 q4) {
    u64 s = x + y;
    u64 d = x + (q4 - y);
    x = shoup_lazy(s, ninv, ninv_pre, q);
    y = shoup_lazy(d, wn.w, wn.wp, q);
}

__device__ __forceinline__ u64 canon8(u64 x, u64 q) {  // [0, 8q) -> [0, q)
    x = csub(x, 4 * q);
    x = csub(x, 2 * q);
    return csub(x, q);
}
__device__ __forceinline__ u64 canon4(u64 x, u64 q) {  // [0, 4q) -> [0, q)
    x = csub(x, 2 * q);
    return csub(x, q);
}

// ---------------------------------------------------------------------------
// Register radix-16 rounds.  A thread holds v[k] = x[p0 + k*st], k < 16, where
// p0 = hb*16*st + r (r < st).  Stage s (s = 0..3, t = st * 2^(3-s)) pairs
// (k, k + 2^(3-s)); its twiddle index is 2^s * M0 + (k >> (4 - s)) with
// M0 = N/(16 st) + (global index of the 16*st super-group).
// ---------------------------------------------------------------------------
template <int S>
__device__ __forceinline__ void fwd_stage16(u64 (&v)[16], const u64* tw, u32 M0, u64 q, u64 q3,
                                            u64 q4) {
    constexpr int half = 8 >> S;
#pragma unroll
    for (int j = 0; j < (1 << S); j++) {
        Tw w = ldtw(tw, (M0 << S) + j);
#pragma unroll
        for (int k = j * 2 * half; k < j * 2 * half + half; k++) ct_bfly(v[k], v[k + half], w, q, q3, q4);
    }
}

template <int S>
__device__ __forceinline__ void inv_stage16(u64 (&v)[16], const u64* itw, u32 M0, u64 q, u64 q4) {
    constexpr int half = 8 >> S;
#pragma unroll
    for (int j = 0; j < (1 << S); j++) {
        Tw w = ldtw(itw, (M0 << S) + j);
#pragma unroll
        for (int k = j * 2 * half; k < j * 2 * half + half; k++) gs_bfly(v[k], v[k + half], w, q, q4);
    }
}

// last inverse round stage s = 3 at global t = 1: uses the N^-1-folded table.
// itwn is indexed by i = (M0 << 3) + j - N/2.
__device__ __forceinline__ void inv_stage16_first(u64 (&v)[16], const u64* itwn, u32 i0,
                                                  const TowerConst& tc, u64 q4) {
#pragma unroll
    for (int j = 0; j < 8; j++) {
        Tw w = ldtw(itwn, i0 + j);
        gs_bfly_ninv(v[2 * j], v[2 * j + 1], w, tc.ninv, tc.ninv_pre, tc.q, q4);
    }
}

__device__ __forceinline__ u32 swz(u32 p) { return p ^ ((p >> 4) & 15u) ^ (((p >> 8) & 15u) << 4); }

// ---------------------------------------------------------------------------
// k_block: the last 12 stages on a 4096-element block; MODE selects
// forward (canonical out), inverse (first 12 inverse stages), or the fused
// forward -> Hadamard -> inverse pipeline.
// ---------------------------------------------------------------------------
template <int MODE>
__global__ __launch_bounds__(256) void k_block(PlanArgs P, const u64* src, u64* dst,
                                               const u64* __restrict__ bdat, u32 batch, u32 nwg) {
    __shared__ u64 lds[4096];
    const u32 tid = threadIdx.x;
    const u32 logn = P.log_n;
    const u32 N = 1u << logn;
    const u32 G = N >> 12;  // blocks per polynomial
    const u32 wid = xcd_remap(blockIdx.x, nwg);
    const u32 g = wid % G;
    const u32 pb = wid / G;
    const u32 t = pb / batch, b = pb % batch;
    const u64 off = ((u64)b * P.towers + t) * N + ((u64)g << 12);
    const u64* blk = src + off;
    u64* oblk = dst + off;
    const TowerConst tc = P.tc[t];
    const u64 q = tc.q, q3 = 3 * q, q4 = 4 * q;
    const u64* tw = P.tw + (u64)t * N * 2;
    const u64* itw = P.itw + (u64)t * N * 2;
    const u64* itwn = P.itwn + (u64)t * N;  // N/2 pairs
    const u32 h = tid >> 4, r = tid & 15;
    u64 v[16];

    if (MODE == MODE_FWD || MODE == MODE_FUSED) {
        // round 1: st = 256, p = tid + 256k
#pragma unroll
        for (int k = 0; k < 16; k++) v[k] = blk[tid + 256 * k];
        {
            const u32 M0 = (N >> 12) + g;
            fwd_stage16<0>(v, tw, M0, q, q3, q4);
            fwd_stage16<1>(v, tw, M0, q, q3, q4);
            fwd_stage16<2>(v, tw, M0, q, q3, q4);
            fwd_stage16<3>(v, tw, M0, q, q3, q4);
        }
#pragma unroll
        for (int k = 0; k < 16; k++) lds[swz(tid + 256 * k)] = v[k];
        __syncthreads();
        // round 2: st = 16, p = h*256 + r + 16k
#pragma unroll
        for (int k = 0; k < 16; k++) v[k] = lds[swz(h * 256 + r + 16 * k)];
        {
            const u32 M0 = (N >> 8) + g * 16 + h;
            fwd_stage16<0>(v, tw, M0, q, q3, q4);
            fwd_stage16<1>(v, tw, M0, q, q3, q4);
            fwd_stage16<2>(v, tw, M0, q, q3, q4);
            fwd_stage16<3>(v, tw, M0, q, q3, q4);
        }
#pragma unroll
        for (int k = 0; k < 16; k++) lds[swz(h * 256 + r + 16 * k)] = v[k];
        __syncthreads();
        // round 3: st = 1, p = 16 tid + k
#pragma unroll
        for (int k = 0; k < 16; k++) v[k] = lds[swz(tid * 16 + k)];
        {
            const u32 M0 = (N >> 4) + g * 256 + tid;
            fwd_stage16<0>(v, tw, M0, q, q3, q4);
            fwd_stage16<1>(v, tw, M0, q, q3, q4);
            fwd_stage16<2>(v, tw, M0, q, q3, q4);
            fwd_stage16<3>(v, tw, M0, q, q3, q4);
        }
#pragma unroll
        for (int k = 0; k < 16; k++) v[k] = canon8(v[k], q);
        if (MODE == MODE_FWD) {
            ulonglong2* o = reinterpret_cast<ulonglong2*>(oblk + tid * 16);
#pragma unroll
            for (int k = 0; k < 8; k++) o[k] = make_ulonglong2(v[2 * k], v[2 * k + 1]);
            return;
        }
        // Hadamard with b (evaluation form), NativeVectorT::ModMulNoCheckEq
        const ulonglong2* bp = reinterpret_cast<const ulonglong2*>(bdat + off + tid * 16);
#pragma unroll
        for (int k = 0; k < 8; k++) {
            ulonglong2 bb = bp[k];
            v[2 * k] = barrett_ref(v[2 * k], bb.x, q, tc.mu, tc.nshift);
            v[2 * k + 1] = barrett_ref(v[2 * k + 1], bb.y, q, tc.mu, tc.nshift);
        }
        // no barrier: round 3' below rewrites only this thread's own LDS slots
    } else {
        const ulonglong2* ip = reinterpret_cast<const ulonglong2*>(blk + tid * 16);
#pragma unroll
        for (int k = 0; k < 8; k++) {
            ulonglong2 a = ip[k];
            v[2 * k] = a.x;
            v[2 * k + 1] = a.y;
        }
    }
    // inverse round 3': st = 1, GS stages t = 1, 2, 4, 8 (s = 3, 2, 1, 0)
    {
        const u32 M0 = (N >> 4) + g * 256 + tid;
        inv_stage16_first(v, itwn, (M0 << 3) - (N >> 1), tc, q4);
        inv_stage16<2>(v, itw, M0, q, q4);
        inv_stage16<1>(v, itw, M0, q, q4);
        inv_stage16<0>(v, itw, M0, q, q4);
    }
#pragma unroll
    for (int k = 0; k < 16; k++) lds[swz(tid * 16 + k)] = v[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 16; k++) v[k] = lds[swz(h * 256 + r + 16 * k)];
    {
        const u32 M0 = (N >> 8) + g * 16 + h;
        inv_stage16<3>(v, itw, M0, q, q4);
        inv_stage16<2>(v, itw, M0, q, q4);
        inv_stage16<1>(v, itw, M0, q, q4);
        inv_stage16<0>(v, itw, M0, q, q4);
    }
#pragma unroll
    for (int k = 0; k < 16; k++) lds[swz(h * 256 + r + 16 * k)] = v[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 16; k++) v[k] = lds[swz(tid + 256 * k)];
    {
        const u32 M0 = (N >> 12) + g;
        inv_stage16<3>(v, itw, M0, q, q4);
        inv_stage16<2>(v, itw, M0, q, q4);
        inv_stage16<1>(v, itw, M0, q, q4);
        inv_stage16<0>(v, itw, M0, q, q4);
    }
    if (logn == 12) {
#pragma unroll
        for (int k = 0; k < 16; k++) v[k] = canon4(v[k], q);
    }
#pragma unroll
    for (int k = 0; k < 16; k++) oblk[tid + 256 * k] = v[k];
}

// ---------------------------------------------------------------------------
// k_cols: the first KA = logN - 12 forward stages (or the last KA inverse
// stages) on columns {c + 4096 k}, k < 2^KA, entirely in registers.
// ---------------------------------------------------------------------------
template <int KA, bool INV>
__global__ __launch_bounds__(256) void k_cols(PlanArgs P, const u64* src, u64* dst, u32 batch,
                                              u32 nwg) {
    constexpr int E = 1 << KA;
    constexpr u32 N = 1u << (KA + 12);
    const u32 wid = xcd_remap(blockIdx.x, nwg);
    const u32 cb = wid & 15;
    const u32 pb = wid >> 4;
    const u32 t = pb / batch, b = pb % batch;
    const u64 off = ((u64)b * P.towers + t) * N + cb * 256 + threadIdx.x;
    const u64* x = src + off;
    u64* y = dst + off;
    const u64 q = P.tc[t].q, q3 = 3 * q, q4 = 4 * q;
    u64 v[E];
#pragma unroll
    for (int k = 0; k < E; k++) v[k] = x[(u64)k * 4096];
    if (!INV) {
        const u64* tw = P.tw + (u64)t * N * 2;
#pragma unroll
        for (int s = 0; s < KA; s++) {
            const int half = E >> (s + 1);
#pragma unroll
            for (int j = 0; j < (1 << s); j++) {
                Tw w = ldtw(tw, (1u << s) + j);
#pragma unroll
                for (int k = j * 2 * half; k < j * 2 * half + half; k++)
                    ct_bfly(v[k], v[k + half], w, q, q3, q4);
            }
        }
    } else {
        const u64* itw = P.itw + (u64)t * N * 2;
#pragma unroll
        for (int s = KA - 1; s >= 0; s--) {
            const int half = E >> (s + 1);
#pragma unroll
            for (int j = 0; j < (1 << s); j++) {
                Tw w = ldtw(itw, (1u << s) + j);
#pragma unroll
                for (int k = j * 2 * half; k < j * 2 * half + half; k++) gs_bfly(v[k], v[k + half], w, q, q4);
            }
        }
#pragma unroll
        for (int k = 0; k < E; k++) v[k] = canon4(v[k], q);
    }
#pragma unroll
    for (int k = 0; k < E; k++) y[(u64)k * 4096] = v[k];
}

// ---------------------------------------------------------------------------
// k_small: N <= 2^11, one workgroup per polynomial, whole tower in LDS.
// ---------------------------------------------------------------------------
template <int MODE>
__global__ __launch_bounds__(256) void k_small(PlanArgs P, const u64* src, u64* dst,
                                               const u64* __restrict__ bdat, u32 batch) {
    __shared__ u64 lds[2048];
    const u32 logn = P.log_n, N = 1u << logn, half = N >> 1;
    const u32 pb = blockIdx.x;
    const u32 b = pb / P.towers, t = pb % P.towers;
    const u64 off = (u64)pb * N;
    const TowerConst tc = P.tc[t];
    const u64 q = tc.q, q3 = 3 * q, q4 = 4 * q;
    const u64* tw = P.tw + (u64)t * N * 2;
    const u64* itw = P.itw + (u64)t * N * 2;
    const u64* itwn = P.itwn + (u64)t * N;
    (void)b;
    for (u32 i = threadIdx.x; i < N; i += blockDim.x) lds[i] = src[off + i];
    __syncthreads();
    if (MODE == MODE_FWD || MODE == MODE_FUSED) {
        for (u32 m = 1, lt = logn - 1; m < N; m <<= 1, lt--) {
            const u32 tt = 1u << lt;
            for (u32 k = threadIdx.x; k < half; k += blockDim.x) {
                const u32 i = k >> lt, j = (i << (lt + 1)) + (k & (tt - 1));
                u64 x = lds[j], y = lds[j + tt];
                ct_bfly(x, y, ldtw(tw, m + i), q, q3, q4);
                lds[j] = x;
                lds[j + tt] = y;
            }
            __syncthreads();
        }
        for (u32 i = threadIdx.x; i < N; i += blockDim.x) {
            u64 x = canon8(lds[i], q);
            if (MODE == MODE_FUSED) x = barrett_ref(x, bdat[off + i], q, tc.mu, tc.nshift);
            lds[i] = x;
        }
        __syncthreads();
        if (MODE == MODE_FWD) {
            for (u32 i = threadIdx.x; i < N; i += blockDim.x) dst[off + i] = lds[i];
            return;
        }
    }
    for (u32 m = half, lt = 0; m >= 1; m >>= 1, lt++) {
        const u32 tt = 1u << lt;
        for (u32 k = threadIdx.x; k < half; k += blockDim.x) {
            const u32 i = k >> lt, j = (i << (lt + 1)) + (k & (tt - 1));
            u64 x = lds[j], y = lds[j + tt];
            if (m == half)
                gs_bfly_ninv(x, y, ldtw(itwn, i), tc.ninv, tc.ninv_pre, q, q4);
            else
                gs_bfly(x, y, ldtw(itw, m + i), q, q4);
            lds[j] = x;
            lds[j + tt] = y;
        }
        __syncthreads();
    }
    for (u32 i = threadIdx.x; i < N; i += blockDim.x) dst[off + i] = canon4(lds[i], q);
}

}  // namespace ofhe
