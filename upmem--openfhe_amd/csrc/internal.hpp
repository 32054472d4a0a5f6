// internal.hpp -- definitions shared by the translation units of the backend
// (ofhe_hip.hip: context, plans, NTT, element-wise ops, base conversion;
// keyswitch.hip: ApproxModUp / ApproxModDown / hybrid key switching).
// Not part of the C ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <map>
#include <set>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/ofhe_hip.h"
#include "eltwise_kernels.hpp"
#include "bconv_mma.hpp"

namespace ofhe {
typedef unsigned __int128 u128;

int fail(int code, const std::string& msg);
int post_launch();

#define HIPCHK(call)                                                                        \
    do {                                                                                    \
        hipError_t e_ = (call);                                                             \
        if (e_ != hipSuccess)                                                               \
            return ofhe::fail(OFHE_ERR_HIP, std::string(#call) + ": " + hipGetErrorString(e_)); \
    } while (0)
#define RCCHK(call)            \
    do {                       \
        int rc_ = (call);      \
        if (rc_) return rc_;   \
    } while (0)

// host-side number theory for table construction (setup, not timed)
inline u64 mulmod(u64 a, u64 b, u64 q) { return (u64)(((u128)a * b) % q); }
inline u64 powmod(u64 b, u64 e, u64 q) {
    u64 r = 1 % q;
    b %= q;
    while (e) {
        if (e & 1) r = mulmod(r, b, q);
        b = mulmod(b, b, q);
        e >>= 1;
    }
    return r;
}
inline u64 invmod(u64 a, u64 q) { return powmod(a, q - 2, q); }  // q prime
inline u64 shoup_pre(u64 w, u64 q) { return (u64)(((u128)w << 64) / q); }
// limb_reduce constants of a modulus m < 2^60: 2^60 mod m, its Shoup
// precon, floor(2^64 / m)
inline void limb_red_consts(u64 m, u64* out) {
    const u64 r60 = (1ull << 60) % m;
    out[0] = r60;
    out[1] = shoup_pre(r60, m);
    out[2] = (u64)(((u128)1 << 64) / m);
}
inline unsigned msb64(u64 x) { return x ? 64u - (unsigned)__builtin_clzll(x) : 0u; }
inline u32 bitrev(u32 x, unsigned bits) {
    u32 r = 0;
    for (unsigned i = 0; i < bits; i++) {
        r = (r << 1) | (x & 1);
        x >>= 1;
    }
    return r;
}

// NULL selects the device's default (null) stream, as the header documents;
// callers that want overlap pass their own stream (e.g. torch's).
inline hipStream_t pick(void* stream) { return (hipStream_t)stream; }

// NTT / INTT of plan towers [t0, t0 + count) over `batch` entries; src and dst
// point at tower t0 of batch entry 0 and advance by sstride / dstride words
// per entry.  src may equal dst (in place).
int plan_ntt_range(ofhe_plan_t p, bool inverse, u32 t0, u32 count, const u64* src, u64* dst, u64 sstride,
                   u64 dstride, u32 batch, hipStream_t s);

// Forward transform of y (towers [t0, t0 + count), in place through the column
// pass) whose block pass writes out = (x - NTT(y)) * s_t mod q_t instead of
// NTT(y); scal = device [count][3] (q, s, s').  log_n >= 12.  parts: 1 = the
// column pass only, 2 = the block pass only (y already through the column
// pass), 3 = both.
int plan_ntt_fwd_sub(ofhe_plan_t p, u32 t0, u32 count, u64* y, u64 ystride, const u64* x, u64 xstride, u64* out,
                     u64 ostride, const u64* scal, u32 batch, hipStream_t s, int parts = 3);

// ApproxSwitchCRTBasis fused with the targets' forward column pass
// (k_bconv_cols, bconv_cols.hpp): N = 2^17, SPLIT_COLS plans, <= 16 sources.
// Target j is written (column-pass output, the block pass's input) at tower
// j (+ B.gap from B.gap_at on) of `out`, transformed with plan tower t0 + that
// index.  bconv_cols_ok says whether it applies.
// src_t0 >= 0: x holds the sources' inverse BLOCK pass output (plan towers
// src_t0 .. src_t0 + B.size_q - 1, plan_ntt_inv_block) and the kernel runs
// their inverse column pass itself before converting.
bool bconv_cols_ok(ofhe_plan_t p, const BconvArgs& B);
int bconv_cols_run(ofhe_plan_t p, u32 t0, const BconvArgs& B, const u64* x, u64* out, u32 batch, hipStream_t s,
                   int src_t0 = -1);

// The inverse transform's first pass only (the block pass, log_n > 12): the
// column pass that completes it is left to the consumer (k_bconv_cols with
// src_t0 >= 0).
int plan_ntt_inv_block(ofhe_plan_t p, u32 t0, u32 count, const u64* src, u64 sstride, u64* dst, u64 dstride, u32 batch,
                       hipStream_t s);

// Forward column pass (2^12 < N; not SPLIT_T9) of the towers
// lifted from `last` ([batch] rows of N, stride lstride, modulus ql; first
// multiplied by pre mod ql unless pre = 1) and
// scaled by tab[6 t + 1] (k_cols / k_tcols <.., SWS>), written to y; the block pass
// (plan_ntt_fwd_sub parts = 2) follows.
int plan_cols_switch(ofhe_plan_t p, u32 t0, u32 count, const u64* last, u64 lstride, u64 ql, u64 pre, const u64* tab,
                     u64* y, u64 ystride, u32 batch, hipStream_t s);

// The block pass of a forward transform (y already through the column pass,
// e.g. plan_cols_switch), in place; log_n > 12.
int plan_ntt_fwd_block(ofhe_plan_t p, u32 t0, u32 count, u64* y, u64 ystride, u32 batch, hipStream_t s);

// Table upload for the one-time (cache-miss / setup) paths: a pageable
// hipMemcpy followed by a wait on the null stream it ran on, so the words are
// in device memory before the call returns and any later launch, on any
// stream, reads them (a pageable copy may return before its DMA has landed).
inline hipError_t upload_blocking(void* dst, const void* src, size_t bytes) {
    hipError_t e = hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice);
    return e == hipSuccess ? hipStreamSynchronize(nullptr) : e;
}

// ApproxSwitchCRTBasis launch (strides and output gap from A)
int bconv_run(const BconvArgs& A, const u64* x, u64* out, u32 batch, hipStream_t s);

}  // namespace ofhe

struct ofhe_ctx_s {
    int device = 0;
    hipMemPool_t pool = nullptr;  // stream-ordered scratch + ofhe_hip_alloc_async (null: the default pool)
    std::atomic<int> live{1};
    // ofhe_hip_alloc_async blocks not yet freed: finalize refuses while any
    // is live.  A set, not a counter, so a pointer the pool never handed out
    // (or one freed twice) cannot make the count wrong; the check and the
    // teardown happen under the same lock as every insert / erase.
    std::mutex blocks_mu;
    std::set<void*> async_blocks;
};

enum { SPLIT_COLS = 0, SPLIT_T8 = 1, SPLIT_T9 = 2, SPLIT_T8B9 = 3 };
// stages of the block pass (its inverse groups have 2^block_stages elements)
inline uint32_t block_stages(int split, uint32_t log_n) {
    if (split == SPLIT_T8 || split == SPLIT_T9) return 8;
    if (split == SPLIT_T8B9) return 9;
    return log_n < 12 ? log_n : 12;
}

struct ofhe_plan_s {
    ofhe_ctx_t ctx = nullptr;
    ofhe::u32 log_n = 0, towers = 0;
    // device
    ofhe::TowerConst* d_tc = nullptr;
    ofhe::u64* d_tw = nullptr;
    ofhe::u64* d_itw = nullptr;
    ofhe::u64* d_tw3 = nullptr;   // round-3 transposed twiddles (log_n >= 12)
    ofhe::u64* d_dtw = nullptr;     // DIT inverse twiddles of the block pass
    ofhe::u64* d_twist = nullptr;   // block-pass inverse twist N^-1 psi^-((2 rev(b) + 1) j0)
    ofhe::u64* d_twist_r = nullptr; // the same times 2^64 mod q (fused pipeline, Montgomery Hadamard)
    // host copies (for ofhe_hip_plan_tables and scalar prep)
    std::vector<ofhe::u64> q, psi, tab, tab_pre, itab, itab_pre, ninv;
    // pipeline tuning (ofhe_hip_plan_tune): batch entries per chunk (0 = all)
    // and internal streams the chunks alternate over (1 = caller's stream).
    ofhe::u32 chunk_batch = 0, nstreams = 1;
    ofhe_plan_options opts{};  // the creation options (ofhe_hip_plan_create_ex)
    bool spq = false;     // every modulus is 2^L - d with d < 2^32 (special-prime kernels)
    // column | block pass split for log_n > 12 (SPLIT_*, ofhe_hip.hip):
    //   SPLIT_COLS  k_cols (log_n - 12 stages) + k_block NR = 3
    //   SPLIT_T8    k_tcols (8) + k_block NR = 2            (N = 2^16)
    //   SPLIT_T9    k_tcols9 (9) + k_block NR = 2           (N = 2^17)
    //   SPLIT_T8B9  k_tcols (8) + k_block NR = 3 whose first round keeps only
    //               its last stage (9 block stages)          (N = 2^17)
    int split = 0;
    hipStream_t st[2] = {nullptr, nullptr};
    hipEvent_t ev_fork = nullptr, ev_join[2] = {nullptr, nullptr};
    std::mutex fork_mu;  // guards st / ev_* (plan_tune, the two-stream pipeline)
    // rescaling scalar tables (keyswitch.hip: DropLastElementAndScale /
    // ModReduce), uploaded once per distinct content into memory no launch
    // has read yet, kept until destroy
    std::mutex tab_mu;
    std::map<std::vector<ofhe::u64>, ofhe::u64*> tabs;
};

struct ofhe_bconv_s {
    ofhe_ctx_t ctx = nullptr;
    ofhe::BconvArgs args{};
    ofhe::u64* d_mem = nullptr;
    // ofhe_hip_approx_mod_down's constant tables (P^-1 mod q_i, and for t > 0
    // t^-1 mod p_j, t mod q_i), uploaded once per distinct (t, P^-1 mod q)
    // into memory no launch has read yet and kept until destroy, so steady-state
    // calls upload nothing and never synchronise
    std::mutex tab_mu;
    std::map<std::vector<ofhe::u64>, ofhe::u64*> tabs;
    // k_bconv_cols in ofhe_hip_approx_mod_up / _down (options.separate_cols = 0)
    bool bcols = true;
};
