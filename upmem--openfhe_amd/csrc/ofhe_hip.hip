// ofhe_hip.hip -- C ABI (include/ofhe_hip.h) of the gfx950 RNS backend.
//
// Replaces the UPMEM interception layer of the reference:
//   PimManager (src/core/include/pim/PimManager.h:21-127, pim/host/PimManager.cpp)
//     -> ofhe_ctx_s: one per device; allocation and
//        transfers are hipMalloc / hipMemcpyAsync instead of per-DPU MRAM
//        chunks (DpuMemory.h) and dpu_push_xfer scatter/gather.
//   PimData + DPU element-wise kernels (PimData.h:46-305, dpu/element-wise/*.c)
//     -> ofhe_hip_mod{mul,add,sub}_vv / ofhe_hip_modmul_scalar.
//   ChineseRemainderTransformFTTNat static tables (transformnat-impl.h:708-763)
//     -> ofhe_plan_s, device-resident twiddles per (q, N).
// No CPU fallback: every compute entry point launches HIP kernels or fails.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <thread>

#include "internal.hpp"
#include "bconv_cols.hpp"

using namespace ofhe;

#define OFHE_VERSION "ofhe-hip 0.2 gfx950"

namespace ofhe {
static thread_local std::string g_err;
int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}
int post_launch() {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(OFHE_ERR_HIP, std::string("kernel launch: ") + hipGetErrorString(e));
    return OFHE_OK;
}
}  // namespace ofhe

// Entry points keep the C linkage of their declarations in include/ofhe_hip.h.
const char* ofhe_hip_last_error(void) { return g_err.c_str(); }
const char* ofhe_hip_version(void) { return OFHE_VERSION; }

int ofhe_hip_device_count(int* count) {
    if (!count) return fail(OFHE_ERR_ARG, "count is NULL");
    HIPCHK(hipGetDeviceCount(count));
    return OFHE_OK;
}

int ofhe_hip_init(int device, ofhe_ctx_t* ctx) {
    if (!ctx) return fail(OFHE_ERR_ARG, "ctx is NULL");
    int n = 0;
    HIPCHK(hipGetDeviceCount(&n));
    if (device < 0 || device >= n) return fail(OFHE_ERR_ARG, "device index out of range");
    HIPCHK(hipSetDevice(device));
    ofhe_ctx_s* c = new (std::nothrow) ofhe_ctx_s();
    if (!c) return fail(OFHE_ERR_NOMEM, "context allocation failed");
    c->device = device;
    // Stream-ordered scratch (ApproxModDown, key switching, rescaling) and
    // ofhe_hip_alloc_async come from a pool of this context's own, which keeps
    // freed blocks across synchronisations instead of returning them to the
    // driver at every sync and mapping them again on the next call (a rescale
    // timed call by call: 0.79 -> 0.62 ms).  The device's default
    // pool, which other libraries in the process share, is left alone;
    // ofhe_hip_trim / ofhe_hip_finalize give the memory back.
    {
        hipMemPoolProps props = {};
        props.allocType = hipMemAllocationTypePinned;
        props.handleTypes = hipMemHandleTypeNone;
        props.location.type = hipMemLocationTypeDevice;
        props.location.id = device;
        hipMemPool_t pool = nullptr;
        if (hipMemPoolCreate(&pool, &props) == hipSuccess && pool) {
            uint64_t keep = UINT64_MAX;
            (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
            c->pool = pool;
        }
    }
    *ctx = c;
    return OFHE_OK;
}

int ofhe_hip_trim(ofhe_ctx_t ctx, size_t keep_bytes) {
    if (!ctx) return fail(OFHE_ERR_ARG, "ctx is NULL");
    if (!ctx->pool) return OFHE_OK;
    HIPCHK(hipSetDevice(ctx->device));
    HIPCHK(hipMemPoolTrimTo(ctx->pool, keep_bytes));
    return OFHE_OK;
}

int ofhe_hip_finalize(ofhe_ctx_t ctx) {
    if (!ctx) return fail(OFHE_ERR_ARG, "ctx is NULL");
    {
        // Destroying the pool would release every block still allocated from
        // it, leaving the caller's ofhe_hip_alloc_async pointers dangling:
        // refuse, and keep the context usable, until all of them are freed.
        std::lock_guard<std::mutex> lk(ctx->blocks_mu);
        if (ctx->live.load() == 0) return fail(OFHE_ERR_STATE, "context already finalized");
        const size_t held = ctx->async_blocks.size();
        if (held > 0)
            return fail(OFHE_ERR_STATE, "ofhe_hip_finalize: " + std::to_string(held) +
                                            " ofhe_hip_alloc_async block(s) still allocated; free them first");
        ctx->live.store(0);
    }
    (void)hipSetDevice(ctx->device);
    (void)hipDeviceSynchronize();
    if (ctx->pool) (void)hipMemPoolDestroy(ctx->pool);  // only the library's own (freed) scratch is left in it
    delete ctx;
    return OFHE_OK;
}

int ofhe_hip_alloc(ofhe_ctx_t ctx, size_t bytes, void** dptr) {
    if (!ctx || !dptr) return fail(OFHE_ERR_ARG, "NULL argument");
    HIPCHK(hipSetDevice(ctx->device));
    hipError_t e = hipMalloc(dptr, bytes ? bytes : 1);
    if (e != hipSuccess) return fail(OFHE_ERR_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
    return OFHE_OK;
}

int ofhe_hip_free(ofhe_ctx_t ctx, void* dptr) {
    if (!ctx) return fail(OFHE_ERR_ARG, "ctx is NULL");
    HIPCHK(hipSetDevice(ctx->device));
    HIPCHK(hipFree(dptr));
    return OFHE_OK;
}


int ofhe_hip_alloc_async(ofhe_ctx_t ctx, size_t bytes, void** dptr, void* stream) {
    if (!ctx || !dptr) return fail(OFHE_ERR_ARG, "NULL argument");
    HIPCHK(hipSetDevice(ctx->device));
    std::lock_guard<std::mutex> lk(ctx->blocks_mu);
    if (ctx->live.load() == 0) return fail(OFHE_ERR_STATE, "context finalized");
    hipError_t e = ctx->pool ? hipMallocFromPoolAsync(dptr, bytes ? bytes : 1, ctx->pool, pick(stream))
                             : hipMallocAsync(dptr, bytes ? bytes : 1, pick(stream));
    if (e != hipSuccess) return fail(OFHE_ERR_NOMEM, std::string("hipMallocAsync: ") + hipGetErrorString(e));
    ctx->async_blocks.insert(*dptr);
    return OFHE_OK;
}

int ofhe_hip_free_async(ofhe_ctx_t ctx, void* dptr, void* stream) {
    if (!ctx) return fail(OFHE_ERR_ARG, "ctx is NULL");
    if (!dptr) return OFHE_OK;
    HIPCHK(hipSetDevice(ctx->device));
    std::lock_guard<std::mutex> lk(ctx->blocks_mu);
    auto it = ctx->async_blocks.find(dptr);
    if (it == ctx->async_blocks.end())
        return fail(OFHE_ERR_ARG, "ofhe_hip_free_async: not a live ofhe_hip_alloc_async block of this context");
    // untracked only once the pool has it back: a failed free leaves the block
    // live, so ofhe_hip_finalize still refuses to destroy the pool under it
    HIPCHK(hipFreeAsync(dptr, pick(stream)));
    ctx->async_blocks.erase(it);
    return OFHE_OK;
}

int ofhe_hip_host_alloc(ofhe_ctx_t ctx, size_t bytes, void** hptr) {
    if (!ctx || !hptr) return fail(OFHE_ERR_ARG, "NULL argument");
    HIPCHK(hipSetDevice(ctx->device));
    hipError_t e = hipHostMalloc(hptr, bytes ? bytes : 1, hipHostMallocDefault);
    if (e != hipSuccess) return fail(OFHE_ERR_NOMEM, std::string("hipHostMalloc: ") + hipGetErrorString(e));
    return OFHE_OK;
}

int ofhe_hip_host_free(ofhe_ctx_t ctx, void* hptr) {
    if (!ctx) return fail(OFHE_ERR_ARG, "ctx is NULL");
    if (!hptr) return OFHE_OK;
    HIPCHK(hipSetDevice(ctx->device));
    HIPCHK(hipHostFree(hptr));
    return OFHE_OK;
}

int ofhe_hip_zero(ofhe_ctx_t ctx, void* dst, size_t bytes, void* stream) {
    if (!ctx || (!dst && bytes)) return fail(OFHE_ERR_ARG, "NULL argument");
    if (!bytes) return OFHE_OK;
    HIPCHK(hipMemsetAsync(dst, 0, bytes, pick(stream)));
    return OFHE_OK;
}

int ofhe_hip_copy_to_device(ofhe_ctx_t ctx, void* dst, const void* src, size_t bytes, void* stream) {
    if (!ctx || (!dst && bytes) || (!src && bytes)) return fail(OFHE_ERR_ARG, "NULL argument");
    HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, pick(stream)));
    return OFHE_OK;
}

int ofhe_hip_copy_to_host(ofhe_ctx_t ctx, void* dst, const void* src, size_t bytes, void* stream) {
    if (!ctx || (!dst && bytes) || (!src && bytes)) return fail(OFHE_ERR_ARG, "NULL argument");
    HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, pick(stream)));
    return OFHE_OK;
}

int ofhe_hip_copy_device(ofhe_ctx_t ctx, void* dst, const void* src, size_t bytes, void* stream) {
    if (!ctx || (!dst && bytes) || (!src && bytes)) return fail(OFHE_ERR_ARG, "NULL argument");
    HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, pick(stream)));
    return OFHE_OK;
}

int ofhe_hip_sync(ofhe_ctx_t ctx, void* stream) {
    if (!ctx) return fail(OFHE_ERR_ARG, "ctx is NULL");
    HIPCHK(hipStreamSynchronize(pick(stream)));
    return OFHE_OK;
}

// A completion marker on one stream: waiting on it waits for that stream's
// work up to the record, nothing queued after it (the adapter's staging
// buffers are reused once their DMA has read them, ofhe_dcrt.hpp).
// It keeps the device id, not the context: an event may outlive the context
// that made it (ofhe_hip_finalize frees the context).
struct ofhe_event_s {
    int device = 0;
    hipEvent_t ev = nullptr;
};

int ofhe_hip_event_create(ofhe_ctx_t ctx, ofhe_event_t* out) {
    if (!ctx || !out) return fail(OFHE_ERR_ARG, "NULL argument");
    if (ctx->live.load() == 0) return fail(OFHE_ERR_STATE, "context finalized");
    HIPCHK(hipSetDevice(ctx->device));
    hipEvent_t e = nullptr;
    HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    *out = new ofhe_event_s{ctx->device, e};
    return OFHE_OK;
}

int ofhe_hip_event_record(ofhe_event_t ev, void* stream) {
    if (!ev) return fail(OFHE_ERR_ARG, "event is NULL");
    HIPCHK(hipEventRecord(ev->ev, pick(stream)));
    return OFHE_OK;
}

int ofhe_hip_event_sync(ofhe_event_t ev) {
    if (!ev) return fail(OFHE_ERR_ARG, "event is NULL");
    HIPCHK(hipEventSynchronize(ev->ev));
    return OFHE_OK;
}

int ofhe_hip_event_destroy(ofhe_event_t ev) {
    if (!ev) return fail(OFHE_ERR_ARG, "event is NULL");
    (void)hipSetDevice(ev->device);
    (void)hipEventDestroy(ev->ev);
    delete ev;
    return OFHE_OK;
}

// ---------------------------------------------------------------------------
// Plans
// ---------------------------------------------------------------------------
int ofhe_hip_plan_create(ofhe_ctx_t ctx, uint32_t log_n, uint32_t towers, const uint64_t* q,
                         const uint64_t* psi, ofhe_plan_t* plan) {
    return ofhe_hip_plan_create_ex(ctx, log_n, towers, q, psi, nullptr, plan);
}

int ofhe_hip_plan_create_ex(ofhe_ctx_t ctx, uint32_t log_n, uint32_t towers, const uint64_t* q,
                            const uint64_t* psi, const ofhe_plan_options* options, ofhe_plan_t* plan) {
    if (!ctx || !q || !psi || !plan) return fail(OFHE_ERR_ARG, "NULL argument");
    if (log_n < 1 || log_n > 17) return fail(OFHE_ERR_ARG, "log_n must be in [1, 17]");
    if (towers < 1 || towers > 4096) return fail(OFHE_ERR_ARG, "towers must be in [1, 4096]");
    const ofhe_plan_options opt = options ? *options : ofhe_plan_options{};
    if (opt.generic_moduli > 1) return fail(OFHE_ERR_ARG, "options.generic_moduli must be 0 or 1");
    // Pass split for log_n > 12 (DESIGN.md "Why not a 10 | 6 split" and the
    // rejected-variant table): 8 | 8 at N = 2^16 (k_tcols + an 8-stage block
    // pass), k_cols + the 12-stage block pass elsewhere; the other splits are
    // selectable for tests and A/B timing.
    int split = log_n == 16 ? SPLIT_T8 : SPLIT_COLS;
    switch (opt.split) {
        case OFHE_SPLIT_AUTO: break;
        case OFHE_SPLIT_COLS:
            if (log_n <= 12) return fail(OFHE_ERR_ARG, "options.split: log_n <= 12 plans have no column pass");
            split = SPLIT_COLS;
            break;
        case OFHE_SPLIT_8_8:
            if (log_n != 16) return fail(OFHE_ERR_ARG, "options.split OFHE_SPLIT_8_8 needs log_n = 16");
            split = SPLIT_T8;
            break;
        case OFHE_SPLIT_9_8:
        case OFHE_SPLIT_8_9:
            if (log_n != 17) return fail(OFHE_ERR_ARG, "options.split OFHE_SPLIT_9_8 / 8_9 need log_n = 17");
            split = opt.split == OFHE_SPLIT_9_8 ? SPLIT_T9 : SPLIT_T8B9;
            break;
        default: return fail(OFHE_ERR_ARG, "options.split is not an OFHE_SPLIT_* value");
    }
    const u32 N = 1u << log_n;
    const u64 m = 2ull * N;
    for (u32 t = 0; t < towers; t++) {
        if (q[t] < 3 || q[t] >= (1ull << 60) || !(q[t] & 1))
            return fail(OFHE_ERR_ARG, "modulus " + std::to_string(t) + " must be odd and in [3, 2^60)");
        if ((q[t] - 1) % m)
            return fail(OFHE_ERR_ARG, "modulus " + std::to_string(t) + " is not 1 mod 2N");
        if (psi[t] < 2 || psi[t] >= q[t] || powmod(psi[t], N, q[t]) != q[t] - 1)
            return fail(OFHE_ERR_ARG, "root " + std::to_string(t) + " is not a primitive 2N-th root of unity");
    }
    ofhe_plan_s* p = new (std::nothrow) ofhe_plan_s();
    if (!p) return fail(OFHE_ERR_NOMEM, "plan allocation failed");
    p->ctx = ctx;
    p->log_n = log_n;
    p->towers = towers;
    const size_t TN = (size_t)towers * N;
    p->q.assign(q, q + towers);
    p->psi.assign(psi, psi + towers);
    p->tab.resize(TN);
    p->tab_pre.resize(TN);
    p->itab.resize(TN);
    p->itab_pre.resize(TN);
    p->ninv.resize(towers);
    std::vector<TowerConst> tc(towers);
    std::vector<u64> tw(2 * TN), itw(2 * TN);
    // round-3 transposed tables (k_block, see ntt_kernels.hpp): per tower
    // 15 U pairs, U = N/16, entry (S, j, u) at (2^S - 1) U + j U + u
    const u32 U3 = N >= 4096 ? N / 16 : 0;
    const size_t W3 = (size_t)15 * U3 * 2;  // words per tower
    std::vector<u64> tw3(W3 * towers);
    // DIT inverse (ntt_kernels.hpp): dtw[t + k] = psi^(-k N / t) for t = 1..N/2,
    // k < t; the block pass's output twist, and twist_r = twist * 2^64 mod q
    std::vector<u64> dtw(2 * TN), twist(2 * TN), twist_r(2 * TN);
    // PreCompute (transformnat-impl.h:708-763), one host thread per tower group
    auto build = [&](u32 t) {
        const u64 qt = q[t], ps = psi[t], psinv = invmod(ps, qt);
        u64* T = &p->tab[(size_t)t * N];
        u64* TI = &p->itab[(size_t)t * N];
        u64 x = 1, xi = 1;
        for (u32 i = 0; i < N; i++) {
            const u32 r = bitrev(i, log_n);
            T[r] = x;
            TI[r] = xi;
            x = mulmod(x, ps, qt);
            xi = mulmod(xi, psinv, qt);
        }
        const u64 ni = invmod(N % qt, qt);
        p->ninv[t] = ni;
        for (u32 i = 0; i < N; i++) {
            const size_t k = (size_t)t * N + i;
            p->tab_pre[k] = shoup_pre(T[i], qt);
            p->itab_pre[k] = shoup_pre(TI[i], qt);
            tw[2 * k] = T[i];
            tw[2 * k + 1] = p->tab_pre[k];
            itw[2 * k] = TI[i];
            itw[2 * k + 1] = p->itab_pre[k];
        }
        for (u32 S = 0; S < 4 && U3; S++)
            for (u32 j = 0; j < (1u << S); j++)
                for (u32 u = 0; u < U3; u++) {
                    const size_t e = (size_t)t * W3 + 2 * ((size_t)((1u << S) - 1) * U3 + (size_t)j * U3 + u);
                    const u32 idx = ((U3 + u) << S) + j;
                    tw3[e] = T[idx];
                    tw3[e + 1] = p->tab_pre[(size_t)t * N + idx];
                }
        {
            u64* D = &dtw[2 * (size_t)t * N];
            u64* F = &twist[2 * (size_t)t * N];
            u64* FR = &twist_r[2 * (size_t)t * N];
            D[0] = 1;
            D[1] = shoup_pre(1, qt);
            for (u32 tt = 1; tt < N; tt <<= 1) {
                const u64 base = powmod(psinv, N / tt, qt);
                u64 w = 1;
                for (u32 k = 0; k < tt; k++) {
                    D[2 * (tt + k)] = w;
                    D[2 * (tt + k) + 1] = shoup_pre(w, qt);
                    w = mulmod(w, base, qt);
                }
            }
            // block-pass twist: group b of G = 2^lb, position j0 ->
            // N^-1 psi^-((2 rev(b) + 1) j0) (ntt_kernels.hpp)
            const u32 lb = block_stages(split, log_n), G = 1u << lb;
            const u64 R = (u64)(((u128)1 << 64) % qt);
            for (u32 b = 0; b < N / G; b++) {
                const u64 step = powmod(psinv, 2 * (u64)bitrev(b, log_n - lb) + 1, qt);
                u64 f = ni;
                for (u32 j0 = 0; j0 < G; j0++) {
                    const u32 j = b * G + j0;
                    F[2 * j] = f;
                    F[2 * j + 1] = shoup_pre(f, qt);
                    const u64 fr = mulmod(f, R, qt);
                    FR[2 * j] = fr;
                    FR[2 * j + 1] = shoup_pre(fr, qt);
                    f = mulmod(f, step, qt);
                }
            }
        }
        TowerConst c{};
        c.q = qt;
        c.ninv = ni;
        c.ninv_pre = shoup_pre(ni, qt);
        const unsigned mb = msb64(qt);
        c.mu = (u64)((((u128)1) << (2 * mb + 3)) / qt);  // ComputeMu, ubintnat.h:651-656
        c.nshift = mb - 2;
        // special prime q = 2^mb - d, d < 2^32: hi32(q) == 2^(mb-32) - 1
        // and 16 d < q, d != 2^32 (canon_spq's single conditional subtract)
        const bool spq = mb >= 33 && (qt >> 32) == ((1ull << (mb - 32)) - 1) && (u32)qt != 0 &&
                         (((1ull << mb) - qt) << 4) < qt;
        c.spq_sh = spq ? mb - 32 : 0;
        c.nq = 0 - qt;
        c.nq4 = 0 - 4 * qt;
        c.one = 1;
        u64 inv = qt;  // q^-1 mod 2^64 by Newton iteration (q odd)
        for (int it = 0; it < 6; it++) inv *= 2 - qt * inv;
        c.qinv = inv;
        tc[t] = c;
    };
    {
        unsigned nth = std::thread::hardware_concurrency();
        if (nth < 1) nth = 1;
        if (nth > towers) nth = towers;
        if (nth > 16) nth = 16;
        std::vector<std::thread> th;
        for (unsigned w = 0; w < nth; w++)
            th.emplace_back([&, w] {
                for (u32 t = w; t < towers; t += nth) build(t);
            });
        for (auto& x : th) x.join();
    }
    p->spq = true;
    for (u32 t = 0; t < towers; t++) p->spq = p->spq && tc[t].spq_sh != 0;
    if (opt.generic_moduli) p->spq = false;
    p->split = split;
    p->opts = opt;
    hipError_t e = hipSetDevice(ctx->device);
    if (e == hipSuccess) e = hipMalloc(&p->d_tc, sizeof(TowerConst) * towers);
    if (e == hipSuccess) e = hipMalloc(&p->d_tw, sizeof(u64) * 2 * TN);
    if (e == hipSuccess) e = hipMalloc(&p->d_itw, sizeof(u64) * 2 * TN);
    if (e == hipSuccess) e = hipMalloc(&p->d_tw3, sizeof(u64) * (tw3.size() ? tw3.size() : 2));
    if (e == hipSuccess && tw3.size())
        e = upload_blocking(p->d_tw3, tw3.data(), sizeof(u64) * tw3.size());
    if (e == hipSuccess) e = hipMalloc(&p->d_dtw, sizeof(u64) * 2 * TN);
    if (e == hipSuccess) e = hipMalloc(&p->d_twist, sizeof(u64) * 2 * TN);
    if (e == hipSuccess) e = hipMalloc(&p->d_twist_r, sizeof(u64) * 2 * TN);
    if (e == hipSuccess) e = upload_blocking(p->d_dtw, dtw.data(), sizeof(u64) * 2 * TN);
    if (e == hipSuccess) e = upload_blocking(p->d_twist, twist.data(), sizeof(u64) * 2 * TN);
    if (e == hipSuccess) e = upload_blocking(p->d_twist_r, twist_r.data(), sizeof(u64) * 2 * TN);
    if (e == hipSuccess) e = upload_blocking(p->d_tc, tc.data(), sizeof(TowerConst) * towers);
    if (e == hipSuccess) e = upload_blocking(p->d_tw, tw.data(), sizeof(u64) * 2 * TN);
    if (e == hipSuccess) e = upload_blocking(p->d_itw, itw.data(), sizeof(u64) * 2 * TN);
    if (e != hipSuccess) {
        ofhe_hip_plan_destroy(p);
        return fail(OFHE_ERR_HIP, std::string("plan upload: ") + hipGetErrorString(e));
    }
    *plan = p;
    return OFHE_OK;
}

int ofhe_hip_plan_tune(ofhe_plan_t p, uint32_t chunk_batch, uint32_t streams) {
    if (!p || !p->ctx) return fail(OFHE_ERR_STATE, "plan is NULL or destroyed");
    if (streams < 1 || streams > 2) return fail(OFHE_ERR_ARG, "streams must be 1 or 2");
    HIPCHK(hipSetDevice(p->ctx->device));
    std::lock_guard<std::mutex> lk(p->fork_mu);
    if (streams == 2 && !p->st[0]) {
        // create everything into locals and commit only when all succeeded,
        // so a failure leaves the plan as it was
        hipStream_t st[2] = {nullptr, nullptr};
        hipEvent_t fork = nullptr, join[2] = {nullptr, nullptr};
        hipError_t e = hipSuccess;
        for (int i = 0; i < 2 && e == hipSuccess; i++) {
            e = hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking);
            if (e == hipSuccess) e = hipEventCreateWithFlags(&join[i], hipEventDisableTiming);
        }
        if (e == hipSuccess) e = hipEventCreateWithFlags(&fork, hipEventDisableTiming);
        if (e != hipSuccess) {
            for (int i = 0; i < 2; i++) {
                if (st[i]) (void)hipStreamDestroy(st[i]);
                if (join[i]) (void)hipEventDestroy(join[i]);
            }
            if (fork) (void)hipEventDestroy(fork);
            return fail(OFHE_ERR_HIP, std::string("plan_tune: ") + hipGetErrorString(e));
        }
        for (int i = 0; i < 2; i++) {
            p->st[i] = st[i];
            p->ev_join[i] = join[i];
        }
        p->ev_fork = fork;
    }
    p->chunk_batch = chunk_batch;
    p->nstreams = streams;
    return OFHE_OK;
}

int ofhe_hip_plan_destroy(ofhe_plan_t p) {
    if (!p) return fail(OFHE_ERR_ARG, "plan is NULL");
    if (p->ctx) (void)hipSetDevice(p->ctx->device);
    for (int i = 0; i < 2; i++) {
        if (p->st[i]) (void)hipStreamSynchronize(p->st[i]);
        if (p->st[i]) (void)hipStreamDestroy(p->st[i]);
        if (p->ev_join[i]) (void)hipEventDestroy(p->ev_join[i]);
    }
    if (p->ev_fork) (void)hipEventDestroy(p->ev_fork);
    (void)hipFree(p->d_tc);
    (void)hipFree(p->d_tw);
    (void)hipFree(p->d_itw);
    (void)hipFree(p->d_tw3);
    (void)hipFree(p->d_dtw);
    (void)hipFree(p->d_twist);
    (void)hipFree(p->d_twist_r);
    for (auto& kv : p->tabs) (void)hipFree(kv.second);
    delete p;
    return OFHE_OK;
}

int ofhe_hip_plan_tables(ofhe_plan_t p, uint64_t* tab, uint64_t* tab_pre, uint64_t* itab,
                         uint64_t* itab_pre, uint64_t* ninv) {
    if (!p) return fail(OFHE_ERR_ARG, "plan is NULL");
    const size_t n = p->tab.size() * sizeof(u64);
    if (tab) memcpy(tab, p->tab.data(), n);
    if (tab_pre) memcpy(tab_pre, p->tab_pre.data(), n);
    if (itab) memcpy(itab, p->itab.data(), n);
    if (itab_pre) memcpy(itab_pre, p->itab_pre.data(), n);
    if (ninv) memcpy(ninv, p->ninv.data(), p->ninv.size() * sizeof(u64));
    return OFHE_OK;
}

// ---------------------------------------------------------------------------
// Launch helpers
// ---------------------------------------------------------------------------
// Device view of plan towers [t0, t0 + count); dense [batch][count][N] strides
// unless the caller overrides them.
static PlanArgs args_of(ofhe_plan_t p, u32 t0 = 0, u32 count = 0) {
    if (!count) count = p->towers - t0;
    const u64 N = 1ull << p->log_n;
    PlanArgs a;
    a.tc = p->d_tc + t0;
    a.tw = p->d_tw + 2 * N * t0;
    a.itw = p->d_itw + 2 * N * t0;
    a.tw3 = p->d_tw3 + (N >= 4096 ? (N / 16) * 30 * t0 : 0);
    a.sstride = a.dstride = a.bstride = N * count;
    a.scal = nullptr;
    a.dtw = p->d_dtw + 2 * N * t0;
    a.twist = p->d_twist + 2 * N * t0;
    a.log_n = p->log_n;
    a.towers = count;
    return a;
}

// Fused pipeline: with the Montgomery Hadamard (kMontFused, log_n >= 12) the
// inverse output twist also carries 2^64 to cancel its 2^-64.
static PlanArgs fused_args(ofhe_plan_t p) {
    PlanArgs a = args_of(p);
    if (kMontFused && p->log_n >= 12) a.twist = p->d_twist_r;
    return a;
}

static int check_common(ofhe_plan_t p, uint32_t batch) {
    if (!p || !p->ctx) return fail(OFHE_ERR_STATE, "plan is NULL or destroyed");
    if (batch == 0) return fail(OFHE_ERR_ARG, "batch must be >= 1");
    const u64 polys = (u64)batch * p->towers;
    if (polys * ((u64)1 << p->log_n) / 4096 >= (1ull << 31))
        return fail(OFHE_ERR_ARG, "batch too large for one launch");
    return OFHE_OK;
}

#ifndef OFHE_COLS_CPT
#define OFHE_COLS_CPT 2
#endif
// Every launcher picks the special-prime instantiation when the plan allows it.
template <int KA, bool INV, bool SPQ>
static void launch_cols_t(const PlanArgs& a, const u64* src, u64* dst, u32 batch, hipStream_t s) {
    // two columns per thread (16-byte accesses) while registers allow
    constexpr int CPT = KA <= 4 ? OFHE_COLS_CPT : 1;
    const u32 nwg = batch * a.towers * (16 / CPT);
    hipLaunchKernelGGL((k_cols<KA, INV, CPT, SPQ>), dim3(nwg), dim3(256), 0, s, a, src, dst, batch, nwg,
                       SwSrc{nullptr, 0, 0, nullptr, 1, 0});
}
template <int KA, bool SPQ>
static void launch_cols_sw(const PlanArgs& a, const SwSrc& S, u64* dst, u32 batch, hipStream_t s) {
    constexpr int CPT = KA <= 4 ? OFHE_COLS_CPT : 1;
    const u32 nwg = batch * a.towers * (16 / CPT);
    hipLaunchKernelGGL((k_cols<KA, false, CPT, SPQ, true>), dim3(nwg), dim3(256), 0, s, a, (const u64*)nullptr, dst,
                       batch, nwg, S);
}

template <bool SPQ>
static void launch_cols_s(const PlanArgs& a, bool inv, const u64* src, u64* dst, u32 batch, hipStream_t s) {
    switch (a.log_n - 12) {
#define CASE(K)                                                 \
    case K:                                                     \
        if (inv)                                                \
            launch_cols_t<K, true, SPQ>(a, src, dst, batch, s); \
        else                                                    \
            launch_cols_t<K, false, SPQ>(a, src, dst, batch, s);\
        break;
        CASE(1) CASE(2) CASE(3) CASE(4) CASE(5)
#undef CASE
        default: break;
    }
}
static void launch_cols(const PlanArgs& a, bool spq, bool inv, const u64* src, u64* dst, u32 batch, hipStream_t s) {
    if (spq)
        launch_cols_s<true>(a, inv, src, dst, batch, s);
    else
        launch_cols_s<false>(a, inv, src, dst, batch, s);
}

// column pass for log_n > 12: k_tcols / k_tcols9 (8 / 9 stages) unless SPLIT_COLS, else k_cols
static void launch_colpass(const PlanArgs& a, bool spq, int split, bool inv, const u64* src, u64* dst, u32 batch,
                           hipStream_t s);

// Pass split for log_n > 12 (the plan's split, internal.hpp): the block pass
// runs the last 8 (SPLIT_T8 / T9: k_block NR = 2), 9 (SPLIT_T8B9: NR = 3
// without the first three stages of its first round) or 12 stages.
template <int MODE>
static void launch_block(const PlanArgs& a, bool spq, const u64* src, u64* dst, const u64* b, u32 batch,
                         hipStream_t s, int split = SPLIT_COLS) {
    const u32 nwg = batch * a.towers * (1u << (a.log_n - 12));
#define LB(SP, NR, SK) \
    hipLaunchKernelGGL((k_block<MODE, SP, NR, SK>), dim3(nwg), dim3(256), 0, s, a, src, dst, b, batch, nwg)
    if (split == SPLIT_T8 || split == SPLIT_T9) {
        if (spq) LB(true, 2, 0); else LB(false, 2, 0);
    } else if (split == SPLIT_T8B9) {
        if (spq) LB(true, 3, 3); else LB(false, 3, 3);
    } else {
        if (spq) LB(true, 3, 0); else LB(false, 3, 0);
    }
#undef LB
}

static void launch_tcols(const PlanArgs& a, bool spq, int split, bool inv, const u64* src, u64* dst, u32 batch,
                         hipStream_t s) {
    if (split == SPLIT_T8B9) {
        const u32 nwg = batch * a.towers * (512 / TCOLS_W);
#define LT17(I, SP)                                                                                           \
    hipLaunchKernelGGL((k_tcols<I, SP, false, 17>), dim3(nwg), dim3(16 * TCOLS_W), 0, s, a, src, dst, batch, nwg, \
                       SwSrc{nullptr, 0, 0, nullptr, 1, 0})
        if (inv) {
            if (spq) LT17(true, true); else LT17(true, false);
        } else {
            if (spq) LT17(false, true); else LT17(false, false);
        }
#undef LT17
        return;
    }
    if (split == SPLIT_T9) {
        const u32 nwg = batch * a.towers * 16;  // 16-column tiles of 512 rows
#define LT9(I, SP) hipLaunchKernelGGL((k_tcols9<I, SP>), dim3(nwg), dim3(512), 0, s, a, src, dst, batch, nwg)
        if (inv) {
            if (spq) LT9(true, true); else LT9(true, false);
        } else {
            if (spq) LT9(false, true); else LT9(false, false);
        }
#undef LT9
        return;
    }
    const u32 nwg = batch * a.towers * (256 / TCOLS_W);
#define LT(I, SP)                                                                                 \
    hipLaunchKernelGGL((k_tcols<I, SP>), dim3(nwg), dim3(16 * TCOLS_W), 0, s, a, src, dst, batch, nwg, \
                       SwSrc{nullptr, 0, 0, nullptr, 1, 0})
    if (inv) {
        if (spq) LT(true, true); else LT(true, false);
    } else {
        if (spq) LT(false, true); else LT(false, false);
    }
#undef LT
}

template <int MODE>
static void launch_small(const PlanArgs& a, bool spq, const u64* src, u64* dst, const u64* b, u32 batch,
                         hipStream_t s) {
    const u32 N = 1u << a.log_n;
    const u32 thr = N / 2 >= 256 ? 256 : (N / 2 < 64 ? 64 : N / 2);
    if (spq)
        hipLaunchKernelGGL((k_small<MODE, true>), dim3(batch * a.towers), dim3(thr), 0, s, a, src, dst, b, batch);
    else
        hipLaunchKernelGGL((k_small<MODE, false>), dim3(batch * a.towers), dim3(thr), 0, s, a, src, dst, b, batch);
}

static void launch_colpass(const PlanArgs& a, bool spq, int split, bool inv, const u64* src, u64* dst, u32 batch,
                           hipStream_t s) {
    if (split != SPLIT_COLS)
        launch_tcols(a, spq, split, inv, src, dst, batch, s);
    else
        launch_cols(a, spq, inv, src, dst, batch, s);
}


namespace ofhe {
int plan_ntt_range(ofhe_plan_t p, bool inverse, u32 t0, u32 count, const u64* src, u64* dst, u64 sstride,
                   u64 dstride, u32 batch, hipStream_t s) {
    if (!p || !p->ctx) return fail(OFHE_ERR_STATE, "plan is NULL or destroyed");
    if (count == 0 || batch == 0) return OFHE_OK;
    if (t0 + count > p->towers || t0 + count < t0) return fail(OFHE_ERR_ARG, "tower range outside the plan");
    if (!src || !dst) return fail(OFHE_ERR_ARG, "data is NULL");
    const u64 N = 1ull << p->log_n;
    if (sstride < N * count || dstride < N * count)
        return fail(OFHE_ERR_ARG, "batch stride smaller than the tower range");
    if ((u64)batch * count * N / 4096 >= (1ull << 31)) return fail(OFHE_ERR_ARG, "batch too large for one launch");
    HIPCHK(hipSetDevice(p->ctx->device));
    PlanArgs a = args_of(p, t0, count);
    PlanArgs ad = a;  // second pass: dst -> dst
    a.sstride = sstride;
    a.dstride = ad.sstride = ad.dstride = dstride;
    if (!inverse) {
        if (p->log_n < 12) {
            launch_small<MODE_FWD>(a, p->spq, src, dst, nullptr, batch, s);
        } else if (p->log_n == 12) {
            launch_block<MODE_FWD>(a, p->spq, src, dst, nullptr, batch, s, p->split);
        } else {
            launch_colpass(a, p->spq, p->split, false, src, dst, batch, s);
            launch_block<MODE_FWD>(ad, p->spq, dst, dst, nullptr, batch, s, p->split);
        }
    } else {
        if (p->log_n < 12) {
            launch_small<MODE_INV>(a, p->spq, src, dst, nullptr, batch, s);
        } else {
            launch_block<MODE_INV>(a, p->spq, src, dst, nullptr, batch, s, p->split);
            if (p->log_n > 12) launch_colpass(ad, p->spq, p->split, true, dst, dst, batch, s);
        }
    }
    return post_launch();
}

int plan_cols_switch(ofhe_plan_t p, u32 t0, u32 count, const u64* last, u64 lstride, u64 ql, u64 pre, const u64* tab,
                     u64* y, u64 ystride, u32 batch, hipStream_t s) {
    if (!p || !p->ctx) return fail(OFHE_ERR_STATE, "plan is NULL or destroyed");
    if (p->log_n <= 12 || p->split == SPLIT_T9) return fail(OFHE_ERR_ARG, "plan_cols_switch: k_cols / k_tcols plans only");
    if (((uintptr_t)last & 15) || (lstride & 1)) return fail(OFHE_ERR_ARG, "plan_cols_switch: misaligned source");
    HIPCHK(hipSetDevice(p->ctx->device));
    PlanArgs a = args_of(p, t0, count);
    a.sstride = a.dstride = ystride;
    pre %= ql;
    const SwSrc S{last, lstride, ql, tab, pre, pre == 1 ? 0 : shoup_pre(pre, ql)};
    if (p->split == SPLIT_T8) {  // N = 2^16: k_tcols
        const u32 nwg = batch * a.towers * (256 / TCOLS_W);
        if (p->spq)
            hipLaunchKernelGGL((k_tcols<false, true, true>), dim3(nwg), dim3(16 * TCOLS_W), 0, s, a,
                               (const u64*)nullptr, y, batch, nwg, S);
        else
            hipLaunchKernelGGL((k_tcols<false, false, true>), dim3(nwg), dim3(16 * TCOLS_W), 0, s, a,
                               (const u64*)nullptr, y, batch, nwg, S);
        return post_launch();
    }
    if (p->split == SPLIT_T8B9) {  // N = 2^17: k_tcols, 512 columns
        const u32 nwg = batch * a.towers * (512 / TCOLS_W);
        if (p->spq)
            hipLaunchKernelGGL((k_tcols<false, true, true, 17>), dim3(nwg), dim3(16 * TCOLS_W), 0, s, a,
                               (const u64*)nullptr, y, batch, nwg, S);
        else
            hipLaunchKernelGGL((k_tcols<false, false, true, 17>), dim3(nwg), dim3(16 * TCOLS_W), 0, s, a,
                               (const u64*)nullptr, y, batch, nwg, S);
        return post_launch();
    }
    switch (p->log_n - 12) {
#define CASE(K)                                                 \
    case K:                                                     \
        if (p->spq)                                             \
            launch_cols_sw<K, true>(a, S, y, batch, s);         \
        else                                                    \
            launch_cols_sw<K, false>(a, S, y, batch, s);        \
        break;
        CASE(1) CASE(2) CASE(3) CASE(4) CASE(5)
#undef CASE
        default: break;
    }
    return post_launch();
}

int plan_ntt_fwd_block(ofhe_plan_t p, u32 t0, u32 count, u64* y, u64 ystride, u32 batch, hipStream_t s) {
    if (!p || !p->ctx) return fail(OFHE_ERR_STATE, "plan is NULL or destroyed");
    if (p->log_n <= 12) return fail(OFHE_ERR_ARG, "plan_ntt_fwd_block: log_n > 12 only");
    HIPCHK(hipSetDevice(p->ctx->device));
    PlanArgs a = args_of(p, t0, count);
    a.sstride = a.dstride = ystride;
    launch_block<MODE_FWD>(a, p->spq, y, y, nullptr, batch, s, p->split);
    return post_launch();
}

int plan_ntt_inv_block(ofhe_plan_t p, u32 t0, u32 count, const u64* src, u64 sstride, u64* dst, u64 dstride, u32 batch,
                       hipStream_t s) {
    if (!p || !p->ctx) return fail(OFHE_ERR_STATE, "plan is NULL or destroyed");
    if (p->log_n <= 12) return fail(OFHE_ERR_ARG, "plan_ntt_inv_block: log_n > 12 only");
    if (count == 0 || batch == 0) return OFHE_OK;
    if (t0 + count > p->towers) return fail(OFHE_ERR_ARG, "tower range outside the plan");
    HIPCHK(hipSetDevice(p->ctx->device));
    PlanArgs a = args_of(p, t0, count);
    a.sstride = sstride;
    a.dstride = dstride;
    launch_block<MODE_INV>(a, p->spq, src, dst, nullptr, batch, s, p->split);
    return post_launch();
}

int plan_ntt_fwd_sub(ofhe_plan_t p, u32 t0, u32 count, u64* y, u64 ystride, const u64* x, u64 xstride, u64* out,
                     u64 ostride, const u64* scal, u32 batch, hipStream_t s, int parts) {
    if (!p || !p->ctx) return fail(OFHE_ERR_STATE, "plan is NULL or destroyed");
    if (p->log_n < 12) return fail(OFHE_ERR_ARG, "fused forward + subtract needs log_n >= 12");
    if (count == 0 || batch == 0) return OFHE_OK;
    if (t0 + count > p->towers) return fail(OFHE_ERR_ARG, "tower range outside the plan");
    HIPCHK(hipSetDevice(p->ctx->device));
    PlanArgs a = args_of(p, t0, count);
    a.sstride = a.dstride = ystride;
    if (p->log_n > 12 && (parts & 1)) launch_colpass(a, p->spq, p->split, false, y, y, batch, s);
    if (!(parts & 2)) return post_launch();
    PlanArgs ab = a;
    ab.sstride = ystride;
    ab.dstride = ostride;
    ab.bstride = xstride;
    ab.scal = scal;
    launch_block<MODE_FWD_SUB>(ab, p->spq, y, out, x, batch, s, p->split);
    return post_launch();
}
}  // namespace ofhe

int ofhe_hip_ntt_fwd(ofhe_plan_t p, uint64_t* data, uint32_t batch, void* stream) {
    RCCHK(check_common(p, batch));
    if (!data) return fail(OFHE_ERR_ARG, "data is NULL");
    const u64 d = (u64)p->towers << p->log_n;
    return plan_ntt_range(p, false, 0, p->towers, data, data, d, d, batch, pick(stream));
}

int ofhe_hip_ntt_inv(ofhe_plan_t p, uint64_t* data, uint32_t batch, void* stream) {
    RCCHK(check_common(p, batch));
    if (!data) return fail(OFHE_ERR_ARG, "data is NULL");
    const u64 d = (u64)p->towers << p->log_n;
    return plan_ntt_range(p, true, 0, p->towers, data, data, d, d, batch, pick(stream));
}

int ofhe_hip_ntt_fwd_range(ofhe_plan_t p, uint32_t t0, uint32_t count, const uint64_t* src, uint64_t* dst,
                           uint64_t src_stride, uint64_t dst_stride, uint32_t batch, void* stream) {
    if (!p || !p->ctx) return fail(OFHE_ERR_STATE, "plan is NULL or destroyed");
    if (batch == 0 || count == 0) return fail(OFHE_ERR_ARG, "batch and count must be >= 1");
    return plan_ntt_range(p, false, t0, count, src, dst, src_stride, dst_stride, batch, pick(stream));
}

int ofhe_hip_ntt_inv_range(ofhe_plan_t p, uint32_t t0, uint32_t count, const uint64_t* src, uint64_t* dst,
                           uint64_t src_stride, uint64_t dst_stride, uint32_t batch, void* stream) {
    if (!p || !p->ctx) return fail(OFHE_ERR_STATE, "plan is NULL or destroyed");
    if (batch == 0 || count == 0) return fail(OFHE_ERR_ARG, "batch and count must be >= 1");
    return plan_ntt_range(p, true, t0, count, src, dst, src_stride, dst_stride, batch, pick(stream));
}

int ofhe_hip_ntt_mul_intt(ofhe_plan_t p, const uint64_t* a_, const uint64_t* b, uint64_t* c,
                          uint32_t batch, void* stream) {
    int rc = check_common(p, batch);
    if (rc) return rc;
    if (!a_ || !b || !c) return fail(OFHE_ERR_ARG, "NULL data pointer");
    if (b == c && a_ != c) return fail(OFHE_ERR_ARG, "c may alias a but not b");
    HIPCHK(hipSetDevice(p->ctx->device));
    const PlanArgs a = fused_args(p);
    hipStream_t s = pick(stream);
    if (p->log_n < 12) {
        launch_small<MODE_FUSED>(a, p->spq, a_, c, b, batch, s);
    } else if (p->log_n == 12) {
        launch_block<MODE_FUSED>(a, p->spq, a_, c, b, batch, s, p->split);
    } else {
        // Chunk the batch so a chunk's intermediates stay in the Infinity
        // Cache between the three passes; optionally alternate two streams so
        // one chunk's HBM-bound column passes overlap another's VALU-bound
        // block pass.
        const u32 cb = (p->chunk_batch && p->chunk_batch < batch) ? p->chunk_batch : batch;
        const u64 words = (u64)p->towers << p->log_n;
        const bool multi = p->nstreams == 2 && cb < batch;
        // the fork / join events and side streams are the plan's: one caller at
        // a time records and waits on them (PlanCache shares plans process-wide)
        std::unique_lock<std::mutex> lk(p->fork_mu, std::defer_lock);
        if (multi) lk.lock();
        if (multi) {
            HIPCHK(hipEventRecord(p->ev_fork, s));
            for (int i = 0; i < 2; i++) HIPCHK(hipStreamWaitEvent(p->st[i], p->ev_fork, 0));
        }
        u32 idx = 0;
        for (u32 b0 = 0; b0 < batch; b0 += cb, idx++) {
            const u32 n = batch - b0 < cb ? batch - b0 : cb;
            hipStream_t sx = multi ? p->st[idx & 1] : s;
            const u64 off = (u64)b0 * words;
            launch_colpass(a, p->spq, p->split, false, a_ + off, c + off, n, sx);
            launch_block<MODE_FUSED>(a, p->spq, c + off, c + off, b + off, n, sx, p->split);
            launch_colpass(a, p->spq, p->split, true, c + off, c + off, n, sx);
        }
        if (multi) {
            for (int i = 0; i < 2; i++) {
                HIPCHK(hipEventRecord(p->ev_join[i], p->st[i]));
                HIPCHK(hipStreamWaitEvent(s, p->ev_join[i], 0));
            }
        }
    }
    return post_launch();
}

int ofhe_hip_ntt_mul_intt_stage(ofhe_plan_t p, int stage, const uint64_t* a_, const uint64_t* b, uint64_t* c,
                                uint32_t batch, void* stream) {
    int rc = check_common(p, batch);
    if (rc) return rc;
    if (!a_ || !b || !c) return fail(OFHE_ERR_ARG, "NULL data pointer");
    if (stage < 0 || stage > 2) return fail(OFHE_ERR_ARG, "stage must be 0, 1 or 2");
    HIPCHK(hipSetDevice(p->ctx->device));
    const PlanArgs a = fused_args(p);
    hipStream_t s = pick(stream);
    if (p->log_n < 12) {
        if (stage == 1) launch_small<MODE_FUSED>(a, p->spq, a_, c, b, batch, s);
    } else if (p->log_n == 12) {
        if (stage == 1) launch_block<MODE_FUSED>(a, p->spq, a_, c, b, batch, s, p->split);
    } else if (stage == 0) {
        launch_colpass(a, p->spq, p->split, false, a_, c, batch, s);
    } else if (stage == 1) {
        launch_block<MODE_FUSED>(a, p->spq, c, c, b, batch, s, p->split);
    } else {
        launch_colpass(a, p->spq, p->split, true, c, c, batch, s);
    }
    return post_launch();
}

// grid cap of the streaming element-wise launches (grid-stride beyond it;
// 2^22 blocks = 2^31 pairs per pass, never reached by a launch of the sizes used)
#ifndef OFHE_ELT_GRID
#define OFHE_ELT_GRID (1u << 22)
#endif
template <int OP>
static int eltwise(ofhe_plan_t p, const u64* a, const u64* b, u64* c, u32 batch, void* stream) {
    int rc = check_common(p, batch);
    if (rc) return rc;
    if (!a || !b || !c) return fail(OFHE_ERR_ARG, "NULL data pointer");
    HIPCHK(hipSetDevice(p->ctx->device));
    const u64 npairs = (u64)batch * p->towers * ((u64)1 << p->log_n) / 2;
    u64 blocks = (npairs + 256 * elt_unroll(OP) - 1) / (256 * elt_unroll(OP));
    if (blocks > OFHE_ELT_GRID) blocks = OFHE_ELT_GRID;
    hipLaunchKernelGGL((k_eltwise<OP>), dim3((u32)blocks), dim3(256), 0, pick(stream), p->d_tc, a, b,
                       c, npairs, p->log_n, p->towers);
    return post_launch();
}

int ofhe_hip_eval_mult_core(ofhe_plan_t p, const uint64_t* c0, const uint64_t* c1, const uint64_t* d0,
                            const uint64_t* d1, uint64_t* out0, uint64_t* out1, uint64_t* out2, uint32_t batch,
                            void* stream) {
    int rc = check_common(p, batch);
    if (rc) return rc;
    if (!c0 || !c1 || !d0 || !d1 || !out0 || !out1 || !out2) return fail(OFHE_ERR_ARG, "NULL data pointer");
    HIPCHK(hipSetDevice(p->ctx->device));
    const u64 N = 1ull << p->log_n;
    const u32 bpr = (u32)((N / 2 + 255) / 256);
    const u64 blocks = (u64)bpr * batch * p->towers;
    if (blocks >= (1ull << 31)) return fail(OFHE_ERR_ARG, "batch too large for one launch");
    hipLaunchKernelGGL(k_tensor2<0>, dim3((u32)blocks), dim3(256), 0, pick(stream), p->d_tc, c0, c1, d0, d1, out0,
                       out1, out2, bpr, p->log_n, p->towers);
    return post_launch();
}

int ofhe_hip_modmul_vv(ofhe_plan_t p, const uint64_t* a, const uint64_t* b, uint64_t* c, uint32_t batch,
                       void* stream) {
    return eltwise<ELT_MUL>(p, a, b, c, batch, stream);
}
int ofhe_hip_modadd_vv(ofhe_plan_t p, const uint64_t* a, const uint64_t* b, uint64_t* c, uint32_t batch,
                       void* stream) {
    return eltwise<ELT_ADD>(p, a, b, c, batch, stream);
}
int ofhe_hip_modsub_vv(ofhe_plan_t p, const uint64_t* a, const uint64_t* b, uint64_t* c, uint32_t batch,
                       void* stream) {
    return eltwise<ELT_SUB>(p, a, b, c, batch, stream);
}

// Vector (.) per-tower scalar.  Each scalar is reduced mod q_t first, as the
// reference does (mubintvecnat.cpp:198-219, 267-288, 310-332), and travels in
// the kernel arguments, SCALAR_MAX towers per launch: nothing is uploaded, so
// concurrent calls on any streams never share state and nothing synchronises.
template <int OP>
static int scalar_op(ofhe_plan_t p, const u64* a, const u64* s, u64* c, u32 batch, bool at_index, u64 idx,
                     void* stream) {
    int rc = check_common(p, batch);
    if (rc) return rc;
    if (!a || !c) return fail(OFHE_ERR_ARG, "NULL data pointer");
    if (!s) return fail(OFHE_ERR_ARG, "scalar array is NULL");
    if (at_index && idx >= (1ull << p->log_n)) return fail(OFHE_ERR_ARG, "index out of range");
    HIPCHK(hipSetDevice(p->ctx->device));
    hipStream_t st = pick(stream);
    for (u32 t0 = 0; t0 < p->towers; t0 += SCALAR_MAX) {
        const u32 cnt = p->towers - t0 < SCALAR_MAX ? p->towers - t0 : SCALAR_MAX;
        ScalarPack S{};
        for (u32 i = 0; i < cnt; i++) {
            const u64 q = p->q[t0 + i], v = s[t0 + i] % q;
            S.v[3 * i] = q;
            S.v[3 * i + 1] = v;
            S.v[3 * i + 2] = shoup_pre(v, q);
        }
        if (at_index) {
            const u64 rows = (u64)batch * cnt;
            hipLaunchKernelGGL(k_scalar_at, dim3((u32)((rows + 255) / 256)), dim3(256), 0, st, S, a, c, batch,
                               p->log_n, cnt, t0, p->towers, idx);
        } else {
            const u64 npairs = ((u64)batch * cnt << p->log_n) / 2;
            u64 blocks = (npairs + 256 * elt_unroll(OP) - 1) / (256 * elt_unroll(OP));
            if (blocks > OFHE_ELT_GRID) blocks = OFHE_ELT_GRID;
            hipLaunchKernelGGL((k_scalar<OP>), dim3((u32)blocks), dim3(256), 0, st, S, a, c, npairs, p->log_n, cnt,
                               t0, p->towers);
        }
        RCCHK(post_launch());
    }
    return OFHE_OK;
}

int ofhe_hip_modmul_scalar(ofhe_plan_t p, const uint64_t* a, const uint64_t* s, uint64_t* c,
                           uint32_t batch, void* stream) {
    return scalar_op<ELT_MULS>(p, a, s, c, batch, false, 0, stream);
}
int ofhe_hip_modadd_scalar(ofhe_plan_t p, const uint64_t* a, const uint64_t* s, uint64_t* c,
                           uint32_t batch, void* stream) {
    return scalar_op<ELT_ADDS>(p, a, s, c, batch, false, 0, stream);
}
int ofhe_hip_modsub_scalar(ofhe_plan_t p, const uint64_t* a, const uint64_t* s, uint64_t* c,
                           uint32_t batch, void* stream) {
    return scalar_op<ELT_SUBS>(p, a, s, c, batch, false, 0, stream);
}
int ofhe_hip_modadd_scalar_at(ofhe_plan_t p, const uint64_t* a, uint64_t index, const uint64_t* s, uint64_t* c,
                              uint32_t batch, void* stream) {
    return scalar_op<ELT_ADDS>(p, a, s, c, batch, true, index, stream);
}

int ofhe_hip_fill_uniform(ofhe_plan_t p, uint64_t* dst, uint32_t batch, uint32_t batch_offset, uint64_t seed,
                          void* stream) {
    int rc = check_common(p, batch);
    if (rc) return rc;
    if (!dst) return fail(OFHE_ERR_ARG, "NULL data pointer");
    HIPCHK(hipSetDevice(p->ctx->device));
    const u64 words = (u64)batch * p->towers << p->log_n;
    u64 blocks = (words + 255) / 256;
    if (blocks > (1u << 22)) blocks = 1u << 22;
    hipLaunchKernelGGL(k_fill_uniform, dim3((u32)blocks), dim3(256), 0, pick(stream), p->d_tc, dst, words,
                       p->log_n, p->towers, batch_offset, seed);
    return post_launch();
}

// ---------------------------------------------------------------------------
// Base conversion
// ---------------------------------------------------------------------------
namespace {
template <class T>
T* pred_of(T* qhlimb, u32 qrows, u32 ppad) { return qhlimb + (size_t)qrows * ppad; }
}  // namespace

// k_bconv_mma's LDS image (bconv_mma.hpp): A-operand fragments
// [tiles][ks][64 lanes][16 int8], then BmRed[4 tiles], then BmSrc[4 ks].
// qhinv: [size_q][2] (canonical QHatInvModq, Shoup precon); qhmodp: [size_q][size_p], canonical.
// A chunk of tpc target tiles per block (blockIdx.y) keeps the LDS image of
// one block within BCONV_MMA_LDS_MAX for any size_p.
static u32 bconv_mma_lds(u32 tpc, u32 ks) { return tpc * (ks * 1024 + 4 * (u32)sizeof(BmRed)) + 4 * ks * (u32)sizeof(BmSrc); }
static bool bconv_mma_table(u32 size_q, u32 size_p, const u64* q, const u64* p, const u64* qhinv,
                            const u64* qhmodp, std::vector<unsigned char>& tab, u32& tiles, u32& ks, u32& tpc,
                            bool& spq) {
    ks = (size_q + 3) / 4;
    if (ks > 8) ks = (ks + 1) & ~1u;  // instantiated K-step counts: 1..8, 10, 12, 14, 16 (zero-padded sources)
    tiles = (size_p + 3) / 4;
    tpc = 0;
    if (size_q > BCONV_MMA_QMAX) {
        tiles = ks = 0;
        return false;
    }
    while (tpc < tiles && bconv_mma_lds(tpc + 1, ks) <= BCONV_MMA_LDS_MAX) tpc++;
    if (tpc == 0) {
        tiles = ks = 0;
        return false;
    }
    const size_t fbytes = (size_t)tiles * ks * 1024;
    const size_t bytes = fbytes + 4 * (size_t)tiles * sizeof(BmRed) + 4 * (size_t)ks * sizeof(BmSrc);
    tab.assign(bytes, 0);
    // h_{(i,a),j} = 2^(8a) QHatModp_{i,j} mod p_j, as signed base-256 digits
    for (u32 t = 0; t < tiles; t++)
        for (u32 s = 0; s < ks; s++)
            for (u32 l = 0; l < 64; l++) {
                const u32 r = l & 31, kh = l >> 5;
                const u32 dh = (r >> 2) & 1, reg = (r & 3) + 4 * (r >> 3);
                const u32 j = 4 * t + 2 * dh + (reg >> 3), bd = reg & 7;
                for (u32 e = 0; e < 16; e++) {
                    const u32 i = 4 * s + 2 * kh + (e >> 3), a = e & 7;
                    if (i >= size_q || j >= size_p) continue;
                    const u64 hv = mulmod(powmod(2, 8 * a, p[j]), qhmodp[(size_t)i * size_p + j], p[j]);
                    const u64 z = hv + DIGIT_BIAS;
                    tab[(((size_t)t * ks + s) * 64 + l) * 16 + e] = (unsigned char)(((z >> (8 * bd)) & 0xFF) ^ 0x80);
                }
            }
    BmRed* red = reinterpret_cast<BmRed*>(tab.data() + fbytes);
    // special-prime reduction (bm_reduce<.., SPQ>) when every target allows it
    spq = OFHE_BCONV_MMA_SPQ != 0;
    for (u32 j = 0; j < size_p && spq; j++) {
        const unsigned L = msb64(p[j]);
        const u64 d = L >= 33 && L <= 60 ? (1ull << L) - p[j] : 0;
        spq = d != 0 && d < (1ull << 32) &&
              (((u128)1 << (81 - L)) + 1) * d + ((u128)1 << 49) + 2 * (u128)d < ((u128)1 << L);
    }
    for (u32 j = 0; j < size_p; j++) {
        BmRed& R = red[j];
        u64 lr[3];
        limb_red_consts(p[j], lr);
        R.p = p[j];
        R.np = 0 - p[j];
        R.r60 = lr[0];
        R.r60p = lr[1];
        R.mu1 = lr[2];
        const u128 k = (((u128)1 << 80) + p[j] - 1) / p[j];
        const u128 bias = k * p[j];  // in [2^80, 2^80 + p)
        R.bhi = (u64)(bias >> 32) - (1ull << 16);
        R.blo = (u64)(bias & 0xFFFFFFFFull) + (1ull << 48);
        R.p2 = 2 * p[j];
        if (spq) {
            const unsigned L = msb64(p[j]);
            R.r60 = (1ull << L) - p[j];                               // d
            R.r60p = (u64)(L - 32) | ((u64)((1u << (L - 32)) - 1) << 32);  // shift | mask << 32
        }
    }
    BmSrc* src = reinterpret_cast<BmSrc*>(red + 4 * tiles);
    for (u32 i = 0; i < size_q; i++) src[i] = BmSrc{q[i], qhinv[2 * i], qhinv[2 * i + 1], 0};
    return true;
}

int ofhe_hip_bconv_create(ofhe_ctx_t ctx, uint32_t log_n, uint32_t size_q, uint32_t size_p,
                          const uint64_t* q, const uint64_t* p, const uint64_t* qhat_inv_modq,
                          const uint64_t* qhat_modp, ofhe_bconv_t* out) {
    return ofhe_hip_bconv_create_ex(ctx, log_n, size_q, size_p, q, p, qhat_inv_modq, qhat_modp, nullptr, out);
}

int ofhe_hip_bconv_create_ex(ofhe_ctx_t ctx, uint32_t log_n, uint32_t size_q, uint32_t size_p,
                             const uint64_t* q, const uint64_t* p, const uint64_t* qhat_inv_modq,
                             const uint64_t* qhat_modp, const ofhe_bconv_options* options, ofhe_bconv_t* out) {
    if (!ctx || !q || !p || !qhat_inv_modq || !qhat_modp || !out) return fail(OFHE_ERR_ARG, "NULL argument");
    const ofhe_bconv_options opt = options ? *options : ofhe_bconv_options{};
    if (opt.kernel > OFHE_BCONV_KERNEL_WIDE) return fail(OFHE_ERR_ARG, "options.kernel is not an OFHE_BCONV_KERNEL_* value");
    if (opt.separate_cols > 1) return fail(OFHE_ERR_ARG, "options.separate_cols must be 0 or 1");
    if (log_n < 1 || log_n > 17) return fail(OFHE_ERR_ARG, "log_n must be in [1, 17]");
    if (size_q < 1 || size_p < 1 || size_q > 256 || size_p > 256)
        return fail(OFHE_ERR_ARG, "size_q and size_p must be in [1, 256]");
    for (u32 i = 0; i < size_q; i++)
        if (q[i] < 2 || q[i] >= (1ull << 60)) return fail(OFHE_ERR_ARG, "q out of range");
    for (u32 j = 0; j < size_p; j++)
        if (p[j] < 2 || p[j] >= (1ull << 60)) return fail(OFHE_ERR_ARG, "p out of range");
    // layout: qv[Q] | qhinv[2Q] | qhmodp[Q*P] | pv[P] | pmu[2P] | qhlimb[Q*Ppad] | pred[3P]
    const u32 ppad = (size_p + BCONV_PT - 1) / BCONV_PT * BCONV_PT;
    const u32 qrows = size_q;
    const size_t words =
        size_q + 2 * size_q + (size_t)size_q * size_p + size_p + 2 * size_p + (size_t)qrows * ppad + 3 * size_p;
    std::vector<u64> h(words);
    u64* qv = h.data();
    u64* qhinv = qv + size_q;
    u64* qhmodp = qhinv + 2 * size_q;
    u64* pv = qhmodp + (size_t)size_q * size_p;
    u64* pmu = pv + size_p;
    for (u32 i = 0; i < size_q; i++) {
        qv[i] = q[i];
        qhinv[2 * i] = qhat_inv_modq[i] % q[i];
        qhinv[2 * i + 1] = shoup_pre(qhinv[2 * i], q[i]);
    }
    u64* qhlimb = pmu + 2 * size_p;
    for (u32 i = 0; i < size_q; i++)
        for (u32 j = 0; j < size_p; j++) {
            const u64 c = qhat_modp[(size_t)i * size_p + j] % p[j];
            qhmodp[(size_t)i * size_p + j] = c;
            qhlimb[(size_t)i * ppad + j] = (c & LIMB_MASK) | ((c >> LIMB) << 32);
        }
    for (u32 j = 0; j < size_p; j++) {
        pv[j] = p[j];
        const u128 mu = (~(u128)0) / p[j];  // floor(2^128 / p), p odd
        pmu[2 * j] = (u64)mu;
        pmu[2 * j + 1] = (u64)(mu >> 64);
        limb_red_consts(p[j], pred_of(qhlimb, qrows, ppad) + 3 * j);
    }
    // the matrix-core kernel's table (bconv_mma.hpp), appended 16-byte aligned
    u32 mm_tiles = 0, mm_ks = 0, mm_tpc = 0;
    bool mm_spq = false;
    size_t mm_off = 0;
    {
        std::vector<unsigned char> tab;
        if (bconv_mma_table(size_q, size_p, q, p, qhinv, qhmodp, tab, mm_tiles, mm_ks, mm_tpc, mm_spq)) {
            mm_off = (h.size() + 1) & ~(size_t)1;
            h.resize(mm_off + tab.size() / 8);
            std::memcpy(h.data() + mm_off, tab.data(), tab.size());
        }
    }
    const size_t words_all = h.size();
    ofhe_bconv_s* b = new (std::nothrow) ofhe_bconv_s();
    if (!b) return fail(OFHE_ERR_NOMEM, "bconv allocation failed");
    b->ctx = ctx;
    b->bcols = !opt.separate_cols;
    hipError_t e = hipSetDevice(ctx->device);
    if (e == hipSuccess) e = hipMalloc(&b->d_mem, words_all * sizeof(u64));
    if (e == hipSuccess) e = upload_blocking(b->d_mem, h.data(), words_all * sizeof(u64));
    if (e != hipSuccess) {
        (void)hipFree(b->d_mem);
        delete b;
        return fail(OFHE_ERR_HIP, std::string("bconv upload: ") + hipGetErrorString(e));
    }
    BconvArgs& A = b->args;
    A.qv = b->d_mem;
    A.qhinv = A.qv + size_q;
    A.qhmodp = A.qhinv + 2 * size_q;
    A.pv = A.qhmodp + (size_t)size_q * size_p;
    A.pmu = A.pv + size_p;
    A.qhlimb = A.pmu + 2 * size_p;
    A.pred = pred_of(A.qhlimb, qrows, ppad);
    A.log_n = log_n;
    A.size_q = size_q;
    A.size_p = size_p;
    A.in_stride = (u64)size_q << log_n;
    A.out_stride = (u64)size_p << log_n;
    A.gap_at = size_p;
    A.gap = 0;
    A.mm_tab = mm_tiles ? (const void*)(b->d_mem + mm_off) : nullptr;
    A.mm_tiles = mm_tiles;
    A.mm_ks = mm_ks;
    A.mm_tpc = mm_tpc;
    A.mm_spq = mm_spq ? 1 : 0;
    A.kernel = opt.kernel;
    *out = b;
    return OFHE_OK;
}

int ofhe_hip_bconv_destroy(ofhe_bconv_t b) {
    if (!b) return fail(OFHE_ERR_ARG, "bconv is NULL");
    if (b->ctx) (void)hipSetDevice(b->ctx->device);
    (void)hipFree(b->d_mem);
    for (auto& kv : b->tabs) (void)hipFree(kv.second);
    delete b;
    return OFHE_OK;
}

namespace ofhe {
// A converter created with an explicit kernel (ofhe_bconv_options.kernel LIMB /
// WIDE) runs that kernel on every path, the fused ModUp / ModDown column
// kernel included: only OFHE_BCONV_KERNEL_AUTO may take k_bconv_cols.
bool bconv_cols_ok(ofhe_plan_t p, const BconvArgs& B) {
    return OFHE_BCONV_MMA && B.kernel == OFHE_BCONV_KERNEL_AUTO && p && p->log_n == 17 && B.log_n == 17 && p->split == SPLIT_COLS && B.mm_tab &&
           B.mm_ks >= 1 && B.mm_ks <= 4 && (B.mm_spq != 0) == p->spq;
}

int bconv_cols_run(ofhe_plan_t p, u32 t0, const BconvArgs& B, const u64* x, u64* out, u32 batch, hipStream_t s,
                   int src_t0) {
    if (!bconv_cols_ok(p, B)) return fail(OFHE_ERR_ARG, "internal: k_bconv_cols does not apply");
    if (src_t0 >= 0 && ((u32)src_t0 < t0 || (u32)src_t0 + B.size_q > p->towers))
        return fail(OFHE_ERR_ARG, "internal: k_bconv_cols sources outside the plan");
    const u32 src_rel = src_t0 >= 0 ? (u32)src_t0 - t0 : 0;
    // the last target's plan tower (after the output gap) must exist
    const u64 last = (u64)B.size_p - 1 + (B.size_p - 1 >= B.gap_at ? B.gap : 0);
    if (t0 + last >= p->towers) return fail(OFHE_ERR_ARG, "internal: k_bconv_cols targets outside the plan");
    const u64 nwg = (u64)batch * (4096 / BC_COLS);
    if (nwg >= (1ull << 31)) return fail(OFHE_ERR_ARG, "batch too large");
    const PlanArgs a = args_of(p, t0);
    switch (B.mm_ks) {
#define BCC1(K, SP, IC) \
    hipLaunchKernelGGL((k_bconv_cols<K, SP, IC>), dim3((u32)nwg), dim3(BC_THREADS), 0, s, B, a, x, out, batch, (u32)nwg, src_rel)
#define BCC(K)                                                   \
    case K:                                                      \
        if (p->spq) {                                            \
            if (src_t0 >= 0) BCC1(K, true, true); else BCC1(K, true, false); \
        } else {                                                 \
            if (src_t0 >= 0) BCC1(K, false, true); else BCC1(K, false, false); \
        }                                                        \
        break;
        BCC(1) BCC(2) BCC(3) BCC(4)
#undef BCC
#undef BCC1
        default: break;
    }
    return post_launch();
}

int bconv_run(const BconvArgs& A, const u64* x, u64* out, u32 batch, hipStream_t s) {
    const u64 total = (u64)batch << A.log_n;
    const u64 blocks = (total + 255) / 256;
    if (blocks >= (1ull << 31)) return fail(OFHE_ERR_ARG, "batch too large");
    const bool generic = A.kernel == OFHE_BCONV_KERNEL_WIDE, limb = A.kernel == OFHE_BCONV_KERNEL_LIMB;
    if (OFHE_BCONV_MMA && A.mm_tab && A.log_n >= 5 && !generic && !limb) {
        const u64 groups = total >> 5;
        const u32 wpb = BCONV_MMA_THREADS / 64;
        const u32 chunks = (A.mm_tiles + A.mm_tpc - 1) / A.mm_tpc;
        u64 gx = (groups + wpb - 1) / wpb;
        u64 cap = 256ull * BCONV_MMA_BLOCKS_PER_CU / chunks;  // about BPC resident blocks per CU in all
        if (cap < 1) cap = 1;
        if (gx > cap) gx = cap;
        const size_t lds = bconv_mma_lds(A.mm_tpc, A.mm_ks);
        const int var = (A.lazy_out ? 1 : 0) | (A.mm_spq ? 2 : 0);
        const dim3 grid((u32)gx, chunks);
        switch (A.mm_ks) {
#define BM_LAUNCH(K, LZ, SP) \
    hipLaunchKernelGGL((k_bconv_mma<K, LZ, SP>), grid, dim3(BCONV_MMA_THREADS), lds, s, A, x, out, batch)
#define BM_CASE(K)                                 \
    case K:                                        \
        if (var == 0) BM_LAUNCH(K, false, false);  \
        if (var == 1) BM_LAUNCH(K, true, false);   \
        if (var == 2) BM_LAUNCH(K, false, true);   \
        if (var == 3) BM_LAUNCH(K, true, true);    \
        break;
            BM_CASE(1) BM_CASE(2) BM_CASE(3) BM_CASE(4) BM_CASE(5) BM_CASE(6) BM_CASE(7) BM_CASE(8)
            BM_CASE(10) BM_CASE(12) BM_CASE(14) BM_CASE(16)
#undef BM_CASE
#undef BM_LAUNCH
            default:
                return fail(OFHE_ERR_STATE, "bconv: bad K-step count");
        }
        return post_launch();
    }
    if (A.size_q <= BCONV_LIMB_QMAX && !generic)
        hipLaunchKernelGGL((k_bconv_limb<BCONV_PT>), dim3((u32)blocks), dim3(256), 0, s, A, x, out, batch);
    else
        hipLaunchKernelGGL((k_bconv<8>), dim3((u32)blocks), dim3(256), 0, s, A, x, out, batch);
    return post_launch();
}
}  // namespace ofhe

int ofhe_hip_approx_switch_crt_basis(ofhe_bconv_t b, const uint64_t* x, uint64_t* out, uint32_t batch,
                                     void* stream) {
    if (!b || !b->ctx) return fail(OFHE_ERR_STATE, "bconv is NULL or destroyed");
    if (!x || !out || batch == 0) return fail(OFHE_ERR_ARG, "bad data argument");
    HIPCHK(hipSetDevice(b->ctx->device));
    return bconv_run(b->args, x, out, batch, pick(stream));
}
