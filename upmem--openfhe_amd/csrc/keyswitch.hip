// keyswitch.hip -- ApproxModUp / ApproxModDown and HYBRID key switching on
// gfx950, composed from the NTT, base-conversion and element kernels.
//
// Reference call stacks restated here (one launch per step covers the whole
// batch; the reference loops over towers with OpenMP):
//   DCRTPolyImpl::ApproxModUp    dcrtpoly-impl.h:1085-1131
//   DCRTPolyImpl::ApproxModDown  dcrtpoly-impl.h:1134-1175
//   KeySwitchHYBRID::EvalKeySwitchPrecomputeCore  keyswitch-hybrid.cpp:330-412
//   KeySwitchHYBRID::EvalFastKeySwitchCoreExt     keyswitch-hybrid.cpp:438-482
//   KeySwitchHYBRID::EvalFastKeySwitchCore        keyswitch-hybrid.cpp:414-436
// CRT tables follow CryptoParametersRNS::PrecomputeCRTTables
// (rns-cryptoparameters.cpp:72-345).  The reference builds them with
// BigInteger quotients (Q/q_i) and reductions; every table entry is a residue
// of a product of the moduli, so it is computed here as that product reduced
// modulo the target prime -- the same integer.
#include <map>
#include <new>

#include "internal.hpp"
#include "ks_kernels.hpp"

using namespace ofhe;

// A/B switches (tools/exp_ks.py): KeySwitchCore reads each digit's own towers
// from the ciphertext instead of a copy (OFHE_KS_OWN); ModUp transforms the
// Q-after-digit and P towers in one launch at full level (OFHE_KS_MERGE).
#ifndef OFHE_KS_OWN
#define OFHE_KS_OWN 1
#endif
#ifndef OFHE_KS_MERGE
#define OFHE_KS_MERGE 1
#endif
// KeySwitchCore's two ModDowns as one set of launches over 2 x batch
// (mod_down_run2) instead of two forked streams (OFHE_KS_MD2)
#ifndef OFHE_KS_MD2
#define OFHE_KS_MD2 1
#endif
// side streams the ModUp digits are spread over (digit j on stream j mod n)
#ifndef OFHE_KS_NSIDE
#define OFHE_KS_NSIDE 2
#endif
constexpr int KS_NSIDE = OFHE_KS_NSIDE;
static_assert(KS_NSIDE >= 2, "KeySwitchCore's two ModDowns use side streams 0 and 1");

namespace {

// prod_{k != skip} ms[k] mod m
u64 prod_mod(const u64* ms, u32 n, u32 skip, u64 m) {
    u64 r = 1 % m;
    for (u32 k = 0; k < n; k++)
        if (k != skip) r = mulmod(r, ms[k] % m, m);
    return r;
}

// one thread per item for the streaming kernels (grid-stride only past 2^30
// threads): a full grid keeps more bytes in flight than a capped grid-stride
// launch (ofhe_hip.hip eltwise, DESIGN.md "Element-wise bandwidth")
u32 grid_for(u64 items) {
    u64 b = (items + 255) / 256;
    if (b > (1u << 22)) b = 1u << 22;
    return (u32)(b ? b : 1);
}

TowerScalar scalar_of(u64 q, u64 s) {
    s %= q;
    return TowerScalar{q, s, shoup_pre(s, q)};
}

int scale_towers(const TowerScalar* d, const u64* x, u64* out, u64 xs, u64 os, u32 batch, u32 towers, u32 log_n,
                 hipStream_t s) {
    const u64 npairs = ((u64)batch * towers << log_n) / 2;
    hipLaunchKernelGGL(k_scale_towers, dim3(grid_for(npairs)), dim3(256), 0, s, d, x, out, xs, os, npairs, log_n,
                       towers);
    return post_launch();
}

int sub_scale(const TowerScalar* d, const u64* x, const u64* y, u64* out, u64 xs, u64 ys, u64 os, u32 batch,
              u32 towers, u32 log_n, hipStream_t s) {
    const u64 npairs = ((u64)batch * towers << log_n) / 2;
    hipLaunchKernelGGL(k_sub_scale, dim3(grid_for(npairs)), dim3(256), 0, s, d, x, y, out, xs, ys, os, npairs,
                       log_n, towers);
    return post_launch();
}

// Stream-ordered scratch from the context's pool: freed on the stream when the
// owner goes out of scope.
struct Scratch {
    void* p = nullptr;
    hipStream_t s = nullptr;
    int alloc(size_t bytes, hipStream_t st, ofhe_ctx_t ctx) {
        s = st;
        hipError_t e = ctx->pool ? hipMallocFromPoolAsync(&p, bytes ? bytes : 8, ctx->pool, st)
                                 : hipMallocAsync(&p, bytes ? bytes : 8, st);
        if (e != hipSuccess) return fail(OFHE_ERR_NOMEM, std::string("scratch: ") + hipGetErrorString(e));
        return OFHE_OK;
    }
    u64* w() const { return (u64*)p; }
    ~Scratch() {
        if (p) (void)hipFreeAsync(p, s);
    }
};

int copy_rows(u64* dst, u64 dstride, const u64* src, u64 sstride, u64 words, u32 rows, hipStream_t s) {
    if (!words || !rows) return OFHE_OK;
    HIPCHK(hipMemcpy2DAsync(dst, dstride * 8, src, sstride * 8, words * 8, rows, hipMemcpyDeviceToDevice, s));
    return OFHE_OK;
}

// ApproxModDown core shared by the generic entry point and the key-switch
// engine.  x: [batch][Q+P] (xstride), the P part at x + Q*N; plan towers
// pq0.. for Q and pp0.. for P (both in `plan_q` / `plan_p`).
struct ModDownArgs {
    ofhe_plan_t plan_q, plan_p;
    u32 q0, p0, size_q, size_p;
    BconvArgs bconv;               // P -> Q
    const TowerScalar* pinv;       // [size_q]
    const TowerScalar* tinv_p;     // [size_p] or NULL (t = 0)
    const TowerScalar* t_q;        // [size_q] or NULL
    bool bcols = false;            // k_bconv_cols for the conversion + column pass when it applies
    bool icol = false;             // ... also fed by the P part's inverse block pass (plan_p == plan_q)
};
// k_bconv_cols also runs the sources' inverse column pass (the INTT's second
// pass) when they come from the same plan and nothing scales them in between
static bool md_icol(const ModDownArgs& A) {
    return A.bcols && A.icol && !A.t_q && !A.tinv_p && A.plan_p == A.plan_q && A.plan_q->log_n == 17;
}

int mod_down_run(const ModDownArgs& A, const u64* x, u64 xstride, u64* out, u64 ostride, u32 batch, hipStream_t s) {
    const u32 log_n = A.plan_q->log_n;
    const u64 N = 1ull << log_n;
    Scratch sp, sq;
    RCCHK(sp.alloc((size_t)batch * A.size_p * N * 8, s, A.plan_q->ctx));
    RCCHK(sq.alloc((size_t)batch * A.size_q * N * 8, s, A.plan_q->ctx));
    const u64 ps = A.size_p * N, qs = A.size_q * N;
    if (md_icol(A)) {
        BconvArgs B = A.bconv;
        B.in_stride = ps;
        B.out_stride = qs;
        B.gap_at = A.size_q;
        B.gap = 0;
        B.lazy_out = 1;
        if (bconv_cols_ok(A.plan_q, B)) {
            // partP's INTT: its block pass here, its column pass inside the conversion
            RCCHK(plan_ntt_inv_block(A.plan_p, A.p0, A.size_p, x + qs, xstride, sp.w(), ps, batch, s));
            RCCHK(bconv_cols_run(A.plan_q, A.q0, B, sp.w(), sq.w(), batch, s, (int)A.p0));
            return plan_ntt_fwd_sub(A.plan_q, A.q0, A.size_q, sq.w(), qs, x, xstride, out, ostride,
                                    reinterpret_cast<const u64*>(A.pinv), batch, s, 2);
        }
    }
    // partP: P towers to coefficient form (dcrtpoly-impl.h:1147-1153)
    RCCHK(plan_ntt_range(A.plan_p, true, A.p0, A.size_p, x + qs, sp.w(), xstride, ps, batch, s));
    if (A.tinv_p) RCCHK(scale_towers(A.tinv_p, sp.w(), sp.w(), ps, ps, batch, A.size_p, log_n, s));
    // partPSwitchedToQ (1156-1157)
    BconvArgs B = A.bconv;
    B.in_stride = ps;
    B.out_stride = qs;
    B.gap_at = A.size_q;
    B.gap = 0;
    B.lazy_out = 1;  // a forward NTT (after an optional tower scale) follows
    if (A.bcols && !A.t_q && bconv_cols_ok(A.plan_q, B)) {
        // the conversion writes the Q towers' column-pass output (k_bconv_cols)
        RCCHK(bconv_cols_run(A.plan_q, A.q0, B, sp.w(), sq.w(), batch, s));
        return plan_ntt_fwd_sub(A.plan_q, A.q0, A.size_q, sq.w(), qs, x, xstride, out, ostride,
                                reinterpret_cast<const u64*>(A.pinv), batch, s, 2);
    }
    RCCHK(bconv_run(B, sp.w(), sq.w(), batch, s));
    if (A.t_q) RCCHK(scale_towers(A.t_q, sq.w(), sq.w(), qs, qs, batch, A.size_q, log_n, s));
    // SetFormat(EVALUATION), then ans_i = (x_i - switched_i) * PInvModq_i
    // (1165-1173): one transform whose block pass applies the subtraction and
    // the scalar while the values are in registers
    if (log_n >= 12)
        return plan_ntt_fwd_sub(A.plan_q, A.q0, A.size_q, sq.w(), qs, x, xstride, out, ostride,
                                reinterpret_cast<const u64*>(A.pinv), batch, s);
    RCCHK(plan_ntt_range(A.plan_q, false, A.q0, A.size_q, sq.w(), sq.w(), qs, qs, batch, s));
    return sub_scale(A.pinv, x, sq.w(), out, xstride, qs, ostride, batch, A.size_q, log_n, s);
}

// The two ApproxModDowns of KeySwitchCore in one set of launches: ct1
// follows ct0 in memory (x1 = x0 + batch * xstride), so the P-part INTT, the
// base conversion and the column pass run once over 2 * batch polynomials;
// only the block pass, which writes the caller's out0 / out1, runs twice.
int mod_down_run2(const ModDownArgs& A, const u64* x0, u64 xstride, u64* out0, u64* out1, u64 ostride, u32 batch,
                  hipStream_t s) {
    const u32 log_n = A.plan_q->log_n;
    const u64 N = 1ull << log_n;
    const u32 b2 = 2 * batch;
    Scratch sp, sq;
    RCCHK(sp.alloc((size_t)b2 * A.size_p * N * 8, s, A.plan_q->ctx));
    RCCHK(sq.alloc((size_t)b2 * A.size_q * N * 8, s, A.plan_q->ctx));
    const u64 ps = A.size_p * N, qs = A.size_q * N;
    BconvArgs B = A.bconv;
    B.in_stride = ps;
    B.out_stride = qs;
    B.gap_at = A.size_q;
    B.gap = 0;
    B.lazy_out = 1;  // a forward NTT (after an optional tower scale) follows
    const bool icol = md_icol(A) && bconv_cols_ok(A.plan_q, B);
    if (icol)  // partP's INTT: its block pass here, its column pass inside the conversion
        RCCHK(plan_ntt_inv_block(A.plan_p, A.p0, A.size_p, x0 + qs, xstride, sp.w(), ps, b2, s));
    else
        RCCHK(plan_ntt_range(A.plan_p, true, A.p0, A.size_p, x0 + qs, sp.w(), xstride, ps, b2, s));
    if (A.tinv_p) RCCHK(scale_towers(A.tinv_p, sp.w(), sp.w(), ps, ps, b2, A.size_p, log_n, s));
    const u64* x1 = x0 + (u64)batch * xstride;
    u64* sq1 = sq.w() + (u64)batch * qs;
    const u64* pinv = reinterpret_cast<const u64*>(A.pinv);
    if (A.bcols && !A.t_q && bconv_cols_ok(A.plan_q, B)) {
        // the conversion writes the Q towers' column-pass output directly
        RCCHK(bconv_cols_run(A.plan_q, A.q0, B, sp.w(), sq.w(), b2, s, icol ? (int)A.p0 : -1));
        RCCHK(plan_ntt_fwd_sub(A.plan_q, A.q0, A.size_q, sq.w(), qs, x0, xstride, out0, ostride, pinv, batch, s, 2));
        return plan_ntt_fwd_sub(A.plan_q, A.q0, A.size_q, sq1, qs, x1, xstride, out1, ostride, pinv, batch, s, 2);
    }
    RCCHK(bconv_run(B, sp.w(), sq.w(), b2, s));
    if (A.t_q) RCCHK(scale_towers(A.t_q, sq.w(), sq.w(), qs, qs, b2, A.size_q, log_n, s));
    if (log_n >= 12) {
        RCCHK(plan_ntt_fwd_sub(A.plan_q, A.q0, A.size_q, sq.w(), qs, x0, xstride, out0, ostride, pinv, b2, s, 1));
        RCCHK(plan_ntt_fwd_sub(A.plan_q, A.q0, A.size_q, sq.w(), qs, x0, xstride, out0, ostride, pinv, batch, s, 2));
        return plan_ntt_fwd_sub(A.plan_q, A.q0, A.size_q, sq1, qs, x1, xstride, out1, ostride, pinv, batch, s, 2);
    }
    RCCHK(plan_ntt_range(A.plan_q, false, A.q0, A.size_q, sq.w(), sq.w(), qs, qs, b2, s));
    RCCHK(sub_scale(A.pinv, x0, sq.w(), out0, xstride, qs, ostride, batch, A.size_q, log_n, s));
    return sub_scale(A.pinv, x1, sq1, out1, xstride, qs, ostride, batch, A.size_q, log_n, s);
}

}  // namespace

// ---------------------------------------------------------------------------
// Generic ApproxModUp / ApproxModDown
// ---------------------------------------------------------------------------
int ofhe_hip_approx_mod_up(ofhe_plan_t pq, ofhe_plan_t pp, ofhe_bconv_t bc, int eval_form, const uint64_t* x,
                           uint64_t* out, uint32_t batch, void* stream) {
    if (!pq || !pp || !bc || !pq->ctx || !pp->ctx || !bc->ctx) return fail(OFHE_ERR_STATE, "NULL or destroyed object");
    if (!x || !out || batch == 0) return fail(OFHE_ERR_ARG, "bad data argument");
    if (pq->log_n != pp->log_n || bc->args.log_n != pq->log_n) return fail(OFHE_ERR_ARG, "ring dimensions differ");
    if (bc->args.size_q != pq->towers || bc->args.size_p != pp->towers)
        return fail(OFHE_ERR_ARG, "base converter does not map plan_q's towers to plan_p's");
    HIPCHK(hipSetDevice(pq->ctx->device));
    hipStream_t s = pick(stream);
    const u64 N = 1ull << pq->log_n, Q = pq->towers, P = pp->towers, qp = (Q + P) * N;
    BconvArgs B = bc->args;
    B.out_stride = qp;
    B.lazy_out = 1;  // the P towers go through a forward NTT below
    const u64* src = x;
    B.in_stride = Q * N;
    if (eval_form) {
        // coefficient copy of x (SetFormat(COEFFICIENT), 1097-1100) into the Q slots
        RCCHK(plan_ntt_range(pq, true, 0, (u32)Q, x, out, Q * N, qp, batch, s));
        src = out;
        B.in_stride = qp;
    }
    if (bc->bcols && bconv_cols_ok(pp, B)) {
        // the conversion writes the P towers' column-pass output (k_bconv_cols),
        // the block pass finishes their forward transform (1112-1116)
        RCCHK(bconv_cols_run(pp, 0, B, src, out + Q * N, batch, s));
        RCCHK(plan_ntt_fwd_block(pp, 0, (u32)P, out + Q * N, qp, batch, s));
    } else {
        RCCHK(bconv_run(B, src, out + Q * N, batch, s));
        // P towers to evaluation form (1112-1116)
        RCCHK(plan_ntt_range(pp, false, 0, (u32)P, out + Q * N, out + Q * N, qp, qp, batch, s));
    }
    // Q towers: the stored evaluation input, or its NTT (1119-1127)
    if (eval_form) return copy_rows(out, qp, x, Q * N, Q * N, batch, s);
    return plan_ntt_range(pq, false, 0, (u32)Q, x, out, Q * N, qp, batch, s);
}

int ofhe_hip_approx_mod_down(ofhe_plan_t pq, ofhe_plan_t pp, ofhe_bconv_t bc, const uint64_t* p_inv_modq,
                             uint64_t t, const uint64_t* x, uint64_t* out, uint32_t batch, void* stream) {
    if (!pq || !pp || !bc || !pq->ctx || !pp->ctx || !bc->ctx) return fail(OFHE_ERR_STATE, "NULL or destroyed object");
    if (!x || !out || !p_inv_modq || batch == 0) return fail(OFHE_ERR_ARG, "bad data argument");
    if (pq->log_n != pp->log_n || bc->args.log_n != pq->log_n) return fail(OFHE_ERR_ARG, "ring dimensions differ");
    if (bc->args.size_q != pp->towers || bc->args.size_p != pq->towers)
        return fail(OFHE_ERR_ARG, "base converter does not map plan_p's towers to plan_q's");
    HIPCHK(hipSetDevice(pq->ctx->device));
    hipStream_t s = pick(stream);
    const u32 Q = pq->towers, P = pp->towers;
    // Tables cached per (t, P^-1 mod q) in the converter: the first call with
    // a key uploads into freshly allocated memory that no launch has read yet
    // and waits for the copy to land (upload_blocking), so the kernels below,
    // on whatever stream, read complete tables; later calls only look the
    // table up and never synchronise.
    std::vector<u64> key(p_inv_modq, p_inv_modq + Q);
    key.push_back(t);
    u64* dtab = nullptr;
    {
        std::lock_guard<std::mutex> lk(bc->tab_mu);
        auto it = bc->tabs.find(key);
        if (it != bc->tabs.end()) {
            dtab = it->second;
        } else {
            std::vector<TowerScalar> tab(Q + (t ? P + Q : 0));
            for (u32 i = 0; i < Q; i++) tab[i] = scalar_of(pq->q[i], p_inv_modq[i]);
            if (t) {
                for (u32 j = 0; j < P; j++) tab[Q + j] = scalar_of(pp->q[j], invmod(t % pp->q[j], pp->q[j]));  // tInvModp
                for (u32 i = 0; i < Q; i++) tab[Q + P + i] = scalar_of(pq->q[i], t);  // t mod q_i
            }
            const size_t words = tab.size() * 3;
            HIPCHK(hipMalloc(&dtab, words * sizeof(u64)));
            hipError_t e = upload_blocking(dtab, tab.data(), words * sizeof(u64));
            if (e != hipSuccess) {
                (void)hipFree(dtab);
                return fail(OFHE_ERR_HIP, std::string("mod-down tables: ") + hipGetErrorString(e));
            }
            bc->tabs.emplace(std::move(key), dtab);
        }
    }
    const TowerScalar* d = (const TowerScalar*)dtab;
    ModDownArgs A{pq, pp, 0, 0, Q, P, bc->args, d, t ? d + Q : nullptr, t ? d + Q + P : nullptr, bc->bcols};
    const u64 N = 1ull << pq->log_n;
    RCCHK(mod_down_run(A, x, (u64)(Q + P) * N, out, (u64)Q * N, batch, s));
    return OFHE_OK;
}

// ---------------------------------------------------------------------------
// HYBRID key switching
// ---------------------------------------------------------------------------
struct KsLevel {
    u32 size_ql = 0, beta = 0;
    std::vector<u32> start, cnt;        // digit j = towers [start, start + cnt)
    std::vector<ofhe_bconv_t> up;       // digit j -> its complement basis (Ql \ digit) | P
    ofhe_bconv_t down = nullptr;        // P -> Ql
    KsTower* d_tow = nullptr;           // [size_ql + size_p]
    TowerScalar* d_pinv = nullptr;      // [size_ql] P^-1 mod q_i
    std::map<u64, TowerScalar*> tscale; // t -> [size_p] t^-1 mod p_j, then [size_ql] t mod q_i
};

struct ofhe_ks_s {
    ofhe_ctx_t ctx = nullptr;
    u32 log_n = 0, size_q = 0, size_p = 0, num_part_q = 0, alpha = 0;
    std::vector<u64> q, p;
    ofhe_plan_t plan = nullptr;  // towers q[0..size_q) then p[0..size_p)
    hipStream_t side[KS_NSIDE] = {};  // fork streams (options.single_stream: none)
    u32 chunk = 0;                    // ciphertexts per ModUp chunk (options.chunk; 0: the whole batch)
    bool bcols = true;                // k_bconv_cols in ModUp / ModDown (options.separate_cols: off)
    bool icol = true;                 // ... with the INTT's column pass inside it (options.separate_icol: off)
    std::mutex mu;
    std::map<u32, KsLevel*> levels;
};

static void level_free(KsLevel* L) {
    if (!L) return;
    for (auto b : L->up) ofhe_hip_bconv_destroy(b);
    if (L->down) ofhe_hip_bconv_destroy(L->down);
    (void)hipFree(L->d_tow);
    (void)hipFree(L->d_pinv);
    for (auto& kv : L->tscale) (void)hipFree(kv.second);
    delete L;
}

int ofhe_hip_ks_create(ofhe_ctx_t ctx, uint32_t log_n, uint32_t size_q, const uint64_t* q, const uint64_t* psi_q,
                       uint32_t size_p, const uint64_t* p, const uint64_t* psi_p, uint32_t num_part_q,
                       ofhe_ks_t* out) {
    return ofhe_hip_ks_create_ex(ctx, log_n, size_q, q, psi_q, size_p, p, psi_p, num_part_q, nullptr, out);
}

int ofhe_hip_ks_create_ex(ofhe_ctx_t ctx, uint32_t log_n, uint32_t size_q, const uint64_t* q, const uint64_t* psi_q,
                          uint32_t size_p, const uint64_t* p, const uint64_t* psi_p, uint32_t num_part_q,
                          const ofhe_ks_options* options, ofhe_ks_t* out) {
    if (!ctx || !q || !psi_q || !p || !psi_p || !out) return fail(OFHE_ERR_ARG, "NULL argument");
    const ofhe_ks_options opt = options ? *options : ofhe_ks_options{};
    if (opt.separate_cols > 1 || opt.separate_icol > 1 || opt.single_stream > 1)
        return fail(OFHE_ERR_ARG, "options.separate_cols / separate_icol / single_stream must be 0 or 1");
    if (size_q < 1 || size_p < 1 || size_q + size_p > 256) return fail(OFHE_ERR_ARG, "size_q + size_p must be in [2, 256]");
    if (num_part_q < 1 || num_part_q > size_q) return fail(OFHE_ERR_ARG, "num_part_q must be in [1, size_q]");
    const u32 alpha = (size_q + num_part_q - 1) / num_part_q;
    // rns-cryptoparameters.cpp:75-83
    if ((int32_t)(size_q - alpha * (num_part_q - 1)) <= 0)
        return fail(OFHE_ERR_ARG, "HYBRID key switching: can't distribute " + std::to_string(size_q) + " towers into " +
                                      std::to_string(num_part_q) + " digits");
    for (u32 j = 0; j < size_p; j++)
        for (u32 i = 0; i < size_q; i++)
            if (p[j] == q[i]) return fail(OFHE_ERR_ARG, "P and Q moduli must be distinct");
    std::vector<u64> mq(q, q + size_q), mp(p, p + size_p), all(mq), roots(psi_q, psi_q + size_q);
    all.insert(all.end(), mp.begin(), mp.end());
    roots.insert(roots.end(), psi_p, psi_p + size_p);
    ofhe_plan_t plan = nullptr;
    RCCHK(ofhe_hip_plan_create_ex(ctx, log_n, size_q + size_p, all.data(), roots.data(), &opt.plan, &plan));
    ofhe_ks_s* k = new (std::nothrow) ofhe_ks_s();
    if (!k) {
        ofhe_hip_plan_destroy(plan);
        return fail(OFHE_ERR_NOMEM, "key-switch allocation failed");
    }
    k->ctx = ctx;
    k->log_n = log_n;
    k->size_q = size_q;
    k->size_p = size_p;
    k->num_part_q = num_part_q;
    k->alpha = alpha;
    k->q = mq;
    k->p = mp;
    k->plan = plan;
    k->bcols = !opt.separate_cols;
    k->icol = !opt.separate_icol;
    k->chunk = opt.chunk;
    if (!opt.single_stream) {
        hipError_t e = hipSetDevice(ctx->device);
        for (int i = 0; i < KS_NSIDE && e == hipSuccess; i++)
            e = hipStreamCreateWithFlags(&k->side[i], hipStreamNonBlocking);
        if (e != hipSuccess) {
            for (auto& st : k->side)
                if (st) (void)hipStreamDestroy(st);
            ofhe_hip_plan_destroy(plan);
            delete k;
            return fail(OFHE_ERR_HIP, std::string("key-switch streams: ") + hipGetErrorString(e));
        }
    }
    *out = k;
    return OFHE_OK;
}

int ofhe_hip_ks_destroy(ofhe_ks_t k) {
    if (!k) return fail(OFHE_ERR_ARG, "key switch is NULL");
    if (k->ctx) (void)hipSetDevice(k->ctx->device);
    (void)hipDeviceSynchronize();
    for (auto& kv : k->levels) level_free(kv.second);
    for (auto& st : k->side)
        if (st) (void)hipStreamDestroy(st);
    if (k->plan) ofhe_hip_plan_destroy(k->plan);
    delete k;
    return OFHE_OK;
}

int ofhe_hip_ks_digits(ofhe_ks_t k, uint32_t size_ql, uint32_t* alpha, uint32_t* beta) {
    if (!k || !k->ctx) return fail(OFHE_ERR_STATE, "key switch is NULL or destroyed");
    if (size_ql < 1 || size_ql > k->size_q) return fail(OFHE_ERR_ARG, "size_ql must be in [1, size_q]");
    // keyswitch-hybrid.cpp:341-345
    u32 b = (size_ql + k->alpha - 1) / k->alpha;
    if (b > k->num_part_q) b = k->num_part_q;
    if (alpha) *alpha = k->alpha;
    if (beta) *beta = b;
    return OFHE_OK;
}

// Tables of one level l = size_ql - 1 (built once, kept resident).
static int level_get(ofhe_ks_t k, u32 size_ql, KsLevel** out) {
    std::lock_guard<std::mutex> lk(k->mu);
    auto it = k->levels.find(size_ql);
    if (it != k->levels.end()) {
        *out = it->second;
        return OFHE_OK;
    }
    u32 beta = 0;
    RCCHK(ofhe_hip_ks_digits(k, size_ql, nullptr, &beta));
    KsLevel* L = new (std::nothrow) KsLevel();
    if (!L) return fail(OFHE_ERR_NOMEM, "level allocation failed");
    const u32 P = k->size_p, l = size_ql;
    L->beta = beta;
    L->size_ql = l;
    int rc = OFHE_OK;
    for (u32 j = 0; j < L->beta && rc == OFHE_OK; j++) {
        // digit j (keyswitch-hybrid.cpp:352-378) and its complement
        // (m_paramsComplPartQ, rns-cryptoparameters.cpp:238-287)
        const u32 st = j * k->alpha, n = std::min(k->alpha, l - st);
        L->start.push_back(st);
        L->cnt.push_back(n);
        const u64* dq = k->q.data() + st;
        std::vector<u64> compl_;
        for (u32 i = 0; i < l; i++)
            if (i < st || i >= st + n) compl_.push_back(k->q[i]);
        compl_.insert(compl_.end(), k->p.begin(), k->p.end());
        const u32 C = (u32)compl_.size();
        std::vector<u64> hinv(n), hmod((size_t)n * C);
        for (u32 i = 0; i < n; i++) {
            // m_PartQlHatInvModq[j][n-1][i] (rns-cryptoparameters.cpp:289-312)
            hinv[i] = invmod(prod_mod(dq, n, i, dq[i]), dq[i]);
            // m_PartQlHatModp[l][j][i][c] (314-341)
            for (u32 c = 0; c < C; c++) hmod[(size_t)i * C + c] = prod_mod(dq, n, i, compl_[c]);
        }
        ofhe_bconv_t b = nullptr;
        rc = ofhe_hip_bconv_create(k->ctx, k->log_n, n, C, dq, compl_.data(), hinv.data(), hmod.data(), &b);
        if (rc == OFHE_OK) L->up.push_back(b);
    }
    if (rc == OFHE_OK) {
        // ApproxModDown tables: PHatInvModp, PHatModq, PInvModq (172-215)
        std::vector<u64> hinv(P), hmod((size_t)P * l);
        for (u32 j = 0; j < P; j++) {
            hinv[j] = invmod(prod_mod(k->p.data(), P, j, k->p[j]), k->p[j]);
            for (u32 i = 0; i < l; i++) hmod[(size_t)j * l + i] = prod_mod(k->p.data(), P, j, k->q[i]);
        }
        rc = ofhe_hip_bconv_create(k->ctx, k->log_n, P, l, k->p.data(), k->q.data(), hinv.data(), hmod.data(),
                                   &L->down);
    }
    if (rc == OFHE_OK) {
        const u64 N = 1ull << k->log_n;
        std::vector<KsTower> tow(l + P);
        for (u32 i = 0; i < l + P; i++) {
            const bool isq = i < l;
            const u64 m = isq ? k->q[i] : k->p[i - l];
            const u128 mu = (~(u128)0) / m;
            u64 lr[3];
            limb_red_consts(m, lr);
            tow[i] = KsTower{m, (u64)mu, (u64)(mu >> 64), (isq ? i : k->size_q + i - l) * N, lr[0], lr[1], lr[2]};
        }
        std::vector<TowerScalar> pinv(l);
        for (u32 i = 0; i < l; i++)
            pinv[i] = scalar_of(k->q[i], invmod(prod_mod(k->p.data(), P, P, k->q[i]), k->q[i]));
        hipError_t e = hipSetDevice(k->ctx->device);
        if (e == hipSuccess) e = hipMalloc(&L->d_tow, sizeof(KsTower) * tow.size());
        if (e == hipSuccess) e = hipMalloc(&L->d_pinv, sizeof(TowerScalar) * pinv.size());
        if (e == hipSuccess) e = upload_blocking(L->d_tow, tow.data(), sizeof(KsTower) * tow.size());
        if (e == hipSuccess)
            e = upload_blocking(L->d_pinv, pinv.data(), sizeof(TowerScalar) * pinv.size());
        if (e != hipSuccess) rc = fail(OFHE_ERR_HIP, std::string("level upload: ") + hipGetErrorString(e));
    }
    if (rc != OFHE_OK) {
        level_free(L);
        return rc;
    }
    k->levels[size_ql] = L;
    *out = L;
    return OFHE_OK;
}

static int level_t_tables(ofhe_ks_t k, KsLevel* L, u64 t, const TowerScalar** out) {
    std::lock_guard<std::mutex> lk(k->mu);
    auto it = L->tscale.find(t);
    if (it != L->tscale.end()) {
        *out = it->second;
        return OFHE_OK;
    }
    const u32 P = k->size_p, l = L->size_ql;
    std::vector<TowerScalar> tab(P + l);
    for (u32 j = 0; j < P; j++) tab[j] = scalar_of(k->p[j], invmod(t % k->p[j], k->p[j]));
    for (u32 i = 0; i < l; i++) tab[P + i] = scalar_of(k->q[i], t);
    TowerScalar* d = nullptr;
    HIPCHK(hipMalloc(&d, sizeof(TowerScalar) * tab.size()));
    hipError_t e = upload_blocking(d, tab.data(), sizeof(TowerScalar) * tab.size());
    if (e != hipSuccess) {
        (void)hipFree(d);
        return fail(OFHE_ERR_HIP, std::string("t tables: ") + hipGetErrorString(e));
    }
    L->tscale[t] = d;
    *out = d;
    return OFHE_OK;
}

// Fork of the caller's stream onto the engine's two side streams, so that
// independent digits (ModUp) and the two ModDowns overlap: each alone is a
// sequence of short launches over a few towers that leaves the chip partly
// idle at its head and tail.  The join (explicit, or in the destructor on an
// error path) puts the caller's stream behind both; declare a KsFork after
// any stream-ordered Scratch its work uses, so it joins before they are freed.
struct KsFork {
    hipStream_t parent = nullptr;
    hipStream_t f[KS_NSIDE] = {};
    hipEvent_t ev[KS_NSIDE + 1] = {};
    bool forked = false;
    int open(ofhe_ks_t k, hipStream_t s) {
        parent = s;
        for (auto& x : f) x = s;
        if (!k->side[0]) return OFHE_OK;
        for (auto& e : ev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        HIPCHK(hipEventRecord(ev[0], s));
        for (int i = 0; i < KS_NSIDE; i++) HIPCHK(hipStreamWaitEvent(k->side[i], ev[0], 0));
        for (int i = 0; i < KS_NSIDE; i++) f[i] = k->side[i];
        forked = true;
        return OFHE_OK;
    }
    int join() {
        if (!forked) return OFHE_OK;
        forked = false;
        for (int i = 0; i < KS_NSIDE; i++) {
            HIPCHK(hipEventRecord(ev[1 + i], f[i]));
            HIPCHK(hipStreamWaitEvent(parent, ev[1 + i], 0));
        }
        return OFHE_OK;
    }
    ~KsFork() {
        (void)join();
        for (auto& e : ev)
            if (e) (void)hipEventDestroy(e);
    }
};

static int ks_check(ofhe_ks_t k, u32 size_ql, u32 batch) {
    if (!k || !k->ctx) return fail(OFHE_ERR_STATE, "key switch is NULL or destroyed");
    if (size_ql < 1 || size_ql > k->size_q) return fail(OFHE_ERR_ARG, "size_ql must be in [1, size_q]");
    if (batch == 0) return fail(OFHE_ERR_ARG, "batch must be >= 1");
    HIPCHK(hipSetDevice(k->ctx->device));
    return OFHE_OK;
}

// EvalKeySwitchPrecomputeCore; with own_copy = false the digit's own towers
// are left out of its slot (KeySwitchCore's inner product reads them from c).
static int ks_precompute_impl(ofhe_ks_t k, KsLevel* L, uint32_t size_ql, const uint64_t* c, uint64_t* digits,
                              uint32_t batch, hipStream_t stream, bool own_copy) {
    KsFork fk;
    RCCHK(fk.open(k, stream));
    const u64 N = 1ull << k->log_n, l = size_ql, P = k->size_p, poly = (l + P) * N, ds = L->beta * poly;
    // ModUp in chunks of ciphertexts (OFHE_KS_CHUNK), so that a chunk's
    // converted towers can still sit in the Infinity Cache when its forward
    // transform reads them
    const u32 cb = k->chunk && k->chunk < batch ? k->chunk : batch;
    for (u32 b0 = 0; b0 < batch; b0 += cb)
    for (u32 j = 0; j < L->beta; j++) {
        const u32 st = L->start[j], n = L->cnt[j];
        const u32 batch_ = std::min(cb, batch - b0);
        hipStream_t s = fk.f[j % KS_NSIDE];  // digits are independent
        u64* slot = digits + (u64)b0 * ds + j * poly;
        const uint64_t* c_ = c + (u64)b0 * l * N;
        // ApproxSwitchCRTBasis to the complement, written around the digit slot (388-406)
        BconvArgs B = L->up[j]->args;
        B.in_stride = B.out_stride = ds;
        B.gap_at = st;
        B.gap = n;
        B.lazy_out = 1;  // every complement tower goes through a forward NTT below
        const bool cols = k->bcols && l == k->size_q && bconv_cols_ok(k->plan, B);
        // partsCt[j] in coefficient form (keyswitch-hybrid.cpp:384-385); with
        // k->icol only its block pass here, its column pass inside the conversion
        if (cols && k->icol)
            RCCHK(plan_ntt_inv_block(k->plan, st, n, c_ + st * N, l * N, slot + st * N, ds, batch_, s));
        else
            RCCHK(plan_ntt_range(k->plan, true, st, n, c_ + st * N, slot + st * N, l * N, ds, batch_, s));
        if (cols) {
            // full level (slot towers = plan towers): the conversion writes the
            // complement's column-pass output, the block passes finish it (394)
            RCCHK(bconv_cols_run(k->plan, 0, B, slot + st * N, slot, batch_, s, k->icol ? (int)st : -1));
            if (st) RCCHK(plan_ntt_fwd_block(k->plan, 0, st, slot, ds, batch_, s));
            RCCHK(plan_ntt_fwd_block(k->plan, st + n, (u32)(l + P) - st - n, slot + (st + n) * N, ds, batch_, s));
            if (own_copy) RCCHK(copy_rows(slot + st * N, ds, c_ + st * N, l * N, (u64)n * N, batch_, s));
            continue;
        }
        RCCHK(bconv_run(B, slot + st * N, slot, batch_, s));
        // complement towers to evaluation form (394)
        RCCHK(plan_ntt_range(k->plan, false, 0, st, slot, slot, ds, ds, batch_, s));
        if (OFHE_KS_MERGE && l == k->size_q) {
            // full level: the Q towers after the digit and the P towers are
            // adjacent both in the plan and in the slot -- one launch
            RCCHK(plan_ntt_range(k->plan, false, st + n, (u32)(l + P) - st - n, slot + (st + n) * N,
                                 slot + (st + n) * N, ds, ds, batch_, s));
        } else {
            RCCHK(plan_ntt_range(k->plan, false, st + n, (u32)l - st - n, slot + (st + n) * N, slot + (st + n) * N,
                                 ds, ds, batch_, s));
            RCCHK(plan_ntt_range(k->plan, false, k->size_q, (u32)P, slot + l * N, slot + l * N, ds, ds, batch_, s));
        }
        // the digit's own towers stay as given (evaluation form, 402-404)
        if (own_copy) RCCHK(copy_rows(slot + st * N, ds, c_ + st * N, l * N, (u64)n * N, batch_, s));
    }
    return fk.join();
}

int ofhe_hip_ks_precompute(ofhe_ks_t k, uint32_t size_ql, const uint64_t* c, uint64_t* digits, uint32_t batch,
                           void* stream) {
    RCCHK(ks_check(k, size_ql, batch));
    if (!c || !digits) return fail(OFHE_ERR_ARG, "NULL data pointer");
    KsLevel* L = nullptr;
    RCCHK(level_get(k, size_ql, &L));
    return ks_precompute_impl(k, L, size_ql, c, digits, batch, pick(stream), true);
}

// EvalFastKeySwitchCoreExt; c != NULL: the digits' own towers come from c
// (see ks_precompute_impl), which only the batch-stationary kernel supports.
static int ks_fast_core_ext_impl(ofhe_ks_t k, KsLevel* L, uint32_t size_ql, const uint64_t* digits,
                                 const uint64_t* key_b, const uint64_t* key_a, uint64_t* ct0, uint64_t* ct1,
                                 uint32_t batch, void* stream, const uint64_t* c) {
    const u32 towers = size_ql + k->size_p;
    const u64 key_stride = (u64)(k->size_q + k->size_p) << k->log_n;
    if (L->beta <= 4) {
        // batch-stationary keys: one thread per (tower, OFHE_KS_CPT coefficients)
        const u64 rows = ((u64)towers << k->log_n) / OFHE_KS_CPT;
        const dim3 g((u32)((rows + 255) / 256)), blk(256);
        hipStream_t s = pick(stream);
        KsOwn own{};
        for (u32 j = 0; j < L->beta; j++) {
            own.start[j] = L->start[j];
            own.cnt[j] = L->cnt[j];
        }
        const u64 c_stride = (u64)size_ql << k->log_n;
#define OFHE_KS_BS(B_)                                                                                      \
    hipLaunchKernelGGL((k_ks_inner_bs<B_, OFHE_KS_CPT>), g, blk, 0, s, L->d_tow, digits, key_b, key_a, ct0, ct1, \
                       key_stride, batch, rows, k->log_n, towers, c, c_stride, own)
        switch (L->beta) {
            case 1: OFHE_KS_BS(1); break;
            case 2: OFHE_KS_BS(2); break;
            case 3: OFHE_KS_BS(3); break;
            default: OFHE_KS_BS(4); break;
        }
#undef OFHE_KS_BS
    } else {
        if (c) return fail(OFHE_ERR_STATE, "internal: own-tower reads need beta <= 4");
        const u64 npairs = ((u64)batch * towers << k->log_n) / 2;
        hipLaunchKernelGGL(k_ks_inner, dim3(grid_for(npairs)), dim3(256), 0, pick(stream), L->d_tow, digits, key_b,
                           key_a, ct0, ct1, key_stride, L->beta, npairs, k->log_n, towers);
    }
    return post_launch();
}

int ofhe_hip_ks_fast_core_ext(ofhe_ks_t k, uint32_t size_ql, const uint64_t* digits, const uint64_t* key_b,
                              const uint64_t* key_a, uint64_t* ct0, uint64_t* ct1, uint32_t batch, void* stream) {
    RCCHK(ks_check(k, size_ql, batch));
    if (!digits || !key_b || !key_a || !ct0 || !ct1) return fail(OFHE_ERR_ARG, "NULL data pointer");
    KsLevel* L = nullptr;
    RCCHK(level_get(k, size_ql, &L));
    return ks_fast_core_ext_impl(k, L, size_ql, digits, key_b, key_a, ct0, ct1, batch, stream, nullptr);
}

static int ks_mod_down_impl(ofhe_ks_t k, KsLevel* L, const u64* x, u64* out, u64 t, u32 batch, hipStream_t s) {
    const TowerScalar* tt = nullptr;
    if (t) RCCHK(level_t_tables(k, L, t, &tt));
    const u32 l = L->size_ql, P = k->size_p;
    ModDownArgs A{k->plan, k->plan, 0, k->size_q, l, P, L->down->args, L->d_pinv,
                  tt ? tt : nullptr, tt ? tt + P : nullptr, k->bcols, k->icol};
    const u64 N = 1ull << k->log_n;
    return mod_down_run(A, x, (u64)(l + P) * N, out, (u64)l * N, batch, s);
}

int ofhe_hip_ks_mod_down(ofhe_ks_t k, uint32_t size_ql, const uint64_t* x, uint64_t* out, uint64_t t, uint32_t batch,
                         void* stream) {
    RCCHK(ks_check(k, size_ql, batch));
    if (!x || !out) return fail(OFHE_ERR_ARG, "NULL data pointer");
    KsLevel* L = nullptr;
    RCCHK(level_get(k, size_ql, &L));
    return ks_mod_down_impl(k, L, x, out, t, batch, pick(stream));
}

int ofhe_hip_ks_core(ofhe_ks_t k, uint32_t size_ql, const uint64_t* c, const uint64_t* key_b, const uint64_t* key_a,
                     uint64_t* out0, uint64_t* out1, uint64_t t, uint32_t batch, void* stream) {
    RCCHK(ks_check(k, size_ql, batch));
    if (!c || !key_b || !key_a || !out0 || !out1) return fail(OFHE_ERR_ARG, "NULL data pointer");
    KsLevel* L = nullptr;
    RCCHK(level_get(k, size_ql, &L));
    hipStream_t s = pick(stream);
    const u64 N = 1ull << k->log_n, poly = (u64)(size_ql + k->size_p) * N;
    Scratch dg, ct;
    RCCHK(dg.alloc((size_t)batch * L->beta * poly * 8, s, k->ctx));
    RCCHK(ct.alloc((size_t)2 * batch * poly * 8, s, k->ctx));
    u64* c0 = ct.w();
    u64* c1 = ct.w() + (u64)batch * poly;
    // the inner product reads each digit's own towers straight from c (beta <= 4),
    // so the precompute skips copying them into the digit slots
    const bool own_from_c = OFHE_KS_OWN && L->beta <= 4;
    RCCHK(ks_precompute_impl(k, L, size_ql, c, dg.w(), batch, s, !own_from_c));
    RCCHK(ks_fast_core_ext_impl(k, L, size_ql, dg.w(), key_b, key_a, c0, c1, batch, s, own_from_c ? c : nullptr));
    if (OFHE_KS_MD2) {
        // both ModDowns in one set of launches (c1 = c0 + batch * poly)
        const TowerScalar* tt = nullptr;
        if (t) RCCHK(level_t_tables(k, L, t, &tt));
        const u32 l = L->size_ql, P = k->size_p;
        ModDownArgs A{k->plan, k->plan, 0, k->size_q, l, P, L->down->args, L->d_pinv,
                      tt ? tt : nullptr, tt ? tt + P : nullptr, k->bcols, k->icol};
        return mod_down_run2(A, c0, poly, out0, out1, (u64)l * N, batch, s);
    }
    KsFork fk;  // after dg, ct: joins before they are freed
    RCCHK(fk.open(k, s));
    RCCHK(ks_mod_down_impl(k, L, c0, out0, t, batch, fk.f[0]));
    RCCHK(ks_mod_down_impl(k, L, c1, out1, t, batch, fk.f[1]));
    return fk.join();
}

// ---------------------------------------------------------------------------
// Element maps
// ---------------------------------------------------------------------------
int ofhe_hip_switch_modulus(ofhe_ctx_t ctx, const uint64_t* src, uint64_t* dst, uint64_t n, uint64_t old_q,
                            uint64_t new_q, void* stream) {
    if (!ctx || ((!src || !dst) && n)) return fail(OFHE_ERR_ARG, "NULL argument");
    if (old_q < 2 || new_q < 2) return fail(OFHE_ERR_ARG, "moduli must be >= 2");
    if (!n) return OFHE_OK;
    HIPCHK(hipSetDevice(ctx->device));
    hipLaunchKernelGGL(k_switch_modulus, dim3(grid_for(n)), dim3(256), 0, pick(stream), src, dst, (u64)n, (u64)old_q,
                       (u64)new_q);
    return post_launch();
}

int ofhe_hip_automorphism(ofhe_plan_t p, uint32_t k, int eval_form, const uint64_t* src, uint64_t* dst,
                          uint32_t batch, void* stream) {
    if (!p || !p->ctx) return fail(OFHE_ERR_STATE, "plan is NULL or destroyed");
    if (!src || !dst || batch == 0) return fail(OFHE_ERR_ARG, "bad data argument");
    if (src == dst) return fail(OFHE_ERR_ARG, "automorphism is out of place (dst must not alias src)");
    if (k % 2 == 0) return fail(OFHE_ERR_ARG, "Automorphism index not odd");  // poly-impl.h:333-334
    HIPCHK(hipSetDevice(p->ctx->device));
    const u64 total = (u64)batch * p->towers << p->log_n;
    if (eval_form)
        hipLaunchKernelGGL(k_automorphism<true>, dim3(grid_for(total)), dim3(256), 0, pick(stream), p->d_tc, src, dst,
                           k, total, p->log_n, p->towers);
    else
        hipLaunchKernelGGL(k_automorphism<false>, dim3(grid_for(total)), dim3(256), 0, pick(stream), p->d_tc, src,
                           dst, k, total, p->log_n, p->towers);
    return post_launch();
}

// ---------------------------------------------------------------------------
// Rescaling on the device: DCRTPolyImpl::DropLastElementAndScale (CKKS / BFV,
// dcrtpoly-impl.h:746-768) and DCRTPolyImpl::ModReduce (BGV, 792-812), the
// callers that take the path's INTT -> SwitchModulus -> NTT steps one tower
// down.  Evaluation form runs INTT(last tower) -> k_switch_scale<SW_SCALE> ->
// the fused forward-subtract block pass, using
//   x a + NTT(sw c) = (x - NTT(sw (-c a^-1))) a      (rescale, a = qlInvModq_i)
//   (x + NTT(sw t)) a = (x - NTT(sw (-t))) a           (mod-reduce)
// with the canonical residues of the reference's own order of operations.
// ---------------------------------------------------------------------------
#ifndef OFHE_RESCALE_FUSE
#define OFHE_RESCALE_FUSE 1  // 0: k_switch_scale then the column pass (A/B)
#endif
static int plan_table(ofhe_plan_t p, const std::vector<u64>& words, const u64** out) {
    std::lock_guard<std::mutex> lk(p->tab_mu);
    auto it = p->tabs.find(words);
    if (it != p->tabs.end()) {
        *out = it->second;
        return OFHE_OK;
    }
    u64* d = nullptr;
    HIPCHK(hipMalloc(&d, words.size() * sizeof(u64)));
    hipError_t e = upload_blocking(d, words.data(), words.size() * sizeof(u64));
    if (e != hipSuccess) {
        (void)hipFree(d);
        return fail(OFHE_ERR_HIP, std::string("rescale tables: ") + hipGetErrorString(e));
    }
    p->tabs.emplace(words, d);
    *out = d;
    return OFHE_OK;
}

static int rescale_check(ofhe_plan_t p, u32 towers, const u64* x, u64 xs, const u64* out, u64 os, u32 batch) {
    if (!p || !p->ctx) return fail(OFHE_ERR_STATE, "plan is NULL or destroyed");
    if (!x || !out || batch == 0) return fail(OFHE_ERR_ARG, "bad data argument");
    // dcrtpoly-impl.h:720-723 (DropLastElement)
    if (towers < 2) return fail(OFHE_ERR_ARG, "Removing last element of DCRTPoly object renders it invalid!");
    if (towers > p->towers) return fail(OFHE_ERR_ARG, "towers exceeds the plan");
    const u64 N = 1ull << p->log_n;
    if (xs < towers * N || os < (towers - 1) * N) return fail(OFHE_ERR_ARG, "batch stride smaller than the towers");
    if (((xs | os) & 1) || (((uintptr_t)x | (uintptr_t)out) & 15))
        return fail(OFHE_ERR_ARG, "strides must be even and buffers 16-byte aligned");
    // In place only with equal strides: every launch then reads and writes a
    // word at the same address from the same thread.  With a packed output
    // (out_stride = (towers-1)N < x_stride) entry b's output would overwrite
    // towers of entry b-1's input that other workgroups still read.
    const u64 x_end = (u64)(uintptr_t)x + 8 * ((u64)(batch - 1) * xs + (u64)towers * N);
    const u64 o_end = (u64)(uintptr_t)out + 8 * ((u64)(batch - 1) * os + (u64)(towers - 1) * N);
    const bool overlap = (u64)(uintptr_t)x < o_end && (u64)(uintptr_t)out < x_end;
    if (overlap && !((const u64*)x == out && xs == os))
        return fail(OFHE_ERR_ARG, "out overlaps x: in place needs out == x and out_stride == x_stride");
    return OFHE_OK;
}

// shared tail: sw[6 L] for k_switch_scale, sc[3 L] (q, a, a') for the
// forward-subtract (evaluation form)
static int rescale_run(ofhe_plan_t p, u32 towers, const u64* x, u64 xs, u64* out, u64 os, bool eval, int mode,
                       const std::vector<u64>& sw, const std::vector<u64>& sc, u64 pre, u32 batch, hipStream_t s) {
    HIPCHK(hipSetDevice(p->ctx->device));
    const u32 L = towers - 1, log_n = p->log_n;
    const u64 N = 1ull << log_n;
    const u64 *dsw = nullptr, *dsc = nullptr;
    RCCHK(plan_table(p, sw, &dsw));
    if (eval) RCCHK(plan_table(p, sc, &dsc));
    const u64 ql = p->q[L];
    SwArgs A{};
    A.tab = dsw;
    A.ql = ql;
    A.pre = pre % ql;
    A.pre_p = shoup_pre(A.pre, ql);
    if (A.pre == 1) A.pre_p = 0;
    A.log_n = log_n;
    A.towers = L;
    const u32 bpr = (u32)((N / 2 + 255) / 256);  // two coefficients per thread
    const u64 blocks = (u64)bpr * batch * L;
    if (blocks >= (1ull << 31)) return fail(OFHE_ERR_ARG, "batch too large for one launch");
    if (!eval) {
        A.last = x + (u64)L * N;
        A.lstride = xs;
        A.x = x;
        A.xstride = xs;
        A.y = out;
        A.ystride = os;
        if (mode == SW_AXPY)
            hipLaunchKernelGGL(k_switch_scale<SW_AXPY>, dim3((u32)blocks), dim3(256), 0, s, A, bpr);
        else
            hipLaunchKernelGGL(k_switch_scale<SW_XPYA>, dim3((u32)blocks), dim3(256), 0, s, A, bpr);
        RCCHK(post_launch());
        // DropLastElementAndScale switches the coefficient-form towers to
        // evaluation form (dcrtpoly-impl.h:765-766); ModReduce does not
        if (mode == SW_AXPY) return plan_ntt_range(p, false, 0, L, out, out, os, os, batch, s);
        return OFHE_OK;
    }
    Scratch sl, sy;
    RCCHK(sl.alloc((size_t)batch * N * 8, s, p->ctx));
    RCCHK(sy.alloc((size_t)batch * L * N * 8, s, p->ctx));
    RCCHK(plan_ntt_range(p, true, L, 1, x + (u64)L * N, sl.w(), xs, N, batch, s));
    const u64 ys = (u64)L * N;
    if (log_n > 12 && p->split != SPLIT_T9 && OFHE_RESCALE_FUSE) {
        // the lift happens in the column pass's loads (k_cols<.., SWS>): the
        // switched towers are never written to HBM before their transform
        RCCHK(plan_cols_switch(p, 0, L, sl.w(), N, ql, A.pre, dsw, sy.w(), ys, batch, s));
        return plan_ntt_fwd_sub(p, 0, L, sy.w(), ys, x, xs, out, os, dsc, batch, s, 2);
    }
    A.last = sl.w();
    A.lstride = N;
    A.y = sy.w();
    A.ystride = ys;
    hipLaunchKernelGGL(k_switch_scale<SW_SCALE>, dim3((u32)blocks), dim3(256), 0, s, A, bpr);
    RCCHK(post_launch());
    if (log_n >= 12) return plan_ntt_fwd_sub(p, 0, L, sy.w(), ys, x, xs, out, os, dsc, batch, s);
    RCCHK(plan_ntt_range(p, false, 0, L, sy.w(), sy.w(), ys, ys, batch, s));
    return sub_scale(reinterpret_cast<const TowerScalar*>(dsc), x, sy.w(), out, xs, ys, os, batch, L, log_n, s);
}

int ofhe_hip_drop_last_and_scale(ofhe_plan_t p, uint32_t towers, const uint64_t* x, uint64_t x_stride,
                                 uint64_t* out, uint64_t out_stride, int eval_form,
                                 const uint64_t* ql_ql_inv_modql_divql_modq, const uint64_t* ql_inv_modq,
                                 uint32_t batch, void* stream) {
    RCCHK(rescale_check(p, towers, x, x_stride, out, out_stride, batch));
    if (!ql_ql_inv_modql_divql_modq || !ql_inv_modq) return fail(OFHE_ERR_ARG, "NULL constants");
    const u32 L = towers - 1;
    std::vector<u64> sw(6 * (size_t)L, 0), sc(3 * (size_t)L, 0);
    for (u32 i = 0; i < L; i++) {
        const u64 q = p->q[i], c = ql_ql_inv_modql_divql_modq[i] % q, a = ql_inv_modq[i] % q;
        if (eval_form) {
            if (a == 0) return fail(OFHE_ERR_ARG, "ql_inv_modq[" + std::to_string(i) + "] is not invertible mod q_i");
            const u64 w = (q - mulmod(c, invmod(a, q), q)) % q;
            const TowerScalar W = scalar_of(q, w), S = scalar_of(q, a);
            sw[6 * i] = q, sw[6 * i + 1] = W.s, sw[6 * i + 2] = W.sp;
            sc[3 * i] = q, sc[3 * i + 1] = S.s, sc[3 * i + 2] = S.sp;
        } else {
            const TowerScalar W = scalar_of(q, c), S = scalar_of(q, a);
            sw[6 * i] = q, sw[6 * i + 1] = W.s, sw[6 * i + 2] = W.sp, sw[6 * i + 3] = S.s, sw[6 * i + 4] = S.sp;
        }
    }
    return rescale_run(p, towers, x, x_stride, out, out_stride, eval_form != 0, SW_AXPY, sw, sc, 1, batch,
                       pick(stream));
}

int ofhe_hip_mod_reduce(ofhe_plan_t p, uint32_t towers, const uint64_t* x, uint64_t x_stride, uint64_t* out,
                        uint64_t out_stride, int eval_form, uint64_t t, uint64_t neg_t_inv_modq,
                        const uint64_t* ql_inv_modq, uint32_t batch, void* stream) {
    RCCHK(rescale_check(p, towers, x, x_stride, out, out_stride, batch));
    if (!ql_inv_modq) return fail(OFHE_ERR_ARG, "NULL constants");
    const u32 L = towers - 1;
    std::vector<u64> sw(6 * (size_t)L, 0), sc(3 * (size_t)L, 0);
    for (u32 i = 0; i < L; i++) {
        const u64 q = p->q[i], tq = t % q, a = ql_inv_modq[i] % q;
        const TowerScalar W = scalar_of(q, eval_form ? (q - tq) % q : tq), S = scalar_of(q, a);
        sw[6 * i] = q, sw[6 * i + 1] = W.s, sw[6 * i + 2] = W.sp, sw[6 * i + 3] = S.s, sw[6 * i + 4] = S.sp;
        sc[3 * i] = q, sc[3 * i + 1] = S.s, sc[3 * i + 2] = S.sp;
    }
    return rescale_run(p, towers, x, x_stride, out, out_stride, eval_form != 0, SW_XPYA, sw, sc, neg_t_inv_modq,
                       batch, pick(stream));
}

// ---------------------------------------------------------------------------
// BV key switching with digitSize = 0 (KeySwitchBV, keyswitch-bv.cpp:302-340):
// digit i of c is CRTDecompose(0)'s tower-i polynomial (dcrtpoly-impl.h:
// 266-288): c_i in coefficient form lifted into every tower (SwitchModulus)
// and transformed -- the fused lift + forward NTT of the rescaling path, one
// launch pair per digit -- then the key inner product (k_bv_inner).
// ---------------------------------------------------------------------------
int ofhe_hip_bv_precompute(ofhe_plan_t p, uint32_t towers, const uint64_t* c, uint64_t* digits, uint32_t batch,
                           void* stream) {
    if (!p || !p->ctx) return fail(OFHE_ERR_STATE, "plan is NULL or destroyed");
    if (!c || !digits || batch == 0) return fail(OFHE_ERR_ARG, "bad data argument");
    if (towers < 1 || towers > p->towers) return fail(OFHE_ERR_ARG, "towers must be in [1, plan towers]");
    if ((((uintptr_t)c | (uintptr_t)digits) & 15)) return fail(OFHE_ERR_ARG, "buffers must be 16-byte aligned");
    HIPCHK(hipSetDevice(p->ctx->device));
    hipStream_t s = pick(stream);
    const u32 T = towers, log_n = p->log_n;
    const u64 N = 1ull << log_n, TN = (u64)T * N;
    std::vector<u64> sw(6 * (size_t)T, 0);
    for (u32 k = 0; k < T; k++) {
        const TowerScalar W = scalar_of(p->q[k], 1);
        sw[6 * k] = p->q[k], sw[6 * k + 1] = W.s, sw[6 * k + 2] = W.sp;
    }
    const u64* dsw = nullptr;
    RCCHK(plan_table(p, sw, &dsw));
    Scratch sc;  // c in coefficient form
    RCCHK(sc.alloc((size_t)batch * TN * 8, s, p->ctx));
    RCCHK(plan_ntt_range(p, true, 0, T, c, sc.w(), TN, TN, batch, s));
    const u64 dstride = (u64)T * TN;  // words per batch entry of digits
    const bool fused = log_n > 12 && p->split != SPLIT_T9 && OFHE_RESCALE_FUSE;
    const u32 bpr = (u32)((N / 2 + 255) / 256);
    if ((u64)bpr * batch * T >= (1ull << 31)) return fail(OFHE_ERR_ARG, "batch too large for one launch");
    for (u32 i = 0; i < T; i++) {
        u64* di = digits + (u64)i * TN;
        if (fused) {
            RCCHK(plan_cols_switch(p, 0, T, sc.w() + (u64)i * N, TN, p->q[i], 1, dsw, di, dstride, batch, s));
            RCCHK(plan_ntt_fwd_block(p, 0, T, di, dstride, batch, s));
            continue;
        }
        SwArgs A{};
        A.last = sc.w() + (u64)i * N;
        A.lstride = TN;
        A.y = di;
        A.ystride = dstride;
        A.tab = dsw;
        A.ql = p->q[i];
        A.pre = 1;
        A.log_n = log_n;
        A.towers = T;
        hipLaunchKernelGGL(k_switch_scale<SW_SCALE>, dim3(bpr * batch * T), dim3(256), 0, s, A, bpr);
        RCCHK(post_launch());
        RCCHK(plan_ntt_range(p, false, 0, T, di, di, dstride, dstride, batch, s));
    }
    return OFHE_OK;
}

int ofhe_hip_bv_core(ofhe_plan_t p, uint32_t towers, const uint64_t* digits, const uint64_t* key_b,
                     const uint64_t* key_a, uint32_t key_towers, uint64_t* out0, uint64_t* out1, uint32_t batch,
                     void* stream) {
    if (!p || !p->ctx) return fail(OFHE_ERR_STATE, "plan is NULL or destroyed");
    if (!digits || !key_b || !key_a || !out0 || !out1 || batch == 0) return fail(OFHE_ERR_ARG, "bad data argument");
    if (towers < 1 || towers > p->towers) return fail(OFHE_ERR_ARG, "towers must be in [1, plan towers]");
    if (key_towers < towers) return fail(OFHE_ERR_ARG, "key_towers smaller than towers");
    if (towers > 256) return fail(OFHE_ERR_ARG, "at most 256 digits (128-bit accumulation)");
    HIPCHK(hipSetDevice(p->ctx->device));
    std::vector<u64> mu(3 * (size_t)towers);
    for (u32 t = 0; t < towers; t++) {
        const u128 m = ~(u128)0 / p->q[t];  // floor((2^128 - 1) / q) = floor(2^128 / q) for q not a power of two
        mu[3 * t] = p->q[t], mu[3 * t + 1] = (u64)m, mu[3 * t + 2] = (u64)(m >> 64);
    }
    const u64* dmu = nullptr;
    RCCHK(plan_table(p, mu, &dmu));
    BvArgs A{digits, key_b, key_a, out0, out1, dmu, towers, towers, key_towers, p->log_n};
    const u64 N = 1ull << p->log_n;
    const u32 bpr = (u32)((N + 255) / 256);
    const u64 blocks = (u64)bpr * batch * towers;
    if (blocks >= (1ull << 31)) return fail(OFHE_ERR_ARG, "batch too large for one launch");
    hipLaunchKernelGGL(k_bv_inner, dim3((u32)blocks), dim3(256), 0, pick(stream), A, bpr);
    return post_launch();
}
