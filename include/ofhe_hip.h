/*
 * ofhe_hip.h -- C ABI of the MI355X (gfx950) RNS polynomial backend.
 *
 * This is the drop-in boundary that replaces the UPMEM interception layer of
 * MpokiAbel/UPMEM--OpenFHE (src/core/include/pim/PimManager.h,
 * src/core/include/pim/PimData.h, src/core/pim/host/PimManager.cpp) and the
 * CPU hot loops it was meant to offload:
 *   - ChineseRemainderTransformFTTNat forward / inverse NTT
 *       (src/core/include/math/hal/intnat/transformnat-impl.h:575-705),
 *   - NativeVectorT element-wise ModMul/ModAdd/ModSub
 *       (src/core/include/math/hal/intnat/mubintvecnat.h:426-432,501-513;
 *        src/core/lib/math/hal/intnat/mubintvecnat.cpp:245-367),
 *   - DCRTPolyImpl::ApproxSwitchCRTBasis / ApproxModUp / ApproxModDown
 *       (src/core/include/lattice/hal/default/dcrtpoly-impl.h:1034-1175),
 *   - the HYBRID key-switching core built on them
 *       (src/pke/lib/keyswitch/keyswitch-hybrid.cpp:325-482),
 *   - NativeVectorT::SwitchModulus and PolyImpl::AutomorphismTransform
 *       (mubintvecnat.cpp:111-136, poly-impl.h:312-365).
 *
 * Conventions
 *   - Plain C, no exceptions cross the ABI. Every entry point returns an int
 *     status (OFHE_OK = 0); ofhe_hip_last_error() gives a thread-local message.
 *     The C++ adapter (upmem--openfhe_amd/host/ofhe_dcrt.hpp) turns non-zero
 *     into lbcrypto-style math_error exceptions, as OPENFHE_THROW does.
 *   - Polynomial data is uint64_t residues laid out [batch][tower][N],
 *     contiguous, in DEVICE memory, unless a function says otherwise.
 *     Inputs must be canonical residues in [0, q_t); outputs are canonical.
 *   - `stream` is a hipStream_t passed as void* (NULL = default stream).
 *     Calls are asynchronous on that stream; nothing here synchronises.
 *   - The caller owns all data buffers; the library owns contexts, plans,
 *     twiddle tables and scratch.
 */
#ifndef OFHE_HIP_H
#define OFHE_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
    OFHE_OK = 0,
    OFHE_ERR_ARG = 1,     /* invalid argument (size, modulus, root ...)     */
    OFHE_ERR_HIP = 2,     /* a HIP runtime call failed                       */
    OFHE_ERR_NOMEM = 3,   /* device or host allocation failed                */
    OFHE_ERR_STATE = 4    /* use of a destroyed / uninitialised object       */
};

typedef struct ofhe_ctx_s* ofhe_ctx_t;   /* one per device (PimManager::getPim) */
typedef struct ofhe_plan_s* ofhe_plan_t; /* NTT plan: (N, towers, q[], psi[])  */

/* Thread-local description of the last failure in this thread: the message
 * OPENFHE_THROW(math_error, msg) carries (src/core/include/utils/exception.h:162);
 * the fork's PIM layer instead aborts in DPU_ASSERT (PimManager.cpp:5-37). */
const char* ofhe_hip_last_error(void);

/* Library version string ("ofhe-hip <ver> gfx950"); no reference counterpart
 * (the fork's kernel binaries are located by path, pim/kernel.h:4-8). */
const char* ofhe_hip_version(void);

/* ---- device context: replaces PimManager::getPim(nr_dpus, profile),
 *      PimManager.h:23-29 (lazily created singleton), and its allocator /
 *      transfers (PimManager.cpp:5-93). --------------------------------- */
int ofhe_hip_device_count(int* count);
int ofhe_hip_init(int device, ofhe_ctx_t* ctx);
int ofhe_hip_finalize(ofhe_ctx_t ctx);
/* PimManager::allocate / deallocate (PimManager.h:83-85) */
int ofhe_hip_alloc(ofhe_ctx_t ctx, size_t bytes, void** dptr);
int ofhe_hip_free(ofhe_ctx_t ctx, void* dptr);
/* Stream-ordered variants (hipMallocAsync / hipFreeAsync): the block is
 * released only after the work already queued on `stream` has finished, so a
 * buffer can be dropped right after the asynchronous calls that use it.
 * The blocks come from the context's own pool: ofhe_hip_finalize returns
 * OFHE_ERR_STATE (and leaves the context usable) while any block obtained
 * here has not been passed to ofhe_hip_free_async. */
int ofhe_hip_alloc_async(ofhe_ctx_t ctx, size_t bytes, void** dptr, void* stream);
int ofhe_hip_free_async(ofhe_ctx_t ctx, void* dptr, void* stream);
/* Pinned (page-locked) host memory for the staging buffers of a host-buffer
 * integration: towers gathered from the reference's per-tower vectors
 * (dcrtpoly.h:421, poly.h:368) into one buffer that DMA can read directly,
 * so host <-> device copies run at the PCIe rate and overlap compute. */
int ofhe_hip_host_alloc(ofhe_ctx_t ctx, size_t bytes, void** hptr);
int ofhe_hip_host_free(ofhe_ctx_t ctx, void* hptr);
/* dst[0..bytes) = 0 on the stream (a zero DCRTPoly, dcrtpoly.h initializing ctor). */
int ofhe_hip_zero(ofhe_ctx_t ctx, void* dst, size_t bytes, void* stream);
/* PimManager::copy_to_pim (scatter, type 0) / copy_from_pim (PimManager.h:44-54) */
int ofhe_hip_copy_to_device(ofhe_ctx_t ctx, void* dst, const void* src, size_t bytes, void* stream);
int ofhe_hip_copy_to_host(ofhe_ctx_t ctx, void* dst, const void* src, size_t bytes, void* stream);
/* device-to-device copy (poly copy constructor, poly.h:368 owns its vector) */
int ofhe_hip_copy_device(ofhe_ctx_t ctx, void* dst, const void* src, size_t bytes, void* stream);
/* PimManager::start_kernel is synchronous (PimManager.h:68); here explicit. */
int ofhe_hip_sync(ofhe_ctx_t ctx, void* stream);
/* A completion marker on one stream.  The reference's copies block until the
 * transfer is done (PimManager::copy_to_pim / copy_from_pim, PimManager.cpp:5-54);
 * with an event the host waits for one staged DMA only, not for every launch
 * queued on the stream (the C++ adapter's pinned staging, ofhe_dcrt.hpp). */
typedef struct ofhe_event_s* ofhe_event_t;
int ofhe_hip_event_create(ofhe_ctx_t ctx, ofhe_event_t* event);
int ofhe_hip_event_record(ofhe_event_t event, void* stream); /* marks the stream's work so far */
int ofhe_hip_event_sync(ofhe_event_t event);                 /* waits for the marked work     */
int ofhe_hip_event_destroy(ofhe_event_t event);
/* Return all but keep_bytes of the context's stream-ordered pool (scratch and
 * ofhe_hip_alloc_async blocks kept across synchronisations) to the device; the
 * reference frees DPU memory per call (PimManager::deallocate, PimManager.h:83-85). */
int ofhe_hip_trim(ofhe_ctx_t ctx, size_t keep_bytes);

/* ---- NTT plan: replaces ChineseRemainderTransformFTTNat::PreCompute and
 *      its static twiddle maps (transformnat-impl.h:708-763,
 *      transformnat.h:352-368).  N = 2^log_n, 1 <= log_n <= 17; q[t] prime,
 *      q[t] = 1 mod 2N, q[t] < 2^60; psi[t] a primitive 2N-th root of unity
 *      mod q[t] (OpenFHE uses the smallest one, nbtheory-impl.h:183-231).
 *      Tables are built on the host once and kept resident on the device. */
int ofhe_hip_plan_create(ofhe_ctx_t ctx, uint32_t log_n, uint32_t towers, const uint64_t* q,
                         const uint64_t* psi, ofhe_plan_t* plan);
/* Kernel choices of a plan, fixed at creation (ofhe_hip_plan_create_ex).  A
 * zero-initialised struct (or NULL) is exactly ofhe_hip_plan_create's choice.
 * Every setting gives the same canonical results; they let tests reach every
 * kernel and A/B timings compare them in one process.  No reference
 * counterpart (the reference has one CPU loop, transformnat-impl.h:300-354). */
enum {
    OFHE_SPLIT_AUTO = 0, /* log_n = 16: OFHE_SPLIT_8_8; other log_n > 12: OFHE_SPLIT_COLS  */
    OFHE_SPLIT_COLS = 1, /* log_n - 12 column stages (k_cols) + a 12-stage block pass     */
    OFHE_SPLIT_8_8 = 2,  /* log_n = 16 only: 8 column stages (k_tcols) + 8-stage block    */
    OFHE_SPLIT_9_8 = 3,  /* log_n = 17 only: 9 column stages (k_tcols9) + 8-stage block   */
    OFHE_SPLIT_8_9 = 4   /* log_n = 17 only: 8 column stages (k_tcols) + 9-stage block    */
};
typedef struct ofhe_plan_options {
    uint32_t split;          /* OFHE_SPLIT_*; log_n <= 12 plans accept only AUTO          */
    uint32_t generic_moduli; /* 1: the generic-modulus kernels even when every q is a
                                special prime 2^L - d (the default picks the faster ones) */
} ofhe_plan_options;
int ofhe_hip_plan_create_ex(ofhe_ctx_t ctx, uint32_t log_n, uint32_t towers, const uint64_t* q,
                            const uint64_t* psi, const ofhe_plan_options* options, ofhe_plan_t* plan);
int ofhe_hip_plan_destroy(ofhe_plan_t plan);
/* Performance knob for ofhe_hip_ntt_mul_intt at log_n > 12: process the batch
 * in chunks of `chunk_batch` entries (0 = whole batch in one pass) and, with
 * streams = 2, alternate the chunks over two internal streams forked from and
 * joined back into the caller's stream.  Results are identical for any
 * setting; only speed changes.  Set it while no other thread launches with
 * the same plan: the launches read the setting without taking the plan's lock. */
int ofhe_hip_plan_tune(ofhe_plan_t plan, uint32_t chunk_batch, uint32_t streams);
/* Copy the plan's host-side tables out (debug / parity tests): any pointer
 * may be NULL.  tab*: [towers][N] in OpenFHE order (Table[rev(i)] = psi^i). */
int ofhe_hip_plan_tables(ofhe_plan_t plan, uint64_t* tab, uint64_t* tab_pre, uint64_t* itab,
                         uint64_t* itab_pre, uint64_t* ninv);

/* Forward negacyclic NTT in place, natural order -> bit-reversed evaluation
 * order: ChineseRemainderTransformFTT<NativeVector>::ForwardTransformToBitReverseInPlace
 * (transformnat-impl.h:575-602 -> 300-354), for every (batch, tower). */
int ofhe_hip_ntt_fwd(ofhe_plan_t plan, uint64_t* data, uint32_t batch, void* stream);
/* Inverse NTT in place, bit-reversed -> natural, n^-1 applied:
 * InverseTransformFromBitReverseInPlace (transformnat-impl.h:637-666 -> 492-552). */
int ofhe_hip_ntt_inv(ofhe_plan_t plan, uint64_t* data, uint32_t batch, void* stream);

/* The same transforms on plan towers [t0, t0 + count) of strided data, in or
 * out of place: src / dst point at tower t0 of batch entry 0 and advance by
 * src_stride / dst_stride words (>= count * N) per batch entry.  This is the
 * per-tower SwitchFormat the DCRTPoly loops issue on sub-bases (e.g. the P
 * towers of a Q|P polynomial in ApproxModUp, dcrtpoly-impl.h:1112-1116). */
int ofhe_hip_ntt_fwd_range(ofhe_plan_t plan, uint32_t t0, uint32_t count, const uint64_t* src,
                           uint64_t* dst, uint64_t src_stride, uint64_t dst_stride, uint32_t batch,
                           void* stream);
int ofhe_hip_ntt_inv_range(ofhe_plan_t plan, uint32_t t0, uint32_t count, const uint64_t* src,
                           uint64_t* dst, uint64_t src_stride, uint64_t dst_stride, uint32_t batch,
                           void* stream);

/* LeveledSHEBase::EvalMultCore for two 2-element ciphertexts
 * (base-leveledshe.cpp:667-672), evaluation form, per (batch, tower) of plan:
 *   out2 = c1 * d1,  out1 = c1 * d0 + c0 * d1,  out0 = d0 * c0
 * (DCRTPoly operator* / += : Barrett ModMul, ModAdd), one pass over HBM.
 * Outputs must not alias inputs. */
int ofhe_hip_eval_mult_core(ofhe_plan_t plan, const uint64_t* c0, const uint64_t* c1, const uint64_t* d0,
                            const uint64_t* d1, uint64_t* out0, uint64_t* out1, uint64_t* out2, uint32_t batch,
                            void* stream);
/* c = a (op) b element-wise per tower: NativeVectorT::ModMul (Barrett,
 * mubintvecnat.cpp:353-367 / .h:501-513), ModAdd (.cpp:245-264 / .h:426-432),
 * ModSub (.cpp:301-307).  c may alias a or b (the *Eq forms). */
int ofhe_hip_modmul_vv(ofhe_plan_t plan, const uint64_t* a, const uint64_t* b, uint64_t* c,
                       uint32_t batch, void* stream);
int ofhe_hip_modadd_vv(ofhe_plan_t plan, const uint64_t* a, const uint64_t* b, uint64_t* c,
                       uint32_t batch, void* stream);
int ofhe_hip_modsub_vv(ofhe_plan_t plan, const uint64_t* a, const uint64_t* b, uint64_t* c,
                       uint32_t batch, void* stream);
/* Vector (.) scalar with one scalar per tower (host array s[towers], any
 * uint64_t; each is reduced mod q[t] first, as the reference does).  The
 * scalars travel in the kernel arguments: nothing is staged, nothing
 * synchronises, and c may alias a.  They replace the DPU SCALAR / SCALAR_EQ
 * kernels (src/core/pim/dpu/element-wise/add-mod.c:23-100, sub-mod.c,
 * mult-mod.c) and the CPU loops of
 *   c = a * s mod q: NativeVectorT::ModMul(Eq)(const IntegerType&)
 *                    (mubintvecnat.cpp:310-332, Shoup), DCRTPoly::Times(Integer);
 *   c = a + s mod q: NativeVectorT::ModAdd(Eq)(const IntegerType&)
 *                    (mubintvecnat.cpp:198-219), DCRTPoly::Plus(Integer) in
 *                    evaluation form (dcrtpoly.h:162-163, poly-impl.h:213-220);
 *   c = a - s mod q: NativeVectorT::ModSub(Eq)(const IntegerType&)
 *                    (mubintvecnat.cpp:267-288), DCRTPoly::Minus(Integer)
 *                    (dcrtpoly.h:182-183, poly-impl.h:223-227). */
int ofhe_hip_modmul_scalar(ofhe_plan_t plan, const uint64_t* a, const uint64_t* s, uint64_t* c,
                           uint32_t batch, void* stream);
int ofhe_hip_modadd_scalar(ofhe_plan_t plan, const uint64_t* a, const uint64_t* s, uint64_t* c,
                           uint32_t batch, void* stream);
int ofhe_hip_modsub_scalar(ofhe_plan_t plan, const uint64_t* a, const uint64_t* s, uint64_t* c,
                           uint32_t batch, void* stream);
/* c[index] = a[index] + s[t] mod q[t] in every (batch, tower); no other word is
 * written (use in place, or copy a to c first): NativeVectorT::ModAddAtIndex(Eq)
 * (mubintvecnat.cpp:221-231), i.e. PolyImpl / DCRTPoly::Plus(Integer) in
 * coefficient form (poly-impl.h:213-220: a constant added to coefficient 0). */
int ofhe_hip_modadd_scalar_at(ofhe_plan_t plan, const uint64_t* a, uint64_t index, const uint64_t* s,
                              uint64_t* c, uint32_t batch, void* stream);

/* Synthetic inputs for benchmarks and tests; no reference
 * counterpart (the benchmark draws uniform vectors on the host,
 * poly-benchmark-16k.cpp:45-70): dst[b][t][i] = splitmix64 draw i + 1 of the stream seeded
 * 0x5EED ^ ((batch_offset + b) << 20) ^ (t << 8) ^ seed, mod q[t] -- what the
 * CPU oracle's generator (oracle_fill_uniform) produces for the same seed. */
int ofhe_hip_fill_uniform(ofhe_plan_t plan, uint64_t* dst, uint32_t batch, uint32_t batch_offset, uint64_t seed,
                          void* stream);

/* The metric pipeline, per (batch, tower): c = INTT(NTT(a) (.) b), a in
 * coefficient form, b in evaluation form, c in coefficient form.  Equals
 * SwitchFormat -> Times -> SwitchFormat on DCRTPoly (dcrtpoly-impl.h:2518-2524,
 * dcrtpoly.h:185-200).  c may alias a. */
int ofhe_hip_ntt_mul_intt(ofhe_plan_t plan, const uint64_t* a, const uint64_t* b, uint64_t* c,
                          uint32_t batch, void* stream);

/* One launch of the pipeline above, for per-kernel timing (bench.py); no
 * reference counterpart (the reference's loop is per tower, dcrtpoly-impl.h:2518-2524):
 * stage 0 = forward column pass (a -> c), 1 = block pass (forward tail,
 * Hadamard with b, inverse head; reads c, or a when log_n <= 12),
 * 2 = inverse column pass (c -> c).  Stages 0 and 2 are no-ops for
 * log_n <= 12.  Running 0, 1, 2 in order equals ofhe_hip_ntt_mul_intt. */
int ofhe_hip_ntt_mul_intt_stage(ofhe_plan_t plan, int stage, const uint64_t* a, const uint64_t* b,
                                uint64_t* c, uint32_t batch, void* stream);

/* ---- RNS base conversion: DCRTPolyImpl::ApproxSwitchCRTBasis
 *      (dcrtpoly-impl.h:1034-1063, Mul128/BarrettUint128ModUint64 in
 *      utils/utilities-int.h:47-103).  x: [batch][size_q][N] coefficient form
 *      mod q[i]; out: [batch][size_p][N] mod p[j].  Precomputations as the pke
 *      layer builds them (pke/lib/schemerns/rns-cryptoparameters.cpp:273-337):
 *      qhat_inv_modq[i] = (Q/q_i)^-1 mod q_i, qhat_modp[i*size_p+j] = (Q/q_i) mod p_j,
 *      all host arrays.  Barrett constants are derived internally. */
typedef struct ofhe_bconv_s* ofhe_bconv_t;
int ofhe_hip_bconv_create(ofhe_ctx_t ctx, uint32_t log_n, uint32_t size_q, uint32_t size_p,
                          const uint64_t* q, const uint64_t* p, const uint64_t* qhat_inv_modq,
                          const uint64_t* qhat_modp, ofhe_bconv_t* bconv);
/* Kernel choices of a converter (ofhe_hip_bconv_create_ex; zero = the default
 * of ofhe_hip_bconv_create).  Same results for every setting. */
enum {
    OFHE_BCONV_KERNEL_AUTO = 0, /* matrix cores (<= 64 sources, N >= 32), else LIMB / WIDE */
    OFHE_BCONV_KERNEL_LIMB = 1, /* 30-bit limb sums on the VALU (<= 16 sources)            */
    OFHE_BCONV_KERNEL_WIDE = 2  /* 128-bit sums on the VALU, any number of sources         */
};
typedef struct ofhe_bconv_options {
    uint32_t kernel;        /* OFHE_BCONV_KERNEL_*; LIMB / WIDE hold on every path that
                               uses the converter (ApproxModUp / ApproxModDown at 2^17
                               then run conversion and column pass as two kernels)     */
    uint32_t separate_cols; /* 1: in ofhe_hip_approx_mod_up / _down at N = 2^17, the
                               conversion and the targets' forward column pass as two
                               kernels instead of the fused k_bconv_cols                  */
} ofhe_bconv_options;
int ofhe_hip_bconv_create_ex(ofhe_ctx_t ctx, uint32_t log_n, uint32_t size_q, uint32_t size_p,
                             const uint64_t* q, const uint64_t* p, const uint64_t* qhat_inv_modq,
                             const uint64_t* qhat_modp, const ofhe_bconv_options* options, ofhe_bconv_t* bconv);
int ofhe_hip_bconv_destroy(ofhe_bconv_t bconv);
int ofhe_hip_approx_switch_crt_basis(ofhe_bconv_t bconv, const uint64_t* x, uint64_t* out,
                                     uint32_t batch, void* stream);

/* DCRTPolyImpl::ApproxModUp (dcrtpoly-impl.h:1085-1131).  x: [batch][Q][N]
 * under plan_q, in evaluation form when eval_form != 0 (else coefficient
 * form); out: [batch][Q+P][N] in evaluation form, towers Q of plan_q then P
 * of plan_p.  q_to_p converts plan_q's basis to plan_p's.  out must not
 * overlap x. */
int ofhe_hip_approx_mod_up(ofhe_plan_t plan_q, ofhe_plan_t plan_p, ofhe_bconv_t q_to_p, int eval_form,
                           const uint64_t* x, uint64_t* out, uint32_t batch, void* stream);
/* DCRTPolyImpl::ApproxModDown (dcrtpoly-impl.h:1134-1175).  x: [batch][Q+P][N]
 * evaluation form; out: [batch][Q][N] evaluation form.  p_to_q converts
 * plan_p's basis to plan_q's (PHatInvModp, PHatModq); p_inv_modq: host
 * [Q] = P^-1 mod q_i.  t = 0 for CKKS / BFV; t > 0 (BGV) multiplies the P part
 * by t^-1 mod p_j and the switched part by t (t_inv_modp derived here).
 * The small constant tables are built and uploaded on the first call with a
 * given (t, p_inv_modq) and cached in p_to_q; no call synchronises. */
int ofhe_hip_approx_mod_down(ofhe_plan_t plan_q, ofhe_plan_t plan_p, ofhe_bconv_t p_to_q,
                             const uint64_t* p_inv_modq, uint64_t t, const uint64_t* x, uint64_t* out,
                             uint32_t batch, void* stream);

/* ---- HYBRID key switching: KeySwitchHYBRID (pke/lib/keyswitch/
 *      keyswitch-hybrid.cpp:325-482) with the CRT tables of
 *      CryptoParametersRNS::PrecomputeCRTTables (pke/lib/schemerns/
 *      rns-cryptoparameters.cpp:72-345) built internally from the moduli.
 *      Q = q[0..size_q) (element params), P = p[0..size_p) (GetParamsP()),
 *      num_part_q = dnum digits of alpha = ceil(size_q / num_part_q) towers.
 *      Every call works at level size_ql (1 <= size_ql <= size_q): the
 *      ciphertext has towers q[0..size_ql).  Evaluation keys are laid out
 *      [num_part_q][size_q + size_p][N] (EvalKey b / a vectors over QP),
 *      shared by the batch. ---- */
typedef struct ofhe_ks_s* ofhe_ks_t;
int ofhe_hip_ks_create(ofhe_ctx_t ctx, uint32_t log_n, uint32_t size_q, const uint64_t* q,
                       const uint64_t* psi_q, uint32_t size_p, const uint64_t* p, const uint64_t* psi_p,
                       uint32_t num_part_q, ofhe_ks_t* ks);
/* Engine choices (ofhe_hip_ks_create_ex; zero / NULL = ofhe_hip_ks_create's
 * defaults).  Same results for every setting. */
typedef struct ofhe_ks_options {
    ofhe_plan_options plan;   /* the engine's Q|P plan                                       */
    uint32_t separate_cols;   /* 1: base conversion and forward column pass as two kernels   */
    uint32_t separate_icol;   /* 1: the digits' inverse column pass as its own kernel        */
    uint32_t chunk;           /* ciphertexts per ModUp chunk (0 = the whole batch)           */
    uint32_t single_stream;   /* 1: every digit on the caller's stream (no side streams)     */
} ofhe_ks_options;
int ofhe_hip_ks_create_ex(ofhe_ctx_t ctx, uint32_t log_n, uint32_t size_q, const uint64_t* q,
                          const uint64_t* psi_q, uint32_t size_p, const uint64_t* p, const uint64_t* psi_p,
                          uint32_t num_part_q, const ofhe_ks_options* options, ofhe_ks_t* ks);
int ofhe_hip_ks_destroy(ofhe_ks_t ks);
/* alpha (towers per digit) and beta (digits at level size_ql, capped at
 * num_part_q), keyswitch-hybrid.cpp:341-345. */
int ofhe_hip_ks_digits(ofhe_ks_t ks, uint32_t size_ql, uint32_t* alpha, uint32_t* beta);
/* EvalKeySwitchPrecomputeCore (keyswitch-hybrid.cpp:330-412): c [batch][size_ql][N]
 * evaluation form -> digits [batch][beta][size_ql + size_p][N] evaluation form. */
int ofhe_hip_ks_precompute(ofhe_ks_t ks, uint32_t size_ql, const uint64_t* c, uint64_t* digits,
                           uint32_t batch, void* stream);
/* EvalFastKeySwitchCoreExt (keyswitch-hybrid.cpp:438-482): ct0 = sum_j digits_j * b_j,
 * ct1 = sum_j digits_j * a_j over Ql|P; ct0, ct1: [batch][size_ql + size_p][N]. */
int ofhe_hip_ks_fast_core_ext(ofhe_ks_t ks, uint32_t size_ql, const uint64_t* digits,
                              const uint64_t* key_b, const uint64_t* key_a, uint64_t* ct0, uint64_t* ct1,
                              uint32_t batch, void* stream);
/* ApproxModDown with the key-switching tables (keyswitch-hybrid.cpp:423-435):
 * x [batch][size_ql + size_p][N] -> out [batch][size_ql][N], evaluation form. */
int ofhe_hip_ks_mod_down(ofhe_ks_t ks, uint32_t size_ql, const uint64_t* x, uint64_t* out, uint64_t t,
                         uint32_t batch, void* stream);
/* KeySwitchCore = EvalFastKeySwitchCore(EvalKeySwitchPrecomputeCore(c))
 * (keyswitch-hybrid.cpp:325-328, 414-436): out0, out1 [batch][size_ql][N]. */
int ofhe_hip_ks_core(ofhe_ks_t ks, uint32_t size_ql, const uint64_t* c, const uint64_t* key_b,
                     const uint64_t* key_a, uint64_t* out0, uint64_t* out1, uint64_t t, uint32_t batch,
                     void* stream);

/* ---- element maps ---- */
/* NativeVectorT::SwitchModulus (mubintvecnat.cpp:111-136) on n words:
 * values of modulus old_q re-centred to new_q, exactly as the reference. */
int ofhe_hip_switch_modulus(ofhe_ctx_t ctx, const uint64_t* src, uint64_t* dst, uint64_t n,
                            uint64_t old_q, uint64_t new_q, void* stream);
/* PolyImpl::AutomorphismTransform(k) (poly-impl.h:312-365), X -> X^k for odd
 * k, per (batch, tower) of plan; eval_form != 0 permutes bit-reversed
 * evaluation slots, else signed permutation of coefficients (a negated zero
 * stays q, as in the reference).  dst must not overlap src. */
int ofhe_hip_automorphism(ofhe_plan_t plan, uint32_t k, int eval_form, const uint64_t* src, uint64_t* dst,
                          uint32_t batch, void* stream);

/* ---- rescaling (callers of the path one tower down) ----
 * x: [batch][towers][N] (x_stride words per batch entry) over plan towers
 * 0..towers-1, canonical, all in evaluation form (eval_form != 0) or all in
 * coefficient form; out: [batch][towers-1][N] (out_stride).  out may be x
 * itself only with out_stride == x_stride (in place); any other overlap of
 * the two ranges is rejected with OFHE_ERR_ARG.
 * DCRTPolyImpl::DropLastElementAndScale (dcrtpoly-impl.h:746-768), CKKS / BFV
 * rescaling with ql_ql_inv_modql_divql_modq[i] and ql_inv_modq[i], i <
 * towers-1 (ckksrns-cryptoparameters.cpp:72-86):
 *   out_i = x_i ql_inv_modq_i + [SwitchModulus(x_last) c_i]   (evaluation:
 *   the last tower through the INTT, the switched term through the NTT);
 *   coefficient form: out_i = NTT(x_i ql_inv_modq_i + SwitchModulus(x_last) c_i)
 *   -- the reference switches these towers to evaluation form (lines 765-766).
 * ql_inv_modq_i must be invertible mod q_i in evaluation form (it is
 * q_last^-1 mod q_i). */
int ofhe_hip_drop_last_and_scale(ofhe_plan_t plan, uint32_t towers, const uint64_t* x, uint64_t x_stride,
                                 uint64_t* out, uint64_t out_stride, int eval_form,
                                 const uint64_t* ql_ql_inv_modql_divql_modq, const uint64_t* ql_inv_modq,
                                 uint32_t batch, void* stream);
/* DCRTPolyImpl::ModReduce (dcrtpoly-impl.h:792-812), BGV modulus switching:
 * delta = [x_last]_coefficient * neg_t_inv_modq mod q_last;
 *   out_i = (x_i + [SwitchModulus(delta)] t) ql_inv_modq_i, the switched term
 * through the NTT in evaluation form; the output keeps the input's form. */
int ofhe_hip_mod_reduce(ofhe_plan_t plan, uint32_t towers, const uint64_t* x, uint64_t x_stride, uint64_t* out,
                        uint64_t out_stride, int eval_form, uint64_t t, uint64_t neg_t_inv_modq,
                        const uint64_t* ql_inv_modq, uint32_t batch, void* stream);

/* ---- BV key switching, digitSize = 0 (KeySwitchBV, keyswitch-bv.cpp:302-340) ----
 * KeySwitchBV::EvalKeySwitchPrecomputeCore -> DCRTPolyImpl::CRTDecompose(0)
 * (keyswitch-bv.cpp:308-312, dcrtpoly-impl.h:266-288): c [batch][towers][N]
 * in evaluation form over plan towers 0..towers-1 -> digits
 * [batch][towers][towers][N], digit i = tower i of c in coefficient form,
 * SwitchModulus'd into every tower, in evaluation form. */
int ofhe_hip_bv_precompute(ofhe_plan_t plan, uint32_t towers, const uint64_t* c, uint64_t* digits, uint32_t batch,
                           void* stream);
/* KeySwitchBV::EvalFastKeySwitchCore (keyswitch-bv.cpp:314-340): ct0 =
 * sum_i bv[i] * d_i, ct1 = sum_i av[i] * d_i over the first `towers` towers of
 * the keys key_b / key_a [towers][key_towers][N] (DropLastElements at lower
 * levels); out0, out1 [batch][towers][N], evaluation form. */
int ofhe_hip_bv_core(ofhe_plan_t plan, uint32_t towers, const uint64_t* digits, const uint64_t* key_b,
                     const uint64_t* key_a, uint32_t key_towers, uint64_t* out0, uint64_t* out1, uint32_t batch,
                     void* stream);

/* ---- multi-GPU: evaluation-key broadcast over RCCL (xGMI) ----
 * the path shards by ciphertext batch with no exchange;
 * the one collective is the broadcast of the key-switching keys from a root
 * GPU (the keys the HYBRID core reads, keyswitch-hybrid.cpp:452-478).  The
 * reference is single-device (PimManager.h:21-127 drives one DPU set), so
 * this has no reference counterpart beyond "the key is in device memory".
 * One communicator per (process, device); the 128-byte id from rank 0's
 * ofhe_hip_comm_unique_id travels to the other ranks out of band. */
#define OFHE_COMM_ID_BYTES 128
typedef struct ofhe_comm_s* ofhe_comm_t;
int ofhe_hip_comm_unique_id(void* id /* OFHE_COMM_ID_BYTES */);
/* Collective over all nranks processes (blocks until they have all joined). */
int ofhe_hip_comm_init(ofhe_ctx_t ctx, int nranks, int rank, const void* id, ofhe_comm_t* out);
int ofhe_hip_comm_destroy(ofhe_comm_t comm);
/* In-place broadcast of `words` u64 of device memory from rank `root`:
 * the root's key is read, every other rank's buffer is overwritten.  Enqueued
 * on `stream` (ncclBroadcast); all ranks must call it with the same words. */
int ofhe_hip_bcast_evalkey(ofhe_comm_t comm, uint64_t* key, size_t words, int root, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* OFHE_HIP_H */
