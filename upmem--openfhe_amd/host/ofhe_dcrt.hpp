// ofhe_dcrt.hpp -- C++ host side of the gfx950 backend, above the C ABI.
//
// Mirrors the reference's interfaces for the hot path so OpenFHE-side code
// (and these tests) read the same way:
//   HipManager::getHip(dev)   <- PimManager::getPim(nr_dpus, profile)
//                                (src/core/include/pim/PimManager.h:23-29,44-85)
//   DeviceBuffer              <- PimData's device allocation (PimData.h:16-34, RAII)
//   DCRTPolyHip               <- DCRTPolyImpl's operator surface used by the
//                                schemes (lattice/hal/default/dcrtpoly.h:142-200,
//                                dcrtpoly-impl.h:410-416, 1034-1063, 2518-2524):
//                                SwitchFormat/SetFormat, Plus/Minus/Times and the
//                                in-place operators, scalar Times, ApproxSwitchCRTBasis.
//   PlanCache                 <- ChineseRemainderTransformFTTNat's static
//                                per-modulus twiddle maps (transformnat.h:352-368)
//   Staging                   <- the per-vector host->DPU push of PimData
//                                (PimData.h:16-21): towers gathered from
//                                separate host vectors into pinned memory, one
//                                transfer each way
//   KsCache / KeyCache        <- the per-parameter-set HYBRID tables
//                                (rns-cryptoparameters.cpp:72-345) and the
//                                evaluation keys kept resident on the device
// Errors: any non-zero C-ABI status becomes ofhe::math_error, the analogue of
// OPENFHE_THROW(math_error, ...) (src/core/include/utils/exception.h:162).
// Device layout: a DCRTPolyHip of `batch` polynomials is one contiguous
// [batch][towers][N] buffer -- towers are contiguous, unlike the reference's
// std::vector<PolyImpl> (dcrtpoly.h:421), so one launch covers every tower.
#pragma once

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <istream>
#include <map>
#include <ostream>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "../../include/ofhe_hip.h"

namespace ofhe {

class math_error : public std::runtime_error {
public:
    explicit math_error(const std::string& m) : std::runtime_error(m) {}
};
class not_implemented_error : public std::runtime_error {
public:
    explicit not_implemented_error(const std::string& m) : std::runtime_error(m) {}
};
class deserialize_error : public std::runtime_error {  // lbcrypto::deserialize_error (utils/exception.h)
public:
    explicit deserialize_error(const std::string& m) : std::runtime_error(m) {}
};

inline void check(int rc, const char* what) {
    if (rc != OFHE_OK) throw math_error(std::string(what) + ": " + ofhe_hip_last_error());
}

// ---------------------------------------------------------------------------
// HipManager: lazily created per-device singleton, creation guarded by a
// mutex (PimManager.h:23-29); owns the device context and its stream.
// ---------------------------------------------------------------------------
class HipManager {
public:
    static HipManager* getHip(int device = 0) {
        static std::mutex mu;
        static std::map<int, std::unique_ptr<HipManager>> inst;
        std::lock_guard<std::mutex> lk(mu);
        auto& p = inst[device];
        if (!p) p.reset(new HipManager(device));
        return p.get();
    }
    ofhe_ctx_t ctx() const { return ctx_; }
    int device() const { return device_; }
    // Every adapter op runs on one stream (the device's null stream), and
    // buffers are allocated and released in that stream's order: a DCRTPoly
    // temporary may die right after the call that reads it -- its memory is
    // returned only once the queued work has finished, and nothing waits.
    void* allocate(size_t bytes) {
        void* p = nullptr;
        check(ofhe_hip_alloc_async(ctx_, bytes, &p, nullptr), "HipManager::allocate");
        return p;
    }
    void deallocate(void* p) { check(ofhe_hip_free_async(ctx_, p, nullptr), "HipManager::deallocate"); }
    void zero(void* dst, size_t bytes) { check(ofhe_hip_zero(ctx_, dst, bytes, nullptr), "HipManager::zero"); }
    // Host <-> device copies of the caller's (pageable) memory go through the
    // manager's two pinned staging buffers: the caller's words are copied into
    // one, a DMA from page-locked memory is queued on the stream (in the
    // stream's order, after the launches that produce or read `dst`), and an
    // event marks it.  A buffer is refilled only after the event of its last
    // DMA -- a wait for that one transfer, not for every launch queued on the
    // stream (round 5 drained the whole stream before and after each round).
    // copy_to_device returns once the caller's buffer has been read (the
    // copy_to_pim contract, PimManager.cpp:5-37), with the DMA possibly still
    // in flight; copy_from_device returns with the words in `dst`
    // (copy_from_pim, PimManager.cpp:39-54), overlapping each chunk's DMA
    // with the previous chunk's host copy.  No pageable hipMemcpyAsync: that
    // path's staging and ordering are the HIP runtime's own (round 4's driver
    // record read back stale words on it, DESIGN.md (c) "The round-4 adapter
    // failure").
    void copy_to_device(void* dst, const void* src, size_t bytes) {
        std::lock_guard<std::mutex> lk(stage_mu_);
        const size_t room = stage_room(bytes);
        for (size_t off = 0; off < bytes;) {
            const size_t n = std::min(bytes - off, room);
            const int k = next_;
            next_ ^= 1;
            stage_wait(k);  // the buffer's previous DMA has read it
            std::memcpy(stage_[k], static_cast<const char*>(src) + off, n);
            check(ofhe_hip_copy_to_device(ctx_, static_cast<char*>(dst) + off, stage_[k], n, nullptr),
                  "HipManager::copy_to_device");
            stage_mark(k);
            off += n;
        }
    }
    void copy_from_device(void* dst, const void* src, size_t bytes) {
        std::lock_guard<std::mutex> lk(stage_mu_);
        const size_t room = stage_room(bytes);
        size_t prev_off = 0, prev_n = 0;
        int prev = -1;
        for (size_t off = 0; off < bytes;) {
            const size_t n = std::min(bytes - off, room);
            const int k = next_;
            next_ ^= 1;
            stage_wait(k);
            check(ofhe_hip_copy_to_host(ctx_, stage_[k], static_cast<const char*>(src) + off, n, nullptr),
                  "HipManager::copy_from_device");
            stage_mark(k);
            if (prev >= 0) drain(prev, dst, prev_off, prev_n);
            prev = k, prev_off = off, prev_n = n;
            off += n;
        }
        if (prev >= 0) drain(prev, dst, prev_off, prev_n);
    }
    void sync() { check(ofhe_hip_sync(ctx_, nullptr), "HipManager::sync"); }
    // ofhe_hip_finalize refuses (OFHE_ERR_STATE) while DeviceBuffers still
    // hold blocks of the context's pool: the context is then left alive for
    // them (they free through the context handle, not through this object),
    // and process exit reclaims it.
    ~HipManager() {
        for (int k = 0; k < 2; k++) {
            if (ev_[k]) {
                (void)ofhe_hip_event_sync(ev_[k]);
                (void)ofhe_hip_event_destroy(ev_[k]);
            }
            if (stage_[k]) (void)ofhe_hip_host_free(ctx_, stage_[k]);
        }
        if (ctx_) (void)ofhe_hip_finalize(ctx_);
    }
    HipManager(const HipManager&) = delete;
    HipManager& operator=(const HipManager&) = delete;

private:
    explicit HipManager(int device) : device_(device) {
        check(ofhe_hip_init(device, &ctx_), "HipManager");
        for (int k = 0; k < 2; k++) check(ofhe_hip_event_create(ctx_, &ev_[k]), "HipManager staging event");
    }
    // bytes each staging buffer takes per round (grown to the request, capped
    // at kStageMax: larger copies go in rounds); caller holds stage_mu_
    static constexpr size_t kStageMax = size_t(32) << 20;
    size_t stage_room(size_t want) {
        want = std::min(std::max<size_t>(want, 1), kStageMax);
        if (stage_bytes_ < want) {
            size_t b = 4096;
            while (b < want) b <<= 1;
            for (int k = 0; k < 2; k++) {
                stage_wait(k);  // a queued DMA may still read the old buffer
                if (stage_[k]) check(ofhe_hip_host_free(ctx_, stage_[k]), "HipManager staging");
                stage_[k] = nullptr;
            }
            stage_bytes_ = 0;
            for (int k = 0; k < 2; k++) check(ofhe_hip_host_alloc(ctx_, b, &stage_[k]), "HipManager staging");
            stage_bytes_ = b;
        }
        return stage_bytes_;
    }
    void stage_mark(int k) {
        check(ofhe_hip_event_record(ev_[k], nullptr), "HipManager staging event");
        pending_[k] = true;
    }
    void stage_wait(int k) {
        if (!pending_[k]) return;
        check(ofhe_hip_event_sync(ev_[k]), "HipManager staging event");
        pending_[k] = false;
    }
    void drain(int k, void* dst, size_t off, size_t n) {
        stage_wait(k);  // the DMA (and, in stream order, its producers) has finished
        std::memcpy(static_cast<char*>(dst) + off, stage_[k], n);
    }
    int device_;
    ofhe_ctx_t ctx_ = nullptr;
    std::mutex stage_mu_;
    void* stage_[2] = {nullptr, nullptr};
    ofhe_event_t ev_[2] = {nullptr, nullptr};
    bool pending_[2] = {false, false};
    int next_ = 0;
    size_t stage_bytes_ = 0;
};

// RAII device buffer of uint64 words.
class DeviceBuffer {
public:
    DeviceBuffer() = default;
    DeviceBuffer(HipManager* m, size_t words) : m_(m), ctx_(m->ctx()), n_(words) {
        if (words) p_ = static_cast<uint64_t*>(m_->allocate(words * sizeof(uint64_t)));
    }
    DeviceBuffer(const DeviceBuffer&) = delete;
    DeviceBuffer& operator=(const DeviceBuffer&) = delete;
    DeviceBuffer(DeviceBuffer&& o) noexcept { swap(o); }
    DeviceBuffer& operator=(DeviceBuffer&& o) noexcept {
        swap(o);
        return *this;
    }
    ~DeviceBuffer() {
        if (p_) (void)ofhe_hip_free_async(ctx_, p_, nullptr);  // stream-ordered, no wait
    }
    uint64_t* get() const { return p_; }
    size_t size() const { return n_; }
    void upload(const uint64_t* h) { m_->copy_to_device(p_, h, n_ * 8); }
    void zero() { m_->zero(p_, n_ * 8); }
    void download(uint64_t* h) const { m_->copy_from_device(h, p_, n_ * 8); }
    void copy_from(const DeviceBuffer& o) {
        check(ofhe_hip_copy_device(m_->ctx(), p_, o.p_, n_ * 8, nullptr), "DeviceBuffer::copy_from");
    }

private:
    void swap(DeviceBuffer& o) {
        std::swap(m_, o.m_);
        std::swap(ctx_, o.ctx_);
        std::swap(p_, o.p_);
        std::swap(n_, o.n_);
    }
    HipManager* m_ = nullptr;
    ofhe_ctx_t ctx_ = nullptr;
    uint64_t* p_ = nullptr;
    size_t n_ = 0;
};

// ---------------------------------------------------------------------------
// PlanCache: one resident NTT plan per (device, N, moduli, roots), shared by
// every DCRTParams over that basis and kept for the process lifetime, as the
// reference's static per-modulus maps keep their tables (transformnat.h:352-368,
// filled in PreCompute, transformnat-impl.h:708-763).
// ---------------------------------------------------------------------------
class PlanHandle {
public:
    PlanHandle(HipManager* m, uint32_t log_n, const std::vector<uint64_t>& q, const std::vector<uint64_t>& r) {
        check(ofhe_hip_plan_create(m->ctx(), log_n, (uint32_t)q.size(), q.data(), r.data(), &p_), "PlanCache");
    }
    ~PlanHandle() {
        if (p_) ofhe_hip_plan_destroy(p_);
    }
    PlanHandle(const PlanHandle&) = delete;
    PlanHandle& operator=(const PlanHandle&) = delete;
    ofhe_plan_t get() const { return p_; }

private:
    ofhe_plan_t p_ = nullptr;
};

class PlanCache {
public:
    static std::shared_ptr<PlanHandle> get(int device, uint32_t log_n, const std::vector<uint64_t>& moduli,
                                           const std::vector<uint64_t>& roots) {
        if (moduli.size() != roots.size() || moduli.empty()) throw math_error("PlanCache: moduli/roots size mismatch");
        // the manager's statics first: destroyed after the cached plans
        HipManager* m = HipManager::getHip(device);
        static std::mutex mu;
        static std::map<Key, std::shared_ptr<PlanHandle>> plans;
        std::lock_guard<std::mutex> lk(mu);
        auto& e = plans[Key{device, log_n, moduli, roots}];
        if (!e) e = std::make_shared<PlanHandle>(m, log_n, moduli, roots);
        return e;
    }

private:
    struct Key {
        int device;
        uint32_t log_n;
        std::vector<uint64_t> q, r;
        bool operator<(const Key& o) const {
            if (device != o.device) return device < o.device;
            if (log_n != o.log_n) return log_n < o.log_n;
            if (q != o.q) return q < o.q;
            return r < o.r;
        }
    };
};

// ---------------------------------------------------------------------------
// Staging: pinned host buffer + device buffer of `words` u64.  A host-buffer
// integration gathers a DCRTPoly's towers (separate std::vectors in the
// reference, dcrtpoly.h:421) into it, uploads once, runs one launch over all
// towers, and scatters the result back.
// ---------------------------------------------------------------------------
class Staging {
public:
    Staging(HipManager* m, size_t words) : m_(m), dev_(m, words), n_(words) {
        void* h = nullptr;
        check(ofhe_hip_host_alloc(m_->ctx(), words * sizeof(uint64_t), &h), "Staging");
        host_ = static_cast<uint64_t*>(h);
        for (auto& e : ev_) check(ofhe_hip_event_create(m_->ctx(), &e), "Staging");
    }
    ~Staging() {
        if (host_) {
            (void)ofhe_hip_sync(m_->ctx(), nullptr);
            (void)ofhe_hip_host_free(m_->ctx(), host_);
        }
        for (auto& e : ev_)
            if (e) (void)ofhe_hip_event_destroy(e);
    }
    Staging(const Staging&) = delete;
    Staging& operator=(const Staging&) = delete;
    uint64_t* host() const { return host_; }
    uint64_t* dev() const { return dev_.get(); }
    size_t words() const { return n_; }
    // towers[t] points at n words (one PolyImpl's values); they land at t*n
    void gather(const std::vector<const uint64_t*>& towers, size_t n) {
        if (towers.size() * n > n_) throw math_error("Staging::gather: more words than the buffer holds");
        for (size_t t = 0; t < towers.size(); t++) std::memcpy(host_ + t * n, towers[t], n * sizeof(uint64_t));
    }
    void scatter(const std::vector<uint64_t*>& towers, size_t n) const {
        if (towers.size() * n > n_) throw math_error("Staging::scatter: more words than the buffer holds");
        for (size_t t = 0; t < towers.size(); t++) std::memcpy(towers[t], host_ + t * n, n * sizeof(uint64_t));
    }
    // pinned memory: DMA straight from / to the staging buffer
    // the first `words` words (default: all) each way
    void upload(size_t words = SIZE_MAX) {
        check(ofhe_hip_copy_to_device(m_->ctx(), dev(), host_, std::min(words, n_) * 8, nullptr), "Staging::upload");
    }
    void download(size_t words = SIZE_MAX) {
        check(ofhe_hip_copy_to_host(m_->ctx(), host_, dev(), std::min(words, n_) * 8, nullptr), "Staging::download");
        m_->sync();
    }

    // gather + upload, pipelined: towers go in chunks of ~kChunkBytes, each
    // chunk's host copies (one tower per OpenMP thread when the caller builds
    // with OpenMP, as OpenFHE does) run while the previous chunk's DMA is in
    // flight.  Chunks land in disjoint parts of the pinned buffer, and every
    // hook ends in get_towers' wait, so no chunk overwrites a buffer a DMA
    // still reads.  Tower t lands at word t * n of the device buffer.
    void put_towers(const std::vector<const uint64_t*>& towers, size_t n) {
        if (towers.size() * n > n_) throw math_error("Staging::put_towers: more words than the buffer holds");
        const size_t per = chunk_towers(n), T = towers.size();
        for (size_t t0 = 0; t0 < T; t0 += per) {
            const size_t t1 = std::min(T, t0 + per);
            copy_towers(t0, t1, [&](size_t t) { std::memcpy(host_ + t * n, towers[t], n * 8); });
            check(ofhe_hip_copy_to_device(m_->ctx(), dev() + t0 * n, host_ + t0 * n, (t1 - t0) * n * 8, nullptr),
                  "Staging::put_towers");
        }
    }
    // download + scatter, pipelined the other way: every chunk's DMA is
    // queued (in stream order, after the launch that produces it), and chunk
    // k is scattered once its event fires while chunk k + 1 is in flight.
    // Returns with every word in place (the reference's synchronous
    // copy_from_pim, PimManager.cpp:39-54).
    void get_towers(const std::vector<uint64_t*>& towers, size_t n) {
        if (towers.size() * n > n_) throw math_error("Staging::get_towers: more words than the buffer holds");
        const size_t per = chunk_towers(n), T = towers.size();
        size_t prev0 = 0, prev1 = 0, k = 0;
        auto scatter_chunk = [&](size_t a, size_t b, int e) {
            check(ofhe_hip_event_sync(ev_[e]), "Staging::get_towers");
            copy_towers(a, b, [&](size_t t) { std::memcpy(towers[t], host_ + t * n, n * 8); });
        };
        for (size_t t0 = 0; t0 < T; t0 += per, k++) {
            const size_t t1 = std::min(T, t0 + per);
            check(ofhe_hip_copy_to_host(m_->ctx(), host_ + t0 * n, dev() + t0 * n, (t1 - t0) * n * 8, nullptr),
                  "Staging::get_towers");
            check(ofhe_hip_event_record(ev_[k & 1], nullptr), "Staging::get_towers");
            if (k) scatter_chunk(prev0, prev1, (int)((k - 1) & 1));
            prev0 = t0, prev1 = t1;
        }
        if (k) scatter_chunk(prev0, prev1, (int)((k - 1) & 1));
    }

private:
    static constexpr size_t kChunkBytes = size_t(8) << 20;
    static size_t chunk_towers(size_t n) { return std::max<size_t>(1, kChunkBytes / (n * 8)); }
    template <class F>
    static void copy_towers(size_t t0, size_t t1, F f) {
#ifdef _OPENMP
#pragma omp parallel for schedule(static) if (t1 - t0 > 1)
#endif
        for (size_t t = t0; t < t1; t++) f(t);
    }
    HipManager* m_;
    DeviceBuffer dev_;
    size_t n_;
    uint64_t* host_ = nullptr;
    ofhe_event_t ev_[2] = {nullptr, nullptr};
};

// ---------------------------------------------------------------------------
// Parameters: (cyclotomic order, moduli, roots) as ILDCRTParams; the NTT plan
// comes from PlanCache, so parameter objects over the same basis share it.
// ---------------------------------------------------------------------------
class DCRTParams {
public:
    DCRTParams(uint32_t cyclotomic_order, std::vector<uint64_t> moduli, std::vector<uint64_t> roots,
               int device = 0)
        : m_(cyclotomic_order), q_(std::move(moduli)), r_(std::move(roots)), mgr_(HipManager::getHip(device)) {
        if (m_ < 4 || (m_ & (m_ - 1))) throw math_error("CyclotomicOrder is not a power of two");
        if (q_.size() != r_.size() || q_.empty()) throw math_error("moduli/roots size mismatch");
        uint32_t n = m_ / 2, lg = 0;
        while ((1u << lg) < n) lg++;
        log_n_ = lg;
        plan_ = PlanCache::get(device, log_n_, q_, r_);
    }
    DCRTParams(const DCRTParams&) = delete;
    DCRTParams& operator=(const DCRTParams&) = delete;
    uint32_t GetCyclotomicOrder() const { return m_; }
    uint32_t GetRingDimension() const { return m_ / 2; }
    uint32_t LogN() const { return log_n_; }
    size_t Towers() const { return q_.size(); }
    const std::vector<uint64_t>& Moduli() const { return q_; }
    const std::vector<uint64_t>& Roots() const { return r_; }
    ofhe_plan_t plan() const { return plan_->get(); }
    HipManager* manager() const { return mgr_; }

private:
    uint32_t m_, log_n_ = 0;
    std::vector<uint64_t> q_, r_;
    HipManager* mgr_;
    std::shared_ptr<PlanHandle> plan_;
};

enum class Format { EVALUATION = 0, COEFFICIENT = 1 };

// ---------------------------------------------------------------------------
// DCRTPolyHip: `batch` DCRT polynomials resident on one device.  With one
// tower it is also the PimData op set (PimData.h:46-168: + - * and
// ModAdd/ModSub/ModMul with vector or scalar right-hand sides).
// ---------------------------------------------------------------------------
class DCRTPolyHip {
public:
    DCRTPolyHip(std::shared_ptr<DCRTParams> p, Format f, uint32_t batch = 1)
        : p_(std::move(p)), f_(f), batch_(batch),
          buf_(p_->manager(), (size_t)batch * p_->Towers() * p_->GetRingDimension()) {
        buf_.zero();
    }
    // a result buffer the producing op overwrites entirely: no zero fill
    struct Uninit {};
    DCRTPolyHip(std::shared_ptr<DCRTParams> p, Format f, uint32_t batch, Uninit)
        : p_(std::move(p)), f_(f), batch_(batch),
          buf_(p_->manager(), (size_t)batch * p_->Towers() * p_->GetRingDimension()) {}
    DCRTPolyHip(const DCRTPolyHip& o) : p_(o.p_), f_(o.f_), batch_(o.batch_), buf_(o.p_->manager(), o.buf_.size()) {
        buf_.copy_from(o.buf_);
    }
    DCRTPolyHip(DCRTPolyHip&&) = default;
    DCRTPolyHip& operator=(DCRTPolyHip&&) = default;

    const std::shared_ptr<DCRTParams>& GetParams() const { return p_; }
    Format GetFormat() const { return f_; }
    uint32_t Batch() const { return batch_; }
    uint64_t* data() const { return buf_.get(); }
    size_t words() const { return buf_.size(); }

    // values[b][t][i] flattened; must be canonical (< q_t)
    void SetValues(const std::vector<uint64_t>& flat, Format f) {
        if (flat.size() != buf_.size()) throw math_error("SetValues: size mismatch");
        buf_.upload(flat.data());
        f_ = f;
    }
    std::vector<uint64_t> GetValues() const {
        std::vector<uint64_t> h(buf_.size());
        buf_.download(h.data());
        return h;
    }
    // tower t of batch entry b (GetElementAtIndex(t) analogue)
    std::vector<uint64_t> GetElementAtIndex(size_t t, uint32_t b = 0) const {
        auto all = GetValues();
        const size_t n = p_->GetRingDimension();
        const size_t off = ((size_t)b * p_->Towers() + t) * n;
        return std::vector<uint64_t>(all.begin() + off, all.begin() + off + n);
    }

    // SwitchFormat (dcrtpoly-impl.h:2518-2524 -> poly-impl.h:412-432)
    void SwitchFormat() {
        if (f_ == Format::COEFFICIENT) {
            check(ofhe_hip_ntt_fwd(p_->plan(), data(), batch_, nullptr), "SwitchFormat");
            f_ = Format::EVALUATION;
        } else {
            check(ofhe_hip_ntt_inv(p_->plan(), data(), batch_, nullptr), "SwitchFormat");
            f_ = Format::COEFFICIENT;
        }
    }
    void SetFormat(Format f) {
        if (f != f_) SwitchFormat();
    }

    DCRTPolyHip Plus(const DCRTPolyHip& rhs) const {
        check_compat(rhs, "Plus", false);
        DCRTPolyHip r(p_, f_, batch_, Uninit{});
        check(ofhe_hip_modadd_vv(p_->plan(), data(), rhs.data(), r.data(), batch_, nullptr), "Plus");
        return r;
    }
    DCRTPolyHip Minus(const DCRTPolyHip& rhs) const {
        check_compat(rhs, "Minus", false);
        DCRTPolyHip r(p_, f_, batch_, Uninit{});
        check(ofhe_hip_modsub_vv(p_->plan(), data(), rhs.data(), r.data(), batch_, nullptr), "Minus");
        return r;
    }
    // Times (dcrtpoly.h:185-200): EVALUATION format only
    DCRTPolyHip Times(const DCRTPolyHip& rhs) const {
        check_compat(rhs, "Times", true);
        DCRTPolyHip r(p_, f_, batch_, Uninit{});
        check(ofhe_hip_modmul_vv(p_->plan(), data(), rhs.data(), r.data(), batch_, nullptr), "Times");
        return r;
    }
    // DropLastElementAndScale (dcrtpoly-impl.h:746-768; CKKS / BFV rescaling):
    // one tower fewer, on the params of the shorter chain.  The reference keeps
    // m_format while its coefficient-form towers come back in evaluation form
    // (lines 765-766); here the format tag follows the data (EVALUATION).
    void DropLastElementAndScale(const std::vector<uint64_t>& QlQlInvModqlDivqlModq,
                                 const std::vector<uint64_t>& qlInvModq) {
        const size_t T = p_->Towers(), n = p_->GetRingDimension();
        if (QlQlInvModqlDivqlModq.size() + 1 < T || qlInvModq.size() + 1 < T)
            throw math_error("DropLastElementAndScale: one constant per remaining tower required");
        auto lp = lower_params();
        DCRTPolyHip r(lp, Format::EVALUATION, batch_, Uninit{});
        check(ofhe_hip_drop_last_and_scale(p_->plan(), (uint32_t)T, data(), T * n, r.data(), (T - 1) * n,
                                           f_ == Format::EVALUATION, QlQlInvModqlDivqlModq.data(), qlInvModq.data(),
                                           batch_, nullptr),
              "DropLastElementAndScale");
        *this = std::move(r);
    }
    // ModReduce (dcrtpoly-impl.h:792-812; BGV modulus switching): one tower
    // fewer, format unchanged
    void ModReduce(uint64_t t, uint64_t negtInvModq, const std::vector<uint64_t>& qlInvModq) {
        const size_t T = p_->Towers(), n = p_->GetRingDimension();
        if (qlInvModq.size() + 1 < T) throw math_error("ModReduce: one constant per remaining tower required");
        auto lp = lower_params();
        DCRTPolyHip r(lp, f_, batch_, Uninit{});
        check(ofhe_hip_mod_reduce(p_->plan(), (uint32_t)T, data(), T * n, r.data(), (T - 1) * n,
                                  f_ == Format::EVALUATION, t, negtInvModq, qlInvModq.data(), batch_, nullptr),
              "ModReduce");
        *this = std::move(r);
    }

    // Times(const std::vector<NativeInteger>&): one scalar per tower (Shoup)
    DCRTPolyHip Times(const std::vector<uint64_t>& scalars) const {
        if (scalars.size() != p_->Towers()) throw math_error("Times: one scalar per tower required");
        DCRTPolyHip r(p_, f_, batch_, Uninit{});
        check(ofhe_hip_modmul_scalar(p_->plan(), data(), scalars.data(), r.data(), batch_, nullptr), "Times");
        return r;
    }
    // Plus / Minus with one integer per tower (dcrtpoly.h:162-163, 182-183;
    // dcrtpoly-impl.h:545-584).  PolyImpl::Plus(Integer) adds the constant
    // polynomial: in COEFFICIENT form only coefficient 0 changes
    // (ModAddAtIndex(0), poly-impl.h:213-220), in EVALUATION form every slot;
    // PolyImpl::Minus(Integer) subtracts from every word in either form
    // (poly-impl.h:223-227), as the reference does.
    DCRTPolyHip Plus(const std::vector<uint64_t>& crt) const {
        if (crt.size() != p_->Towers()) throw math_error("Plus: one integer per tower required");
        DCRTPolyHip r(*this);
        if (f_ == Format::COEFFICIENT)
            check(ofhe_hip_modadd_scalar_at(p_->plan(), r.data(), 0, crt.data(), r.data(), batch_, nullptr), "Plus");
        else
            check(ofhe_hip_modadd_scalar(p_->plan(), data(), crt.data(), r.data(), batch_, nullptr), "Plus");
        return r;
    }
    DCRTPolyHip Minus(const std::vector<uint64_t>& crt) const {
        if (crt.size() != p_->Towers()) throw math_error("Minus: one integer per tower required");
        DCRTPolyHip r(p_, f_, batch_, Uninit{});
        check(ofhe_hip_modsub_scalar(p_->plan(), data(), crt.data(), r.data(), batch_, nullptr), "Minus");
        return r;
    }
    // Plus / Minus(const Integer&): the same integer in every tower
    DCRTPolyHip Plus(uint64_t v) const { return Plus(std::vector<uint64_t>(p_->Towers(), v)); }
    DCRTPolyHip Minus(uint64_t v) const { return Minus(std::vector<uint64_t>(p_->Towers(), v)); }
    DCRTPolyHip& operator+=(const DCRTPolyHip& rhs) {
        check_compat(rhs, "operator+=", false);
        check(ofhe_hip_modadd_vv(p_->plan(), data(), rhs.data(), data(), batch_, nullptr), "operator+=");
        return *this;
    }
    DCRTPolyHip& operator-=(const DCRTPolyHip& rhs) {
        check_compat(rhs, "operator-=", false);
        check(ofhe_hip_modsub_vv(p_->plan(), data(), rhs.data(), data(), batch_, nullptr), "operator-=");
        return *this;
    }
    DCRTPolyHip& operator*=(const DCRTPolyHip& rhs) {
        check_compat(rhs, "operator*=", true);
        check(ofhe_hip_modmul_vv(p_->plan(), data(), rhs.data(), data(), batch_, nullptr), "operator*=");
        return *this;
    }
    DCRTPolyHip operator+(const DCRTPolyHip& rhs) const { return Plus(rhs); }
    DCRTPolyHip operator-(const DCRTPolyHip& rhs) const { return Minus(rhs); }
    DCRTPolyHip operator*(const DCRTPolyHip& rhs) const { return Times(rhs); }

    // c = INTT(NTT(this) (.) rhs): this in COEFFICIENT, rhs in EVALUATION; the
    // result is COEFFICIENT.  Equal to SwitchFormat; *= rhs; SwitchFormat.
    DCRTPolyHip MulViaNTT(const DCRTPolyHip& rhs) const {
        if (f_ != Format::COEFFICIENT || rhs.f_ != Format::EVALUATION)
            throw not_implemented_error("MulViaNTT: needs COEFFICIENT x EVALUATION");
        check_compat(rhs, "MulViaNTT", false, false);
        DCRTPolyHip r(p_, Format::COEFFICIENT, batch_, Uninit{});
        check(ofhe_hip_ntt_mul_intt(p_->plan(), data(), rhs.data(), r.data(), batch_, nullptr), "MulViaNTT");
        return r;
    }

    // AutomorphismTransform(k) (dcrtpoly-impl.h:350-358 -> poly-impl.h:312-365)
    DCRTPolyHip AutomorphismTransform(uint32_t k) const {
        DCRTPolyHip r(p_, f_, batch_, Uninit{});
        check(ofhe_hip_automorphism(p_->plan(), k, f_ == Format::EVALUATION, data(), r.data(), batch_, nullptr),
              "AutomorphismTransform");
        return r;
    }

    bool operator==(const DCRTPolyHip& o) const {
        return f_ == o.f_ && p_->Moduli() == o.p_->Moduli() && GetValues() == o.GetValues();
    }

    // Serialization in the reference's field order, one DCRTPoly record per
    // batch entry:
    //   DCRTPolyImpl::save (dcrtpoly.h:349-354): "v" towers, "f" format, "p" params
    //   PolyImpl::save (poly.h:322-327):         "v" values, "f" format, "p" params
    //   NativeVectorT::save, binary (mubintvecnat.h:665-674): size_type count, the
    //     words as binary_data, then the modulus (one NativeInteger word)
    //   ElemParams::save (elemparams.h:224-231): "co", "rd", "cm", "ru"
    //   ILDCRTParams::save (ildcrtparams.h:351-355): its ElemParams, then "p" the
    //     per-tower ILNativeParams
    // Little-endian, with cereal's binary conventions for what the reference
    // writes itself: a uint64 size_type before every vector, enums as uint32
    // (Format, utils/inttypes.h:65).  Not written: cereal's own framing
    // (class-version words, shared_ptr ids, the polymorphic params' type
    // names) and the BigInteger fields ("bm", "br", ILDCRTParams' "m"); cereal
    // is an empty submodule in the reference snapshot, so its byte stream is
    // not reproduced or pinned here.
    void Save(std::ostream& os) const {
        const auto h = GetValues();
        const size_t T = p_->Towers(), n = p_->GetRingDimension();
        const uint32_t co = p_->GetCyclotomicOrder(), rd = p_->GetRingDimension();
        for (uint32_t b = 0; b < batch_; b++) {
            put<uint64_t>(os, T);
            for (size_t t = 0; t < T; t++) {
                put<uint64_t>(os, n);
                os.write(reinterpret_cast<const char*>(h.data() + ((size_t)b * T + t) * n), n * 8);
                put<uint64_t>(os, p_->Moduli()[t]);
                put<uint32_t>(os, (uint32_t)f_);
                put_native_params(os, co, rd, p_->Moduli()[t], p_->Roots()[t]);
            }
            put<uint32_t>(os, (uint32_t)f_);
            put<uint32_t>(os, co);
            put<uint32_t>(os, rd);
            put<uint64_t>(os, T);
            for (size_t t = 0; t < T; t++) put_native_params(os, co, rd, p_->Moduli()[t], p_->Roots()[t]);
        }
        if (!os) throw math_error("DCRTPolyHip::Save: stream write failed");
    }
    // The inverse of Save for `batch` consecutive records; every record must
    // carry the same basis and format, and every value must be <= its modulus.
    static DCRTPolyHip Load(std::istream& is, uint32_t batch = 1, int device = 0) {
        if (batch == 0) throw deserialize_error("DCRTPolyHip::Load: batch must be >= 1");
        std::vector<uint64_t> flat, q0, r0;
        uint32_t co0 = 0, f0 = 0;
        for (uint32_t b = 0; b < batch; b++) {
            const uint64_t T = get<uint64_t>(is);
            if (T < 1 || T > 4096) throw deserialize_error("DCRTPolyHip::Load: tower count out of range");
            std::vector<uint64_t> q(T), r(T), vals;
            uint32_t co = 0, f = 0;
            for (uint64_t t = 0; t < T; t++) {
                const uint64_t n = get<uint64_t>(is);
                if (n < 2 || n > (1u << 17) || (n & (n - 1))) throw deserialize_error("DCRTPolyHip::Load: ring dimension");
                const size_t off = vals.size();
                vals.resize(off + n);
                is.read(reinterpret_cast<char*>(vals.data() + off), n * 8);
                const uint64_t m = get<uint64_t>(is);
                const uint32_t tf = get<uint32_t>(is);
                uint32_t tco, trd;
                uint64_t tq, tr;
                get_native_params(is, tco, trd, tq, tr);
                if (tq != m || trd != n || tco != 2 * n) throw deserialize_error("DCRTPolyHip::Load: tower params disagree");
                if (t == 0) co = tco, f = tf;
                if (tco != co || tf != f) throw deserialize_error("DCRTPolyHip::Load: towers of different rings / formats");
                // NativeVectorT::load (mubintvecnat.h:684-702) takes the words as
                // they are; the library itself writes the representative q (a
                // negated zero of a coefficient-form AutomorphismTransform), so
                // words <= m load unchanged and Save -> Load round-trips every
                // library output.  Larger words are refused: the device kernels'
                // lazy bounds assume inputs below 2q.
                for (size_t i = off; i < off + n; i++)
                    if (vals[i] > m) throw deserialize_error("DCRTPolyHip::Load: value above its modulus");
                q[t] = m;
                r[t] = tr;
            }
            const uint32_t pf = get<uint32_t>(is), pco = get<uint32_t>(is), prd = get<uint32_t>(is);
            const uint64_t pT = get<uint64_t>(is);
            if (pf != f || pco != co || prd != co / 2 || pT != T) throw deserialize_error("DCRTPolyHip::Load: params disagree");
            for (uint64_t t = 0; t < T; t++) {
                uint32_t tco, trd;
                uint64_t tq, tr;
                get_native_params(is, tco, trd, tq, tr);
                if (tco != co || tq != q[t] || tr != r[t]) throw deserialize_error("DCRTPolyHip::Load: params disagree");
            }
            if (f > 1) throw deserialize_error("DCRTPolyHip::Load: unknown format");
            if (b == 0) q0 = q, r0 = r, co0 = co, f0 = f;
            if (q != q0 || r != r0 || co != co0 || f != f0)
                throw deserialize_error("DCRTPolyHip::Load: batch entries over different bases / formats");
            flat.insert(flat.end(), vals.begin(), vals.end());
        }
        auto P = std::make_shared<DCRTParams>(co0, q0, r0, device);
        DCRTPolyHip x(P, (Format)f0, batch, Uninit{});
        x.SetValues(flat, (Format)f0);
        return x;
    }

private:
    template <class T>
    static void put(std::ostream& os, T v) {
        os.write(reinterpret_cast<const char*>(&v), sizeof v);  // little-endian host (x86-64)
    }
    template <class T>
    static T get(std::istream& is) {
        T v{};
        if (!is.read(reinterpret_cast<char*>(&v), sizeof v)) throw deserialize_error("DCRTPolyHip::Load: truncated stream");
        return v;
    }
    // ILNativeParams = ElemParams' "co", "rd", "cm" (the tower modulus), "ru"
    static void put_native_params(std::ostream& os, uint32_t co, uint32_t rd, uint64_t q, uint64_t r) {
        put<uint32_t>(os, co);
        put<uint32_t>(os, rd);
        put<uint64_t>(os, q);
        put<uint64_t>(os, r);
    }
    static void get_native_params(std::istream& is, uint32_t& co, uint32_t& rd, uint64_t& q, uint64_t& r) {
        co = get<uint32_t>(is);
        rd = get<uint32_t>(is);
        q = get<uint64_t>(is);
        r = get<uint64_t>(is);
    }
    // DropLastElement (dcrtpoly-impl.h:719-728): the params of the chain
    // without its last tower (a cached plan of that basis)
    std::shared_ptr<DCRTParams> lower_params() const {
        if (p_->Towers() < 2) throw math_error("Removing last element of DCRTPoly object renders it invalid!");
        std::vector<uint64_t> q(p_->Moduli().begin(), p_->Moduli().end() - 1);
        std::vector<uint64_t> r(p_->Roots().begin(), p_->Roots().end() - 1);
        return std::make_shared<DCRTParams>(p_->GetCyclotomicOrder(), q, r, p_->manager()->device());
    }

    void check_compat(const DCRTPolyHip& rhs, const char* op, bool eval_only, bool same_format = true) const {
        if (p_->GetRingDimension() != rhs.p_->GetRingDimension())
            throw math_error(std::string(op) + ": RingDimension missmatch");
        if (same_format && f_ != rhs.f_) throw not_implemented_error(std::string(op) + ": Format missmatch");
        if (eval_only && (f_ != Format::EVALUATION || rhs.f_ != Format::EVALUATION))
            throw not_implemented_error(std::string(op) + " for DCRTPolyHip supported only in Format::EVALUATION");
        if (p_->Towers() != rhs.p_->Towers()) throw math_error(std::string(op) + ": tower size mismatch");
        if (p_->Moduli() != rhs.p_->Moduli()) throw math_error(std::string(op) + ": Modulus missmatch");
        if (batch_ != rhs.batch_) throw math_error(std::string(op) + ": batch mismatch");
    }

    std::shared_ptr<DCRTParams> p_;
    Format f_;
    uint32_t batch_;
    DeviceBuffer buf_;
};

// ---------------------------------------------------------------------------
// ApproxSwitchCRTBasis (dcrtpoly-impl.h:1034-1063): x over basis Q (params of
// x) -> basis P (paramsP), both COEFFICIENT form.
// ---------------------------------------------------------------------------
class BaseConverter {
public:
    BaseConverter(const DCRTParams& Q, const DCRTParams& P, const std::vector<uint64_t>& QHatInvModq,
                  const std::vector<uint64_t>& QHatModp /* [sizeQ][sizeP] */) {
        check(ofhe_hip_bconv_create(Q.manager()->ctx(), Q.LogN(), (uint32_t)Q.Towers(), (uint32_t)P.Towers(),
                                    Q.Moduli().data(), P.Moduli().data(), QHatInvModq.data(), QHatModp.data(), &h_),
              "BaseConverter");
    }
    ~BaseConverter() {
        if (h_) ofhe_hip_bconv_destroy(h_);
    }
    BaseConverter(const BaseConverter&) = delete;
    BaseConverter& operator=(const BaseConverter&) = delete;
    DCRTPolyHip ApproxSwitchCRTBasis(const DCRTPolyHip& x, const std::shared_ptr<DCRTParams>& paramsP) const {
        if (x.GetFormat() != Format::COEFFICIENT) throw math_error("ApproxSwitchCRTBasis: COEFFICIENT form expected");
        DCRTPolyHip out(paramsP, Format::COEFFICIENT, x.Batch(), DCRTPolyHip::Uninit{});
        check(ofhe_hip_approx_switch_crt_basis(h_, x.data(), out.data(), x.Batch(), nullptr), "ApproxSwitchCRTBasis");
        return out;
    }

    ofhe_bconv_t handle() const { return h_; }

private:
    ofhe_bconv_t h_ = nullptr;
};

// ApproxModUp (dcrtpoly-impl.h:1085-1131): x over Q (either format) -> a
// polynomial over paramsQP = Q|P in EVALUATION form.  q_to_p converts Q -> P.
inline DCRTPolyHip ApproxModUp(const DCRTPolyHip& x, const std::shared_ptr<DCRTParams>& paramsP,
                               const std::shared_ptr<DCRTParams>& paramsQP, const BaseConverter& q_to_p) {
    const auto& Q = x.GetParams();
    if (paramsQP->Towers() != Q->Towers() + paramsP->Towers()) throw math_error("ApproxModUp: paramsQP size");
    DCRTPolyHip out(paramsQP, Format::EVALUATION, x.Batch(), DCRTPolyHip::Uninit{});
    check(ofhe_hip_approx_mod_up(Q->plan(), paramsP->plan(), q_to_p.handle(), x.GetFormat() == Format::EVALUATION,
                                 x.data(), out.data(), x.Batch(), nullptr),
          "ApproxModUp");
    return out;
}

// ApproxModDown (dcrtpoly-impl.h:1134-1175): x over Q|P (EVALUATION) -> Q.
inline DCRTPolyHip ApproxModDown(const DCRTPolyHip& x, const std::shared_ptr<DCRTParams>& paramsQ,
                                 const std::shared_ptr<DCRTParams>& paramsP, const BaseConverter& p_to_q,
                                 const std::vector<uint64_t>& PInvModq, uint64_t t = 0) {
    if (x.GetFormat() != Format::EVALUATION) throw math_error("ApproxModDown: EVALUATION form expected");
    if (x.GetParams()->Towers() != paramsQ->Towers() + paramsP->Towers())
        throw math_error("ApproxModDown: tower count mismatch");
    if (PInvModq.size() != paramsQ->Towers()) throw math_error("ApproxModDown: PInvModq size");
    DCRTPolyHip out(paramsQ, Format::EVALUATION, x.Batch(), DCRTPolyHip::Uninit{});
    check(ofhe_hip_approx_mod_down(paramsQ->plan(), paramsP->plan(), p_to_q.handle(), PInvModq.data(), t, x.data(),
                                   out.data(), x.Batch(), nullptr),
          "ApproxModDown");
    return out;
}

// KeySwitchHYBRID (pke/lib/keyswitch/keyswitch-hybrid.cpp) for one parameter
// set: Q (element params), P (GetParamsP()) and dnum = numPartQ.  An
// evaluation key is a pair of DCRTPolyHip over Q|P with batch = numPartQ
// (the b and a vectors of EvalKeyRelin).
class KeySwitchHybrid {
public:
    KeySwitchHybrid(const DCRTParams& Q, const DCRTParams& P, uint32_t numPartQ) {
        check(ofhe_hip_ks_create(Q.manager()->ctx(), Q.LogN(), (uint32_t)Q.Towers(), Q.Moduli().data(),
                                 Q.Roots().data(), (uint32_t)P.Towers(), P.Moduli().data(), P.Roots().data(), numPartQ,
                                 &h_),
              "KeySwitchHybrid");
        sizeQ_ = Q.Towers();
        sizeP_ = P.Towers();
        numPartQ_ = numPartQ;
    }
    ~KeySwitchHybrid() {
        if (h_) ofhe_hip_ks_destroy(h_);
    }
    KeySwitchHybrid(const KeySwitchHybrid&) = delete;
    KeySwitchHybrid& operator=(const KeySwitchHybrid&) = delete;

    // KeySwitchCore(a, evalKey) (keyswitch-hybrid.cpp:325-328): c is over Ql
    // (its params give the level), EVALUATION form.  t > 0 for BGV.
    std::pair<DCRTPolyHip, DCRTPolyHip> KeySwitchCore(const DCRTPolyHip& c, const DCRTPolyHip& key_b,
                                                      const DCRTPolyHip& key_a, uint64_t t = 0) const {
        if (c.GetFormat() != Format::EVALUATION) throw math_error("KeySwitchCore: EVALUATION form expected");
        const uint32_t l = (uint32_t)c.GetParams()->Towers();
        if (l > sizeQ_) throw math_error("KeySwitchCore: ciphertext has more towers than Q");
        if (key_b.Batch() != numPartQ_ || key_a.Batch() != numPartQ_ ||
            key_b.GetParams()->Towers() != sizeQ_ + sizeP_ || key_a.GetParams()->Towers() != sizeQ_ + sizeP_)
            throw math_error("KeySwitchCore: evaluation key must be numPartQ polynomials over Q|P");
        DCRTPolyHip o0(c.GetParams(), Format::EVALUATION, c.Batch(), DCRTPolyHip::Uninit{}),
            o1(c.GetParams(), Format::EVALUATION, c.Batch(), DCRTPolyHip::Uninit{});
        check(ofhe_hip_ks_core(h_, l, c.data(), key_b.data(), key_a.data(), o0.data(), o1.data(), t, c.Batch(),
                               nullptr),
              "KeySwitchCore");
        return {std::move(o0), std::move(o1)};
    }

    ofhe_ks_t handle() const { return h_; }

private:
    ofhe_ks_t h_ = nullptr;
    size_t sizeQ_ = 0, sizeP_ = 0;
    uint32_t numPartQ_ = 0;
};

// KsCache: one KeySwitchHybrid per (device, N, Q, P, dnum) -- the reference
// precomputes its HYBRID CRT tables once per CryptoParametersRNS
// (rns-cryptoparameters.cpp:72-345).
class KsCache {
public:
    static std::shared_ptr<KeySwitchHybrid> get(const DCRTParams& Q, const DCRTParams& P, uint32_t numPartQ) {
        static std::mutex mu;
        static std::map<std::vector<uint64_t>, std::shared_ptr<KeySwitchHybrid>> cache;
        std::vector<uint64_t> key{(uint64_t)Q.manager()->device(), Q.LogN(), numPartQ, Q.Towers()};
        key.insert(key.end(), Q.Moduli().begin(), Q.Moduli().end());
        key.insert(key.end(), P.Moduli().begin(), P.Moduli().end());
        std::lock_guard<std::mutex> lk(mu);
        auto& e = cache[key];
        if (!e) e = std::make_shared<KeySwitchHybrid>(Q, P, numPartQ);
        return e;
    }
};

// KeyCache: evaluation keys resident on the device, uploaded once per key
// (when EvalMultKeyGen / EvalAtIndexKeyGen store them) and looked up by the
// caller's key id (e.g. the EvalKey's tag) at every key switch.
class KeyCache {
public:
    struct Key {
        DCRTPolyHip b, a;  // numPartQ polynomials over Q|P each (EvalKeyRelin's b and a vectors)
    };
    static std::shared_ptr<const Key> put(const std::string& id, DCRTPolyHip b, DCRTPolyHip a) {
        auto k = std::make_shared<const Key>(Key{std::move(b), std::move(a)});
        std::lock_guard<std::mutex> lk(mu());
        map()[id] = k;
        return k;
    }
    static std::shared_ptr<const Key> get(const std::string& id) {
        std::lock_guard<std::mutex> lk(mu());
        auto it = map().find(id);
        if (it == map().end()) throw math_error("KeyCache: no evaluation key '" + id + "'");
        return it->second;
    }
    static void erase(const std::string& id) {
        std::lock_guard<std::mutex> lk(mu());
        map().erase(id);
    }

private:
    static std::mutex& mu() {
        static std::mutex m;
        return m;
    }
    static std::map<std::string, std::shared_ptr<const Key>>& map() {
        static std::map<std::string, std::shared_ptr<const Key>> m;
        return m;
    }
};

}  // namespace ofhe
