// A test double of the reference's tower types, written to the reference's
// accessor names, with the RUN_ON_HIP hooks inserted exactly where
// INTEGRATION.md §3 puts them and the reference's own CPU loops (OpenMP over
// the towers, as dcrtpoly-impl.h runs them) as the fallback when a hook
// declines.  The CPU loops run on the C oracle (oracle/libofhe_oracle.so):
// test infrastructure, the checker and the stand-in for the reference's
// native backend, which cannot be built here.
//
// Names and shapes followed (not copied):
//   PolyImpl::GetParams() / operator[] / GetFormat / OverrideFormat   poly.h:114-119,179,209-215
//   ILNativeParams::GetModulus / GetRootOfUnity / GetRingDimension   ilparams.h, elemparams.h
//   NativeIntegerT: one uint64_t m_value, ConvertToInt()             ubintnat.h:139-141,1659
//   DCRTPolyImpl::m_vectors and the members below                    dcrtpoly.h:142-200,421;
//                                                                     dcrtpoly-impl.h:349-357,410-416,
//                                                                     565-661,1034-1175,2516-2523
//   KeySwitchHYBRID::KeySwitchCore and its three stages                keyswitch-hybrid.cpp:324-482
#pragma once
#include <omp.h>

#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#include "../../upmem--openfhe_amd/host/ofhe_openfhe_hooks.hpp"

extern "C" {
int oracle_moduli_chain(unsigned bits, uint64_t cyclo_order, unsigned count, uint64_t* q_out, uint64_t* psi_out);
int oracle_ntt_tables(uint64_t n, uint64_t q, uint64_t psi, uint64_t* tab, uint64_t* tab_pre, uint64_t* itab,
                      uint64_t* itab_pre, uint64_t* coi, uint64_t* coi_pre);
void oracle_ntt_fwd(uint64_t* x, uint64_t len, uint64_t q, const uint64_t* tab, const uint64_t* tab_pre);
void oracle_ntt_inv(uint64_t* x, uint64_t n, uint64_t q, const uint64_t* itab, const uint64_t* itab_pre,
                    uint64_t ninv, uint64_t ninv_pre);
void oracle_vec_modmul(const uint64_t* a, const uint64_t* b, uint64_t* c, uint64_t n, uint64_t q);
void oracle_vec_modadd(const uint64_t* a, const uint64_t* b, uint64_t* c, uint64_t n, uint64_t q);
void oracle_vec_modsub(const uint64_t* a, const uint64_t* b, uint64_t* c, uint64_t n, uint64_t q);
void oracle_base_conv_precompute(unsigned sizeQ, unsigned sizeP, const uint64_t* q, const uint64_t* p,
                                 uint64_t* qhatinv_modq, uint64_t* qhatinv_modq_pre, uint64_t* qhat_modp,
                                 uint64_t* mu_lo, uint64_t* mu_hi);
void oracle_approx_switch_crt_basis(const uint64_t* x, uint64_t* out, uint64_t n, unsigned sizeQ, unsigned sizeP,
                                    const uint64_t* q, const uint64_t* p, const uint64_t* qhatinv_modq,
                                    const uint64_t* qhatinv_modq_pre, const uint64_t* qhat_modp,
                                    const uint64_t* mu_lo, const uint64_t* mu_hi);
void oracle_vec_modmul_scalar(const uint64_t* a, uint64_t s, uint64_t* c, uint64_t n, uint64_t q);
void oracle_vec_modsub_scalar(const uint64_t* a, uint64_t s, uint64_t* c, uint64_t n, uint64_t q);
uint64_t oracle_modinv(uint64_t a, uint64_t q);
void oracle_automorphism(const uint64_t* x, uint64_t* out, uint64_t n, uint32_t k, int eval_form, uint64_t q);
}

namespace mock {
enum class Format { EVALUATION = 0, COEFFICIENT = 1 };  // the reference's enumerators (utils/inttypes.h)
struct NativeInteger {                                  // NativeIntegerT<uint64_t>: one word
    uint64_t m_value = 0;
    uint64_t ConvertToInt() const { return m_value; }
};
struct ILNativeParams {
    NativeInteger modulus, root;
    uint32_t ring;
    const NativeInteger& GetModulus() const { return modulus; }
    const NativeInteger& GetRootOfUnity() const { return root; }
    uint32_t GetRingDimension() const { return ring; }
    uint32_t GetCyclotomicOrder() const { return 2 * ring; }  // power-of-two cyclotomic
};

// The reference caches its twiddle tables per modulus (transformnat.h:352-368):
// the CPU loops look them up here, built once per (n, q, psi).
struct NttTables {
    std::vector<uint64_t> tab, tp, it, ip, coi, cp;
    uint32_t log_n = 0;
};
inline const NttTables& tables(uint32_t n, uint64_t q, uint64_t psi) {
    static std::mutex mu;
    static std::map<std::tuple<uint32_t, uint64_t, uint64_t>, std::unique_ptr<NttTables>> cache;
    std::lock_guard<std::mutex> lk(mu);
    auto& e = cache[{n, q, psi}];
    if (!e) {
        e.reset(new NttTables);
        while ((1u << e->log_n) < n) e->log_n++;
        e->tab.resize(n), e->tp.resize(n), e->it.resize(n), e->ip.resize(n);
        e->coi.resize(e->log_n + 1), e->cp.resize(e->log_n + 1);
        oracle_ntt_tables(n, q, psi, e->tab.data(), e->tp.data(), e->it.data(), e->ip.data(), e->coi.data(),
                          e->cp.data());
    }
    return *e;
}
inline void ntt_words(uint64_t* x, uint32_t n, uint64_t q, uint64_t psi, bool fwd) {
    const NttTables& t = tables(n, q, psi);
    if (fwd)
        oracle_ntt_fwd(x, n, q, t.tab.data(), t.tp.data());
    else
        oracle_ntt_inv(x, n, q, t.it.data(), t.ip.data(), t.coi[t.log_n], t.cp[t.log_n]);
}

inline int g_cpu_switches = 0;  // towers transformed by PolyImpl::SwitchFormat (the CPU loop)
struct PolyImpl {
    std::shared_ptr<ILNativeParams> params;
    std::vector<NativeInteger> values;
    Format m_format = Format::COEFFICIENT;
    const std::shared_ptr<ILNativeParams>& GetParams() const { return params; }
    NativeInteger& operator[](uint32_t i) { return values[i]; }
    const NativeInteger& operator[](uint32_t i) const { return values[i]; }
    Format GetFormat() const { return m_format; }
    void OverrideFormat(Format f) { m_format = f; }  // poly.h:179
    uint64_t q() const { return params->modulus.m_value; }
    uint64_t* w() { return reinterpret_cast<uint64_t*>(values.data()); }
    const uint64_t* w() const { return reinterpret_cast<const uint64_t*>(values.data()); }
    uint32_t n() const { return params->ring; }
    // poly-impl.h:412-432, on the oracle
    void SwitchFormat() {
        ntt_words(w(), n(), q(), params->root.m_value, m_format == Format::COEFFICIENT);
        m_format = m_format == Format::COEFFICIENT ? Format::EVALUATION : Format::COEFFICIENT;
#pragma omp atomic
        g_cpu_switches++;
    }
};
using Towers = std::vector<PolyImpl>;

inline uint64_t mulmod(uint64_t a, uint64_t b, uint64_t m) { return (uint64_t)((unsigned __int128)a * b % m); }
inline std::vector<uint64_t> moduli(const Towers& t) {
    std::vector<uint64_t> q;
    for (auto& p : t) q.push_back(p.q());
    return q;
}

// ApproxSwitchCRTBasis on the oracle (its own OpenMP loop over coefficients,
// as dcrtpoly-impl.h:1040-1061), x's towers -> out's towers, with the
// caller's QHatInvModq / QHatModp; the Shoup and Barrett constants derived
// from the moduli (the reference's ...Precon / modpBarrettMu tables)
inline void cpu_switch_basis(const Towers& x, Towers& out, const std::vector<uint64_t>& hinv,
                             const std::vector<uint64_t>& hmod) {
    const auto q = moduli(x), p = moduli(out);
    const unsigned sq = (unsigned)q.size(), sp = (unsigned)p.size();
    std::vector<uint64_t> h0(sq), hpre(sq), hm0(sq * sp), mlo(sp), mhi(sp);
    oracle_base_conv_precompute(sq, sp, q.data(), p.data(), h0.data(), hpre.data(), hm0.data(), mlo.data(), mhi.data());
    for (unsigned i = 0; i < sq; i++) hpre[i] = (uint64_t)(((unsigned __int128)hinv[i] << 64) / q[i]);
    const uint32_t n = x[0].n();
    std::vector<uint64_t> in((size_t)sq * n), o((size_t)sp * n);
    for (unsigned i = 0; i < sq; i++) std::copy(x[i].w(), x[i].w() + n, in.begin() + (size_t)i * n);
    oracle_approx_switch_crt_basis(in.data(), o.data(), n, sq, sp, q.data(), p.data(), hinv.data(), hpre.data(),
                                   hmod.data(), mlo.data(), mhi.data());
    for (unsigned j = 0; j < sp; j++) std::copy(o.begin() + (size_t)j * n, o.begin() + (size_t)(j + 1) * n, out[j].w());
}
// the reference's per-tower OpenMP loop (e.g. dcrtpoly-impl.h:2519-2523)
template <class F>
inline void each_tower(size_t T, F f) {
#pragma omp parallel for schedule(static)
    for (size_t i = 0; i < T; i++) f(i);
}
inline void set_format(Towers& t, Format f) {
    each_tower(t.size(), [&](size_t i) {
        if (t[i].GetFormat() != f) t[i].SwitchFormat();
    });
}

struct DCRTPolyImpl {
    Format m_format = Format::COEFFICIENT;
    Towers m_vectors;

    // dcrtpoly-impl.h:2516-2523 with the hook, as INTEGRATION.md §3 shows it
    void SwitchFormat() {
        m_format = (m_format == Format::COEFFICIENT) ? Format::EVALUATION : Format::COEFFICIENT;
        if (ofhe::hooks::SwitchFormat(m_vectors)) return;
        each_tower(m_vectors.size(), [&](size_t i) { m_vectors[i].SwitchFormat(); });
    }
    // operator*= / += / -= (dcrtpoly.h:142-148, dcrtpoly-impl.h:410-416)
    DCRTPolyImpl& operator*=(const DCRTPolyImpl& rhs) {
        if (!ofhe::hooks::TimesEq(m_vectors, rhs.m_vectors)) binary(rhs, oracle_vec_modmul);
        return *this;
    }
    DCRTPolyImpl& operator+=(const DCRTPolyImpl& rhs) {
        if (!ofhe::hooks::PlusEq(m_vectors, rhs.m_vectors)) binary(rhs, oracle_vec_modadd);
        return *this;
    }
    DCRTPolyImpl& operator-=(const DCRTPolyImpl& rhs) {
        if (!ofhe::hooks::MinusEq(m_vectors, rhs.m_vectors)) binary(rhs, oracle_vec_modsub);
        return *this;
    }
    // operator*=(std::vector<NativeInteger>) / Minus(std::vector<Integer>) in place (dcrtpoly-impl.h:565-661)
    void TimesScalarEq(const std::vector<uint64_t>& s) {
        if (ofhe::hooks::TimesScalarEq(m_vectors, s)) return;
        each_tower(m_vectors.size(), [&](size_t i) {
            auto& t = m_vectors[i];
            oracle_vec_modmul_scalar(t.w(), s[i] % t.q(), t.w(), t.n(), t.q());
        });
    }
    void MinusScalarEq(const std::vector<uint64_t>& s) {
        if (ofhe::hooks::MinusScalarEq(m_vectors, s)) return;
        each_tower(m_vectors.size(), [&](size_t i) {
            auto& t = m_vectors[i];
            oracle_vec_modsub_scalar(t.w(), s[i] % t.q(), t.w(), t.n(), t.q());
        });
    }
    // AutomorphismTransform(k) (dcrtpoly-impl.h:349-357)
    DCRTPolyImpl AutomorphismTransform(uint32_t k) const {
        DCRTPolyImpl result(*this);
        if (ofhe::hooks::AutomorphismTransform(m_vectors, result.m_vectors, k)) return result;
        if (k % 2 == 0) throw ofhe::math_error("Automorphism index not odd");
        each_tower(m_vectors.size(), [&](size_t i) {
            const auto& t = m_vectors[i];
            oracle_automorphism(t.w(), result.m_vectors[i].w(), t.n(), k, t.GetFormat() == Format::EVALUATION, t.q());
        });
        return result;
    }
    // ApproxSwitchCRTBasis (dcrtpoly-impl.h:1034-1063): ans over `paramsP`
    DCRTPolyImpl ApproxSwitchCRTBasis(const Towers& paramsP, const std::vector<uint64_t>& hinv,
                                      const std::vector<uint64_t>& hmod) const {
        DCRTPolyImpl ans{m_format, paramsP};
        if (!ofhe::hooks::ApproxSwitchCRTBasis(m_vectors, ans.m_vectors, hinv, hmod))
            cpu_switch_basis(m_vectors, ans.m_vectors, hinv, hmod);
        return ans;
    }
    // ApproxModUp (dcrtpoly-impl.h:1084-1131): `paramsP` carries the P towers'
    // params (values ignored); the hook takes it only when the gate says so,
    // then the P towers are appended first
    void ApproxModUp(const Towers& paramsP, const std::vector<uint64_t>& hinv, const std::vector<uint64_t>& hmod) {
        const size_t sizeQ = m_vectors.size();
        if (ofhe::hooks::device_takes(ofhe::hooks::HookOp::ApproxModUp, m_vectors[0].n(), sizeQ + paramsP.size())) {
            m_vectors.insert(m_vectors.end(), paramsP.begin(), paramsP.end());
            ofhe::hooks::ApproxModUp(m_vectors, sizeQ, hinv, hmod);
            m_format = Format::EVALUATION;
            return;
        }
        Towers cp(m_vectors);
        if (m_format == Format::EVALUATION) set_format(cp, Format::COEFFICIENT);
        Towers partP(paramsP);
        cpu_switch_basis(cp, partP, hinv, hmod);
        for (auto& t : partP) t.OverrideFormat(Format::COEFFICIENT);
        set_format(partP, Format::EVALUATION);
        if (m_format == Format::COEFFICIENT) set_format(m_vectors, Format::EVALUATION);
        m_vectors.insert(m_vectors.end(), partP.begin(), partP.end());
        m_format = Format::EVALUATION;
    }
    // ApproxModDown (dcrtpoly-impl.h:1133-1175): ans over the first sizeQ towers
    DCRTPolyImpl ApproxModDown(size_t sizeQ, const std::vector<uint64_t>& pinv, const std::vector<uint64_t>& phinv,
                               const std::vector<uint64_t>& phmodq, uint64_t t) const {
        DCRTPolyImpl ans{Format::EVALUATION, Towers(m_vectors.begin(), m_vectors.begin() + sizeQ)};
        if (ofhe::hooks::ApproxModDown(m_vectors, ans.m_vectors, pinv, phinv, phmodq, t)) return ans;
        Towers partP(m_vectors.begin() + sizeQ, m_vectors.end());
        set_format(partP, Format::COEFFICIENT);
        if (t > 0)
            each_tower(partP.size(), [&](size_t j) {
                auto& x = partP[j];
                oracle_vec_modmul_scalar(x.w(), oracle_modinv(t % x.q(), x.q()), x.w(), x.n(), x.q());
            });
        Towers sw(ans.m_vectors);
        cpu_switch_basis(partP, sw, phinv, phmodq);
        for (auto& x : sw) x.OverrideFormat(Format::COEFFICIENT);
        if (t > 0)
            each_tower(sw.size(), [&](size_t i) { oracle_vec_modmul_scalar(sw[i].w(), t % sw[i].q(), sw[i].w(), sw[i].n(), sw[i].q()); });
        set_format(sw, Format::EVALUATION);
        each_tower(sizeQ, [&](size_t i) {
            auto& o = ans.m_vectors[i];
            oracle_vec_modsub(m_vectors[i].w(), sw[i].w(), o.w(), o.n(), o.q());
            oracle_vec_modmul_scalar(o.w(), pinv[i], o.w(), o.n(), o.q());
        });
        return ans;
    }

private:
    void binary(const DCRTPolyImpl& rhs, void (*op)(const uint64_t*, const uint64_t*, uint64_t*, uint64_t, uint64_t)) {
        if (moduli(m_vectors) != moduli(rhs.m_vectors)) throw ofhe::math_error("Modulus missmatch");
        each_tower(m_vectors.size(), [&](size_t i) {
            auto& t = m_vectors[i];
            op(t.w(), rhs.m_vectors[i].w(), t.w(), t.n(), t.q());
        });
    }
};

// Products of moduli mod m (the BigInteger quotients the pke layer reduces,
// rns-cryptoparameters.cpp:72-345), excluding index `skip`.
inline uint64_t prod_mod(const std::vector<uint64_t>& ms, size_t skip, uint64_t m) {
    uint64_t r = 1 % m;
    for (size_t i = 0; i < ms.size(); i++)
        if (i != skip) r = mulmod(r, ms[i] % m, m);
    return r;
}
// QHatInvModq / QHatModp of a basis switch src -> dst ([src][dst] row-major)
inline void switch_tables(const std::vector<uint64_t>& src, const std::vector<uint64_t>& dst, std::vector<uint64_t>& hinv,
                          std::vector<uint64_t>& hmod) {
    hinv.assign(src.size(), 0);
    hmod.assign(src.size() * dst.size(), 0);
    for (size_t i = 0; i < src.size(); i++) {
        hinv[i] = oracle_modinv(prod_mod(src, i, src[i]), src[i]);
        for (size_t j = 0; j < dst.size(); j++) hmod[i * dst.size() + j] = prod_mod(src, i, dst[j]);
    }
}
// ModDown tables: PInvModq, PHatInvModp, PHatModq ([P][Q])
inline void moddown_tables(const std::vector<uint64_t>& q, const std::vector<uint64_t>& p, std::vector<uint64_t>& pinv,
                           std::vector<uint64_t>& phinv, std::vector<uint64_t>& phmodq) {
    pinv.clear();
    for (auto qi : q) pinv.push_back(oracle_modinv(prod_mod(p, SIZE_MAX, qi), qi));
    switch_tables(p, q, phinv, phmodq);
}

// KeySwitchHYBRID::KeySwitchCore on the CPU (keyswitch-hybrid.cpp:324-482):
// digit decomposition + per-digit ApproxSwitchCRTBasis to the complement,
// the key inner product, two ApproxModDown.  key: bv / av [dnum] polynomials
// over Q|P (sizeQ + sizeP towers).  The hook runs first, as INTEGRATION.md §3
// places it; this body is the reference's.
struct KeySwitchHYBRID {
    size_t sizeQ, sizeP;
    uint32_t dnum;
    std::vector<Towers> bv, av;
    std::string tag;
    std::pair<DCRTPolyImpl, DCRTPolyImpl> KeySwitchCore(const DCRTPolyImpl& a, uint64_t t) const {
        DCRTPolyImpl ct0{Format::EVALUATION, a.m_vectors}, ct1{Format::EVALUATION, a.m_vectors};
        if (ofhe::hooks::KeySwitchCore(a.m_vectors, tag, t, ct0.m_vectors, ct1.m_vectors)) return {ct0, ct1};
        const size_t l = a.m_vectors.size();
        const size_t alpha = (sizeQ + dnum - 1) / dnum;
        const size_t beta = std::min<size_t>((l + alpha - 1) / alpha, dnum);
        // Ql|P towers: a's, then P (params from the key's last sizeP towers)
        Towers QlP(a.m_vectors);
        for (size_t k = 0; k < sizeP; k++) QlP.push_back(bv[0][sizeQ + k]);
        DCRTPolyImpl c0{Format::EVALUATION, QlP}, c1{Format::EVALUATION, QlP};
        for (auto* c : {&c0, &c1})
            for (auto& tw : c->m_vectors) std::fill(tw.values.begin(), tw.values.end(), NativeInteger{0});
        for (size_t j = 0; j < beta; j++) {
            const size_t st = alpha * j, cnt = std::min(alpha, l - st);
            Towers part(a.m_vectors.begin() + st, a.m_vectors.begin() + st + cnt);  // 350-374
            Towers coeff(part);
            set_format(coeff, Format::COEFFICIENT);                                    // 384-385
            Towers compl_;                                                             // the complement: Ql \ digit, then P
            for (size_t i = 0; i < l + sizeP; i++)
                if (i < st || i >= st + cnt) compl_.push_back(QlP[i]);
            std::vector<uint64_t> hinv, hmod;
            switch_tables(moduli(part), moduli(compl_), hinv, hmod);
            cpu_switch_basis(coeff, compl_, hinv, hmod);                               // 386-394
            for (auto& x : compl_) x.OverrideFormat(Format::COEFFICIENT);
            set_format(compl_, Format::EVALUATION);
            Towers ext;                                                                // 396-409
            for (size_t i = 0; i < st; i++) ext.push_back(compl_[i]);
            for (size_t i = 0; i < cnt; i++) ext.push_back(part[i]);
            for (size_t i = st + cnt; i < l + sizeP; i++) ext.push_back(compl_[i - cnt]);
            each_tower(l + sizeP, [&](size_t i) {                                      // 459-476
                const size_t k = i < l ? i : sizeQ + (i - l);
                const uint64_t q = QlP[i].q();
                const uint32_t n = QlP[i].n();
                std::vector<uint64_t> tmp(n);
                oracle_vec_modmul(ext[i].w(), bv[j][k].w(), tmp.data(), n, q);
                oracle_vec_modadd(c0.m_vectors[i].w(), tmp.data(), c0.m_vectors[i].w(), n, q);
                oracle_vec_modmul(ext[i].w(), av[j][k].w(), tmp.data(), n, q);
                oracle_vec_modadd(c1.m_vectors[i].w(), tmp.data(), c1.m_vectors[i].w(), n, q);
            });
        }
        std::vector<uint64_t> ql(moduli(a.m_vectors)), p, pinv, phinv, phmodq;
        for (size_t k = 0; k < sizeP; k++) p.push_back(bv[0][sizeQ + k].q());
        moddown_tables(ql, p, pinv, phinv, phmodq);
        return {c0.ApproxModDown(l, pinv, phinv, phmodq, t), c1.ApproxModDown(l, pinv, phinv, phmodq, t)};  // 414-435
    }
};

// Towers of ring n over moduli q / roots r with uniform values
template <class Rng>
Towers make_towers(uint32_t n, const std::vector<uint64_t>& q, const std::vector<uint64_t>& r, Rng& rng,
                   Format f = Format::COEFFICIENT) {
    Towers out;
    for (size_t t = 0; t < q.size(); t++) {
        auto p = std::make_shared<ILNativeParams>(ILNativeParams{{q[t]}, {r[t]}, n});
        PolyImpl x{p, std::vector<NativeInteger>(n), f};
        for (auto& v : x.values) v.m_value = rng() % q[t];
        out.push_back(std::move(x));
    }
    return out;
}
inline std::vector<uint64_t> words(const PolyImpl& p) { return std::vector<uint64_t>(p.w(), p.w() + p.n()); }

}  // namespace mock
