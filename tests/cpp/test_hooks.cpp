// The RUN_ON_HIP hook bodies (upmem--openfhe_amd/host/ofhe_openfhe_hooks.hpp)
// instantiated on a tower type with the reference's accessor surface and
// checked against the CPU oracle (oracle/libofhe_oracle.so, test
// infrastructure).  The mock below is this repo's own test double written to
// the reference's method names -- PolyImpl::GetParams() / operator[]
// (poly.h:209-215), ILNativeParams::GetModulus() / GetRootOfUnity() /
// GetRingDimension(), NativeIntegerT::ConvertToInt() with one uint64_t member
// (ubintnat.h:139-141, 1659) -- not a copy of any reference header: it shows
// that the hooks compile against, and only need, that surface.
#include <cstdint>
#include <cstdio>
#include <memory>
#include <string>
#include <random>
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
struct NativeInteger {  // NativeIntegerT<uint64_t>: one word
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
int g_cpu_switches = 0;  // towers transformed by the CPU loop (PolyImpl::SwitchFormat)
struct PolyImpl {
    std::shared_ptr<ILNativeParams> params;
    std::vector<NativeInteger> values;
    Format m_format = Format::COEFFICIENT;
    const std::shared_ptr<ILNativeParams>& GetParams() const { return params; }
    NativeInteger& operator[](uint32_t i) { return values[i]; }
    const NativeInteger& operator[](uint32_t i) const { return values[i]; }
    Format GetFormat() const { return m_format; }
    void OverrideFormat(Format f) { m_format = f; }  // poly.h:179
    void SwitchFormat();                              // poly-impl.h:412-432, on the oracle
};
// DCRTPolyImpl with the RUN_ON_HIP SwitchFormat exactly as INTEGRATION.md §3
// shows it for dcrtpoly-impl.h:2516-2523: the hook, else the reference loop
struct DCRTPolyImpl {
    Format m_format = Format::COEFFICIENT;
    std::vector<PolyImpl> m_vectors;
    void SwitchFormat() {
        m_format = (m_format == Format::COEFFICIENT) ? Format::EVALUATION : Format::COEFFICIENT;
        if (ofhe::hooks::SwitchFormat(m_vectors)) return;
        size_t size{m_vectors.size()};
        for (size_t i = 0; i < size; ++i) m_vectors[i].SwitchFormat();
    }
};
}  // namespace mock

void mock::PolyImpl::SwitchFormat() {
    const uint32_t n = params->ring;
    uint32_t log_n = 0;
    while ((1u << log_n) < n) log_n++;
    std::vector<uint64_t> tab(n), tp(n), it(n), ip(n), coi(log_n + 1), cp(log_n + 1), x(n);
    const uint64_t q = params->modulus.m_value;
    oracle_ntt_tables(n, q, params->root.m_value, tab.data(), tp.data(), it.data(), ip.data(), coi.data(), cp.data());
    for (uint32_t i = 0; i < n; i++) x[i] = values[i].m_value;
    if (m_format == Format::COEFFICIENT) {
        oracle_ntt_fwd(x.data(), n, q, tab.data(), tp.data());
        m_format = Format::EVALUATION;
    } else {
        oracle_ntt_inv(x.data(), n, q, it.data(), ip.data(), coi[log_n], cp[log_n]);
        m_format = Format::COEFFICIENT;
    }
    for (uint32_t i = 0; i < n; i++) values[i].m_value = x[i];
    g_cpu_switches++;
}

static int g_fail = 0;
#define CHECK(c, msg)                                      \
    do {                                                   \
        if (!(c)) {                                        \
            std::printf("  FAIL %s:%d %s\n", __FILE__, __LINE__, msg); \
            g_fail++;                                      \
        }                                                  \
    } while (0)

static std::vector<mock::PolyImpl> towers(uint32_t n, const std::vector<uint64_t>& q, const std::vector<uint64_t>& r,
                                          std::mt19937_64& rng) {
    std::vector<mock::PolyImpl> out;
    for (size_t t = 0; t < q.size(); t++) {
        auto p = std::make_shared<mock::ILNativeParams>(mock::ILNativeParams{{q[t]}, {r[t]}, n});
        mock::PolyImpl x{p, std::vector<mock::NativeInteger>(n)};
        for (auto& v : x.values) v.m_value = rng() % q[t];
        out.push_back(std::move(x));
    }
    return out;
}
static std::vector<uint64_t> words(const mock::PolyImpl& p) {
    std::vector<uint64_t> w;
    for (auto& v : p.values) w.push_back(v.m_value);
    return w;
}

// The oracle's per-tower transforms (ChineseRemainderTransformFTT, on the C
// restatement): fwd = COEFFICIENT -> EVALUATION, else back.
static std::vector<uint64_t> ntt(const std::vector<uint64_t>& x, uint64_t q, uint64_t psi, bool fwd) {
    const uint64_t n = x.size();
    uint32_t log_n = 0;
    while ((1ull << log_n) < n) log_n++;
    std::vector<uint64_t> tab(n), tp(n), it(n), ip(n), coi(log_n + 1), cp(log_n + 1), y(x);
    oracle_ntt_tables(n, q, psi, tab.data(), tp.data(), it.data(), ip.data(), coi.data(), cp.data());
    if (fwd)
        oracle_ntt_fwd(y.data(), n, q, tab.data(), tp.data());
    else
        oracle_ntt_inv(y.data(), n, q, it.data(), ip.data(), coi[log_n], cp[log_n]);
    return y;
}
// ApproxSwitchCRTBasis src -> dst on the oracle, with the oracle's tables;
// the tables go to the hook too (hinv, hmod)
struct Switch {
    std::vector<uint64_t> hinv, hinvp, hmod, mlo, mhi;
    Switch(const std::vector<uint64_t>& a, const std::vector<uint64_t>& b)
        : hinv(a.size()), hinvp(a.size()), hmod(a.size() * b.size()), mlo(b.size()), mhi(b.size()) {
        oracle_base_conv_precompute((unsigned)a.size(), (unsigned)b.size(), a.data(), b.data(), hinv.data(), hinvp.data(),
                                    hmod.data(), mlo.data(), mhi.data());
    }
    std::vector<std::vector<uint64_t>> run(const std::vector<std::vector<uint64_t>>& x, const std::vector<uint64_t>& a,
                                           const std::vector<uint64_t>& b) const {
        const uint64_t n = x[0].size();
        std::vector<uint64_t> in, out(b.size() * n);
        for (auto& t : x) in.insert(in.end(), t.begin(), t.end());
        oracle_approx_switch_crt_basis(in.data(), out.data(), n, (unsigned)a.size(), (unsigned)b.size(), a.data(),
                                       b.data(), hinv.data(), hinvp.data(), hmod.data(), mlo.data(), mhi.data());
        std::vector<std::vector<uint64_t>> r;
        for (size_t j = 0; j < b.size(); j++) r.emplace_back(out.begin() + j * n, out.begin() + (j + 1) * n);
        return r;
    }
};
static uint64_t prod_inv(const std::vector<uint64_t>& ms, uint64_t q) {  // (prod ms)^-1 mod q
    unsigned __int128 r = 1;
    for (auto m : ms) r = r * (m % q) % q;
    return oracle_modinv((uint64_t)r, q);
}

int main() {
    const uint32_t log_n = 12, n = 1u << log_n, T = 5, P = 3;
    std::vector<uint64_t> all(T + P), roots(T + P);
    oracle_moduli_chain(60, 2 * n, T + P, all.data(), roots.data());
    std::vector<uint64_t> q(all.begin(), all.begin() + T), r(roots.begin(), roots.begin() + T);
    std::vector<uint64_t> p(all.begin() + T, all.end()), rp(roots.begin() + T, roots.end());
    std::mt19937_64 rng(77);
    try {
        // DCRTPolyImpl::SwitchFormat through the hook (N = 2^12: the device)
        // against the reference's own per-tower loop on the oracle
        auto a = towers(n, q, r, rng);
        auto a0 = a;
        {
            mock::DCRTPolyImpl d{mock::Format::COEFFICIENT, a}, ref{mock::Format::COEFFICIENT, a};
            mock::g_cpu_switches = 0;
            d.SwitchFormat();
            CHECK(mock::g_cpu_switches == 0, "N = 2^12 SwitchFormat ran on the device");
            for (auto& t : ref.m_vectors) t.SwitchFormat();
            bool ok = d.m_format == mock::Format::EVALUATION;
            for (uint32_t t = 0; t < T; t++)
                ok = ok && words(d.m_vectors[t]) == words(ref.m_vectors[t]) &&
                     d.m_vectors[t].GetFormat() == mock::Format::EVALUATION;
            CHECK(ok, "hooks::SwitchFormat (forward) vs oracle, formats flipped");
            a = d.m_vectors;
            d.SwitchFormat();
            ok = d.m_format == mock::Format::COEFFICIENT && mock::g_cpu_switches == (int)T;  // T: the ref loop above
            for (uint32_t t = 0; t < T; t++)
                ok = ok && words(d.m_vectors[t]) == words(a0[t]) && d.m_vectors[t].GetFormat() == mock::Format::COEFFICIENT;
            CHECK(ok, "hooks::SwitchFormat round trip");
        }
        // small ring (binfhe-sized N = 2^10): the hook declines, the reference
        // loop runs, the format still flips and the values equal the oracle's
        {
            const uint32_t ns = 1u << 10;
            std::vector<uint64_t> qs(3), rs(3);
            oracle_moduli_chain(60, 2 * ns, 3, qs.data(), rs.data());
            auto sm = towers(ns, qs, rs, rng);
            mock::DCRTPolyImpl d{mock::Format::COEFFICIENT, sm}, ref{mock::Format::COEFFICIENT, sm};
            mock::g_cpu_switches = 0;
            d.SwitchFormat();
            bool ok = mock::g_cpu_switches == 3 && d.m_format == mock::Format::EVALUATION;
            for (auto& t : ref.m_vectors) t.SwitchFormat();
            for (size_t t = 0; t < 3; t++) ok = ok && words(d.m_vectors[t]) == words(ref.m_vectors[t]);
            CHECK(ok, "N = 2^10 SwitchFormat takes the CPU loop and flips m_format");
            CHECK(!ofhe::hooks::device_switch_format(d.m_vectors), "device_switch_format(N = 2^10) is false");
        }
        bool ok = true;
        // element-wise *=, +=, -= against the oracle
        auto b = towers(n, q, r, rng);
        for (int op = 0; op < 3; op++) {
            auto x = a0;
            if (op == 0) ofhe::hooks::TimesEq(x, b);
            if (op == 1) ofhe::hooks::PlusEq(x, b);
            if (op == 2) ofhe::hooks::MinusEq(x, b);
            ok = true;
            for (uint32_t t = 0; t < T; t++) {
                std::vector<uint64_t> wa = words(a0[t]), wb = words(b[t]), wc(n);
                (op == 0 ? oracle_vec_modmul : op == 1 ? oracle_vec_modadd : oracle_vec_modsub)(wa.data(), wb.data(),
                                                                                               wc.data(), n, q[t]);
                ok = ok && wc == words(x[t]);
            }
            CHECK(ok, op == 0 ? "hooks::TimesEq" : op == 1 ? "hooks::PlusEq" : "hooks::MinusEq");
        }
        // ApproxSwitchCRTBasis Q -> P against the oracle
        std::vector<uint64_t> hinv(T), hinvp(T), hmod(T * P), mlo(P), mhi(P);
        oracle_base_conv_precompute(T, P, q.data(), p.data(), hinv.data(), hinvp.data(), hmod.data(), mlo.data(),
                                    mhi.data());
        auto out = towers(n, p, rp, rng);
        ofhe::hooks::ApproxSwitchCRTBasis(a0, out, hinv, hmod);
        std::vector<uint64_t> xin, want(P * (size_t)n);
        for (auto& t : a0) {
            auto w = words(t);
            xin.insert(xin.end(), w.begin(), w.end());
        }
        oracle_approx_switch_crt_basis(xin.data(), want.data(), n, T, P, q.data(), p.data(), hinv.data(), hinvp.data(),
                                       hmod.data(), mlo.data(), mhi.data());
        ok = true;
        for (uint32_t j = 0; j < P; j++)
            ok = ok && std::vector<uint64_t>(want.begin() + j * (size_t)n, want.begin() + (j + 1) * (size_t)n) ==
                           words(out[j]);
        CHECK(ok, "hooks::ApproxSwitchCRTBasis vs oracle");
        // ApproxModUp (dcrtpoly-impl.h:1084-1131) from either format: the
        // caller appends the P towers (their params set, values ignored), the
        // hook fills all of them in EVALUATION form.  Oracle: the reference's
        // steps -- INTT of an evaluation-form input, ApproxSwitchCRTBasis,
        // NTT of the P towers, the Q towers in evaluation form.
        Switch up(q, p);
        for (int ev = 0; ev < 2; ev++) {
            auto x = towers(n, q, r, rng);
            std::vector<std::vector<uint64_t>> coeff, wantQ;
            for (uint32_t t = 0; t < T; t++) {
                coeff.push_back(words(x[t]));
                wantQ.push_back(ntt(coeff.back(), q[t], r[t], true));
            }
            if (ev)
                for (uint32_t t = 0; t < T; t++) {
                    for (uint32_t i = 0; i < n; i++) x[t].values[i].m_value = wantQ[t][i];
                    x[t].m_format = mock::Format::EVALUATION;
                }
            auto ext = towers(n, p, rp, rng);  // the appended P towers (garbage values)
            x.insert(x.end(), ext.begin(), ext.end());
            ofhe::hooks::ApproxModUp(x, T, up.hinv, up.hmod);
            auto pp = up.run(coeff, q, p);
            ok = true;
            for (uint32_t t = 0; t < T; t++) ok = ok && words(x[t]) == wantQ[t];
            for (uint32_t j = 0; j < P; j++) ok = ok && words(x[T + j]) == ntt(pp[j], p[j], rp[j], true);
            for (auto& tw : x) ok = ok && tw.GetFormat() == mock::Format::EVALUATION;
            CHECK(ok, ev ? "hooks::ApproxModUp (evaluation input) vs oracle" : "hooks::ApproxModUp (coefficient input) vs oracle");
        }
        // ApproxModDown (dcrtpoly-impl.h:1133-1175), t = 0 (CKKS) and t = 65537
        // (BGV): out_i = (x_i - NTT(t ApproxSwitch(t^-1 INTT(x_P)))_i) PInvModq_i
        Switch down(p, q);
        std::vector<uint64_t> pinv;
        for (auto qi : q) pinv.push_back(prod_inv(p, qi));
        for (uint64_t tt : {uint64_t(0), uint64_t(65537)}) {
            std::vector<uint64_t> all_r(r);
            all_r.insert(all_r.end(), rp.begin(), rp.end());
            auto x = towers(n, all, all_r, rng);
            for (auto& tw : x) tw.m_format = mock::Format::EVALUATION;
            std::vector<std::vector<uint64_t>> partP;
            for (uint32_t j = 0; j < P; j++) {
                auto c = ntt(words(x[T + j]), p[j], rp[j], false);
                if (tt) oracle_vec_modmul_scalar(c.data(), oracle_modinv(tt % p[j], p[j]), c.data(), n, p[j]);
                partP.push_back(c);
            }
            auto sw = down.run(partP, p, q);
            auto out = towers(n, q, r, rng);  // the caller's ans (values overwritten)
            ofhe::hooks::ApproxModDown(x, out, pinv, down.hinv, down.hmod, tt);
            ok = true;
            for (uint32_t i = 0; i < T; i++) {
                if (tt) oracle_vec_modmul_scalar(sw[i].data(), tt, sw[i].data(), n, q[i]);
                auto e = ntt(sw[i], q[i], r[i], true);
                std::vector<uint64_t> want(n, 0);
                auto xi = words(x[i]);
                oracle_vec_modsub(xi.data(), e.data(), want.data(), n, q[i]);
                oracle_vec_modmul_scalar(want.data(), pinv[i], want.data(), n, q[i]);
                ok = ok && words(out[i]) == want && out[i].GetFormat() == mock::Format::EVALUATION;
            }
            CHECK(ok, tt ? "hooks::ApproxModDown (t = 65537) vs oracle" : "hooks::ApproxModDown (t = 0) vs oracle");
        }
        // AutomorphismTransform (poly-impl.h:312-365), both formats, k = 5 and
        // the transposition k = m - 1; an even index throws math_error
        for (int ev = 0; ev < 2; ev++)
            for (uint32_t k : {5u, 2 * n - 1}) {
                auto x = towers(n, q, r, rng);
                if (ev)
                    for (auto& tw : x) tw.m_format = mock::Format::EVALUATION;
                auto out = x;
                ofhe::hooks::AutomorphismTransform(x, out, k);
                ok = true;
                for (uint32_t t = 0; t < T; t++) {
                    auto xi = words(x[t]);
                    std::vector<uint64_t> want(n);
                    oracle_automorphism(xi.data(), want.data(), n, k, ev, q[t]);
                    ok = ok && words(out[t]) == want && out[t].GetFormat() == x[t].GetFormat();
                }
                CHECK(ok, ev ? "hooks::AutomorphismTransform (evaluation) vs oracle"
                             : "hooks::AutomorphismTransform (coefficient) vs oracle");
            }
        {
            bool thrown = false;
            try {
                auto x = towers(n, q, r, rng);
                auto out = x;
                ofhe::hooks::AutomorphismTransform(x, out, 4);
            } catch (const ofhe::math_error&) {
                thrown = true;
            }
            CHECK(thrown, "AutomorphismTransform with an even index throws math_error");
        }
        // scalar Times (one scalar per tower, any 64-bit value), signed Times
        // (negative, INT64_MIN, -q), Minus
        {
            std::vector<uint64_t> sc;
            for (uint32_t t = 0; t < T; t++) sc.push_back(rng());
            auto x = a0;
            ofhe::hooks::TimesScalarEq(x, sc);
            ok = true;
            for (uint32_t t = 0; t < T; t++) {
                auto w = words(a0[t]);
                oracle_vec_modmul_scalar(w.data(), sc[t] % q[t], w.data(), n, q[t]);
                ok = ok && words(x[t]) == w;
            }
            CHECK(ok, "hooks::TimesScalarEq vs oracle");
            for (int64_t v : {int64_t(-12345), INT64_MIN, -(int64_t)q[0], int64_t(7)}) {
                auto y = a0;
                ofhe::hooks::TimesSignedEq(y, v);
                ok = true;
                for (uint32_t t = 0; t < T; t++) {
                    const uint64_t mag = v < 0 ? (uint64_t)0 - (uint64_t)v : (uint64_t)v;
                    const uint64_t s1 = v < 0 ? (q[t] - mag % q[t]) % q[t] : mag % q[t];
                    auto w = words(a0[t]);
                    oracle_vec_modmul_scalar(w.data(), s1, w.data(), n, q[t]);
                    ok = ok && words(y[t]) == w;
                }
                CHECK(ok, ("hooks::TimesSignedEq(" + std::to_string(v) + ") vs oracle").c_str());
            }
            auto z = a0;
            ofhe::hooks::MinusScalarEq(z, sc);
            ok = true;
            for (uint32_t t = 0; t < T; t++) {
                auto w = words(a0[t]);
                oracle_vec_modsub_scalar(w.data(), sc[t] % q[t], w.data(), n, q[t]);
                ok = ok && words(z[t]) == w;
            }
            CHECK(ok, "hooks::MinusScalarEq vs oracle");
        }
        // the reference's error behaviour: mismatched bases throw math_error
        bool thrown = false;
        try {
            auto x = a0;
            auto y = towers(n, p, rp, rng);
            y.resize(x.size(), y[0]);
            ofhe::hooks::PlusEq(x, y);
        } catch (const ofhe::math_error&) {
            thrown = true;
        }
        CHECK(thrown, "PlusEq over different moduli throws math_error");
    } catch (const std::exception& e) {
        std::printf("  FAIL exception %s\n", e.what());
        g_fail++;
    }
    std::printf("hooks: %d failures\n", g_fail);
    return g_fail ? 1 : 0;
}
