// ofhe_openfhe_hooks.hpp -- the bodies of the RUN_ON_HIP hooks a maintainer
// adds to OpenFHE's DCRTPolyImpl, as templates over the
// reference's own tower type, so the hook inside the member function is one
// call and this code is compiled and tested here (tests/cpp/test_hooks.cpp).
//
// `Towers` is DCRTPolyImpl::m_vectors, a std::vector<PolyImpl<NativeVector>>
// (dcrtpoly.h:421).  The templates use only what the reference's PolyImpl /
// ILNativeParams / NativeIntegerT expose:
//   tower.GetParams()->GetModulus().ConvertToInt()      (poly.h:114, ubintnat.h:1659)
//   tower.GetParams()->GetRootOfUnity().ConvertToInt()  (poly.h:115)
//   tower.GetParams()->GetRingDimension()               (poly.h:119)
//   &tower[0]: NativeIntegerT is one uint64_t m_value    (ubintnat.h:139-141), the
//              N values of a tower are contiguous      (mubintvecnat.h:127,671)
//
// Each hook gathers the towers into pinned staging memory, makes ONE launch
// over every tower and scatters back (the host-buffer integration; the
// resident integration keeps DCRTPolyHip objects instead, ofhe_dcrt.hpp).
//
//   DCRTPolyImpl::SwitchFormat          dcrtpoly-impl.h:2516-2523 -> if (!SwitchFormat(m_vectors)) <reference loop>
//   DCRTPolyImpl::operator*= / Times    dcrtpoly.h:142-148, 185-200 -> TimesEq(m_vectors, rhs.m_vectors)
//   DCRTPolyImpl::operator+= / -=       dcrtpoly-impl.h:410-416     -> PlusEq / MinusEq
//   DCRTPolyImpl::ApproxSwitchCRTBasis  dcrtpoly-impl.h:1034-1063   -> ApproxSwitchCRTBasis(...)
//   DCRTPolyImpl::ApproxModUp           dcrtpoly-impl.h:1084-1131   -> ApproxModUp(m_vectors, sizeQ, ...)
//   DCRTPolyImpl::ApproxModDown         dcrtpoly-impl.h:1133-1175   -> ApproxModDown(m_vectors, ans.m_vectors, ...)
//   DCRTPolyImpl::AutomorphismTransform dcrtpoly-impl.h:349-357     -> AutomorphismTransform(m_vectors, result.m_vectors, k)
//   DCRTPolyImpl::Times / operator*= by scalar   dcrtpoly-impl.h:586-661 -> TimesScalarEq / TimesSignedEq
//   DCRTPolyImpl::Minus by scalar       dcrtpoly-impl.h:565-584     -> MinusScalarEq
#pragma once

#include <algorithm>
#include <cstdint>
#include <map>
#include <memory>
#include <type_traits>
#include <utility>
#include <vector>

#include "ofhe_dcrt.hpp"

namespace ofhe {
namespace hooks {

// The basis of a tower vector (moduli, roots, ring dimension) and raw word
// pointers into each tower's values.
struct TowerView {
    uint32_t n = 0, log_n = 0;
    std::vector<uint64_t> q, psi;
    std::vector<uint64_t*> data;
};

template <class Towers>
TowerView view(Towers& towers) {
    TowerView v;
    if (towers.empty()) throw math_error("hooks: no towers");
    for (auto& t : towers) {
        const auto& prm = *t.GetParams();
        const uint32_t n = (uint32_t)prm.GetRingDimension();
        if (v.n == 0) v.n = n;
        if (n != v.n) throw math_error("hooks: towers of different ring dimension");
        static_assert(sizeof(t[0]) == sizeof(uint64_t), "NativeInteger must be one 64-bit word");
        v.q.push_back((uint64_t)prm.GetModulus().ConvertToInt());
        v.psi.push_back((uint64_t)prm.GetRootOfUnity().ConvertToInt());
        v.data.push_back(reinterpret_cast<uint64_t*>(&t[0]));
    }
    while ((1u << v.log_n) < v.n) v.log_n++;
    if ((1u << v.log_n) != v.n) throw math_error("hooks: ring dimension is not a power of two");
    return v;
}

inline std::vector<const uint64_t*> cptr(const std::vector<uint64_t*>& p) {
    return std::vector<const uint64_t*>(p.begin(), p.end());
}

// Pinned staging reused across hook calls: a hook runs once per DCRTPoly
// operation, and page-locking host memory costs far more than the transfer.
// One pool per (thread, device), slots grow to the largest size asked for;
// every hook ends with a synchronous download, so a slot is idle when reused.
inline Staging& staging(int device, size_t words, int slot = 0) {
    thread_local std::map<std::pair<int, int>, std::unique_ptr<Staging>> pool;
    auto& s = pool[{device, slot}];
    if (!s || s->words() < words) {
        s.reset();  // release the smaller buffer first
        s.reset(new Staging(HipManager::getHip(device), words));
    }
    return *s;
}

// Rings below this stay on the reference's CPU loop: binfhe's rings (N <= 2^11,
// rgsw-acc-*.cpp) are launch-latency bound on the GPU and PCIe-bound through
// the host-buffer hooks.
constexpr uint32_t kDeviceMinRing = 4096;

// Whether the device takes DCRTPolyImpl::SwitchFormat for these towers: a
// power-of-two cyclotomic (PolyImpl::SwitchFormat sends rd != co / 2 to
// ArbitrarySwitchFormat, poly-impl.h:412-420), ring dimension >= kDeviceMinRing,
// every tower in the same format.
template <class Towers>
bool device_switch_format(const Towers& towers) {
    if (towers.empty()) return false;
    const auto& p0 = *towers[0].GetParams();
    const uint32_t n = (uint32_t)p0.GetRingDimension();
    if (n < kDeviceMinRing || (uint64_t)p0.GetCyclotomicOrder() != 2 * (uint64_t)n) return false;
    for (const auto& t : towers)
        if (t.GetFormat() != towers[0].GetFormat()) return false;
    return true;
}

// DCRTPolyImpl::SwitchFormat (dcrtpoly-impl.h:2516-2523): every tower
// COEFFICIENT -> EVALUATION (ForwardTransformToBitReverseInPlace) or back
// (InverseTransformFromBitReverseInPlace) in one launch, then each tower's
// format flipped with PolyImpl::OverrideFormat (poly.h:179), as
// PolyImpl::SwitchFormat does per tower (poly-impl.h:412-432).  Returns false,
// touching nothing, when device_switch_format() says no: the caller then runs
// the reference's own per-tower loop.
template <class Towers>
bool SwitchFormat(Towers& towers, int device = 0) {
    if (!device_switch_format(towers)) return false;
    using Fmt = std::decay_t<decltype(towers[0].GetFormat())>;
    const bool to_eval = towers[0].GetFormat() == Fmt::COEFFICIENT;
    TowerView v = view(towers);
    auto plan = PlanCache::get(device, v.log_n, v.q, v.psi);
    const size_t words = v.q.size() * (size_t)v.n;
    Staging& st = staging(device, words);
    st.gather(cptr(v.data), v.n);
    st.upload(words);
    check(to_eval ? ofhe_hip_ntt_fwd(plan->get(), st.dev(), 1, nullptr)
                  : ofhe_hip_ntt_inv(plan->get(), st.dev(), 1, nullptr),
          "hooks::SwitchFormat");
    st.download(words);
    st.scatter(v.data, v.n);
    for (auto& t : towers) t.OverrideFormat(to_eval ? Fmt::EVALUATION : Fmt::COEFFICIENT);
    return true;
}

namespace detail {
// a (op)= b over all towers in one launch; op 0 ModMul (Barrett), 1 ModAdd, 2 ModSub
template <class Towers>
void binary_eq(Towers& a, const Towers& b, int op, const char* what, int device) {
    TowerView va = view(a);
    TowerView vb = view(const_cast<Towers&>(b));
    if (va.q != vb.q || va.n != vb.n) throw math_error(std::string(what) + ": Modulus missmatch");
    auto plan = PlanCache::get(device, va.log_n, va.q, va.psi);
    const size_t words = va.q.size() * (size_t)va.n;
    Staging& sa = staging(device, words, 0);
    Staging& sb = staging(device, words, 1);
    sa.gather(cptr(va.data), va.n);
    sb.gather(cptr(vb.data), vb.n);
    sa.upload(words);
    sb.upload(words);
    int rc = op == 0   ? ofhe_hip_modmul_vv(plan->get(), sa.dev(), sb.dev(), sa.dev(), 1, nullptr)
             : op == 1 ? ofhe_hip_modadd_vv(plan->get(), sa.dev(), sb.dev(), sa.dev(), 1, nullptr)
                       : ofhe_hip_modsub_vv(plan->get(), sa.dev(), sb.dev(), sa.dev(), 1, nullptr);
    check(rc, what);
    sa.download(words);
    sa.scatter(va.data, va.n);
}
}  // namespace detail

// DCRTPolyImpl::operator*= (dcrtpoly.h:142-148; EVALUATION form, the caller checks)
template <class Towers>
void TimesEq(Towers& a, const Towers& b, int device = 0) {
    detail::binary_eq(a, b, 0, "hooks::TimesEq", device);
}
// DCRTPolyImpl::operator+= (dcrtpoly-impl.h:410-416)
template <class Towers>
void PlusEq(Towers& a, const Towers& b, int device = 0) {
    detail::binary_eq(a, b, 1, "hooks::PlusEq", device);
}
// DCRTPolyImpl::operator-=
template <class Towers>
void MinusEq(Towers& a, const Towers& b, int device = 0) {
    detail::binary_eq(a, b, 2, "hooks::MinusEq", device);
}

// NTT plan over towers [t0, t0 + count) of a view (PlanCache: one per basis)
inline std::shared_ptr<PlanHandle> plan_of(const TowerView& v, size_t t0, size_t count, int device) {
    std::vector<uint64_t> q(v.q.begin() + t0, v.q.begin() + t0 + count);
    std::vector<uint64_t> r(v.psi.begin() + t0, v.psi.begin() + t0 + count);
    return PlanCache::get(device, v.log_n, q, r);
}

// Base converter src -> dst with the pke layer's tables (rns-cryptoparameters.cpp
// :273-337; hmod row-major [src][dst]), built once per (basis pair, tables) and
// cached process-wide, as the reference precomputes them once per parameter set.
inline std::shared_ptr<ofhe_bconv_s> converter(int device, uint32_t log_n, const std::vector<uint64_t>& src,
                                               const std::vector<uint64_t>& dst, const std::vector<uint64_t>& hinv,
                                               const std::vector<uint64_t>& hmod, const char* what) {
    if (hinv.size() != src.size() || hmod.size() != src.size() * dst.size())
        throw math_error(std::string(what) + ": table sizes");
    HipManager* m = HipManager::getHip(device);
    static std::mutex mu;
    static std::map<std::vector<uint64_t>, std::shared_ptr<ofhe_bconv_s>> cache;
    std::vector<uint64_t> key{(uint64_t)device, log_n, src.size()};
    key.insert(key.end(), src.begin(), src.end());
    key.insert(key.end(), dst.begin(), dst.end());
    key.insert(key.end(), hinv.begin(), hinv.end());
    key.insert(key.end(), hmod.begin(), hmod.end());
    std::lock_guard<std::mutex> lk(mu);
    auto& e = cache[key];
    if (!e) {
        ofhe_bconv_t h = nullptr;
        check(ofhe_hip_bconv_create(m->ctx(), log_n, (uint32_t)src.size(), (uint32_t)dst.size(), src.data(), dst.data(),
                                    hinv.data(), hmod.data(), &h),
              what);
        e = std::shared_ptr<ofhe_bconv_s>(h, [](ofhe_bconv_t p) { ofhe_hip_bconv_destroy(p); });
    }
    return e;
}

// DCRTPolyImpl::ApproxSwitchCRTBasis (dcrtpoly-impl.h:1034-1063): x's towers
// (basis Q, COEFFICIENT form) -> out's towers (basis P, already sized by the
// caller as the reference's `ans(paramsP, m_format, true)`), with the
// QHatInvModq / QHatModp tables the pke layer precomputes
// (rns-cryptoparameters.cpp:273-337; QHatModp row-major [sizeQ][sizeP]).
template <class TowersQ, class TowersP>
void ApproxSwitchCRTBasis(const TowersQ& x, TowersP& out, const std::vector<uint64_t>& QHatInvModq,
                          const std::vector<uint64_t>& QHatModp, int device = 0) {
    TowerView vx = view(const_cast<TowersQ&>(x)), vo = view(out);
    if (vx.n != vo.n) throw math_error("hooks::ApproxSwitchCRTBasis: ring dimensions differ");
    auto bc = converter(device, vx.log_n, vx.q, vo.q, QHatInvModq, QHatModp, "hooks::ApproxSwitchCRTBasis");
    const size_t wx = vx.q.size() * (size_t)vx.n, wo = vo.q.size() * (size_t)vo.n;
    Staging& sx = staging(device, wx, 0);
    Staging& so = staging(device, wo, 1);
    sx.gather(cptr(vx.data), vx.n);
    sx.upload(wx);
    check(ofhe_hip_approx_switch_crt_basis(bc.get(), sx.dev(), so.dev(), 1, nullptr), "hooks::ApproxSwitchCRTBasis");
    so.download(wo);
    so.scatter(vo.data, vo.n);
}

// DCRTPolyImpl::ApproxModUp (dcrtpoly-impl.h:1084-1131).  `towers` is
// m_vectors after the caller's resize to Q|P: the sizeQ towers of x (all in
// one format) followed by sizeP towers whose params are paramsP's (their
// values are ignored).  On return every tower holds ApproxModUp(x) in
// EVALUATION form -- the Q towers x itself in evaluation form, the P towers
// NTT(ApproxSwitchCRTBasis(x)) -- and says so (OverrideFormat), as the
// reference's m_format = EVALUATION, m_params = paramsQP leave it.
template <class Towers>
void ApproxModUp(Towers& towers, size_t sizeQ, const std::vector<uint64_t>& QHatInvModq,
                 const std::vector<uint64_t>& QHatModp, int device = 0) {
    using Fmt = std::decay_t<decltype(towers[0].GetFormat())>;
    if (sizeQ < 1 || sizeQ >= towers.size()) throw math_error("hooks::ApproxModUp: sizeQ outside (0, towers)");
    const bool eval = towers[0].GetFormat() == Fmt::EVALUATION;
    for (size_t i = 0; i < sizeQ; i++)
        if (towers[i].GetFormat() != towers[0].GetFormat()) throw math_error("hooks::ApproxModUp: mixed formats");
    TowerView v = view(towers);
    const size_t sizeP = v.q.size() - sizeQ;
    auto pq = plan_of(v, 0, sizeQ, device), pp = plan_of(v, sizeQ, sizeP, device);
    std::vector<uint64_t> q(v.q.begin(), v.q.begin() + sizeQ), p(v.q.begin() + sizeQ, v.q.end());
    auto bc = converter(device, v.log_n, q, p, QHatInvModq, QHatModp, "hooks::ApproxModUp");
    const size_t wx = sizeQ * (size_t)v.n, wo = v.q.size() * (size_t)v.n;
    Staging& sx = staging(device, wx, 0);
    Staging& so = staging(device, wo, 1);
    sx.gather(cptr(std::vector<uint64_t*>(v.data.begin(), v.data.begin() + sizeQ)), v.n);
    sx.upload(wx);
    check(ofhe_hip_approx_mod_up(pq->get(), pp->get(), bc.get(), eval ? 1 : 0, sx.dev(), so.dev(), 1, nullptr),
          "hooks::ApproxModUp");
    so.download(wo);
    so.scatter(v.data, v.n);
    for (auto& t : towers) t.OverrideFormat(Fmt::EVALUATION);
}

// DCRTPolyImpl::ApproxModDown (dcrtpoly-impl.h:1133-1175): x = the Q|P towers
// in EVALUATION form -> out, the caller's `ans` (sizeQ = out.size() towers over
// paramsQ, after its DropLastElements), in EVALUATION form:
//   out_i = (x_i - NTT(t * ApproxSwitchCRTBasis_{P->Q}(t^-1 * INTT(x_P)))_i) * PInvModq_i
// with the t factors only when t > 0 (BGV; the reference's tInvModp is
// t.ModInverse(p_j), bgvrns-cryptoparameters.cpp:83-88, derived here from t).
// PHatInvModp / PHatModq ([sizeP][sizeQ]) as rns-cryptoparameters.cpp:172-215.
template <class TowersQP, class TowersQ>
void ApproxModDown(const TowersQP& x, TowersQ& out, const std::vector<uint64_t>& PInvModq,
                   const std::vector<uint64_t>& PHatInvModp, const std::vector<uint64_t>& PHatModq, uint64_t t = 0,
                   int device = 0) {
    using Fmt = std::decay_t<decltype(x[0].GetFormat())>;
    for (const auto& tw : x)
        if (tw.GetFormat() != Fmt::EVALUATION) throw math_error("hooks::ApproxModDown: EVALUATION form expected");
    TowerView vx = view(const_cast<TowersQP&>(x)), vo = view(out);
    const size_t sizeQ = vo.q.size();
    if (sizeQ >= vx.q.size()) throw math_error("hooks::ApproxModDown: output has as many towers as the input");
    if (!std::equal(vo.q.begin(), vo.q.end(), vx.q.begin()) || vo.n != vx.n)
        throw math_error("hooks::ApproxModDown: output basis is not the input's Q part");
    if (PInvModq.size() != sizeQ) throw math_error("hooks::ApproxModDown: PInvModq size");
    const size_t sizeP = vx.q.size() - sizeQ;
    auto pq = plan_of(vx, 0, sizeQ, device), pp = plan_of(vx, sizeQ, sizeP, device);
    std::vector<uint64_t> q(vx.q.begin(), vx.q.begin() + sizeQ), p(vx.q.begin() + sizeQ, vx.q.end());
    auto bc = converter(device, vx.log_n, p, q, PHatInvModp, PHatModq, "hooks::ApproxModDown");
    const size_t wx = vx.q.size() * (size_t)vx.n, wo = sizeQ * (size_t)vx.n;
    Staging& sx = staging(device, wx, 0);
    Staging& so = staging(device, wo, 1);
    sx.gather(cptr(vx.data), vx.n);
    sx.upload(wx);
    check(ofhe_hip_approx_mod_down(pq->get(), pp->get(), bc.get(), PInvModq.data(), t, sx.dev(), so.dev(), 1,
                                   nullptr),
          "hooks::ApproxModDown");
    so.download(wo);
    so.scatter(vo.data, vo.n);
    for (auto& tw : out) tw.OverrideFormat(Fmt::EVALUATION);
}

// DCRTPolyImpl::AutomorphismTransform(k) (dcrtpoly-impl.h:349-357 ->
// PolyImpl::AutomorphismTransform, poly-impl.h:312-365): out (the caller's
// result, same params and size as x) = sigma_k(x) tower by tower, in x's
// format (evaluation: bit-reversed slot permutation; coefficient: signed
// permutation).  An even k throws math_error as the reference does.
template <class Towers>
void AutomorphismTransform(const Towers& x, Towers& out, uint32_t k, int device = 0) {
    using Fmt = std::decay_t<decltype(x[0].GetFormat())>;
    const bool eval = x[0].GetFormat() == Fmt::EVALUATION;
    for (const auto& tw : x)
        if (tw.GetFormat() != x[0].GetFormat()) throw math_error("hooks::AutomorphismTransform: mixed formats");
    TowerView vx = view(const_cast<Towers&>(x)), vo = view(out);
    if (vx.q != vo.q || vx.n != vo.n) throw math_error("hooks::AutomorphismTransform: output basis differs");
    auto plan = plan_of(vx, 0, vx.q.size(), device);
    const size_t words = vx.q.size() * (size_t)vx.n;
    Staging& sx = staging(device, words, 0);
    Staging& so = staging(device, words, 1);
    sx.gather(cptr(vx.data), vx.n);
    sx.upload(words);
    check(ofhe_hip_automorphism(plan->get(), k, eval ? 1 : 0, sx.dev(), so.dev(), 1, nullptr),
          "hooks::AutomorphismTransform");
    so.download(words);
    so.scatter(vo.data, vo.n);
    for (auto& tw : out) tw.OverrideFormat(x[0].GetFormat());
}

namespace detail {
// x_t (op)= s_t over all towers in one launch; op 0 ModMul (Shoup), 2 ModSub
template <class Towers>
void scalar_eq(Towers& x, const std::vector<uint64_t>& s, int op, const char* what, int device) {
    TowerView v = view(x);
    if (s.size() != v.q.size()) throw math_error(std::string(what) + ": one scalar per tower required");
    auto plan = plan_of(v, 0, v.q.size(), device);
    const size_t words = v.q.size() * (size_t)v.n;
    Staging& st = staging(device, words, 0);
    st.gather(cptr(v.data), v.n);
    st.upload(words);
    check(op == 0 ? ofhe_hip_modmul_scalar(plan->get(), st.dev(), s.data(), st.dev(), 1, nullptr)
                  : ofhe_hip_modsub_scalar(plan->get(), st.dev(), s.data(), st.dev(), 1, nullptr),
          what);
    st.download(words);
    st.scatter(v.data, v.n);
}
}  // namespace detail

// DCRTPolyImpl::Times(const std::vector<NativeInteger>&) / Times(Integer) /
// operator*=(NativeInteger) (dcrtpoly-impl.h:586-661 -> PolyImpl::Times,
// NativeVectorT::ModMul(Eq)(const IntegerType&), mubintvecnat.cpp:310-332):
// tower t times s[t] mod q_t, in place (the caller copies first for Times).
template <class Towers>
void TimesScalarEq(Towers& x, const std::vector<uint64_t>& s, int device = 0) {
    detail::scalar_eq(x, s, 0, "hooks::TimesScalarEq", device);
}
// DCRTPolyImpl::Times(NativeInteger::SignedNativeInt) (dcrtpoly-impl.h:597-605
// -> PolyImpl::Times, poly-impl.h:237-252): a negative v multiplies by
// q - (|v| mod q) in every tower.
template <class Towers>
void TimesSignedEq(Towers& x, int64_t v, int device = 0) {
    std::vector<uint64_t> s;
    for (auto& tw : x) {
        const uint64_t q = (uint64_t)tw.GetParams()->GetModulus().ConvertToInt();
        const uint64_t mag = v < 0 ? (uint64_t)0 - (uint64_t)v : (uint64_t)v;  // |v| without overflow at INT64_MIN
        s.push_back(v < 0 ? q - mag % q : mag);                              // q - 0 = q reduces to 0
    }
    detail::scalar_eq(x, s, 0, "hooks::TimesSignedEq", device);
}
// DCRTPolyImpl::Minus(const Integer&) / Minus(const std::vector<Integer>&)
// (dcrtpoly-impl.h:565-584 -> PolyImpl::Minus, poly-impl.h:223-227): every word
// of tower t minus s[t] mod q_t, in either format.
template <class Towers>
void MinusScalarEq(Towers& x, const std::vector<uint64_t>& s, int device = 0) {
    detail::scalar_eq(x, s, 2, "hooks::MinusScalarEq", device);
}

}  // namespace hooks
}  // namespace ofhe
