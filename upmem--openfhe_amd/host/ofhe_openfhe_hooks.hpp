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
#pragma once

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

// DCRTPolyImpl::ApproxSwitchCRTBasis (dcrtpoly-impl.h:1034-1063): x's towers
// (basis Q, COEFFICIENT form) -> out's towers (basis P, already sized by the
// caller as the reference's `ans(paramsP, m_format, true)`), with the
// QHatInvModq / QHatModp tables the pke layer precomputes
// (rns-cryptoparameters.cpp:273-337; QHatModp row-major [sizeQ][sizeP]).
// The converter is built once per (Q, P) and cached.
template <class TowersQ, class TowersP>
void ApproxSwitchCRTBasis(const TowersQ& x, TowersP& out, const std::vector<uint64_t>& QHatInvModq,
                          const std::vector<uint64_t>& QHatModp, int device = 0) {
    TowerView vx = view(const_cast<TowersQ&>(x)), vo = view(out);
    if (vx.n != vo.n) throw math_error("hooks::ApproxSwitchCRTBasis: ring dimensions differ");
    if (QHatInvModq.size() != vx.q.size() || QHatModp.size() != vx.q.size() * vo.q.size())
        throw math_error("hooks::ApproxSwitchCRTBasis: table sizes");
    HipManager* m = HipManager::getHip(device);
    static std::mutex mu;  // the converter cache is process-wide
    static std::map<std::vector<uint64_t>, std::shared_ptr<ofhe_bconv_s>> cache;
    std::shared_ptr<ofhe_bconv_s> bc;
    {
        std::vector<uint64_t> key{(uint64_t)device, vx.log_n, vx.q.size()};
        key.insert(key.end(), vx.q.begin(), vx.q.end());
        key.insert(key.end(), vo.q.begin(), vo.q.end());
        key.insert(key.end(), QHatInvModq.begin(), QHatInvModq.end());
        key.insert(key.end(), QHatModp.begin(), QHatModp.end());
        std::lock_guard<std::mutex> lk(mu);
        auto& e = cache[key];
        if (!e) {
            ofhe_bconv_t h = nullptr;
            check(ofhe_hip_bconv_create(m->ctx(), vx.log_n, (uint32_t)vx.q.size(), (uint32_t)vo.q.size(), vx.q.data(),
                                        vo.q.data(), QHatInvModq.data(), QHatModp.data(), &h),
                  "hooks::ApproxSwitchCRTBasis");
            e = std::shared_ptr<ofhe_bconv_s>(h, [](ofhe_bconv_t p) { ofhe_hip_bconv_destroy(p); });
        }
        bc = e;
    }
    const size_t wx = vx.q.size() * (size_t)vx.n, wo = vo.q.size() * (size_t)vo.n;
    Staging& sx = staging(device, wx, 0);
    Staging& so = staging(device, wo, 1);
    sx.gather(cptr(vx.data), vx.n);
    sx.upload(wx);
    check(ofhe_hip_approx_switch_crt_basis(bc.get(), sx.dev(), so.dev(), 1, nullptr), "hooks::ApproxSwitchCRTBasis");
    so.download(wo);
    so.scatter(vo.data, vo.n);
}

}  // namespace hooks
}  // namespace ofhe
