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
// Every hook is gated: it returns false, touching nothing, unless the device
// (PCIe both ways included) beats the reference's own OpenMP loop over the
// towers for this ring dimension and tower count -- the crossover measured by
// tests/cpp/hook_crossover.cpp (profiles/r06_hook_crossover.txt)
// -- and the caller then runs that loop unchanged.
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
//   KeySwitchHYBRID::KeySwitchCore      keyswitch-hybrid.cpp:324-328 -> KeySwitchCore(a, tag, ...)
//     with the evaluation key made resident once by PutEvalKey (the
//     EvalMultKeyGen / EvalAtIndexKeyGen hook, evalkeyrelin.h:136,166)
#pragma once

#include <algorithm>
#include <cstdint>
#include <map>
#include <mutex>
#include <string>
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
// Cost: each calling thread keeps two pinned slots (plus their device
// twins) as large as its largest hooked call -- 48 + 96 MiB for a key switch at
// N = 2^17, 48 towers -- until the thread exits.
inline Staging& staging(int device, size_t words, int slot = 0) {
    thread_local std::map<std::pair<int, int>, std::unique_ptr<Staging>> pool;
    auto& s = pool[{device, slot}];
    if (!s || s->words() < words) {
        s.reset();  // release the smaller buffer first
        s.reset(new Staging(HipManager::getHip(device), words));
    }
    return *s;
}

// ---------------------------------------------------------------------------
// The gate.  HookOp names a hook; the device takes a call when the ring
// dimension n >= 2^min_log_n[op][tower class].  Tower classes bracket the
// tower counts the crossover was measured at, T = 1, 8, 16, 48 Q towers:
// T < 8, 8 <= T < 16, 16 <= T < 48, T >= 48, counted as the hook sees them
// (the basis ops and the key switch count Q + P with P = ceil(Q / 3), which
// falls in the same class as Q for every measured point).  kNever keeps an op
// on the CPU loop at every measured size (the element-wise hooks: at 16-24
// PCIe bytes per coefficient the host-buffer path cannot beat a host loop
// over the same words in the host's memory and caches; they pay only in the
// resident integration, DCRTPolyHip).  Rings below kDeviceMinRing
// (binfhe's, N <= 2^11, rgsw-acc-*.cpp) always stay on the CPU.
// ---------------------------------------------------------------------------
enum class HookOp : int {
    SwitchFormat = 0,
    TimesEq,
    PlusEq,
    MinusEq,
    ApproxSwitchCRTBasis,
    ApproxModUp,
    ApproxModDown,
    AutomorphismTransform,
    ScalarEq,  // TimesScalarEq / TimesSignedEq / MinusScalarEq
    KeySwitchCore,
    Count
};
constexpr int kHookOps = (int)HookOp::Count;
constexpr uint8_t kNever = 255, kAlways = 0;
constexpr uint32_t kDeviceMinRing = 4096;

inline const char* hook_name(HookOp op) {
    static const char* names[kHookOps] = {"SwitchFormat",  "TimesEq",     "PlusEq",
                                          "MinusEq",       "ApproxSwitchCRTBasis", "ApproxModUp",
                                          "ApproxModDown", "AutomorphismTransform", "ScalarEq",
                                          "KeySwitchCore"};
    return names[(int)op];
}
inline int tower_class(size_t towers) { return towers < 8 ? 0 : towers < 16 ? 1 : towers < 48 ? 2 : 3; }

struct Policy {
    uint8_t min_log_n[kHookOps][4];
    // measured: tests/cpp/hook_crossover.cpp on the MI355X box (host
    // buffers, pipelined pinned staging, both PCIe directions; the CPU loop
    // on 16 OpenMP threads), device taken where it wins by >= 10 % at that
    // N and every larger one; two runs on two boxes
    // (profiles/r06_hook_crossover.txt, r06m_hook_crossover.txt), entry by
    // entry the larger (the CPU kept where either run put the crossover
    // higher; the runs differ by one step at four borderline entries).
    // DESIGN.md (b).
    static Policy measured() {
        Policy p{};
        const uint8_t table[kHookOps][4] = {
            /* SwitchFormat          */ {13, 14, 14, 13},
            /* TimesEq               */ {16, kNever, kNever, kNever},
            /* PlusEq                */ {kNever, kNever, kNever, kNever},
            /* MinusEq               */ {kNever, kNever, kNever, kNever},
            /* ApproxSwitchCRTBasis  */ {17, 14, 12, 12},
            /* ApproxModUp           */ {14, 12, 12, 12},
            /* ApproxModDown         */ {12, 12, 12, 12},
            /* AutomorphismTransform */ {13, 14, 14, 14},
            /* ScalarEq              */ {kNever, kNever, kNever, kNever},
            /* KeySwitchCore         */ {12, 12, 12, 12},
        };
        for (int o = 0; o < kHookOps; o++)
            for (int c = 0; c < 4; c++) p.min_log_n[o][c] = table[o][c];
        return p;
    }
    static Policy all(uint8_t v) {  // kAlways / kNever everywhere (tests, A/B timing)
        Policy p{};
        for (auto& r : p.min_log_n)
            for (auto& c : r) c = v;
        return p;
    }
};
namespace detail {
inline std::mutex& policy_mu() {
    static std::mutex m;
    return m;
}
inline Policy& policy_ref() {
    static Policy p = Policy::measured();
    return p;
}
}  // namespace detail
inline Policy policy() {
    std::lock_guard<std::mutex> lk(detail::policy_mu());
    return detail::policy_ref();
}
inline void set_policy(const Policy& p) {
    std::lock_guard<std::mutex> lk(detail::policy_mu());
    detail::policy_ref() = p;
}
// Whether the device takes `op` on `towers` towers of ring dimension n.
inline bool device_takes(HookOp op, uint32_t n, size_t towers) {
    if (n < kDeviceMinRing || towers == 0) return false;
    const uint8_t need = policy().min_log_n[(int)op][tower_class(towers)];
    if (need == kNever) return false;
    uint32_t lg = 0;
    while ((1u << lg) < n) lg++;
    return lg >= need;
}
template <class Towers>
uint32_t ring_of(const Towers& towers) {
    return towers.empty() ? 0 : (uint32_t)towers[0].GetParams()->GetRingDimension();
}

// Whether the device takes DCRTPolyImpl::SwitchFormat for these towers: a
// power-of-two cyclotomic (PolyImpl::SwitchFormat sends rd != co / 2 to
// ArbitrarySwitchFormat, poly-impl.h:412-420), every tower in the same
// format, and the gate.
template <class Towers>
bool device_switch_format(const Towers& towers) {
    if (towers.empty()) return false;
    const auto& p0 = *towers[0].GetParams();
    const uint32_t n = (uint32_t)p0.GetRingDimension();
    if ((uint64_t)p0.GetCyclotomicOrder() != 2 * (uint64_t)n) return false;
    for (const auto& t : towers)
        if (t.GetFormat() != towers[0].GetFormat()) return false;
    return device_takes(HookOp::SwitchFormat, n, towers.size());
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
    st.put_towers(cptr(v.data), v.n);
    check(to_eval ? ofhe_hip_ntt_fwd(plan->get(), st.dev(), 1, nullptr)
                  : ofhe_hip_ntt_inv(plan->get(), st.dev(), 1, nullptr),
          "hooks::SwitchFormat");
    st.get_towers(v.data, v.n);
    for (auto& t : towers) t.OverrideFormat(to_eval ? Fmt::EVALUATION : Fmt::COEFFICIENT);
    return true;
}

namespace detail {
// a (op)= b over all towers in one launch; op 0 ModMul (Barrett), 1 ModAdd, 2 ModSub
template <class Towers>
bool binary_eq(Towers& a, const Towers& b, int op, const char* what, int device) {
    const HookOp hop = op == 0 ? HookOp::TimesEq : op == 1 ? HookOp::PlusEq : HookOp::MinusEq;
    if (!device_takes(hop, ring_of(a), a.size())) return false;
    TowerView va = view(a);
    TowerView vb = view(const_cast<Towers&>(b));
    if (va.q != vb.q || va.n != vb.n) throw math_error(std::string(what) + ": Modulus missmatch");
    auto plan = PlanCache::get(device, va.log_n, va.q, va.psi);
    const size_t words = va.q.size() * (size_t)va.n;
    Staging& sa = staging(device, words, 0);
    Staging& sb = staging(device, words, 1);
    sa.put_towers(cptr(va.data), va.n);
    sb.put_towers(cptr(vb.data), vb.n);
    int rc = op == 0   ? ofhe_hip_modmul_vv(plan->get(), sa.dev(), sb.dev(), sa.dev(), 1, nullptr)
             : op == 1 ? ofhe_hip_modadd_vv(plan->get(), sa.dev(), sb.dev(), sa.dev(), 1, nullptr)
                       : ofhe_hip_modsub_vv(plan->get(), sa.dev(), sb.dev(), sa.dev(), 1, nullptr);
    check(rc, what);
    sa.get_towers(va.data, va.n);
    return true;
}
}  // namespace detail

// DCRTPolyImpl::operator*= (dcrtpoly.h:142-148; EVALUATION form, the caller
// checks).  Each returns false, touching nothing, when the gate keeps the op
// on the caller's loop.
template <class Towers>
bool TimesEq(Towers& a, const Towers& b, int device = 0) {
    return detail::binary_eq(a, b, 0, "hooks::TimesEq", device);
}
// DCRTPolyImpl::operator+= (dcrtpoly-impl.h:410-416)
template <class Towers>
bool PlusEq(Towers& a, const Towers& b, int device = 0) {
    return detail::binary_eq(a, b, 1, "hooks::PlusEq", device);
}
// DCRTPolyImpl::operator-=
template <class Towers>
bool MinusEq(Towers& a, const Towers& b, int device = 0) {
    return detail::binary_eq(a, b, 2, "hooks::MinusEq", device);
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
bool ApproxSwitchCRTBasis(const TowersQ& x, TowersP& out, const std::vector<uint64_t>& QHatInvModq,
                          const std::vector<uint64_t>& QHatModp, int device = 0) {
    if (!device_takes(HookOp::ApproxSwitchCRTBasis, ring_of(x), x.size() + out.size())) return false;
    TowerView vx = view(const_cast<TowersQ&>(x)), vo = view(out);
    if (vx.n != vo.n) throw math_error("hooks::ApproxSwitchCRTBasis: ring dimensions differ");
    auto bc = converter(device, vx.log_n, vx.q, vo.q, QHatInvModq, QHatModp, "hooks::ApproxSwitchCRTBasis");
    const size_t wx = vx.q.size() * (size_t)vx.n, wo = vo.q.size() * (size_t)vo.n;
    Staging& sx = staging(device, wx, 0);
    Staging& so = staging(device, wo, 1);
    sx.put_towers(cptr(vx.data), vx.n);
    check(ofhe_hip_approx_switch_crt_basis(bc.get(), sx.dev(), so.dev(), 1, nullptr), "hooks::ApproxSwitchCRTBasis");
    so.get_towers(vo.data, vo.n);
    return true;
}

// DCRTPolyImpl::ApproxModUp (dcrtpoly-impl.h:1084-1131).  `towers` is
// m_vectors after the caller's resize to Q|P: the sizeQ towers of x (all in
// one format) followed by sizeP towers whose params are paramsP's (their
// values are ignored).  On return every tower holds ApproxModUp(x) in
// EVALUATION form -- the Q towers x itself in evaluation form, the P towers
// NTT(ApproxSwitchCRTBasis(x)) -- and says so (OverrideFormat), as the
// reference's m_format = EVALUATION, m_params = paramsQP leave it.  The caller
// appends the P towers only when device_takes(HookOp::ApproxModUp, n, sizeQ +
// sizeP); a false return leaves `towers` untouched.
template <class Towers>
bool ApproxModUp(Towers& towers, size_t sizeQ, const std::vector<uint64_t>& QHatInvModq,
                 const std::vector<uint64_t>& QHatModp, int device = 0) {
    if (!device_takes(HookOp::ApproxModUp, ring_of(towers), towers.size())) return false;
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
    sx.put_towers(cptr(std::vector<uint64_t*>(v.data.begin(), v.data.begin() + sizeQ)), v.n);
    check(ofhe_hip_approx_mod_up(pq->get(), pp->get(), bc.get(), eval ? 1 : 0, sx.dev(), so.dev(), 1, nullptr),
          "hooks::ApproxModUp");
    so.get_towers(v.data, v.n);
    for (auto& t : towers) t.OverrideFormat(Fmt::EVALUATION);
    return true;
}

// DCRTPolyImpl::ApproxModDown (dcrtpoly-impl.h:1133-1175): x = the Q|P towers
// in EVALUATION form -> out, the caller's `ans` (sizeQ = out.size() towers over
// paramsQ, after its DropLastElements), in EVALUATION form:
//   out_i = (x_i - NTT(t * ApproxSwitchCRTBasis_{P->Q}(t^-1 * INTT(x_P)))_i) * PInvModq_i
// with the t factors only when t > 0 (BGV; the reference's tInvModp is
// t.ModInverse(p_j), bgvrns-cryptoparameters.cpp:83-88, derived here from t).
// PHatInvModp / PHatModq ([sizeP][sizeQ]) as rns-cryptoparameters.cpp:172-215.
template <class TowersQP, class TowersQ>
bool ApproxModDown(const TowersQP& x, TowersQ& out, const std::vector<uint64_t>& PInvModq,
                   const std::vector<uint64_t>& PHatInvModp, const std::vector<uint64_t>& PHatModq, uint64_t t = 0,
                   int device = 0) {
    if (!device_takes(HookOp::ApproxModDown, ring_of(x), x.size())) return false;
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
    sx.put_towers(cptr(vx.data), vx.n);
    check(ofhe_hip_approx_mod_down(pq->get(), pp->get(), bc.get(), PInvModq.data(), t, sx.dev(), so.dev(), 1,
                                   nullptr),
          "hooks::ApproxModDown");
    so.get_towers(vo.data, vo.n);
    for (auto& tw : out) tw.OverrideFormat(Fmt::EVALUATION);
    return true;
}

// DCRTPolyImpl::AutomorphismTransform(k) (dcrtpoly-impl.h:349-357 ->
// PolyImpl::AutomorphismTransform, poly-impl.h:312-365): out (the caller's
// result, same params and size as x) = sigma_k(x) tower by tower, in x's
// format (evaluation: bit-reversed slot permutation; coefficient: signed
// permutation).  An even k throws math_error as the reference does.
template <class Towers>
bool AutomorphismTransform(const Towers& x, Towers& out, uint32_t k, int device = 0) {
    if (!device_takes(HookOp::AutomorphismTransform, ring_of(x), x.size())) return false;
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
    sx.put_towers(cptr(vx.data), vx.n);
    check(ofhe_hip_automorphism(plan->get(), k, eval ? 1 : 0, sx.dev(), so.dev(), 1, nullptr),
          "hooks::AutomorphismTransform");
    so.get_towers(vo.data, vo.n);
    for (auto& tw : out) tw.OverrideFormat(x[0].GetFormat());
    return true;
}

namespace detail {
// x_t (op)= s_t over all towers in one launch; op 0 ModMul (Shoup), 2 ModSub
template <class Towers>
bool scalar_eq(Towers& x, const std::vector<uint64_t>& s, int op, const char* what, int device) {
    if (!device_takes(HookOp::ScalarEq, ring_of(x), x.size())) return false;
    TowerView v = view(x);
    if (s.size() != v.q.size()) throw math_error(std::string(what) + ": one scalar per tower required");
    auto plan = plan_of(v, 0, v.q.size(), device);
    const size_t words = v.q.size() * (size_t)v.n;
    Staging& st = staging(device, words, 0);
    st.put_towers(cptr(v.data), v.n);
    check(op == 0 ? ofhe_hip_modmul_scalar(plan->get(), st.dev(), s.data(), st.dev(), 1, nullptr)
                  : ofhe_hip_modsub_scalar(plan->get(), st.dev(), s.data(), st.dev(), 1, nullptr),
          what);
    st.get_towers(v.data, v.n);
    return true;
}
}  // namespace detail

// DCRTPolyImpl::Times(const std::vector<NativeInteger>&) / Times(Integer) /
// operator*=(NativeInteger) (dcrtpoly-impl.h:586-661 -> PolyImpl::Times,
// NativeVectorT::ModMul(Eq)(const IntegerType&), mubintvecnat.cpp:310-332):
// tower t times s[t] mod q_t, in place (the caller copies first for Times).
template <class Towers>
bool TimesScalarEq(Towers& x, const std::vector<uint64_t>& s, int device = 0) {
    return detail::scalar_eq(x, s, 0, "hooks::TimesScalarEq", device);
}
// DCRTPolyImpl::Times(NativeInteger::SignedNativeInt) (dcrtpoly-impl.h:597-605
// -> PolyImpl::Times, poly-impl.h:237-252): a negative v multiplies by
// q - (|v| mod q) in every tower.
template <class Towers>
bool TimesSignedEq(Towers& x, int64_t v, int device = 0) {
    if (!device_takes(HookOp::ScalarEq, ring_of(x), x.size())) return false;
    std::vector<uint64_t> s;
    for (auto& tw : x) {
        const uint64_t q = (uint64_t)tw.GetParams()->GetModulus().ConvertToInt();
        const uint64_t mag = v < 0 ? (uint64_t)0 - (uint64_t)v : (uint64_t)v;  // |v| without overflow at INT64_MIN
        s.push_back(v < 0 ? q - mag % q : mag);                              // q - 0 = q reduces to 0
    }
    return detail::scalar_eq(x, s, 0, "hooks::TimesSignedEq", device);
}
// DCRTPolyImpl::Minus(const Integer&) / Minus(const std::vector<Integer>&)
// (dcrtpoly-impl.h:565-584 -> PolyImpl::Minus, poly-impl.h:223-227): every word
// of tower t minus s[t] mod q_t, in either format.
template <class Towers>
bool MinusScalarEq(Towers& x, const std::vector<uint64_t>& s, int device = 0) {
    return detail::scalar_eq(x, s, 2, "hooks::MinusScalarEq", device);
}

// ---------------------------------------------------------------------------
// HYBRID key switching, hooked one level up: KeySwitchHYBRID::KeySwitchCore
// (keyswitch-hybrid.cpp:324-328) = EvalKeySwitchPrecomputeCore (digit
// decomposition, per-digit ApproxSwitchCRTBasis, 330-412) ->
// EvalFastKeySwitchCoreExt (key inner product, 438-482) -> two ApproxModDown
// (414-435), all in one ofhe_hip_ks_core call on device-resident keys.
// ---------------------------------------------------------------------------
// One evaluation key on the device: EvalKeyRelinImpl's b and a vectors
// (evalkeyrelin.h:136,166; numPartQ DCRTPolys over Q|P each) as two
// DCRTPolyHip of batch numPartQ, with the bases they came with.
struct HookEvalKey {
    std::shared_ptr<DCRTParams> Q, P, QP;
    uint32_t num_part_q = 0;
    std::shared_ptr<const KeyCache::Key> key;
};
namespace detail {
inline std::mutex& keys_mu() {
    static std::mutex m;
    return m;
}
inline std::map<std::string, std::shared_ptr<const HookEvalKey>>& keys() {
    static std::map<std::string, std::shared_ptr<const HookEvalKey>> m;
    return m;
}
}  // namespace detail

// The EvalMultKeyGen / EvalAtIndexKeyGen side: uploads the key once, keyed by
// its tag (Key::GetKeyTag).  bv[j] / av[j] are the tower vectors of
// GetBVector()[j] / GetAVector()[j] (DCRTPolyImpl::GetAllElements,
// dcrtpoly.h:391-397), all over the same Q|P basis in EVALUATION form, whose
// last sizeP towers are P (CryptoParametersRNS::GetParamsP).
template <class Towers>
void PutEvalKey(const std::string& tag, const std::vector<const Towers*>& bv, const std::vector<const Towers*>& av,
                size_t sizeP, int device = 0) {
    if (bv.empty() || bv.size() != av.size()) throw math_error("hooks::PutEvalKey: b and a need numPartQ polynomials each");
    TowerView v0 = view(const_cast<Towers&>(*bv[0]));
    if (sizeP < 1 || sizeP >= v0.q.size()) throw math_error("hooks::PutEvalKey: sizeP outside (0, towers)");
    const size_t T = v0.q.size(), n = v0.n, dnum = bv.size();
    auto HK = std::make_shared<HookEvalKey>();
    const size_t sizeQ = T - sizeP;
    HK->Q = std::make_shared<DCRTParams>(2 * (uint32_t)n, std::vector<uint64_t>(v0.q.begin(), v0.q.begin() + sizeQ),
                                         std::vector<uint64_t>(v0.psi.begin(), v0.psi.begin() + sizeQ), device);
    HK->P = std::make_shared<DCRTParams>(2 * (uint32_t)n, std::vector<uint64_t>(v0.q.begin() + sizeQ, v0.q.end()),
                                         std::vector<uint64_t>(v0.psi.begin() + sizeQ, v0.psi.end()), device);
    HK->QP = std::make_shared<DCRTParams>(2 * (uint32_t)n, v0.q, v0.psi, device);
    HK->num_part_q = (uint32_t)dnum;
    std::vector<uint64_t> fb, fa;
    fb.reserve(dnum * T * n);
    fa.reserve(dnum * T * n);
    for (size_t j = 0; j < dnum; j++) {
        for (int which = 0; which < 2; which++) {
            const Towers& tj = *(which ? av[j] : bv[j]);
            using Fmt = std::decay_t<decltype(tj[0].GetFormat())>;
            for (const auto& tw : tj)
                if (tw.GetFormat() != Fmt::EVALUATION) throw math_error("hooks::PutEvalKey: EVALUATION form expected");
            TowerView vj = view(const_cast<Towers&>(tj));
            if (vj.q != v0.q || vj.psi != v0.psi || vj.n != v0.n)
                throw math_error("hooks::PutEvalKey: key polynomials over different bases");
            auto& f = which ? fa : fb;
            for (size_t t = 0; t < T; t++) f.insert(f.end(), vj.data[t], vj.data[t] + n);
        }
    }
    DCRTPolyHip b(HK->QP, Format::EVALUATION, (uint32_t)dnum, DCRTPolyHip::Uninit{});
    DCRTPolyHip a(HK->QP, Format::EVALUATION, (uint32_t)dnum, DCRTPolyHip::Uninit{});
    b.SetValues(fb, Format::EVALUATION);
    a.SetValues(fa, Format::EVALUATION);
    HK->key = KeyCache::put("hooks:" + tag, std::move(b), std::move(a));
    std::lock_guard<std::mutex> lk(detail::keys_mu());
    detail::keys()[tag] = HK;
}
inline void EraseEvalKey(const std::string& tag) {
    KeyCache::erase("hooks:" + tag);
    std::lock_guard<std::mutex> lk(detail::keys_mu());
    detail::keys().erase(tag);
}
inline std::shared_ptr<const HookEvalKey> GetEvalKey(const std::string& tag) {
    std::lock_guard<std::mutex> lk(detail::keys_mu());
    auto it = detail::keys().find(tag);
    if (it == detail::keys().end()) throw math_error("hooks::KeySwitchCore: no resident evaluation key '" + tag + "'");
    return it->second;
}

// KeySwitchCore(a, evalKey) for the key PutEvalKey stored under `tag`: a's
// towers (Ql, a prefix of Q, EVALUATION form) -> ct0, ct1 (the caller's two
// DCRTPoly(paramsQl, EVALUATION) outputs, l towers each), t = the BGV
// plaintext modulus or 0 (cryptoParams->GetNoiseScale() == 1, 313).  Gather
// a, one upload, one ofhe_hip_ks_core, one download of both outputs, scatter.
// Returns false, touching nothing, when the gate keeps it on the CPU.
template <class TowersQl, class TowersOut>
bool KeySwitchCore(const TowersQl& a, const std::string& tag, uint64_t t, TowersOut& ct0, TowersOut& ct1,
                   int device = 0) {
    auto HK = GetEvalKey(tag);
    const size_t T = HK->QP->Towers();
    if (!device_takes(HookOp::KeySwitchCore, ring_of(a), T)) return false;
    using Fmt = std::decay_t<decltype(a[0].GetFormat())>;
    for (const auto& tw : a)
        if (tw.GetFormat() != Fmt::EVALUATION) throw math_error("hooks::KeySwitchCore: EVALUATION form expected");
    TowerView va = view(const_cast<TowersQl&>(a)), v0 = view(ct0), v1 = view(ct1);
    const size_t l = va.q.size(), n = va.n;
    const auto& Qm = HK->Q->Moduli();
    if (n != HK->QP->GetRingDimension()) throw math_error("hooks::KeySwitchCore: ring dimension differs from the key's");
    if (l > Qm.size() || !std::equal(va.q.begin(), va.q.end(), Qm.begin()))
        throw math_error("hooks::KeySwitchCore: ciphertext basis is not a prefix of the key's Q");
    if (v0.q != va.q || v1.q != va.q || v0.n != n || v1.n != n)
        throw math_error("hooks::KeySwitchCore: outputs must be over the ciphertext's basis");
    auto ks = KsCache::get(*HK->Q, *HK->P, HK->num_part_q);
    const size_t words = l * n;
    Staging& sx = staging(device, words, 0);
    Staging& so = staging(device, 2 * words, 1);
    sx.put_towers(cptr(va.data), n);
    check(ofhe_hip_ks_core(ks->handle(), (uint32_t)l, sx.dev(), HK->key->b.data(), HK->key->a.data(), so.dev(),
                           so.dev() + words, t, 1, nullptr),
          "hooks::KeySwitchCore");
    std::vector<uint64_t*> both(v0.data);
    both.insert(both.end(), v1.data.begin(), v1.data.end());
    so.get_towers(both, n);
    for (auto& tw : ct0) tw.OverrideFormat(Fmt::EVALUATION);
    for (auto& tw : ct1) tw.OverrideFormat(Fmt::EVALUATION);
    return true;
}

}  // namespace hooks
}  // namespace ofhe
