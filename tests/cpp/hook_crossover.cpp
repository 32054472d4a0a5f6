// Measures every RUN_ON_HIP hook against the CPU loop it replaces, to set the
// gate in ofhe_openfhe_hooks.hpp (Policy::measured).  Same calls, same mock
// objects (mock_openfhe.hpp), the gate forced to the device and then to the
// CPU: the device leg is gather + PCIe up + launch + PCIe down + scatter,
// the CPU leg the reference's OpenMP loop over towers on the oracle (the
// stand-in for the reference's native backend), on
// OMP_NUM_THREADS threads.  Test infrastructure, run on the GPU box:
//
//   hook_crossover_bin [min_log_n max_log_n]  > profiles/r06_hook_crossover.txt
//
// Prints one line per (op, N, T): median ms of each leg, then the table the
// gate takes: per op and tower class the smallest log N from which the device
// wins (by kMargin) at every measured N up to 2^max, else kNever.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <random>
#include <string>
#include <vector>

#include "mock_openfhe.hpp"

using mock::Format;
using mock::Towers;
using ofhe::hooks::HookOp;
using Clock = std::chrono::steady_clock;
// the device must beat the CPU loop by this factor for the gate to take it
// (run-to-run noise of either leg is a few per cent)
constexpr double kMargin = 1.10;

// median of reps (>= 3, until ~budget seconds) of fn in ms
static double time_ms(const std::function<void()>& fn, double budget = 0.25) {
    fn();  // warm: tables, plans, staging, converters
    std::vector<double> t;
    const auto start = Clock::now();
    while (t.size() < 3 || (t.size() < 15 && std::chrono::duration<double>(Clock::now() - start).count() < budget)) {
        const auto a = Clock::now();
        fn();
        t.push_back(std::chrono::duration<double, std::milli>(Clock::now() - a).count());
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

int main(int argc, char** argv) {
    const uint32_t lo = argc > 2 ? (uint32_t)std::atoi(argv[1]) : 12, hi = argc > 2 ? (uint32_t)std::atoi(argv[2]) : 17;
    const size_t Ts[4] = {1, 8, 16, 48};
    std::printf("# hook crossover: device (host buffers, PCIe both ways) vs CPU loop (oracle, %d OpenMP threads)\n",
                omp_get_max_threads());
    std::printf("# %-22s %6s %4s %11s %11s %7s\n", "op", "log_n", "T", "device_ms", "cpu_ms", "cpu/dev");
    // wins[op][class][log_n]
    std::vector<std::vector<std::vector<int>>> wins(ofhe::hooks::kHookOps,
                                                    std::vector<std::vector<int>>(4, std::vector<int>(32, -1)));
    std::mt19937_64 rng(3);
    for (int c = 0; c < 4; c++) {
        const size_t T = Ts[c];
        for (uint32_t lg = lo; lg <= hi; lg++) {
            const uint32_t n = 1u << lg;
            // Q = T towers; P = alpha = ceil(T / dnum) with dnum = min(3, T) (HYBRID: P covers one digit)
            const uint32_t dnum = (uint32_t)std::min<size_t>(3, T);
            const size_t P = (T + dnum - 1) / dnum;
            std::vector<uint64_t> all(T + P), roots(T + P);
            oracle_moduli_chain(60, 2 * n, (unsigned)(T + P), all.data(), roots.data());
            std::vector<uint64_t> q(all.begin(), all.begin() + T), r(roots.begin(), roots.begin() + T);
            std::vector<uint64_t> p(all.begin() + T, all.end()), rp(roots.begin() + T, roots.end());
            auto A = mock::make_towers(n, q, r, rng, Format::EVALUATION);
            auto B = mock::make_towers(n, q, r, rng, Format::EVALUATION);
            auto Pt = mock::make_towers(n, p, rp, rng, Format::EVALUATION);
            auto QP = mock::make_towers(n, all, roots, rng, Format::EVALUATION);
            std::vector<uint64_t> hinv, hmod, pinv, phinv, phmodq, sc;
            mock::switch_tables(q, p, hinv, hmod);
            mock::moddown_tables(q, p, pinv, phinv, phmodq);
            for (size_t t = 0; t < T; t++) sc.push_back(rng());
            mock::KeySwitchHYBRID ks{T, P, dnum, {}, {}, "x"};
            for (uint32_t j = 0; j < dnum; j++) {
                ks.bv.push_back(QP);
                ks.av.push_back(QP);
            }
            {
                std::vector<const Towers*> bp, ap;
                for (uint32_t j = 0; j < dnum; j++) bp.push_back(&ks.bv[j]), ap.push_back(&ks.av[j]);
                ofhe::hooks::PutEvalKey("x", bp, ap, P);
            }
            mock::DCRTPolyImpl x{Format::EVALUATION, A}, y{Format::EVALUATION, B};
            mock::DCRTPolyImpl xc{Format::COEFFICIENT, A};
            for (auto& t : xc.m_vectors) t.OverrideFormat(Format::COEFFICIENT);
            mock::DCRTPolyImpl xqp{Format::EVALUATION, QP};
            struct Case {
                HookOp op;
                std::function<void()> fn;
            };
            std::vector<Case> cases = {
                {HookOp::SwitchFormat, [&] { x.SwitchFormat(); }},
                {HookOp::TimesEq, [&] { x *= y; }},
                {HookOp::PlusEq, [&] { x += y; }},
                {HookOp::MinusEq, [&] { x -= y; }},
                {HookOp::ApproxSwitchCRTBasis, [&] { (void)xc.ApproxSwitchCRTBasis(Pt, hinv, hmod); }},
                {HookOp::ApproxModUp,
                 [&] {
                     mock::DCRTPolyImpl u{Format::COEFFICIENT, xc.m_vectors};
                     u.ApproxModUp(Pt, hinv, hmod);
                 }},
                {HookOp::ApproxModDown, [&] { (void)xqp.ApproxModDown(T, pinv, phinv, phmodq, 0); }},
                {HookOp::AutomorphismTransform, [&] { (void)x.AutomorphismTransform(5); }},
                {HookOp::ScalarEq, [&] { x.TimesScalarEq(sc); }},
                {HookOp::KeySwitchCore, [&] { (void)ks.KeySwitchCore(x, 0); }},
            };
            for (auto& cs : cases) {
                ofhe::hooks::set_policy(ofhe::hooks::Policy::all(ofhe::hooks::kAlways));
                const double dev = time_ms(cs.fn);
                ofhe::hooks::set_policy(ofhe::hooks::Policy::all(ofhe::hooks::kNever));
                const double cpu = time_ms(cs.fn);
                wins[(int)cs.op][c][lg] = cpu >= kMargin * dev;
                std::printf("  %-22s %6u %4zu %11.3f %11.3f %7.2f\n", ofhe::hooks::hook_name(cs.op), lg, T, dev, cpu,
                            cpu / dev);
                std::fflush(stdout);
            }
            ofhe::hooks::EraseEvalKey("x");
        }
    }
    std::printf("# Policy::measured() table: min log N per tower class {T<8, 8<=T<16, 16<=T<48, T>=48}\n");
    for (int op = 0; op < ofhe::hooks::kHookOps; op++) {
        std::printf("  /* %-21s */ {", ofhe::hooks::hook_name((HookOp)op));
        for (int c = 0; c < 4; c++) {
            // smallest lg such that the device wins at lg and every larger measured lg
            int need = -1;
            for (int lg = (int)hi; lg >= (int)lo; lg--) {
                if (wins[op][c][lg] == 1)
                    need = lg;
                else
                    break;
            }
            if (need < 0)
                std::printf("kNever");
            else
                std::printf("%d", need);
            std::printf(c < 3 ? ", " : "},\n");
        }
    }
    return 0;
}
