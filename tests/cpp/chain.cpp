// Device-resident operator chain through the C++ adapter (ofhe_dcrt.hpp), the
// way an OpenFHE evaluation strings DCRTPoly calls together: nothing returns
// to the host between the steps.
//
//   X  = SwitchFormat(A)                      dcrtpoly-impl.h:2518-2524   (COEFFICIENT -> EVALUATION)
//   Y  = X * B                                dcrtpoly.h:185-200          (Hadamard)
//   Z  = SwitchFormat(Y)                      (EVALUATION -> COEFFICIENT)
//   Z1 = Z.Plus(s) ; Z2 = Z1.Minus(s')        dcrtpoly-impl.h:545-584      (scalar, coefficient form)
//   U  = ApproxModUp(Z2)                      dcrtpoly-impl.h:1085-1131    (Q -> Q|P, EVALUATION)
//   (K0, K1) = KeySwitchCore(Y, kb, ka)       keyswitch-hybrid.cpp:325-328
//   D  = ApproxModDown(U * P)                 dcrtpoly-impl.h:1134-1175    (== SwitchFormat(Z2))
//
// usage: chain_bin <out.bin> [reps]
// Writes the parameters, inputs and every intermediate to <out.bin> for
// tests/test_cpp_host.py, which checks each against the CPU oracle, and prints
// the chain's wall time per repetition (inputs resident, one sync at the end).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../../upmem--openfhe_amd/host/ofhe_dcrt.hpp"

using namespace ofhe;
typedef unsigned __int128 u128;

static uint64_t mulmod(uint64_t a, uint64_t b, uint64_t q) { return (uint64_t)((u128)a * b % q); }
static uint64_t powmod(uint64_t b, uint64_t e, uint64_t q) {
    uint64_t r = 1 % q;
    b %= q;
    for (; e; e >>= 1, b = mulmod(b, b, q))
        if (e & 1) r = mulmod(r, b, q);
    return r;
}
static bool is_prime(uint64_t n) {
    if (n < 2) return false;
    const uint64_t bases[] = {2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37};
    for (auto b : bases)
        if (n % b == 0) return n == b;
    uint64_t d = n - 1;
    int s = 0;
    while (!(d & 1)) d >>= 1, s++;
    for (auto b : bases) {
        uint64_t x = powmod(b, d, n);
        if (x == 1 || x == n - 1) continue;
        bool comp = true;
        for (int r = 1; r < s && comp; r++)
            if ((x = mulmod(x, x, n)) == n - 1) comp = false;
        if (comp) return false;
    }
    return true;
}
// poly-benchmark chain (poly-benchmark-16k.cpp:89-96), minimal roots (nbtheory-impl.h:183-231)
static std::vector<uint64_t> chain(uint32_t m, int count) {
    uint64_t q = (1ull << 60) + 1;
    while (!is_prime(q)) q += m;
    std::vector<uint64_t> out;
    for (int i = 0; i < count; i++) {
        q -= m;
        while (!is_prime(q)) q -= m;
        out.push_back(q);
    }
    return out;
}
static uint64_t root_of_unity(uint64_t m, uint64_t q) {
    uint64_t psi = 0;
    for (uint64_t c = 2;; c++)
        if (powmod(psi = powmod(c, (q - 1) / m, q), m / 2, q) == q - 1) break;
    uint64_t p2 = mulmod(psi, psi, q), x = psi, best = psi;
    for (uint64_t k = 3; k < m; k += 2)
        if ((x = mulmod(x, p2, q)) < best) best = x;
    return best;
}
static uint64_t prod_mod(const std::vector<uint64_t>& v, size_t skip, uint64_t m) {
    uint64_t r = 1 % m;
    for (size_t k = 0; k < v.size(); k++)
        if (k != skip) r = mulmod(r, v[k] % m, m);
    return r;
}
static std::shared_ptr<DCRTParams> params(uint32_t m, const std::vector<uint64_t>& q) {
    std::vector<uint64_t> r;
    for (auto x : q) r.push_back(root_of_unity(m, x));
    return std::make_shared<DCRTParams>(m, q, r);
}
static std::unique_ptr<BaseConverter> converter(const DCRTParams& A, const DCRTParams& B) {
    std::vector<uint64_t> hinv, hmod;
    const auto& a = A.Moduli();
    for (size_t i = 0; i < a.size(); i++) {
        hinv.push_back(powmod(prod_mod(a, i, a[i]), a[i] - 2, a[i]));
        for (auto bj : B.Moduli()) hmod.push_back(prod_mod(a, i, bj));
    }
    return std::unique_ptr<BaseConverter>(new BaseConverter(A, B, hinv, hmod));
}

static void put(FILE* f, const std::vector<uint64_t>& v) {
    const uint64_t n = v.size();
    std::fwrite(&n, 8, 1, f);
    std::fwrite(v.data(), 8, n, f);
}

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s out.bin [reps]\n", argv[0]);
        return 2;
    }
    const int reps = argc > 2 ? std::atoi(argv[2]) : 5;
    const uint32_t log_n = 13, m = 2u << log_n, n = m / 2, batch = 2, sq = 6, sp = 2, dnum = 3;
    try {
        auto all = chain(m, sq + sp);
        std::vector<uint64_t> q(all.begin(), all.begin() + sq), p(all.begin() + sq, all.end());
        auto PQ = params(m, q), PP = params(m, p), PQP = params(m, all);
        auto up = converter(*PQ, *PP), down = converter(*PP, *PQ);
        auto ks = KsCache::get(*PQ, *PP, dnum);
        std::vector<uint64_t> pinv, pmod;
        for (auto qi : q) pinv.push_back(powmod(prod_mod(p, p.size(), qi), qi - 2, qi));
        for (auto mm : all) pmod.push_back(prod_mod(p, p.size(), mm));

        std::mt19937_64 rng(2024);
        auto uniform = [&](const std::vector<uint64_t>& mods, uint32_t rows) {
            std::vector<uint64_t> v((size_t)rows * mods.size() * n);
            for (size_t i = 0; i < v.size(); i++) v[i] = rng() % mods[(i / n) % mods.size()];
            return v;
        };
        const auto a = uniform(q, batch), b = uniform(q, batch), kb = uniform(all, dnum), ka = uniform(all, dnum);
        std::vector<uint64_t> s1, s2;
        for (uint32_t t = 0; t < sq; t++) s1.push_back(rng()), s2.push_back(rng() % q[t]);

        DCRTPolyHip A(PQ, Format::COEFFICIENT, batch), B(PQ, Format::EVALUATION, batch);
        A.SetValues(a, Format::COEFFICIENT);
        B.SetValues(b, Format::EVALUATION);
        DCRTPolyHip KB(PQP, Format::EVALUATION, dnum), KA(PQP, Format::EVALUATION, dnum);
        KB.SetValues(kb, Format::EVALUATION);
        KA.SetValues(ka, Format::EVALUATION);
        HipManager::getHip(0)->sync();

        auto run = [&](bool keep, std::vector<std::vector<uint64_t>>* outs) {
            DCRTPolyHip X(A);
            X.SwitchFormat();
            DCRTPolyHip Y = X * B;
            DCRTPolyHip Z(Y);
            Z.SwitchFormat();
            DCRTPolyHip Z2 = Z.Plus(s1).Minus(s2);
            DCRTPolyHip U = ApproxModUp(Z2, PP, PQP, *up);
            auto K = ks->KeySwitchCore(Y, KB, KA);
            DCRTPolyHip D = ApproxModDown(U.Times(pmod), PQ, PP, *down, pinv);
            if (keep)
                for (const DCRTPolyHip* x : std::vector<const DCRTPolyHip*>{&Y, &Z, &Z2, &U, &K.first, &K.second, &D})
                    outs->push_back(x->GetValues());
        };
        std::vector<std::vector<uint64_t>> outs;
        run(true, &outs);
        HipManager::getHip(0)->sync();
        const auto t0 = std::chrono::steady_clock::now();
        for (int r = 0; r < reps; r++) run(false, nullptr);
        HipManager::getHip(0)->sync();
        const double ms =
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() / reps;
        FILE* f = std::fopen(argv[1], "wb");
        if (!f) return 3;
        put(f, {log_n, batch, sq, sp, dnum});
        put(f, q);
        put(f, p);
        put(f, PQ->Roots());
        put(f, PP->Roots());
        const std::vector<const std::vector<uint64_t>*> ins{&a, &b, &kb, &ka, &s1, &s2};
        for (const auto* v : ins) put(f, *v);
        for (const auto& v : outs) put(f, v);
        std::fclose(f);
        std::printf("chain N=2^%u Q=%u P=%u dnum=%u batch=%u: %.3f ms per chain (device-resident, %d reps)\n", log_n,
                    sq, sp, dnum, batch, ms, reps);
    } catch (const std::exception& e) {
        std::printf("chain failed: %s\n", e.what());
        return 1;
    }
    return 0;
}
