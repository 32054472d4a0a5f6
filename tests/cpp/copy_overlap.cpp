// Host-side cost of DCRTPolyHip::SetValues while device work is queued on the
// adapter's stream (round 6: HipManager's staged copies wait on their own
// DMA's event instead of draining the stream).  A batch of forward
// transforms (~several ms of GPU work) is queued, then SetValues uploads an
// unrelated polynomial; the host time of that call is printed, and the
// uploaded words are read back and checked.  Before round 6 the call
// synchronised the stream first, so it took the queued work's time.
//
//   copy_overlap_bin      (GPU box; prints one line, exit 1 on a wrong word)
#include <chrono>
#include <cstdio>
#include <random>
#include <vector>

#include "../../upmem--openfhe_amd/host/ofhe_dcrt.hpp"

using namespace ofhe;
using Clock = std::chrono::steady_clock;

static uint64_t prev_prime(uint64_t q, uint64_t m) {
    auto is_prime = [](uint64_t n) {
        if (n < 2) return false;
        for (uint64_t p : {2ull, 3ull, 5ull, 7ull, 11ull, 13ull, 17ull, 19ull, 23ull, 29ull, 31ull, 37ull}) {
            if (n % p == 0) return n == p;
        }
        uint64_t d = n - 1;
        int r = 0;
        while (!(d & 1)) d >>= 1, r++;
        auto mulmod = [](uint64_t a, uint64_t b, uint64_t m) { return (uint64_t)((unsigned __int128)a * b % m); };
        for (uint64_t a : {2ull, 3ull, 5ull, 7ull, 11ull, 13ull, 17ull, 19ull, 23ull, 29ull, 31ull, 37ull}) {
            uint64_t x = 1, b = a % n, e = d;
            while (e) {
                if (e & 1) x = mulmod(x, b, n);
                b = mulmod(b, b, n);
                e >>= 1;
            }
            if (x == 1 || x == n - 1) continue;
            bool comp = true;
            for (int i = 1; i < r && comp; i++) {
                x = mulmod(x, x, n);
                if (x == n - 1) comp = false;
            }
            if (comp) return false;
        }
        return true;
    };
    do q -= m;
    while (!is_prime(q));
    return q;
}
static uint64_t root(uint64_t m, uint64_t q) {  // a primitive m-th root (not the minimal one: any works here)
    auto pw = [](uint64_t b, uint64_t e, uint64_t q) {
        uint64_t r = 1;
        b %= q;
        while (e) {
            if (e & 1) r = (uint64_t)((unsigned __int128)r * b % q);
            b = (uint64_t)((unsigned __int128)b * b % q);
            e >>= 1;
        }
        return r;
    };
    for (uint64_t g = 2;; g++) {
        const uint64_t x = pw(g, (q - 1) / m, q);
        if (pw(x, m / 2, q) == q - 1) return x;
    }
}

int main() {
    const uint32_t log_n = 16, n = 1u << log_n, m = 2 * n, T = 16, big = 1024;
    std::vector<uint64_t> q, r;
    uint64_t x = (1ull << 60) + 1;
    for (uint32_t t = 0; t < T; t++) {
        x = prev_prime(x, m);
        q.push_back(x);
        r.push_back(root(m, x));
    }
    auto P = std::make_shared<DCRTParams>(m, q, r);
    DCRTPolyHip A(P, Format::COEFFICIENT, big), B(P, Format::COEFFICIENT, 1);
    std::mt19937_64 rng(5);
    std::vector<uint64_t> v((size_t)T * n);
    for (size_t i = 0; i < v.size(); i++) v[i] = rng() % q[i / n];
    B.SetValues(v, Format::COEFFICIENT);  // warm: staging buffers
    A.SwitchFormat();
    A.SwitchFormat();
    P->manager()->sync();
    double queued = 0, alone = 0;
    for (int rep = 0; rep < 5; rep++) {
        auto t0 = Clock::now();
        B.SetValues(v, Format::COEFFICIENT);
        P->manager()->sync();
        alone += std::chrono::duration<double, std::milli>(Clock::now() - t0).count();
        A.SwitchFormat();  // queued: `big` polynomials x T towers of forward transforms
        t0 = Clock::now();
        B.SetValues(v, Format::COEFFICIENT);
        queued += std::chrono::duration<double, std::milli>(Clock::now() - t0).count();
        P->manager()->sync();
    }
    const auto t1 = Clock::now();
    A.SwitchFormat();
    P->manager()->sync();
    const double work = std::chrono::duration<double, std::milli>(Clock::now() - t1).count();
    const bool ok = B.GetValues() == v;
    std::printf("SetValues of %u x 2^%u words: %.3f ms with %.2f ms of transforms queued ahead, %.3f ms on an idle "
                "stream (upload + sync); read-back %s\n",
                T, log_n, queued / 5, work, alone / 5, ok ? "exact" : "WRONG");
    return ok ? 0 : 1;
}
