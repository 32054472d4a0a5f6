// copy_soak.cpp -- soak of the adapter's buffer path (diagnosis of the
// round-4 driver record: UTDCRTPoly.DCRT_mod_ops_on_two_elements read back
// wrong sums and products for every word).  Each iteration runs the exact
// sequence DCRTPolyHip uses for `(A + B).GetValues()` on a fresh 3-tower N = 8
// plan -- stream-ordered pool blocks, a zero fill, a pageable upload bracketed
// by syncs, k_eltwise, a pageable download -- under one of several variants,
// with a larger transform between iterations to churn the pool and the L2s.
// It classifies every mismatch: result all zeros, operands lost on the device,
// stale read-back (a second download differs from the first) or wrong residues.
//
//   copy_soak <variant> <iterations>
//   variant 0: as DCRTPolyHip (pool blocks, zero fill, pageable copies)
//   variant 1: no zero fill before the upload
//   variant 2: hipMalloc blocks instead of the pool
//   variant 3: pinned staging for both copies
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "../../include/ofhe_hip.h"

typedef unsigned __int128 u128;
#define CK(x)                                                                     \
    do {                                                                          \
        int rc_ = (x);                                                            \
        if (rc_) {                                                                \
            std::printf("error %d at %s:%d: %s\n", rc_, __FILE__, __LINE__, ofhe_hip_last_error()); \
            std::exit(3);                                                         \
        }                                                                         \
    } while (0)

static uint64_t mulmod(uint64_t a, uint64_t b, uint64_t q) { return (uint64_t)((u128)a * b % q); }
static uint64_t powmod(uint64_t b, uint64_t e, uint64_t q) {
    uint64_t r = 1 % q;
    for (b %= q; e; e >>= 1, b = mulmod(b, b, q))
        if (e & 1) r = mulmod(r, b, q);
    return r;
}
static bool is_prime(uint64_t n) {
    if (n < 2) return false;
    for (uint64_t p : {2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37})
        if (n % p == 0) return n == p;
    uint64_t d = n - 1;
    int s = 0;
    while (!(d & 1)) d >>= 1, s++;
    for (uint64_t a : {2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37}) {
        uint64_t x = powmod(a, d, n);
        if (x == 1 || x == n - 1) continue;
        bool comp = true;
        for (int r = 1; r < s && comp; r++) {
            x = mulmod(x, x, n);
            if (x == n - 1) comp = false;
        }
        if (comp) return false;
    }
    return true;
}
static uint64_t root(uint64_t m, uint64_t q) {
    for (uint64_t c = 2;; c++) {
        uint64_t psi = powmod(c, (q - 1) / m, q);
        if (powmod(psi, m / 2, q) == q - 1) return psi;
    }
}

int main(int argc, char** argv) {
    const int variant = argc > 1 ? std::atoi(argv[1]) : 0;
    const int iters = argc > 2 ? std::atoi(argv[2]) : 1000;
    ofhe_ctx_t ctx;
    CK(ofhe_hip_init(0, &ctx));
    // 16 bases of 3 moduli ~2^(20+k) (plans created on first use, as PlanCache does)
    const uint32_t m = 16, T = 3;
    std::vector<std::vector<uint64_t>> qs(16);
    std::vector<ofhe_plan_t> plans(16, nullptr);
    for (int k = 0; k < 16; k++) {
        uint64_t x = (1ull << (20 + k)) + 1;
        while (qs[k].size() < T) {
            if (is_prime(x)) qs[k].push_back(x);
            x += m;
        }
    }
    // churn: a 2^14 x 4 transform on its own buffers between iterations
    ofhe_plan_t big;
    std::vector<uint64_t> bq, br;
    for (uint64_t x = (1ull << 59) + 1; bq.size() < 4; x += 1ull << 15)
        if (is_prime(x)) bq.push_back(x), br.push_back(root(1ull << 15, x));
    CK(ofhe_hip_plan_create(ctx, 14, 4, bq.data(), br.data(), &big));
    void* churn = nullptr;
    CK(ofhe_hip_alloc(ctx, (size_t)4 << 17, &churn));
    CK(ofhe_hip_zero(ctx, churn, (size_t)4 << 17, nullptr));

    uint64_t *pin_in = nullptr, *pin_out = nullptr;
    CK(ofhe_hip_host_alloc(ctx, 2 * 24 * 8, (void**)&pin_in));
    CK(ofhe_hip_host_alloc(ctx, 24 * 8, (void**)&pin_out));
    std::mt19937_64 rng(11);
    long bad_zero = 0, bad_operand = 0, bad_stale = 0, bad_other = 0, bad_total = 0;
    const auto t0 = std::chrono::steady_clock::now();
    for (int it = 0; it < iters; it++) {
        const int k = it % 16;
        if (!plans[k]) {
            std::vector<uint64_t> r;
            for (auto q : qs[k]) r.push_back(root(m, q));
            CK(ofhe_hip_plan_create(ctx, 3, T, qs[k].data(), r.data(), &plans[k]));
        }
        std::vector<uint64_t> a(24), b(24), want(24), got(24), again(24), ra(24);
        for (int i = 0; i < 24; i++) {
            const uint64_t q = qs[k][i / 8];
            a[i] = rng() % q;
            b[i] = rng() % q;
            want[i] = (a[i] + b[i]) % q;
        }
        void *A = nullptr, *B = nullptr, *S = nullptr;
        auto alloc = [&](void** p) {
            if (variant == 2) CK(ofhe_hip_alloc(ctx, 192, p));
            else CK(ofhe_hip_alloc_async(ctx, 192, p, nullptr));
        };
        auto release = [&](void* p) {
            if (variant == 2) CK(ofhe_hip_free(ctx, p));
            else CK(ofhe_hip_free_async(ctx, p, nullptr));
        };
        auto up = [&](void* d, const uint64_t* h, int slot) {
            CK(ofhe_hip_sync(ctx, nullptr));
            if (variant == 3) {
                std::memcpy(pin_in + 24 * slot, h, 192);
                CK(ofhe_hip_copy_to_device(ctx, d, pin_in + 24 * slot, 192, nullptr));
            } else {
                CK(ofhe_hip_copy_to_device(ctx, d, h, 192, nullptr));
            }
            CK(ofhe_hip_sync(ctx, nullptr));
        };
        auto down = [&](uint64_t* h, const void* d) {
            CK(ofhe_hip_sync(ctx, nullptr));
            if (variant == 3) {
                CK(ofhe_hip_copy_to_host(ctx, pin_out, d, 192, nullptr));
                CK(ofhe_hip_sync(ctx, nullptr));
                std::memcpy(h, pin_out, 192);
            } else {
                CK(ofhe_hip_copy_to_host(ctx, h, d, 192, nullptr));
            }
            CK(ofhe_hip_sync(ctx, nullptr));
        };
        alloc(&A);
        if (variant != 1) CK(ofhe_hip_zero(ctx, A, 192, nullptr));
        alloc(&B);
        if (variant != 1) CK(ofhe_hip_zero(ctx, B, 192, nullptr));
        up(A, a.data(), 0);
        up(B, b.data(), 1);
        alloc(&S);
        CK(ofhe_hip_modadd_vv(plans[k], (const uint64_t*)A, (const uint64_t*)B, (uint64_t*)S, 1, nullptr));
        down(got.data(), S);
        if (got != want) {
            bad_total++;
            down(again.data(), S);
            down(ra.data(), A);
            bool zero = true;
            for (auto v : got) zero = zero && v == 0;
            if (zero) bad_zero++;
            else if (again != got) bad_stale++;
            else if (ra != a) bad_operand++;
            else bad_other++;
            if (bad_total <= 5)
                std::printf("iter %d: got[0]=%llu want[0]=%llu again[0]=%llu A[0]=%llu a[0]=%llu\n", it,
                            (unsigned long long)got[0], (unsigned long long)want[0], (unsigned long long)again[0],
                            (unsigned long long)ra[0], (unsigned long long)a[0]);
        }
        release(S);
        release(B);
        release(A);
        if (it % 4 == 3) CK(ofhe_hip_ntt_fwd(big, (uint64_t*)churn, 1, nullptr));
        if (it % 2000 == 1999)
            std::printf("variant %d: %d iterations, %ld mismatches so far\n", variant, it + 1, bad_total), std::fflush(stdout);
    }
    CK(ofhe_hip_sync(ctx, nullptr));
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::printf("variant %d: %d iterations in %.1f s: %ld mismatches (all-zero %ld, stale read-back %ld, operand "
                "lost %ld, other %ld)\n",
                variant, iters, s, bad_total, bad_zero, bad_stale, bad_operand, bad_other);
    return bad_total ? 1 : 0;
}
