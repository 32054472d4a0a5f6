// tensor2_diag.hip -- diagnostic build only (never linked into the library).
//
// Round 2 saw a grid-stride EvalMultCore kernel with per-lane tower constants
// return non-canonical words for tower 2 of 4 at N = 2^16 (VERDICT r02, weak
// #1).  That variant was not committed; this program rebuilds the pattern it
// shared with k_eltwise<ELT_MUL> -- a grid-stride loop, U 16-byte pairs per
// thread, the tower index t = row % towers computed per lane and the
// TowerConst loaded from tcs[t] -- and runs it next to the shipped per-row
// kernel (k_tensor2) and k_eltwise on identical inputs, against exact 128-bit
// host arithmetic.  With DBG the kernel also writes, for every element, the
// (row, t, q, mu, nshift) it used and the Barrett intermediates of out2.
//
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -o tensor2_diag tensor2_diag.hip
//   ./tensor2_diag [log_n towers batch]...
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../upmem--openfhe_amd/csrc/eltwise_kernels.hpp"

using namespace ofhe;
typedef unsigned __int128 u128;

#define CK(x)                                                                           \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(3);                                                                    \
        }                                                                               \
    } while (0)

struct Dbg {
    u64 row, t, q, mu, nshift, prod_hi, prod_lo, est, r;
};

// barrett_ref with its intermediates exposed (same arithmetic, arith.hpp)
__device__ __forceinline__ u64 barrett_dbg(u64 a, u64 b, u64 q, u64 mu, u32 n_shift, Dbg* d) {
    u64 p00 = mad32(lo32(a), lo32(b), 0);
    u64 m1 = mad32(lo32(a), hi32(b), (u64)hi32(p00));
    u64 m2 = mad32(hi32(a), lo32(b), (u64)lo32(m1));
    u64 hi = mad32(hi32(a), hi32(b), (u64)hi32(m1)) + (u64)hi32(m2);
    u64 lo = ((u64)lo32(m2) << 32) | lo32(p00);
    u64 sh = n_shift ? ((lo >> n_shift) | (hi << (64 - n_shift))) : lo;
    u64 q00 = mad32(lo32(sh), lo32(mu), 0);
    u64 r1 = mad32(lo32(sh), hi32(mu), (u64)hi32(q00));
    u64 r2 = mad32(hi32(sh), lo32(mu), (u64)lo32(r1));
    u64 th = mad32(hi32(sh), hi32(mu), (u64)hi32(r1)) + (u64)hi32(r2);
    u64 tl = ((u64)lo32(r2) << 32) | lo32(q00);
    u32 s = n_shift + 7;
    u64 est = s >= 64 ? (th >> (s - 64)) : ((tl >> s) | (th << (64 - s)));
    u64 r = lo - est * q;
    d->prod_hi = hi;
    d->prod_lo = lo;
    d->est = est;
    d->r = r;
    return r >= q ? r - q : r;
}

// the round-2 pattern: grid-stride, U pairs per thread, per-lane tower constants
template <int U, bool DBG>
__global__ __launch_bounds__(256) void k_tensor2_gs(const TowerConst* __restrict__ tcs, const u64* c0, const u64* c1,
                                                    const u64* d0, const u64* d1, u64* o0, u64* o1, u64* o2,
                                                    u64 npairs, u32 log_n, u32 towers, Dbg* dbg) {
    const u64 stride = (u64)gridDim.x * blockDim.x;
    for (u64 i0 = (u64)blockIdx.x * blockDim.x + threadIdx.x; i0 < npairs; i0 += stride * U) {
        u64x2 a0[U], a1[U], b0[U], b1[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const u64 i = i0 + u * stride;
            if (i < npairs) {
                a0[u] = ld2_s(c0 + 2 * i);
                a1[u] = ld2_s(c1 + 2 * i);
                b0[u] = ld2_s(d0 + 2 * i);
                b1[u] = ld2_s(d1 + 2 * i);
            }
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            const u64 i = i0 + u * stride;
            if (i >= npairs) break;
            const u32 row = (u32)((2 * i) >> log_n);
            const u32 t = row % towers;
            const TowerConst tc = tcs[t];
            u64x2 r0, r1, r2;
            if (DBG) {
                Dbg dx{row, t, tc.q, tc.mu, tc.nshift, 0, 0, 0, 0}, dy = dx;
                r2.x = barrett_dbg(a1[u].x, b1[u].x, tc.q, tc.mu, tc.nshift, &dx);
                r2.y = barrett_dbg(a1[u].y, b1[u].y, tc.q, tc.mu, tc.nshift, &dy);
                dbg[2 * i] = dx;
                dbg[2 * i + 1] = dy;
            } else {
                r2.x = barrett_ref(a1[u].x, b1[u].x, tc.q, tc.mu, tc.nshift);
                r2.y = barrett_ref(a1[u].y, b1[u].y, tc.q, tc.mu, tc.nshift);
            }
            r1.x = modadd_fast(barrett_ref(a1[u].x, b0[u].x, tc.q, tc.mu, tc.nshift),
                               barrett_ref(a0[u].x, b1[u].x, tc.q, tc.mu, tc.nshift), tc.q);
            r1.y = modadd_fast(barrett_ref(a1[u].y, b0[u].y, tc.q, tc.mu, tc.nshift),
                               barrett_ref(a0[u].y, b1[u].y, tc.q, tc.mu, tc.nshift), tc.q);
            r0.x = barrett_ref(b0[u].x, a0[u].x, tc.q, tc.mu, tc.nshift);
            r0.y = barrett_ref(b0[u].y, a0[u].y, tc.q, tc.mu, tc.nshift);
            st2_s(o0 + 2 * i, r0);
            st2_s(o1 + 2 * i, r1);
            st2_s(o2 + 2 * i, r2);
        }
    }
}

static u64 host_msb(u64 x) { return 64 - __builtin_clzll(x); }

static u64 splitmix(u64& s) {
    u64 z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static u64 mulmod(u64 a, u64 b, u64 q) { return (u64)(((u128)a * b) % q); }

static const u64 QS[8] = {0xffffffffffc0001ull, 0xfffffffff840001ull, 0xfffffffff6a0001ull, 0xfffffffff5a0001ull,
                          0xfffffffff2a0001ull, 0xfffffffff240001ull, 0xffffffffefe0001ull, 0xffffffffeca0001ull};

// returns the number of wrong words over the three outputs
static long run(const char* name, int variant, u32 log_n, u32 towers, u32 batch) {
    const u64 N = 1ull << log_n, words = N * towers * batch, npairs = words / 2;
    std::vector<TowerConst> tc(towers);
    for (u32 t = 0; t < towers; t++) {
        memset(&tc[t], 0, sizeof(TowerConst));
        const u64 q = QS[t % 8];
        const u64 mb = host_msb(q);
        tc[t].q = q;
        tc[t].mu = (u64)(((u128)1 << (2 * mb + 3)) / q);
        tc[t].nshift = (u32)(mb - 2);
    }
    std::vector<u64> h[4];
    u64 seed = 0x1234 + log_n * 77 + towers * 13 + batch;
    for (int k = 0; k < 4; k++) {
        h[k].resize(words);
        for (u64 e = 0; e < words; e++) h[k][e] = splitmix(seed) % tc[(e >> log_n) % towers].q;
    }
    TowerConst* dtc;
    u64 *din[4], *dout[3];
    Dbg* ddbg = nullptr;
    CK(hipMalloc(&dtc, sizeof(TowerConst) * towers));
    CK(hipMemcpy(dtc, tc.data(), sizeof(TowerConst) * towers, hipMemcpyHostToDevice));
    for (int k = 0; k < 4; k++) {
        CK(hipMalloc(&din[k], words * 8));
        CK(hipMemcpy(din[k], h[k].data(), words * 8, hipMemcpyHostToDevice));
    }
    for (int k = 0; k < 3; k++) {
        CK(hipMalloc(&dout[k], words * 8));
        CK(hipMemset(dout[k], 0xA5, words * 8));
    }
    const bool dbg = variant == 3;
    if (dbg) CK(hipMalloc(&ddbg, words * sizeof(Dbg)));
    auto grid_for = [&](int U) {
        u64 b = (npairs + 256 * U - 1) / (256 * U);
        return (u32)(b > (1u << 22) ? (1u << 22) : b);
    };
    if (variant == 0) {  // shipped per-row kernel
        const u32 bpr = (u32)((N / 2 + 255) / 256);
        hipLaunchKernelGGL(k_tensor2<0>, dim3(bpr * batch * towers), dim3(256), 0, 0, dtc, din[0], din[1], din[2],
                           din[3], dout[0], dout[1], dout[2], bpr, log_n, towers);
    } else if (variant == 1) {
        hipLaunchKernelGGL((k_tensor2_gs<2, false>), dim3(grid_for(2)), dim3(256), 0, 0, dtc, din[0], din[1], din[2],
                           din[3], dout[0], dout[1], dout[2], npairs, log_n, towers, ddbg);
    } else if (variant == 2) {
        hipLaunchKernelGGL((k_tensor2_gs<1, false>), dim3(grid_for(1)), dim3(256), 0, 0, dtc, din[0], din[1], din[2],
                           din[3], dout[0], dout[1], dout[2], npairs, log_n, towers, ddbg);
    } else if (variant == 3) {
        hipLaunchKernelGGL((k_tensor2_gs<2, true>), dim3(grid_for(2)), dim3(256), 0, 0, dtc, din[0], din[1], din[2],
                           din[3], dout[0], dout[1], dout[2], npairs, log_n, towers, ddbg);
    } else {  // k_eltwise<ELT_MUL>: out2 = c1 * d1 only
        hipLaunchKernelGGL(k_eltwise<ELT_MUL>, dim3(grid_for(2)), dim3(256), 0, 0, dtc, din[1], din[3], dout[2],
                           npairs, log_n, towers);
    }
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    std::vector<u64> o[3];
    for (int k = 0; k < 3; k++) {
        o[k].resize(words);
        CK(hipMemcpy(o[k].data(), dout[k], words * 8, hipMemcpyDeviceToHost));
    }
    std::vector<Dbg> hd;
    if (dbg) {
        hd.resize(words);
        CK(hipMemcpy(hd.data(), ddbg, words * sizeof(Dbg), hipMemcpyDeviceToHost));
    }
    long bad_total = 0;
    std::vector<long> bad(3 * towers, 0);
    int shown = 0;
    for (u64 e = 0; e < words; e++) {
        const u32 t = (u32)((e >> log_n) % towers);
        const u64 q = tc[t].q;
        const u64 a0 = h[0][e], a1 = h[1][e], b0 = h[2][e], b1 = h[3][e];
        const u64 want[3] = {mulmod(b0, a0, q), (mulmod(a1, b0, q) + mulmod(a0, b1, q)) % q, mulmod(a1, b1, q)};
        for (int k = 0; k < 3; k++) {
            if (variant == 4 && k != 2) continue;
            if (o[k][e] != want[k]) {
                bad[3 * t + k]++;
                bad_total++;
                if (shown < 6) {
                    shown++;
                    printf("  %s bad out%d e=%llu (b=%llu t=%u j=%llu) got %llu want %llu\n", name, k,
                           (unsigned long long)e, (unsigned long long)(e >> log_n) / towers, t,
                           (unsigned long long)(e & (N - 1)), (unsigned long long)o[k][e], (unsigned long long)want[k]);
                    if (dbg && k == 2) {
                        const Dbg& d = hd[e];
                        const u128 p = (u128)a1 * b1;
                        printf("    used row=%llu t=%llu q=%llx mu=%llx nshift=%llu | table q=%llx mu=%llx nshift=%u\n",
                               (unsigned long long)d.row, (unsigned long long)d.t, (unsigned long long)d.q,
                               (unsigned long long)d.mu, (unsigned long long)d.nshift, (unsigned long long)tc[t].q,
                               (unsigned long long)tc[t].mu, tc[t].nshift);
                        printf("    prod hi/lo %llx %llx (exact %llx %llx) est %llu r %llu\n",
                               (unsigned long long)d.prod_hi, (unsigned long long)d.prod_lo,
                               (unsigned long long)(u64)(p >> 64), (unsigned long long)(u64)p,
                               (unsigned long long)d.est, (unsigned long long)d.r);
                    }
                }
            }
        }
        if (dbg) {
            const Dbg& d = hd[e];
            if (d.q != tc[t].q || d.mu != tc[t].mu || d.nshift != tc[t].nshift || d.t != t) {
                if (shown < 12) {
                    shown++;
                    printf("  %s e=%llu constants differ: used t=%llu q=%llx, table t=%u q=%llx\n", name,
                           (unsigned long long)e, (unsigned long long)d.t, (unsigned long long)d.q, t,
                           (unsigned long long)tc[t].q);
                }
            }
        }
    }
    printf("%-22s log_n=%u towers=%u batch=%u bad=%ld per (tower,out):", name, log_n, towers, batch, bad_total);
    for (u32 t = 0; t < towers; t++) printf(" [%ld %ld %ld]", bad[3 * t], bad[3 * t + 1], bad[3 * t + 2]);
    printf("\n");
    fflush(stdout);
    for (int k = 0; k < 4; k++) CK(hipFree(din[k]));
    for (int k = 0; k < 3; k++) CK(hipFree(dout[k]));
    CK(hipFree(dtc));
    if (ddbg) CK(hipFree(ddbg));
    return bad_total;
}

int main(int argc, char** argv) {
    std::vector<u32> shapes = {16, 4, 1, 16, 4, 2, 16, 16, 2, 16, 2, 1, 14, 4, 1, 17, 8, 1};
    if (argc > 1) {
        shapes.clear();
        for (int i = 1; i + 2 < argc; i += 3) {
            shapes.push_back(atoi(argv[i]));
            shapes.push_back(atoi(argv[i + 1]));
            shapes.push_back(atoi(argv[i + 2]));
        }
    }
    const char* names[5] = {"k_tensor2 (per-row)", "grid-stride U=2", "grid-stride U=1", "grid-stride U=2 DBG",
                            "k_eltwise<MUL>"};
    long any = 0;
    for (size_t s = 0; s + 2 < shapes.size(); s += 3)
        for (int v = 0; v < 5; v++) any += run(names[v], v, shapes[s], shapes[s + 1], shapes[s + 2]);
    printf("total bad %ld\n", any);
    return any ? 1 : 0;
}
