// tensor2_asm_diag.hip -- diagnostic build only.  Runs the round-2 EvalMultCore
// machine code (t2_orig.hsaco, reassembled by t2asm_build.py from that build's
// compiler output) and its patched variants (t2_nop, t2_carry) on identical
// inputs against exact 128-bit host arithmetic, at the shapes of the round-2
// failure (N = 2^16, 4 towers, batch 1 / 2) and others.
//
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -o tensor2_asm_diag_bin tensor2_asm_diag.hip
//   ./tensor2_asm_diag_bin <dir with the .hsaco files>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

typedef unsigned long long u64;
typedef unsigned int u32;
typedef unsigned __int128 u128;

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(3);                                                                           \
        }                                                                                      \
    } while (0)

struct TowerConst {  // csrc/ntt_kernels.hpp layout at round 2 (64 bytes)
    u64 q, ninv, ninv_pre, mu, nq, nq4;
    u32 nshift, spq_sh;
    u64 qinv;
};
static_assert(sizeof(TowerConst) == 64, "layout");

static const u64 QS[4] = {0xffffffffffc0001ull, 0xfffffffff840001ull, 0xfffffffff6a0001ull, 0xfffffffff5a0001ull};

static u64 splitmix(u64& s) {
    u64 z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static u64 mulmod(u64 a, u64 b, u64 q) { return (u64)(((u128)a * b) % q); }

static long run(hipFunction_t fn, const char* name, u32 log_n, u32 towers, u32 batch, u32 grid_cap, int reps,
                u32 lds = 0, u32 bdim = 256) {
    const u64 N = 1ull << log_n, words = N * towers * batch;
    u64 npairs = words / 2;
    std::vector<TowerConst> tc(towers);
    for (u32 t = 0; t < towers; t++) {
        memset(&tc[t], 0, sizeof(TowerConst));
        const u64 q = QS[t % 4];
        const u32 mb = 64 - __builtin_clzll(q);
        tc[t].q = q;
        tc[t].mu = (u64)(((u128)1 << (2 * mb + 3)) / q);
        tc[t].nshift = mb - 2;
    }
    std::vector<u64> h[4];
    u64 seed = 0x77 + log_n * 31 + towers * 7 + batch;
    for (int k = 0; k < 4; k++) {
        h[k].resize(words);
        for (u64 e = 0; e < words; e++) h[k][e] = splitmix(seed) % tc[(e >> log_n) % towers].q;
    }
    TowerConst* dtc;
    u64 *din[4], *dout[3];
    CK(hipMalloc(&dtc, sizeof(TowerConst) * towers));
    CK(hipMemcpy(dtc, tc.data(), sizeof(TowerConst) * towers, hipMemcpyHostToDevice));
    for (int k = 0; k < 4; k++) {
        CK(hipMalloc(&din[k], words * 8));
        CK(hipMemcpy(din[k], h[k].data(), words * 8, hipMemcpyHostToDevice));
    }
    for (int k = 0; k < 3; k++) CK(hipMalloc(&dout[k], words * 8));
    u64 blocks = (npairs + bdim - 1) / bdim;
    if (blocks > grid_cap) blocks = grid_cap;
    long worst = 0;
    std::vector<long> bad(3 * towers);
    for (int rep = 0; rep < reps; rep++) {
        for (int k = 0; k < 3; k++) CK(hipMemset(dout[k], 0xA5, words * 8));
        void* args[] = {&dtc, &din[0], &din[1], &din[2], &din[3], &dout[0], &dout[1], &dout[2], &npairs, &log_n, &towers};
        CK(hipModuleLaunchKernel(fn, (u32)blocks, 1, 1, bdim, 1, 1, lds, 0, args, nullptr));
        CK(hipDeviceSynchronize());
        std::vector<u64> o[3];
        for (int k = 0; k < 3; k++) {
            o[k].resize(words);
            CK(hipMemcpy(o[k].data(), dout[k], words * 8, hipMemcpyDeviceToHost));
        }
        long tot = 0;
        std::fill(bad.begin(), bad.end(), 0);
        int shown = 0;
        for (u64 e = 0; e < words; e++) {
            const u32 t = (u32)((e >> log_n) % towers);
            const u64 q = tc[t].q;
            const u64 a0 = h[0][e], a1 = h[1][e], b0 = h[2][e], b1 = h[3][e];
            const u64 want[3] = {mulmod(b0, a0, q), (mulmod(a1, b0, q) + mulmod(a0, b1, q)) % q, mulmod(a1, b1, q)};
            for (int k = 0; k < 3; k++)
                if (o[k][e] != want[k]) {
                    bad[3 * t + k]++;
                    tot++;
                    if (rep == 0 && shown < 3) {
                        shown++;
                        printf("    %s out%d e=%llu (t=%u j=%llu) got %llu (%s q) want %llu\n", name, k, e, t, e & (N - 1),
                               o[k][e], o[k][e] >= q ? ">=" : "<", want[k]);
                    }
                }
        }
        if (!strcmp(name, "dump")) {
            // out0 holds (q, nshift) as the lane had them; out2 as computed
            long cbad = 0, both = 0, o2bad = 0, shownd = 0;
            for (u64 i = 0; i < npairs; i++) {
                const u64 e = 2 * i;
                const u32 t = (u32)((e >> log_n) % towers);
                const bool cb = o[0][e] != tc[t].q || (u32)o[0][e + 1] != tc[t].nshift;
                const bool b2 = o[2][e] != mulmod(h[1][e], h[3][e], tc[t].q) ||
                                o[2][e + 1] != mulmod(h[1][e + 1], h[3][e + 1], tc[t].q);
                cbad += cb;
                o2bad += b2;
                both += cb && b2;
                if (cb && shownd++ < 4)
                    printf("    pair %llu (t=%u): held q=%llx nshift=%u, table q=%llx nshift=%u\n", i, t, o[0][e],
                           (u32)o[0][e + 1], tc[t].q, tc[t].nshift);
            }
            printf("    pairs with wrong constants %ld, with a wrong out2 %ld, both %ld (of %llu)\n", cbad, o2bad, both,
                   npairs);
        }
        if (!strcmp(name, "dumpin")) {
            long ibad = 0, both = 0, o2bad = 0, showni = 0;
            for (u64 i = 0; i < npairs; i++) {
                const u64 e = 2 * i;
                const u32 t = (u32)((e >> log_n) % towers);
                const bool ib = o[0][e] != h[1][e] || o[0][e + 1] != h[1][e + 1];
                const bool b2 = o[2][e] != mulmod(h[1][e], h[3][e], tc[t].q) ||
                                o[2][e + 1] != mulmod(h[1][e + 1], h[3][e + 1], tc[t].q);
                ibad += ib;
                o2bad += b2;
                both += ib && b2;
                if (ib && showni++ < 4)
                    printf("    pair %llu: loaded c1 %llx %llx, memory holds %llx %llx\n", i, o[0][e], o[0][e + 1],
                           h[1][e], h[1][e + 1]);
            }
            printf("    pairs whose c1 load differs from memory %ld, with a wrong out2 %ld, both %ld (of %llu)\n", ibad,
                   o2bad, both, npairs);
        }
        if (tot && rep == 0 && getenv("T2_MATCH")) {
            // is a wrong word some other element's correct result?
            std::unordered_map<u64, u64> where;
            for (u64 e = 0; e < words; e++) {
                const u32 t = (u32)((e >> log_n) % towers);
                const u64 q = tc[t].q;
                where[mulmod(h[1][e], h[3][e], q)] = e * 4 + 2;
                where[mulmod(h[2][e], h[0][e], q)] = e * 4 + 0;
                where[(mulmod(h[1][e], h[2][e], q) + mulmod(h[0][e], h[3][e], q)) % q] = e * 4 + 1;
                where[mulmod(h[1][e], h[2][e], q)] = e * 4 + 3;  // c1 d0 alone
            }
            long found = 0, shownm = 0, checked = 0;
            for (u64 e = 0; e < words && checked < 20000; e++) {
                const u32 t = (u32)((e >> log_n) % towers);
                const u64 q = tc[t].q;
                const u64 w2 = mulmod(h[1][e], h[3][e], q);
                if (o[2][e] == w2) continue;
                checked++;
                auto it = where.find(o[2][e]);
                if (it != where.end()) {
                    found++;
                    if (shownm++ < 8)
                        printf("    out2[%llu] = result %llu of element %llu (delta %lld)\n", e, it->second & 3,
                               it->second >> 2, (long long)(it->second >> 2) - (long long)e);
                }
            }
            printf("    %ld of %ld wrong out2 words are another element's correct result\n", found, checked);
        }
        if (tot > worst) worst = tot;
        printf("%-7s log_n=%u towers=%u batch=%u grid=%llu x %u lds=%u rep=%d bad=%ld per (tower,out):", name, log_n,
               towers, batch, blocks, bdim, lds, rep, tot);
        for (u32 t = 0; t < towers; t++) printf(" [%ld %ld %ld]", bad[3 * t], bad[3 * t + 1], bad[3 * t + 2]);
        printf("\n");
        fflush(stdout);
    }
    for (int k = 0; k < 4; k++) CK(hipFree(din[k]));
    for (int k = 0; k < 3; k++) CK(hipFree(dout[k]));
    CK(hipFree(dtc));
    return worst;
}

int main(int argc, char** argv) {
    const std::string dir = argc > 1 ? argv[1] : ".";
    const char* kname = "_ZN4ofhe9k_tensor2ILi0EEEvPKNS_10TowerConstEPKmS5_S5_S5_PmS6_S6_mjj";
    const char* kinds_all[] = {"vgpr64", "vgpr48x", "orig", "dumpin", "dump", "allnop", "nont", "vmwait", "rcpnop", "nobranch", "vnop", "endwait", "zero",
                           "execnop", "nop", "carry"};
    // T2_SWEEP (round 4): the allocation sweep, 56 (orig) .. 128 VGPRs
    const char* kinds_sweep[] = {"orig", "vgpr64", "vgpr48x", "vgpr80", "vgpr88", "vgpr96", "vgpr104", "vgpr112", "vgpr120", "vgpr128"};
    const bool sweep = getenv("T2_SWEEP") != nullptr;
    const char** kinds = sweep ? kinds_sweep : kinds_all;
    const int nall = sweep ? (int)(sizeof(kinds_sweep) / sizeof(kinds_sweep[0])) : (int)(sizeof(kinds_all) / sizeof(kinds_all[0]));
    const int only = getenv("T2_ONLY") ? atoi(getenv("T2_ONLY")) : 99;
    const int nk = only < 99 ? only : nall;
    long bad[16] = {};
    for (int v = 0; v < nk; v++) {
        hipModule_t m;
        hipFunction_t f;
        CK(hipModuleLoad(&m, (dir + "/t2_" + kinds[v] + ".hsaco").c_str()));
        CK(hipModuleGetFunction(&f, m, kname));
        bad[v] += run(f, kinds[v], 16, 4, 1, 1u << 22, 2);
        bad[v] += run(f, kinds[v], 16, 16, 2, 1u << 22, 1);
        if (v == 0 && getenv("T2_PLACEMENT")) {
            // occupancy / placement of the original code: one workgroup per CU
            // (160 KiB of dynamic LDS), 64-thread workgroups, a capped grid
            run(f, "orig-lds", 16, 4, 1, 1u << 22, 2, 160 * 1024);
            run(f, "orig-lds", 16, 16, 2, 1u << 22, 1, 160 * 1024);
            run(f, "orig-b64", 16, 4, 1, 1u << 22, 1, 0, 64);
            run(f, "orig-g64", 16, 16, 2, 64, 1);
            run(f, "orig", 14, 4, 1, 1u << 22, 1);
            run(f, "orig", 16, 2, 1, 1u << 22, 1);
            run(f, "orig", 14, 16, 4, 1u << 22, 1);
        }
        CK(hipModuleUnload(m));
    }
    printf("summary:");
    for (int v = 0; v < nk; v++) printf(" %s %ld", kinds[v], bad[v]);
    printf(" wrong words\n");
    return 0;
}
