// Package power per byte moved at each level of the memory hierarchy: every
// workgroup streams read-modify-write passes over its own private region, so
// the footprint alone decides where the bytes live (per-XCD L2, Infinity
// Cache, HBM) and the kernel shape is the same for all three.  Run back to
// back for a given time so rocm-smi can read package power and sclk
// (tools/power_l2.sh).  Regions are >= 32 KiB per workgroup and walked in
// order, so the 32 KiB vector L1 holds none of a pass's reads.
//   mempower_bin <workgroups> <KiB per workgroup> <passes per launch> <seconds>
// Build: hipcc -O3 --offload-arch=gfx950 -o mempower_bin mempower.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <chrono>

typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void k_rmw(u64x2* buf, uint32_t vecs_per_wg, int passes) {
    u64x2* r = buf + (size_t)blockIdx.x * vecs_per_wg;
    for (int p = 0; p < passes; p++) {
        for (uint32_t i = threadIdx.x; i < vecs_per_wg; i += 4 * 256) {
            u64x2 v[4];
#pragma unroll
            for (int k = 0; k < 4; k++) v[k] = r[i + 256 * k];
#pragma unroll
            for (int k = 0; k < 4; k++) r[i + 256 * k] = v[k] + (u64x2){1, 1};
        }
    }
}

int main(int argc, char** argv) {
    if (argc < 5) {
        fprintf(stderr, "usage: %s <workgroups> <KiB per wg> <passes> <seconds>\n", argv[0]);
        return 2;
    }
    const uint32_t nwg = atoi(argv[1]);
    const uint32_t kib = atoi(argv[2]);
    const int passes = atoi(argv[3]);
    const double secs = atof(argv[4]);
    const uint32_t vecs = kib * 1024 / 16;
    if (nwg == 0 || kib < 32 || vecs % 1024 || passes < 1) {
        fprintf(stderr, "need workgroups > 0, KiB >= 32 and a multiple of 16, passes >= 1\n");
        return 2;
    }
    const size_t bytes = (size_t)nwg * kib * 1024;
    u64x2* d = nullptr;
    if (hipMalloc(&d, bytes) != hipSuccess) return 1;
    if (hipMemset(d, 0, bytes) != hipSuccess) return 1;
    k_rmw<<<nwg, 256>>>(d, vecs, passes);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    auto t0 = std::chrono::steady_clock::now();
    double el = 0;
    long launches = 0;
    while (el < secs) {
        for (int i = 0; i < 8; i++) k_rmw<<<nwg, 256>>>(d, vecs, passes);
        launches += 8;
        if (hipDeviceSynchronize() != hipSuccess) return 1;
        el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    }
    const double moved = 2.0 * bytes * passes * launches;
    printf("rmw %u wg x %u KiB (%.1f MiB total) x %d passes: %.0f GB/s (read + write), %.3f ms per launch\n", nwg, kib,
           bytes / 1048576.0, passes, moved / el / 1e9, el / launches * 1e3);
    hipFree(d);
    return 0;
}
