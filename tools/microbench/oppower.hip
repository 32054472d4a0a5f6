// Power per instruction type: one gfx950 VALU instruction (oprate3.hip's
// kernels) run back to back for a given time so rocm-smi can read the package
// power and sclk it settles at (tools/power_ops.sh).  Prints wave-instructions
// per second.  Build: hipcc -O3 --offload-arch=gfx950 -o oppower_bin oppower.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#define IT 256
#define CH 16

#define K32(NAME, ASM)                                                                     \
    __global__ __launch_bounds__(256) void NAME(uint32_t* out, uint32_t s1) {            \
        uint32_t y[CH];                                                                   \
        _Pragma("unroll") for (int c = 0; c < CH; c++) y[c] = threadIdx.x * 977u + c + s1; \
        uint32_t z = s1 ^ 0x1234567u;                                                     \
        for (int i = 0; i < IT; i++) {                                                    \
            _Pragma("unroll") for (int c = 0; c < CH; c++) asm volatile(ASM : "+v"(y[c]) : "v"(z)); \
        }                                                                                 \
        uint32_t r = 0;                                                                   \
        _Pragma("unroll") for (int c = 0; c < CH; c++) r ^= y[c];                         \
        out[blockIdx.x * blockDim.x + threadIdx.x] = r;                                   \
    }
#define K64(NAME, ASM)                                                                     \
    __global__ __launch_bounds__(256) void NAME(uint32_t* out, uint32_t s1) {            \
        uint64_t y[CH];                                                                   \
        _Pragma("unroll") for (int c = 0; c < CH; c++) y[c] = threadIdx.x * 977u + c + s1; \
        uint64_t z = s1 ^ 0x1234567u;                                                     \
        for (int i = 0; i < IT; i++) {                                                    \
            _Pragma("unroll") for (int c = 0; c < CH; c++) asm volatile(ASM : "+v"(y[c]) : "v"(z)); \
        }                                                                                 \
        uint64_t r = 0;                                                                   \
        _Pragma("unroll") for (int c = 0; c < CH; c++) r ^= y[c];                         \
        out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(r ^ (r >> 32));           \
    }

K32(k_add_u32, "v_add_u32 %0, %0, %1")
K32(k_add3_u32, "v_add3_u32 %0, %0, %1, %0")
K32(k_xor, "v_xor_b32 %0, %0, %1")
K32(k_lshl_b32, "v_lshlrev_b32 %0, 3, %0")
K32(k_mul_lo, "v_mul_lo_u32 %0, %0, %1")
K32(k_mul_hi, "v_mul_hi_u32 %0, %0, %1")
K32(k_mul_u24, "v_mul_u32_u24 %0, %0, %1")
K32(k_mulhi_u24, "v_mul_hi_u32_u24 %0, %0, %1")
K32(k_mad_u24, "v_mad_u32_u24 %0, %0, %1, %0")
K32(k_cndmask, "v_cndmask_b32 %0, %0, %1, vcc")
K32(k_add_co, "v_add_co_u32 %0, vcc, %0, %1")
K32(k_fma_f32, "v_fma_f32 %0, %0, %1, %0")
K32(k_pk_add_u16, "v_pk_add_u16 %0, %0, %1")
__global__ __launch_bounds__(256) void k_mad_u64(uint32_t* out, uint32_t s1) {
    uint64_t y[CH];
    uint32_t a[CH];
#pragma unroll
    for (int c = 0; c < CH; c++) y[c] = threadIdx.x * 977u + c + s1, a[c] = threadIdx.x + c;
    uint32_t z = s1 ^ 0x1234567u;
    for (int i = 0; i < IT; i++) {
#pragma unroll
        for (int c = 0; c < CH; c++) asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(y[c]) : "v"(a[c]), "v"(z) : "s0", "s1");
    }
    uint64_t r = 0;
#pragma unroll
    for (int c = 0; c < CH; c++) r ^= y[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(r ^ (r >> 32));
}
K64(k_lshl_add_u64, "v_lshl_add_u64 %0, %0, 0, %1")
K64(k_cmp_u64, "v_cmp_le_u64 vcc, %0, %1")
K64(k_lshr_b64, "v_lshrrev_b64 %0, 3, %0")
K64(k_fma_f64, "v_fma_f64 %0, %0, %1, %0")
K64(k_mov_b64, "v_mov_b64 %0, %1")

#include <chrono>
#include <cstring>
#include <cstdlib>
typedef void (*KF)(uint32_t*, uint32_t);
struct Op { const char* name; KF k; };
int main(int argc, char** argv) {
    const Op ops[] = {{"add_u32", k_add_u32}, {"xor_b32", k_xor}, {"add_co_u32", k_add_co}, {"cndmask_b32", k_cndmask},
                      {"mul_lo_u32", k_mul_lo}, {"mul_hi_u32", k_mul_hi}, {"mul_u32_u24", k_mul_u24},
                      {"mad_u64_u32", k_mad_u64}, {"lshl_add_u64", k_lshl_add_u64}, {"mov_b64", k_mov_b64},
                      {"fma_f32", k_fma_f32}, {"fma_f64", k_fma_f64}};
    if (argc < 3) { fprintf(stderr, "usage: oppower_bin <op> <seconds>\n"); return 2; }
    KF k = nullptr;
    for (const Op& o : ops) if (!strcmp(o.name, argv[1])) k = o.k;
    if (!k) { fprintf(stderr, "unknown op %s\n", argv[1]); return 2; }
    const double secs = atof(argv[2]);
    int blocks = 256 * 16;
    uint32_t* buf;
    if (hipMalloc(&buf, (size_t)blocks * 256 * 4) != hipSuccess) return 1;
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, buf, 12345u);
    (void)hipDeviceSynchronize();
    long launches = 0;
    auto t0 = std::chrono::steady_clock::now();
    double el = 0;
    while (el < secs) {
        for (int r = 0; r < 20; r++) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, buf, 12345u);
        launches += 20;
        (void)hipDeviceSynchronize();
        el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    }
    const double waveinst = (double)blocks * 4 * IT * CH * launches;
    printf("%-14s %.3e wave-inst/s  (%.3f per SIMD per ns)\n", argv[1], waveinst / el, waveinst / el / 1024 / 1e9);
    (void)hipFree(buf);
    return 0;
}
