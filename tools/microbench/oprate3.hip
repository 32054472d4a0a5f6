// Issue rate of single gfx950 VALU instructions (inline asm, 16 independent
// chains per thread, 16 waves per CU).  Prints wave-instructions per SIMD
// cycle at the nominal 2.4 GHz: 0.5 = one wave64 instruction every 2 cycles.
// Build: hipcc -O3 --offload-arch=gfx950 -o oprate3_bin oprate3.hip
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

template <class F>
void run(const char* name, F kern, uint32_t* buf, int blocks) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, buf, 12345u);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int r = 0; r < 5; r++) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, buf, 12345u);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    double waveinst = (double)blocks * 4 * IT * CH * 5;
    double simd_cycles = 1024.0 * 2.4e9 * ms / 1e3;
    printf("%-16s %.3f wave-inst/SIMD-cycle  (%.2f cycles per wave64 instruction)\n", name, waveinst / simd_cycles,
           simd_cycles / waveinst);
}

int main() {
    int blocks = 256 * 16;
    uint32_t* buf;
    (void)hipMalloc(&buf, (size_t)blocks * 256 * 4);
    run("add_u32", k_add_u32, buf, blocks);
    run("add3_u32", k_add3_u32, buf, blocks);
    run("xor_b32", k_xor, buf, blocks);
    run("lshlrev_b32", k_lshl_b32, buf, blocks);
    run("cndmask_b32", k_cndmask, buf, blocks);
    run("add_co_u32", k_add_co, buf, blocks);
    run("fma_f32", k_fma_f32, buf, blocks);
    run("pk_add_u16", k_pk_add_u16, buf, blocks);
    run("mul_lo_u32", k_mul_lo, buf, blocks);
    run("mul_hi_u32", k_mul_hi, buf, blocks);
    run("mul_u32_u24", k_mul_u24, buf, blocks);
    run("mul_hi_u32_u24", k_mulhi_u24, buf, blocks);
    run("mad_u32_u24", k_mad_u24, buf, blocks);
    run("mad_u64_u32", k_mad_u64, buf, blocks);
    run("lshl_add_u64", k_lshl_add_u64, buf, blocks);
    run("cmp_le_u64", k_cmp_u64, buf, blocks);
    run("lshrrev_b64", k_lshr_b64, buf, blocks);
    run("fma_f64", k_fma_f64, buf, blocks);
    run("mov_b64", k_mov_b64, buf, blocks);
    return 0;
}
