// oprate4.hip -- per-instruction VALU issue cost on gfx950 in SHADER CYCLES.
//
// oprate3 timed launches with events and normalised to a nominal 2.4 GHz; the
// clock under load is lower (DVFS under the package power cap), so its
// "cycles" overstate the cost.  Here every wave reads s_memtime (the shader
// clock, MI355X_MICROARCH.md "s_memtime tick = shader cycle") around its own
// loop, so the result does not depend on the clock the box runs at.
//
// One workgroup per CU (grid = CUs), W waves per SIMD (blockDim = 256 W),
// CH independent chains per thread, IT iterations.  Per SIMD the W waves
// issue W * IT * CH instructions in (median wave elapsed) cycles.
//   CH = 16, W = 1..4 -> throughput (cycles per wave64 instruction per SIMD);
//   one 256 W-thread workgroup per CU, so W waves share each SIMD
//   CH = 1,  W = 1    -> dependent-issue latency of one chain
// Build: hipcc -O3 --offload-arch=gfx950 -o oprate4_bin oprate4.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#define IT 512

#define K32(NAME, ASM)                                                                              \
    template <int CH>                                                                               \
    __global__ __launch_bounds__(1024) void NAME(uint64_t* cyc, uint32_t* out, uint32_t s1) {      \
        uint32_t y[CH];                                                                             \
        _Pragma("unroll") for (int c = 0; c < CH; c++) y[c] = threadIdx.x * 977u + c + s1;          \
        uint32_t z = s1 ^ 0x1234567u;                                                               \
        __builtin_amdgcn_s_waitcnt(0);                                                              \
        const uint64_t t0 = __builtin_amdgcn_s_memtime();                                           \
        for (int i = 0; i < IT; i++) {                                                              \
            _Pragma("unroll") for (int c = 0; c < CH; c++) asm volatile(ASM : "+v"(y[c]) : "v"(z) : "vcc"); \
        }                                                                                           \
        const uint64_t t1 = __builtin_amdgcn_s_memtime();                                           \
        uint32_t r = 0;                                                                             \
        _Pragma("unroll") for (int c = 0; c < CH; c++) r ^= y[c];                                   \
        out[blockIdx.x * blockDim.x + threadIdx.x] = r;                                             \
        if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0; \
    }
#define K64Z(NAME, ZT, ASM)                                                                              \
    template <int CH>                                                                               \
    __global__ __launch_bounds__(1024) void NAME(uint64_t* cyc, uint32_t* out, uint32_t s1) {      \
        uint64_t y[CH];                                                                             \
        _Pragma("unroll") for (int c = 0; c < CH; c++) y[c] = threadIdx.x * 977u + c + s1;          \
        ZT z = s1 ^ 0x1234567u;                                                               \
        __builtin_amdgcn_s_waitcnt(0);                                                              \
        const uint64_t t0 = __builtin_amdgcn_s_memtime();                                           \
        for (int i = 0; i < IT; i++) {                                                              \
            _Pragma("unroll") for (int c = 0; c < CH; c++) asm volatile(ASM : "+v"(y[c]) : "v"(z) : "vcc"); \
        }                                                                                           \
        const uint64_t t1 = __builtin_amdgcn_s_memtime();                                           \
        uint64_t r = 0;                                                                             \
        _Pragma("unroll") for (int c = 0; c < CH; c++) r ^= y[c];                                   \
        out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(r ^ (r >> 32));                     \
        if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0; \
    }

#define K64(NAME, ASM) K64Z(NAME, uint64_t, ASM)
K32(k_add_u32, "v_add_u32 %0, %0, %1")
K32(k_add3_u32, "v_add3_u32 %0, %0, %1, %0")
K32(k_xor, "v_xor_b32 %0, %0, %1")
K32(k_lshl_b32, "v_lshlrev_b32 %0, 3, %0")
K32(k_mul_lo, "v_mul_lo_u32 %0, %0, %1")
K32(k_mul_hi, "v_mul_hi_u32 %0, %0, %1")
K32(k_mul_u24, "v_mul_u32_u24 %0, %0, %1")
K32(k_mul_hi_u24, "v_mul_hi_u32_u24 %0, %0, %1")
K32(k_add_co, "v_add_co_u32 %0, vcc, %0, %1")
K32(k_addc_co, "v_addc_co_u32 %0, vcc, %0, %1, vcc")
K32(k_cndmask, "v_cndmask_b32 %0, %0, %1, vcc")
K32(k_fma_f32, "v_fma_f32 %0, %0, %1, %0")
K32(k_mov_b32, "v_mov_b32 %0, %1")
K64Z(k_mad_u64, uint32_t, "v_mad_u64_u32 %0, vcc, %1, %1, %0")
K64(k_lshl_add_u64, "v_lshl_add_u64 %0, %0, 0, %1")
K64(k_cmp_u64, "v_cmp_le_u64 vcc, %0, %1")
K64(k_lshr_b64, "v_lshrrev_b64 %0, 3, %0")
K64(k_fma_f64, "v_fma_f64 %0, %0, %1, %0")
K64(k_mov_b64, "v_mov_b64 %0, %1")

typedef void (*KFn)(uint64_t*, uint32_t*, uint32_t);

static double run(KFn kern, int ch, int waves, int ncu, uint64_t* dcyc, uint32_t* dout, int reps = 3) {
    const int threads = 256 * waves, nw = ncu * threads / 64;
    std::vector<uint64_t> c(nw);
    double best = 1e30;
    for (int r = 0; r < reps; r++) {
        hipLaunchKernelGGL(kern, dim3(ncu), dim3(threads), 0, 0, dcyc, dout, 12345u + r);
        hipError_t e = hipGetLastError();
        if (e == hipSuccess) e = hipDeviceSynchronize();
        if (e != hipSuccess) {
            std::printf("launch failed: %s\n", hipGetErrorString(e));
            std::exit(1);
        }
        (void)hipMemcpy(c.data(), dcyc, nw * 8, hipMemcpyDeviceToHost);
        std::sort(c.begin(), c.end());
        const double med = (double)c[nw / 2];
        // per SIMD: `waves` waves each issued IT * ch instructions in ~med cycles
        best = std::min(best, med / ((double)IT * ch * waves));
    }
    return best;
}

int main() {
    int ncu = 0;
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    uint64_t* dcyc;
    uint32_t* dout;
    (void)hipMalloc(&dcyc, (size_t)ncu * 32 * 8);
    (void)hipMalloc(&dout, (size_t)ncu * 2048 * 4);
    struct Op {
        const char* name;
        KFn thr, lat;
    };
#define OP(N, K) {N, K<16>, K<1>}
    Op ops[] = {OP("v_add_u32", k_add_u32),         OP("v_add3_u32", k_add3_u32),     OP("v_xor_b32", k_xor),
                OP("v_lshlrev_b32", k_lshl_b32),    OP("v_mul_lo_u32", k_mul_lo),     OP("v_mul_hi_u32", k_mul_hi),
                OP("v_mul_u32_u24", k_mul_u24),     OP("v_mul_hi_u32_u24", k_mul_hi_u24),
                OP("v_add_co_u32", k_add_co),       OP("v_addc_co_u32", k_addc_co),   OP("v_cndmask_b32", k_cndmask),
                OP("v_fma_f32", k_fma_f32),         OP("v_mov_b32", k_mov_b32),       OP("v_mad_u64_u32", k_mad_u64),
                OP("v_lshl_add_u64", k_lshl_add_u64), OP("v_cmp_le_u64", k_cmp_u64), OP("v_lshrrev_b64", k_lshr_b64),
                OP("v_fma_f64", k_fma_f64),         OP("v_mov_b64", k_mov_b64)};
    std::printf("# shader cycles per wave64 instruction per SIMD (s_memtime), %d CUs\n", ncu);
    std::printf("%-18s %8s %8s %8s %8s %10s\n", "instruction", "W=1", "W=2", "W=3", "W=4", "latency");
    for (auto& o : ops) {
        double t[4];
        const int ws[4] = {1, 2, 3, 4};
        for (int i = 0; i < 4; i++) t[i] = run(o.thr, 16, ws[i], ncu, dcyc, dout);
        const double lat = run(o.lat, 1, 1, ncu, dcyc, dout);
        std::printf("%-18s %8.2f %8.2f %8.2f %8.2f %10.2f\n", o.name, t[0], t[1], t[2], t[3], lat);
    }
    return 0;
}
