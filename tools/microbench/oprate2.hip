// Instruction throughput on gfx950 with 16 independent chains per thread and
// 16 waves/CU, compiled from C (the forms the NTT kernels use).  Reports
// wave-instructions per SIMD-cycle relative to the 2-cycle full-rate issue.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define IT 512
#define CH 16
template <int OP>
__global__ __launch_bounds__(256) void k(uint64_t* out, uint32_t s1, uint32_t s2) {
  uint64_t x[CH];
  uint32_t y[CH];
#pragma unroll
  for (int c = 0; c < CH; c++) { x[c] = threadIdx.x * 977u + c * 131u + s1; y[c] = (uint32_t)x[c] ^ s2; }
  for (int i = 0; i < IT; i++) {
#pragma unroll
    for (int c = 0; c < CH; c++) {
      if (OP == 0) x[c] = (uint64_t)(uint32_t)x[c] * (uint64_t)(s1 + c) + x[c];                 // v_mad_u64_u32
      if (OP == 1) y[c] = y[c] * (s1 | c) + 1;                                                  // v_mul_lo_u32 (+add)
      if (OP == 2) y[c] = __umulhi(y[c], s1 + c) ^ c;                                            // v_mul_hi_u32 (+xor)
      if (OP == 3) x[c] = x[c] + ((uint64_t)s1 << 3) + c;                                       // v_lshl_add_u64
      if (OP == 4) y[c] = y[c] + (s1 ^ c);                                                      // v_add_u32
      if (OP == 5) x[c] = x[c] >= s1 ? x[c] - s1 : x[c] + 7;                                    // cmp64 + cndmask + sub
      if (OP == 6) y[c] = (y[c] << (c & 7)) ^ s1;                                               // v_lshlrev_b32 + xor
      if (OP == 7) y[c] = y[c] * (s1 | c);                                                      // bare v_mul_lo_u32
    }
  }
  uint64_t r = 0;
#pragma unroll
  for (int c = 0; c < CH; c++) r ^= x[c] ^ y[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
template <int OP>
void run(const char* name, uint64_t* buf, int blocks, double ops_per_iter) {
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, buf, 12345u, 678u);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, buf, 12345u, 678u);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  double waveinst = (double)blocks * 4 * IT * CH * ops_per_iter * 5;  // wave-instructions
  double simd_cycles = 1024.0 * 2.4e9 * ms / 1e3;                     // at 2.4 GHz nominal
  printf("%-34s %.3f wave-inst per SIMD-cycle (1/%.1f)  [%.2f ms]\n", name, waveinst / simd_cycles,
         simd_cycles / waveinst, ms / 5);
}
int main() {
  int blocks = 256 * 16; uint64_t* buf; (void)hipMalloc(&buf, (size_t)blocks * 256 * 8);
  run<0>("mad_u64_u32 (x=lo*s+x)", buf, blocks, 1);
  run<7>("mul_lo_u32 bare", buf, blocks, 1);
  run<1>("mul_lo_u32 + add", buf, blocks, 2);
  run<2>("mul_hi_u32 + xor", buf, blocks, 2);
  run<3>("lshl_add_u64 (x+=c)", buf, blocks, 1);
  run<4>("add_u32", buf, blocks, 1);
  run<5>("csub64 (cmp,cndmask,sub)", buf, blocks, 5);
  run<6>("lshl_b32 + xor", buf, blocks, 2);
  return 0;
}
