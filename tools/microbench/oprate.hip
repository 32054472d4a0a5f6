// Throughput of individual gfx950 VALU instructions relevant to 64-bit modular
// arithmetic (8 independent chains per thread, 16 waves/CU).  tools/microbench.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define ITERS 1024
#define OP_KERNEL(NAME, BODY)                                                   \
__global__ void NAME(uint64_t* out, uint64_t seed) {                            \
  uint64_t x0 = seed + threadIdx.x, x1 = x0 * 3, x2 = x0 * 5, x3 = x0 * 7;      \
  uint64_t x4 = x0 * 11, x5 = x0 * 13, x6 = x0 * 17, x7 = x0 * 19;              \
  uint64_t k = seed | 1;                                                        \
  for (int i = 0; i < ITERS; i++) {                                             \
    BODY(x0) BODY(x1) BODY(x2) BODY(x3) BODY(x4) BODY(x5) BODY(x6) BODY(x7)      \
  }                                                                             \
  out[blockIdx.x * blockDim.x + threadIdx.x] = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7; \
}
#define B_LSHLADD(x) asm volatile("v_lshl_add_u64 %0, %0, 1, %1" : "+v"(x) : "v"(k));
#define B_ADD32(x) { uint32_t l = (uint32_t)x; asm volatile("v_add_u32 %0, %0, %1" : "+v"(l) : "v"((uint32_t)k)); x = (x & ~0xffffffffull) | l; }
#define B_LSHL64(x) asm volatile("v_lshlrev_b64 %0, 1, %0" : "+v"(x));
#define B_ASHR64(x) asm volatile("v_ashrrev_i64 %0, 1, %0" : "+v"(x));
#define B_MAD(x) { uint32_t l = (uint32_t)(x >> 7); asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(x) : "v"(l), "v"((uint32_t)k) : "s0", "s1"); }
#define B_MULLO(x) { uint32_t l = (uint32_t)x; asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(l) : "v"((uint32_t)k)); x = (x & ~0xffffffffull) | l; }
#define B_CNDMASK(x) { uint32_t l = (uint32_t)x; asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(l) : "v"((uint32_t)k)); x = (x & ~0xffffffffull) | l; }
#define B_CMP64(x) asm volatile("v_cmp_gt_u64 vcc, %0, %1" :: "v"(x), "v"(k) : "vcc");
#define B_MOV(x) { uint32_t l; asm volatile("v_mov_b32 %0, %1" : "=v"(l) : "v"((uint32_t)k)); x ^= l; }
OP_KERNEL(k_lshladd, B_LSHLADD)
OP_KERNEL(k_add32, B_ADD32)
OP_KERNEL(k_lshl64, B_LSHL64)
OP_KERNEL(k_ashr64, B_ASHR64)
OP_KERNEL(k_mad, B_MAD)
OP_KERNEL(k_mullo, B_MULLO)
OP_KERNEL(k_cndmask, B_CNDMASK)
OP_KERNEL(k_cmp64, B_CMP64)
OP_KERNEL(k_mov, B_MOV)

template <typename K>
void run(const char* name, K k, uint64_t* buf, int blocks) {
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, buf, 3ull);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, buf, 3ull);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  double ops = (double)blocks * 256 * ITERS * 8 * 5;
  printf("%-12s %8.2f Gop/s  (%.2f of 78.6T full rate)\n", name, ops / ms / 1e6, ops / ms / 1e6 / 78643.2);
}
int main() {
  int blocks = 256 * 16; uint64_t* buf; (void)hipMalloc(&buf, (size_t)blocks * 256 * 8);
  run("lshl_add_u64", k_lshladd, buf, blocks);
  run("add_u32", k_add32, buf, blocks);
  run("lshlrev_b64", k_lshl64, buf, blocks);
  run("ashrrev_i64", k_ashr64, buf, blocks);
  run("mad_u64_u32", k_mad, buf, blocks);
  run("mul_lo_u32", k_mullo, buf, blocks);
  run("cndmask", k_cndmask, buf, blocks);
  run("cmp_gt_u64", k_cmp64, buf, blocks);
  run("mov_b32", k_mov, buf, blocks);
  return 0;
}
