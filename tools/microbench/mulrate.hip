// Microbenchmark: 32/64-bit integer multiply and modmul throughput on gfx950.
// Used once to size the NTT design (DESIGN.md "VALU budget").
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define ITERS 2048
#define CHAINS 8

__global__ void k_mullo32(uint32_t* out, uint32_t seed) {
  uint32_t x[CHAINS];
  for (int c = 0; c < CHAINS; c++) x[c] = threadIdx.x * 7 + c + seed;
  for (int i = 0; i < ITERS; i++) {
#pragma unroll
    for (int c = 0; c < CHAINS; c++) x[c] = x[c] * (x[c] | 1u);
  }
  uint32_t s = 0; for (int c = 0; c < CHAINS; c++) s ^= x[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_mulhi32(uint32_t* out, uint32_t seed) {
  uint32_t x[CHAINS];
  for (int c = 0; c < CHAINS; c++) x[c] = threadIdx.x * 7 + c + seed;
  for (int i = 0; i < ITERS; i++) {
#pragma unroll
    for (int c = 0; c < CHAINS; c++) x[c] = __umulhi(x[c], x[c] ^ 0x9e3779b9u) + 1;
  }
  uint32_t s = 0; for (int c = 0; c < CHAINS; c++) s ^= x[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_mad64(uint64_t* out, uint32_t seed) {
  uint64_t x[CHAINS];
  for (int c = 0; c < CHAINS; c++) x[c] = threadIdx.x * 7 + c + seed;
  for (int i = 0; i < ITERS; i++) {
#pragma unroll
    for (int c = 0; c < CHAINS; c++) x[c] = (uint64_t)(uint32_t)x[c] * (uint32_t)(x[c] >> 17) + x[c];
  }
  uint64_t s = 0; for (int c = 0; c < CHAINS; c++) s ^= x[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_fma32(float* out, uint32_t seed) {
  float x[CHAINS];
  for (int c = 0; c < CHAINS; c++) x[c] = threadIdx.x * 7 + c + seed;
  for (int i = 0; i < ITERS; i++) {
#pragma unroll
    for (int c = 0; c < CHAINS; c++) x[c] = fmaf(x[c], 0.999f, 0.5f);
  }
  float s = 0; for (int c = 0; c < CHAINS; c++) s += x[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_fma64(double* out, uint32_t seed) {
  double x[CHAINS];
  for (int c = 0; c < CHAINS; c++) x[c] = threadIdx.x * 7 + c + seed;
  for (int i = 0; i < ITERS; i++) {
#pragma unroll
    for (int c = 0; c < CHAINS; c++) x[c] = fma(x[c], 0.999, 0.5);
  }
  double s = 0; for (int c = 0; c < CHAINS; c++) s += x[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__device__ __forceinline__ uint64_t shoup(uint64_t a, uint64_t w, uint64_t wp, uint64_t q) {
  uint64_t qh = __umul64hi(a, wp);
  uint64_t r = a * w - qh * q;
  return r >= q ? r - q : r;
}
__global__ void k_shoup(uint64_t* out, uint64_t q, uint64_t w, uint64_t wp) {
  uint64_t x[CHAINS];
  for (int c = 0; c < CHAINS; c++) x[c] = (threadIdx.x * 7919ull + c) % q;
  for (int i = 0; i < ITERS; i++) {
#pragma unroll
    for (int c = 0; c < CHAINS; c++) x[c] = shoup(x[c], w, wp, q);
  }
  uint64_t s = 0; for (int c = 0; c < CHAINS; c++) s ^= x[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename T, typename K, typename... A>
double run(K k, T* buf, int blocks, A... a) {
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, buf, a...);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, buf, a...);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  return ms / 5;
}

int main() {
  int blocks = 256 * 16;
  size_t n = (size_t)blocks * 256;
  void* buf; hipMalloc(&buf, n * 8);
  double ops = (double)n * ITERS * CHAINS;
  double t;
  t = run(k_mullo32, (uint32_t*)buf, blocks, 1u); printf("mul_lo_u32   : %.2f Gop/s\n", ops / t / 1e6);
  t = run(k_mulhi32, (uint32_t*)buf, blocks, 1u); printf("mul_hi_u32   : %.2f Gop/s\n", ops / t / 1e6);
  t = run(k_mad64, (uint64_t*)buf, blocks, 1u);   printf("mad_u64_u32  : %.2f Gop/s\n", ops / t / 1e6);
  t = run(k_fma32, (float*)buf, blocks, 1u);      printf("fma_f32      : %.2f Gop/s\n", ops / t / 1e6);
  t = run(k_fma64, (double*)buf, blocks, 1u);     printf("fma_f64      : %.2f Gop/s\n", ops / t / 1e6);
  uint64_t q = 1152921504606748673ull, w = 62213374832584ull;
  unsigned __int128 wp = ((unsigned __int128)w << 64) / q;
  t = run(k_shoup, (uint64_t*)buf, blocks, q, w, (uint64_t)wp); printf("shoup modmul : %.2f Gop/s\n", ops / t / 1e6);
  hipFree(buf);
  return 0;
}
