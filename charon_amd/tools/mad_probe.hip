// Microbenchmark: sustained 32x32->64 integer multiply-add rate (v_mad_u64_u32) on one GPU.
// Output feeds bench.py's roofline peak (profiles/r01_mad_probe.txt).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

__global__ void k_mad(uint64_t* out, uint32_t c, int iters) {
  uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      a0 = (uint64_t)(uint32_t)a0 * c + a0;
      a1 = (uint64_t)(uint32_t)a1 * c + a1;
      a2 = (uint64_t)(uint32_t)a2 * c + a2;
      a3 = (uint64_t)(uint32_t)a3 * c + a3;
      a4 = (uint64_t)(uint32_t)a4 * c + a4;
      a5 = (uint64_t)(uint32_t)a5 * c + a5;
      a6 = (uint64_t)(uint32_t)a6 * c + a6;
      a7 = (uint64_t)(uint32_t)a7 * c + a7;
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

int main() {
  const int blocks = 256 * 16, threads = 256, iters = 1000;
  uint64_t* d;
  if (hipMalloc(&d, (size_t)blocks * threads * 8) != hipSuccess) return 1;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(k_mad, dim3(blocks), dim3(threads), 0, 0, d, 0x9E3779B9u, 10);
  (void)hipDeviceSynchronize();
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(k_mad, dim3(blocks), dim3(threads), 0, 0, d, 0x9E3779B9u, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) best = ms;
  }
  const double mads = (double)blocks * threads * iters * 16 * 8;
  printf("v_mad_u64_u32 sustained: %.2f T/s (best of 5, %.3f ms, %d blocks x %d threads)\n", mads / best / 1e9,
         best, blocks, threads);
  printf("nominal full-rate int32 lane-ops: 256 CU x 4 SIMD x 32 lanes x 2.4 GHz = 78.6 T/s\n");
  return 0;
}
