// Microbenchmark: latency vs issue cost of the integer multiply-add chains the Fp product is built
// from, and the Fp product itself at 1..8 waves per SIMD.  Decides how much ILP the gfx950 Montgomery
// kernels need (DESIGN.md "Latency").  Output: profiles/r01_lat_probe.txt
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include "field.h"

using namespace bls;

#define MAD1(acc, x, y) "v_mad_u64_u32 " acc ", vcc, " x ", " y ", " acc "\n\t"

template <int CH>
__global__ void __launch_bounds__(64) k_chain(uint64_t* out, uint32_t seed, long long* cyc) {
  uint32_t x = threadIdx.x + seed, y = seed * 3 + 1;
  uint64_t a0 = x, a1 = x + 1, a2 = x + 2, a3 = x + 3;
  long long t0 = clock64();
  for (int it = 0; it < 64; ++it) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      if (CH == 1) {
        asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0\n\t" : "+v"(a0) : "v"(x), "v"(y) : "vcc");
      } else if (CH == 2) {
        asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_mad_u64_u32 %1, vcc, %2, %3, %1\n\t"
                     : "+v"(a0), "+v"(a1) : "v"(x), "v"(y) : "vcc");
      } else if (CH == 3) {  // mad + addc on vcc, one chain (the shape of fp_asm_gfx950.h)
        uint32_t t = 0;
        asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\t"
                     : "+v"(a0), "+v"(t) : "v"(x), "v"(y) : "vcc");
        a1 += t;
      } else {  // 4 independent chains
        asm volatile("v_mad_u64_u32 %0, vcc, %4, %5, %0\n\tv_mad_u64_u32 %1, vcc, %4, %5, %1\n\t"
                     "v_mad_u64_u32 %2, vcc, %4, %5, %2\n\tv_mad_u64_u32 %3, vcc, %4, %5, %3\n\t"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(x), "v"(y) : "vcc");
      }
    }
  }
  long long t1 = clock64();
  out[blockIdx.x * 64 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

__global__ void __launch_bounds__(64) k_fpmul(uint32_t* out, int iters) {
  fp a, b;
  for (int i = 0; i < 12; ++i) {
    a.v[i] = (threadIdx.x * 2654435761u + i) & 0x0fffffff;
    b.v[i] = (blockIdx.x * 40503u + 7 * i) & 0x0fffffff;
  }
  for (int i = 0; i < iters; ++i) fp_mul(a, a, b);
  for (int i = 0; i < 12; ++i) out[(blockIdx.x * 64 + threadIdx.x) * 12 + i] = a.v[i];
}

int main() {
  uint64_t* d;
  long long* dc;
  uint32_t* dm;
  (void)hipMalloc(&d, 1 << 24);
  (void)hipMalloc(&dc, 8);
  (void)hipMalloc(&dm, 64ull << 20);
  long long c;
  const char* names[] = {"", "1 dependent mad chain", "2 interleaved mad chains", "mad+addc(vcc) chain",
                         "4 interleaved mad chains"};
  for (int ch = 1; ch <= 4; ++ch) {
    for (int rep = 0; rep < 2; ++rep) {
      if (ch == 1) hipLaunchKernelGGL(k_chain<1>, dim3(1), dim3(64), 0, 0, d, 7u, dc);
      if (ch == 2) hipLaunchKernelGGL(k_chain<2>, dim3(1), dim3(64), 0, 0, d, 7u, dc);
      if (ch == 3) hipLaunchKernelGGL(k_chain<3>, dim3(1), dim3(64), 0, 0, d, 7u, dc);
      if (ch == 4) hipLaunchKernelGGL(k_chain<4>, dim3(1), dim3(64), 0, 0, d, 7u, dc);
      (void)hipDeviceSynchronize();
    }
    (void)hipMemcpy(&c, dc, 8, hipMemcpyDeviceToHost);
    const int per = ch == 2 ? 2 : ch == 4 ? 4 : 1;
    printf("%-28s: %.2f cycles per group (%d mad per group), one wave\n", names[ch], (double)c / 1024, per);
  }
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int iters = 2000;
  for (int wps = 1; wps <= 8; wps *= 2) {
    const int blocks = 1024 * wps;
    hipLaunchKernelGGL(k_fpmul, dim3(blocks), dim3(64), 0, 0, dm, 10);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(k_fpmul, dim3(blocks), dim3(64), 0, 0, dm, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double muls = (double)blocks * 64 * iters;
    printf("fp_mul chain, %d wave(s)/SIMD: %.3f ms, %.1f G fp_mul/s, %.0f ns per mul per wave\n", wps, ms,
           muls / ms / 1e6, ms * 1e6 / iters);
  }
  return 0;
}
