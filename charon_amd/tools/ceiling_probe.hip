// The practical ceiling of k_verify_fused's arithmetic on MI355X: every lane of every SIMD
// runs nothing but the shipped product routines (tools/gen_fp_asm.py: the Fp2 product and square, the Fp product,
// reached by s_swappc exactly as the verify kernels reach them) in a dependent chain, for ~40 ms, at one wave per
// SIMD (the C2 kernel's occupancy: 36 KiB of LDS per one-wave workgroup, as BLS_LANE_F12) and at two.  It prints
// Fp-mul-equivalent products per second (an Fp2 product = 3, a square = 2, the roofline unit of bench.py) and the
// wall-clock SIMD cycles implied at the nominal 2.4 GHz, and checks a few lanes against the host build of the same
// field code.  k_verify_fused's own rate (24,247 products per Verify x C2 verifies/s) divided by this figure is the
// fraction of the attainable product rate the kernel reaches.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../csrc -I../../include -o ceiling_probe ceiling_probe.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "tower.h"

using namespace bls;

#define CK(x)                                                                                 \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess) {                                                                   \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));      \
      exit(1);                                                                                \
    }                                                                                         \
  } while (0)

// MODE 0: Fp2 product a <- a b; 1: Fp2 square a <- a^2 + b (the add keeps the chain from collapsing);
// 2: Fp product a.c0 <- a.c0 b.c0.  LDS_KB pins the occupancy: 36 -> 4 one-wave workgroups per CU (one per SIMD).
template <int MODE, int LDS_KB>
__global__ void __launch_bounds__(64) k_chain(const fp2* in, fp2* out, int iters) {
  __shared__ uint32_t pad[LDS_KB * 256];
  const int lane = blockIdx.x * 64 + threadIdx.x;
  fp2 a = in[2 * (lane & 1023)], b = in[2 * (lane & 1023) + 1];
  if (iters < 0) pad[threadIdx.x] = a.c0.v[0];  // never: keeps the LDS allocation
  for (int k = 0; k < iters; ++k) {
    if (MODE == 0) {
      fp2_mul(a, a, b);
    } else if (MODE == 1) {
      fp2_sqr(a, a);
      fp2_add(a, a, b);
    } else {
      fp_mul(a.c0, a.c0, b.c0);
    }
  }
  out[lane] = a;
}

static void host_chain(int mode, fp2& a, const fp2& b, int iters) {
  for (int k = 0; k < iters; ++k) {
    if (mode == 0) {
      fp2_mul(a, a, b);
    } else if (mode == 1) {
      fp2_sqr(a, a);
      fp2_add(a, a, b);
    } else {
      fp_mul(a.c0, a.c0, b.c0);
    }
  }
}

template <int MODE, int LDS_KB>
static double run(const fp2* d_in, fp2* d_out, const std::vector<fp2>& h_in, int blocks, int iters, const char* name,
                  double units) {
  hipLaunchKernelGGL((k_chain<MODE, LDS_KB>), dim3(blocks), dim3(64), 0, 0, d_in, d_out, 8);  // warm-up
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, 0));
  hipLaunchKernelGGL((k_chain<MODE, LDS_KB>), dim3(blocks), dim3(64), 0, 0, d_in, d_out, iters);
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<fp2> got(blocks * 64);
  CK(hipMemcpy(got.data(), d_out, sizeof(fp2) * got.size(), hipMemcpyDeviceToHost));
  int bad = 0;
  for (int lane : {0, 1, 63, 64 * 37 + 5}) {
    fp2 a = h_in[2 * (lane & 1023)];
    host_chain(MODE, a, h_in[2 * (lane & 1023) + 1], iters);
    for (int j = 0; j < 12; ++j) {
      bad += a.c0.v[j] != got[lane].c0.v[j];
      if (MODE != 2) bad += a.c1.v[j] != got[lane].c1.v[j];
    }
  }
  const double lanes = blocks * 64.0;
  const double rate = lanes * iters * units / (ms * 1e-3);
  const double waves_per_simd = blocks / 1024.0;
  printf("%-34s waves/SIMD %.0f: %8.3f ms  %7.2f G products/s  %7.1f ns per chain step per wave  check %s\n", name,
         waves_per_simd, ms, rate / 1e9, ms * 1e6 / iters, bad ? "FAILED" : "ok");
  return rate;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 4000;
  std::vector<fp2> h(2048);
  uint64_t s = 0x636861726f6e;
  for (auto& x : h) {
    for (int j = 0; j < 12; ++j) {
      s = s * 6364136223846793005ull + 1442695040888963407ull;
      x.c0.v[j] = (uint32_t)(s >> 32);
      s = s * 6364136223846793005ull + 1442695040888963407ull;
      x.c1.v[j] = (uint32_t)(s >> 32);
    }
    x.c0.v[11] &= 0x0fffffff;  // < p
    x.c1.v[11] &= 0x0fffffff;
  }
  fp2 *d_in, *d_out;
  CK(hipMalloc(&d_in, sizeof(fp2) * h.size()));
  CK(hipMalloc(&d_out, sizeof(fp2) * 2048 * 64));
  CK(hipMemcpy(d_in, h.data(), sizeof(fp2) * h.size(), hipMemcpyHostToDevice));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int one = 4 * cus;  // one wave per SIMD
  printf("CUs %d, %d iterations per lane\n", cus, iters);
  run<0, 36>(d_in, d_out, h, one, iters, "Fp2 product (3 units)", 3.0);
  run<1, 36>(d_in, d_out, h, one, iters, "Fp2 square + add (2 units)", 2.0);
  run<2, 36>(d_in, d_out, h, one, iters, "Fp product (1 unit)", 1.0);
  run<0, 18>(d_in, d_out, h, 2 * one, iters / 2, "Fp2 product (3 units)", 3.0);
  run<2, 18>(d_in, d_out, h, 2 * one, iters / 2, "Fp product (1 unit)", 1.0);
  CK(hipFree(d_in));
  CK(hipFree(d_out));
  return 0;
}
