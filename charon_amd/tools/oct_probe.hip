// Microbenchmark of the split-Fp2 build (verify_lat.hip): cycles per operation for eight lanes per value (the Fp2
// twins l, l ^ 4 and the quad), at one wave per SIMD, to see what the octet check's latency is made of.  Each
// octet holds one value (identical on its eight lanes, as the kernels require); s_memtime around a dependent chain;
// median over waves.  Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o charon_amd/tools/oct_probe oct_probe.hip
#define BLS_FP2_PAIR 1
#define bls bls_fp2p
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>

#include "../csrc/lg2.h"

using namespace bls;

template <int K>
__global__ void __launch_bounds__(64) k_op(const uint32_t* in, uint32_t* out, uint64_t* cyc, int iters) {
  const int lane = threadIdx.x;
  const int oct = lane >> 3;
  const quad_m qm(lane & 3);
  const uint32_t m = (lane & 1) ? ~0u : 0u;
  fp12 f;
  uint32_t* fw = &f.c0.c0.c0.v[0];
  for (int w = 0; w < 144; ++w) fw[w] = in[(oct * 144 + w) % 4096] & 0x0fffffffu;
  cyc_c c;
  c.z2 = f.c0.c0;
  c.z3 = f.c0.c1;
  c.z4 = f.c0.c2;
  c.z5 = f.c1.c0;
  g1a P;
  P.x = f.c1.c1.c0;
  P.y = f.c1.c1.c1;
  g2a Q;
  Q.x = f.c1.c2;
  Q.y = f.c1.c1;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    if (K == 0) fp_mul(f.c0.c0.c0, f.c0.c0.c0, f.c0.c0.c1);
    if (K == 1) fp2_mul(f.c0.c0, f.c0.c0, f.c0.c1);
    if (K == 2) fp2_sqr(f.c0.c0, f.c0.c0);
    if (K == 3) fp2_add(f.c0.c0, f.c0.c0, f.c0.c1);
    if (K == 4) cyc_sqr_compressed_quad(c, qm);
    if (K == 5) fp12q_mul(f, f, f, qm);
    if (K == 6) fp12q_exp_xabs(f, f, qm);
    if (K == 7) final_exponentiation_quad(f, f, qm);
    if (K == 8) {
      fp6 h;
      miller_loop_split(h, P, Q, m);
      f.c0 = h;
    }
    if (K == 9) fp2_inv(f.c0.c0, f.c0.c0);
    if (K == 10) fp12_inv(f, f);
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  const uint32_t* cw = &c.z2.c0.v[0];
  uint32_t acc = 0;
  for (int w = 0; w < 144; ++w) acc ^= fw[w];
  for (int w = 0; w < 96; ++w) acc ^= cw[w];
  out[blockIdx.x * 64 + lane] = acc;
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  constexpr int NOPS = 11;
  const char* names[NOPS] = {"fp_mul (not split)", "fp2_mul (twins)", "fp2_sqr (twins)", "fp2_add", "cyc_sqr_compressed_quad",
                             "fp12q_mul", "fp12q_exp_xabs", "final_exponentiation_quad", "miller_loop_split",
                             "fp2_inv", "fp12_inv"};
  const int iters[NOPS] = {400, 200, 200, 400, 40, 20, 2, 1, 1, 10, 4};
  uint32_t *d_in, *d_out;
  uint64_t* d_cyc;
  uint32_t h_in[4096];
  for (int i = 0; i < 4096; ++i) h_in[i] = 0x9E3779B9u * (i + 7);
  if (hipMalloc(&d_in, sizeof(h_in)) || hipMalloc(&d_out, 1024 * 64 * 4) || hipMalloc(&d_cyc, 1024 * 8)) return 1;
  (void)hipMemcpy(d_in, h_in, sizeof(h_in), hipMemcpyHostToDevice);
  uint64_t h_cyc[1024];
  double per_product = 0;
  for (int k = 0; k < NOPS; ++k) {
    for (int rep = 0; rep < 2; ++rep) {
      switch (k) {
#define L(K) case K: hipLaunchKernelGGL(k_op<K>, dim3(1024), dim3(64), 0, 0, d_in, d_out, d_cyc, iters[K]); break;
        L(0) L(1) L(2) L(3) L(4) L(5) L(6) L(7) L(8) L(9) L(10)
      }
      if (hipDeviceSynchronize() != hipSuccess) return 2;
    }
    (void)hipMemcpy(h_cyc, d_cyc, sizeof(h_cyc), hipMemcpyDeviceToHost);
    std::sort(h_cyc, h_cyc + 1024);
    const double cy = (double)h_cyc[512] / iters[k];
    if (k == 0) per_product = cy;
    printf("%-28s %10.0f cycles/op  = %7.1f fp_mul-worth\n", names[k], cy, cy / per_product);
  }
  return 0;
}
