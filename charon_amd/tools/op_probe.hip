// Microbenchmark: cycles per tower / curve operation at one wave per SIMD (the C2 regime), against the
// cost of the Fp products each one performs (profiles/r02_op_probe.txt).  Each lane runs a dependent chain of
// one operation; s_memtime around the loop; median over waves.  Shows how much of an operation's time is
// products and how much is operand traffic (scratch/flat loads), adds and selects.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#include "../csrc/ops.h"

using namespace bls;

template <int K>
__global__ void __launch_bounds__(64) k_op(const uint32_t* in, uint32_t* out, uint64_t* cyc, int iters) {
  const int lane = threadIdx.x;
  fp12 f;
  uint32_t* fw = &f.c0.c0.c0.v[0];
  for (int w = 0; w < 144; ++w) fw[w] = in[(lane * 144 + w) % 4096] & 0x0fffffffu;
  fp2 g0 = f.c0.c0, g1 = f.c0.c1, h1 = f.c0.c2;
  g2j T;
  T.x = f.c1.c0;
  T.y = f.c1.c1;
  T.z = f.c1.c2;
  g1a P;
  P.x = f.c0.c0.c0;
  P.y = f.c0.c0.c1;
  uint8_t valid96[96];
  if (K == 25) {  // a valid compressed G2 point per lane (outside the timed loop)
    uint8_t m[32];
    for (int b = 0; b < 32; ++b) m[b] = (uint8_t)(lane + 7 * b);
    g2j hj;
    hash_to_g2(hj, m, 32, DST_POP, 43);
    g2_compress(valid96, hj);
  }
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    if (K == 0) fp_mul(f.c0.c0.c0, f.c0.c0.c0, f.c0.c0.c1);
    if (K == 1) fp_add(f.c0.c0.c0, f.c0.c0.c0, f.c0.c0.c1);
    if (K == 2) fp2_mul(f.c0.c0, f.c0.c0, f.c0.c1);
    if (K == 3) fp6_mul(f.c0, f.c0, f.c1);
    if (K == 4) fp12_sqr(f, f);
    if (K == 5) fp12_mul(f, f, f);
    if (K == 6) fp12_mul_line2(f, g0, g1, h1, g1, h1, g0);
    if (K == 7) fp12_cyclotomic_sqr(f, f);
    if (K == 8) miller_dbl_step(T, g0, g1, h1, P.x, P.y);
    if (K == 9) jac_dbl(T, T);
    if (K == 10) fp_sub(f.c0.c0.c0, f.c0.c0.c0, f.c0.c0.c1);
    if (K == 11) final_exponentiation(f, f);
    if (K == 12) fp12_cyc_exp_xabs(f, f);
    if (K == 13) {
      g1a Ps[2];
      g2a Qs[2];
      bool skip[2] = {false, false};
      Ps[0] = P;
      Ps[1] = P;
      Qs[0].x = T.x;
      Qs[0].y = T.y;
      Qs[1].x = T.y;
      Qs[1].y = T.x;
      miller_loop_n(f, Ps, Qs, skip, 2);
    }
    if (K == 14) {
      uint8_t m[32];
      for (int b = 0; b < 32; ++b) m[b] = (uint8_t)(f.c0.c0.c0.v[b & 7] >> (b & 24));
      g2j hj;
      hash_to_g2(hj, m, 32, DST_POP, 43);
      f.c0.c0 = hj.x;
    }
    if (K == 15) {
      uint8_t b[96];
      b[0] = 0xa0;
      for (int k = 1; k < 96; ++k) b[k] = (uint8_t)(f.c0.c0.c0.v[k % 12] >> (k & 24));
      g2a a;
      const int st = g2_decompress(a, b, true);
      f.c0.c0 = a.x;
      f.c0.c1.c0.v[0] ^= (uint32_t)st;
    }
    if (K == 21) {
      uint8_t b[96];
      b[0] = 0xa0;
      for (int k = 1; k < 96; ++k) b[k] = (uint8_t)(f.c0.c0.c0.v[k % 12] >> (k & 24));
      g2a a;
      const int st = g2_decompress(a, b, false);
      f.c0.c0 = a.x;
      f.c0.c1.c0.v[0] ^= (uint32_t)st;
    }
    if (K == 22) {
      g2j pj;
      pj.x = T.x;
      pj.y = T.y;
      fp2_set_one(pj.z);
      f.c0.c1.c0.v[1] ^= g2_in_subgroup(pj) ? 1u : 0u;
      T.x = T.y;
    }
    if (K == 23 || K == 24) {  // g2_decompress without the square root (23) / with it (24), inlined here
      uint8_t b[96];
      b[0] = 0xa0;
      for (int k = 1; k < 96; ++k) b[k] = (uint8_t)(f.c0.c0.c0.v[k % 12] >> (k & 24));
      uint8_t buf[96];
      for (int i = 0; i < 96; ++i) buf[i] = b[i];
      buf[0] &= 0x1f;
      fp2 x;
      fp_plain_from_be48(x.c1, buf);
      fp_plain_from_be48(x.c0, buf + 48);
      int st = (!fp_plain_lt_p(x.c0) || !fp_plain_lt_p(x.c1)) ? 1 : 0;
      fp_to_mont(x.c0, x.c0);
      fp_to_mont(x.c1, x.c1);
      fp2 y2, y;
      fp2_sqr(y2, x);
      fp2_mul(y2, y2, x);
      fp2_add(y2, y2, FP2_B2);
      if (K == 24) {
        if (!fp2_sqrt(y, y2)) st |= 2;
      } else {
        y = y2;
      }
      if (fp2_is_lex_largest(y)) fp2_neg(y, y);
      f.c0.c0 = y;
      f.c0.c1.c0.v[0] ^= (uint32_t)st;
    }
    if (K == 25) {
      g2a a;
      const int st = g2_decompress(a, valid96, false);
      f.c0.c0 = a.x;
      f.c0.c1.c0.v[0] ^= (uint32_t)st;
      valid96[95] ^= (uint8_t)(a.y.c0.v[0] & 0);  // keep the input live per iteration
    }
    if (K == 16) fp_pow(f.c0.c0.c0, f.c0.c0.c0, EXP_SQRT, 378);
    if (K == 18) {
      fp2 y;
      const bool ok = fp2_sqrt(y, f.c0.c0);
      f.c0.c0 = y;
      f.c0.c1.c0.v[0] ^= ok ? 1u : 0u;
    }
    if (K == 19) f.c0.c1.c0.v[1] ^= g2_in_subgroup(T) ? 1u : 0u;
    if (K == 20) {
      g1j q, p1;
      p1.x = P.x;
      p1.y = P.y;
      fp_set_one(p1.z);
      jac_mul_u64(q, p1, X_ABS);
      P.x = q.x;
      P.y = q.y;
    }
    if (K == 17) {
      g1a a;
      uint8_t b[48];
      b[0] = 0x80 | (uint8_t)(f.c0.c0.c0.v[0] & 0x1f);
      for (int k = 1; k < 48; ++k) b[k] = (uint8_t)(f.c0.c0.c1.v[k % 12] >> (k & 24));
      const int st = g1_decompress(a, b, true);
      f.c0.c0.c0 = a.x;
      f.c0.c1.c0.v[0] ^= (uint32_t)st;
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  uint32_t acc = 0;
  for (int w = 0; w < 144; ++w) acc ^= fw[w];
  acc ^= g0.c0.v[0] ^ T.x.c0.v[1] ^ T.z.c1.v[2];
  out[blockIdx.x * 64 + lane] = acc;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

static double median(uint64_t* h, int n) {
  for (int i = 1; i < n; ++i)
    for (int j = i; j > 0 && h[j - 1] > h[j]; --j) {
      const uint64_t t = h[j];
      h[j] = h[j - 1];
      h[j - 1] = t;
    }
  return (double)h[n / 2];
}

int main() {
  constexpr int NOPS = 26;
  const char* names[NOPS] = {"fp_mul", "fp_add", "fp2_mul", "fp6_mul", "fp12_sqr", "fp12_mul", "fp12_mul_line2",
                           "fp12_cyclotomic_sqr", "miller_dbl_step", "jac_dbl<fp2>", "fp_sub",
                           "final_exponentiation", "fp12_cyc_exp_xabs", "miller_loop_n(2)", "hash_to_g2",
                           "g2_decompress+subgroup", "fp_pow(sqrt)", "g1_decompress+subgroup", "fp2_sqrt", "g2_in_subgroup", "jac_mul_u64<fp>(|x|)", "g2_decompress(no sub)", "g2_in_subgroup(z=1)", "g2dec parts w/o sqrt", "g2dec parts + sqrt", "g2_decompress(valid, no sub)"};
  // Fp products per op (host instrumented build: tests/test_work_counts.py); 0 = not a product count
  const int products[NOPS] = {1, 0, 3, 18, 36, 54, 69, 18, 25, 16, 0, 8150, 1404, 10700, 5740, 2203, 458, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  const int iters[NOPS] = {400, 400, 200, 40, 20, 20, 20, 40, 40, 40, 400, 1, 2, 1, 2, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4};
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
        L(0) L(1) L(2) L(3) L(4) L(5) L(6) L(7) L(8) L(9) L(10) L(11) L(12) L(13) L(14) L(15) L(16) L(17) L(18) L(19) L(20) L(21) L(22) L(23) L(24) L(25)
      }
      if (hipDeviceSynchronize() != hipSuccess) return 2;
    }
    (void)hipMemcpy(h_cyc, d_cyc, sizeof(h_cyc), hipMemcpyDeviceToHost);
    const double c = median(h_cyc, 1024) / iters[k];
    if (k == 0) per_product = c;
    printf("%-22s %9.0f cycles/op  products %3d  = %5.2f products-worth  (overhead %5.1f %%)\n", names[k], c,
           products[k], c / per_product, products[k] ? 100.0 * (c / per_product - products[k]) / (c / per_product) : 100.0);
  }
  return 0;
}
