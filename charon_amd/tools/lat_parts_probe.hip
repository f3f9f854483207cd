// Where the n = 1 latency goes: each building block of the octet prep and check (verify_lat.hip), timed on its own
// in the split-Fp2 build at the n = 1 placement (one octet per wave, `waves` waves: 8 = the latency regime, 1024 = the
// whole chip), s_memrealtime (100 MHz) around a dependent chain, median over waves.  Inputs are arbitrary field
// elements (timing only; the point operations do not check their inputs, decompression gets the flag bits set).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I charon_amd/csrc -o charon_amd/tools/lat_parts_probe \
//          charon_amd/tools/lat_parts_probe.hip
// Run:   charon_amd/tools/lat_parts_probe [waves]
#include "../csrc/verify_lat.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>

namespace bls {

template <int K>
__global__ void __launch_bounds__(64) k_part(const uint32_t* in, uint32_t* out, uint64_t* us100, int iters) {
  bls_race::init(nullptr, 0);
  const int lane = threadIdx.x;
  const int oct = lane >> 3;
  const int q = lane & 3;
  const quad_m qm(q);
  const uint32_t m = (lane & 1) ? ~0u : 0u;
  fp12 f;
  uint32_t* fw = &f.c0.c0.c0.v[0];
  for (int w = 0; w < 144; ++w) fw[w] = in[(oct * 144 + w + 7 * blockIdx.x) % 4096] & 0x0fffffffu;
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
  g2j J;
  J.x = f.c0.c1;
  J.y = f.c0.c2;
  J.z = f.c1.c0;
  uint8_t bytes[96];
  for (int k = 0; k < 96; ++k) bytes[k] = (uint8_t)(in[(oct * 96 + k) % 4096] >> 3);
  bytes[0] = (uint8_t)(0x80 | (bytes[0] & 0x1f));
  uint32_t acc = 0;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
    if (K == 0) fp_mul(f.c0.c0.c0, f.c0.c0.c0, f.c0.c0.c1);
    if (K == 1) fp2_mul(f.c0.c0, f.c0.c0, f.c0.c1);
    if (K == 2) fp2_sqr(f.c0.c0, f.c0.c0);
    if (K == 3) fp_pow(f.c0.c0.c0, f.c0.c0.c0, EXP_SQRT, 378);
    if (K == 4) fp2_inv(f.c0.c0, f.c0.c0);
    if (K == 5) fp12_inv(f, f);
    if (K == 6) cyc_sqr_compressed_quad(c, qm);
    if (K == 7) fp12q_mul(f, f, f, qm);
    if (K == 8) fp12q_exp_xabs(f, f, qm);
    if (K == 9) final_exponentiation_quad(f, f, qm);
    if (K == 10) fp12h_sqr_split(f.c0, m);
    if (K == 11) {
      fp2 g0, g1, h1;
      miller_dbl_step_split(J, g0, g1, h1, P.x, P.y, m);
      fp2_add(J.x, J.x, g0);
      fp2_add(J.y, J.y, h1);
    }
    if (K == 12) fp12h_mul_line_split(f.c0, f.c1.c0, f.c1.c1, f.c1.c2, m);
    if (K == 13) {
      fp6 h;
      miller_loop_split(h, P, Q, m);
      f.c0 = h;
    }
    if (K == 14) {
      g2j t;
      g2_dbl_quad(t, J, q);
      J = t;
    }
    if (K == 15) g2_clear_cofactor_quad(J, J, q);
    if (K == 16) {
      g2a qa;
      map_to_curve_sswu_tv(qa, f.c0.c0, f.c0.c1, f.c0.c2);
      f.c0.c0 = qa.x;
      f.c0.c1 = qa.y;
    }
    if (K == 17) {
      iso_map_g2(J, Q);
      Q.x = J.x;
    }
    if (K == 18) {
      g2j s;
      hash_to_g2_pair_sum(s, bytes, 32, DST_POP, 43, m);
      bytes[1] ^= (uint8_t)s.x.c0.v[0];
    }
    if (K == 19) {
      g2a sig;
      acc += (uint32_t)g2_decompress(sig, bytes, false);
      bytes[5] ^= (uint8_t)sig.x.c0.v[0];
    }
    if (K == 20) {
      g1a pk;
      acc += (uint32_t)g1_decompress(pk, bytes, true);
      bytes[5] ^= (uint8_t)pk.x.v[0];
    }
    if (K == 21) {
      g2a hm;
      hm.x = f.c0.c1;
      hm.y = f.c0.c2;
      acc += (uint32_t)lq4_verify(P, hm, Q, q);
      P.x.v[0] ^= acc;
    }
    if (K == 22) {
      uint32_t uni[64];
      expand_message_xmd_256(uni, bytes, 32, DST_POP, 43);
      bytes[2] ^= (uint8_t)uni[5];
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
  const uint32_t* cw = &c.z2.c0.v[0];
  for (int w = 0; w < 144; ++w) acc ^= fw[w];
  for (int w = 0; w < 96; ++w) acc ^= cw[w];
  acc ^= J.x.c0.v[0] ^ bytes[1] ^ bytes[2] ^ bytes[5] ^ P.x.v[0];
  out[blockIdx.x * 64 + lane] = acc;
  if (lane == 0) us100[blockIdx.x] = t1 - t0;
}

}  // namespace bls

int main(int argc, char** argv) {
  const int waves = argc > 1 ? atoi(argv[1]) : 8;
  constexpr int NOPS = 23;
  const char* names[NOPS] = {"fp_mul (one lane)", "fp2_mul (twins)", "fp2_sqr (twins)", "fp_pow (p+1)/4 (one lane)",
                             "fp2_inv", "fp12_inv", "cyc_sqr_compressed_quad", "fp12q_mul", "fp12q_exp_xabs",
                             "final_exponentiation_quad", "fp12h_sqr_split", "miller_dbl_step_split",
                             "fp12h_mul_line_split", "miller_loop_split", "g2_dbl_quad", "g2_clear_cofactor_quad",
                             "map_to_curve_sswu_tv", "iso_map_g2", "hash_to_g2_pair_sum", "g2_decompress",
                             "g1_decompress (+subgroup)", "lq4_verify (octet check)", "expand_message_xmd_256"};
  const int iters[NOPS] = {200, 100, 100, 2, 10, 4, 40, 20, 2, 1, 20, 20, 20, 1, 40, 1, 2, 10, 1, 2, 2, 1, 10};
  uint32_t *d_in, *d_out;
  uint64_t* d_t;
  static uint32_t h_in[4096];
  for (int i = 0; i < 4096; ++i) h_in[i] = 0x9E3779B9u * (i + 7);
  if (hipMalloc(&d_in, sizeof(h_in)) || hipMalloc(&d_out, 1024 * 64 * 4) || hipMalloc(&d_t, 1024 * 8)) return 1;
  (void)hipMemcpy(d_in, h_in, sizeof(h_in), hipMemcpyHostToDevice);
  static uint64_t h_t[1024];
  printf("waves %d (one octet each); microseconds per op (s_memrealtime, median over waves)\n", waves);
  for (int k = 0; k < NOPS; ++k) {
    for (int rep = 0; rep < 2; ++rep) {
      switch (k) {
#define L(K) \
  case K: hipLaunchKernelGGL(bls_fp2p::k_part<K>, dim3(waves), dim3(64), 0, 0, d_in, d_out, d_t, iters[K]); break;
        L(0) L(1) L(2) L(3) L(4) L(5) L(6) L(7) L(8) L(9) L(10) L(11) L(12) L(13) L(14) L(15) L(16) L(17) L(18) L(19)
        L(20) L(21) L(22)
#undef L
      }
      if (hipDeviceSynchronize() != hipSuccess) return 2;
    }
    (void)hipMemcpy(h_t, d_t, waves * 8, hipMemcpyDeviceToHost);
    std::sort(h_t, h_t + waves);
    const double us = (double)h_t[waves / 2] / iters[k] / 100.0;
    const double us_min = (double)h_t[0] / iters[k] / 100.0;
    printf("%-30s %10.2f us/op  (min %.2f)\n", names[k], us, us_min);
  }
  return 0;
}
