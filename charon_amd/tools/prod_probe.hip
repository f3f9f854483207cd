// Microbenchmark: Fp Montgomery product routines on gfx950 (profiles/r02_prod_probe.txt).
//   * PROBE_OLD  : round-1 radix-2^32 routine (mad + addc carry capture, canonical output)
//   * PROBE_NEW1 : radix-2^29, one accumulator chain, lazy [0, 2p) output
//   * PROBE_NEW2 : radix-2^29, two accumulator chains (the shipped routine)
//   * PROBE_SQR2 : radix-2^29 squaring variant
// Each lane runs a dependent chain of `iters` products a <- a*b (b restored every step), at 1, 2 and 4
// waves per SIMD; cycles per product per wave come from s_memtime around the loop.  A few lanes'
// results are written out and checked on the host (tools/run_prod_probe.py) against big integers.
// Also: issue/latency of single instructions used by the routines.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include "probe_bodies.h"

typedef uint32_t u32x12 __attribute__((ext_vector_type(12)));

#define CLOB_OLD "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34", "v35", "v36", \
  "v37", "v38", "v39", "vcc", "s16", "s17", "s18", "s19", "s20", "s21", "s22", "s23", "s24", "s25", "s26", "s27", "s28"
#define CLOB_NEW CLOB_OLD, "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "s40", "s41", "s42", \
  "s43", "s44", "s45", "s46", "s47"

template <int V>
__global__ void __launch_bounds__(64) k_prod(const uint32_t* in, uint32_t* out, uint64_t* cyc, int iters) {
  const int lane = blockIdx.x * 64 + threadIdx.x;
  u32x12 a, b, b0;
  for (int i = 0; i < 12; ++i) {
    a[i] = in[(lane % 64) * 24 + i];
    b0[i] = in[(lane % 64) * 24 + 12 + i];
  }
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    b = b0;
    if (V == 0) asm volatile(PROBE_V0 : "+{v[0:11]}"(a), "+{v[12:23]}"(b) : : CLOB_OLD);
    if (V == 1) asm volatile(PROBE_V1 : "+{v[0:11]}"(a), "+{v[12:23]}"(b) : : CLOB_NEW);
    if (V == 2) asm volatile(PROBE_V2 : "+{v[0:11]}"(a), "+{v[12:23]}"(b) : : CLOB_NEW);
    if (V == 3) asm volatile(PROBE_V3 : "+{v[0:11]}"(a), "+{v[12:23]}"(b) : : CLOB_NEW);
    if (V == 4) asm volatile(PROBE_V4 : "+{v[0:11]}"(a), "+{v[12:23]}"(b) : : CLOB_NEW);
    if (V == 5) asm volatile(PROBE_V5 : "+{v[0:11]}"(a), "+{v[12:23]}"(b) : : CLOB_NEW);
    if (V == 6) asm volatile(PROBE_V6 : "+{v[0:11]}"(a), "+{v[12:23]}"(b) : : CLOB_NEW);
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 12; ++i) out[lane * 12 + i] = a[i];
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// Single-instruction probes: 8 independent streams x 32 unrolled per iteration, or 1 dependent stream.
template <int K>
__global__ void __launch_bounds__(64) k_ins(uint32_t* out, uint64_t* cyc, int iters) {
  uint32_t x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
  uint64_t y0 = x0, y1 = x1, y2 = x2, y3 = x3;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#define R8(S) S S S S S S S S
    if (K == 0)  // dependent mad chain, rotating carry-out SGPR pairs
      asm volatile(R8("v_mad_u64_u32 %0, s[40:41], %1, %2, %0\n\tv_mad_u64_u32 %0, s[42:43], %1, %2, %0\n\tv_mad_u64_u32 %0, s[44:45], %1, %2, %0\n\tv_mad_u64_u32 %0, s[46:47], %1, %2, %0\n\t")
                   : "+v"(y0) : "v"(x1), "v"(x2) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47");
    if (K == 1)  // 2 independent mad chains
      asm volatile(R8("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_mad_u64_u32 %1, vcc, %2, %3, %1\n\tv_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_mad_u64_u32 %1, vcc, %2, %3, %1\n\t")
                   : "+v"(y0), "+v"(y1) : "v"(x1), "v"(x2) : "vcc");
    if (K == 2)  // 4 independent mad chains, rotating carry-out SGPR pairs
      asm volatile(R8("v_mad_u64_u32 %0, s[40:41], %4, %5, %0\n\tv_mad_u64_u32 %1, s[42:43], %4, %5, %1\n\tv_mad_u64_u32 %2, s[44:45], %4, %5, %2\n\tv_mad_u64_u32 %3, s[46:47], %4, %5, %3\n\t")
                   : "+v"(y0), "+v"(y1), "+v"(y2), "+v"(y3) : "v"(x1), "v"(x2) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47");
    if (K == 3)  // mad + addc(vcc) pairs (round-1 pattern), one chain
      asm volatile(R8("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\t")
                   : "+v"(y0), "+v"(x0) : "v"(x1), "v"(x2) : "vcc");
    if (K == 4)  // independent 64-bit shifts
      asm volatile(R8("v_lshrrev_b64 %0, 29, %0\n\tv_lshrrev_b64 %1, 29, %1\n\tv_lshrrev_b64 %2, 29, %2\n\tv_lshrrev_b64 %3, 29, %3\n\t")
                   : "+v"(y0), "+v"(y1), "+v"(y2), "+v"(y3));
    if (K == 5)  // independent v_lshl_add_u64
      asm volatile(R8("v_lshl_add_u64 %0, %1, 0, %0\n\tv_lshl_add_u64 %1, %2, 0, %1\n\tv_lshl_add_u64 %2, %3, 0, %2\n\tv_lshl_add_u64 %3, %0, 0, %3\n\t")
                   : "+v"(y0), "+v"(y1), "+v"(y2), "+v"(y3));
    if (K == 6)  // independent v_mul_lo_u32
      asm volatile(R8("v_mul_lo_u32 %0, %0, %4\n\tv_mul_lo_u32 %1, %1, %4\n\tv_mul_lo_u32 %2, %2, %4\n\tv_mul_lo_u32 %3, %3, %4\n\t")
                   : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : "v"(x7));
    if (K == 7)  // independent v_alignbit_b32 / v_and_b32
      asm volatile(R8("v_alignbit_b32 %0, %0, %4, 5\n\tv_and_b32_e32 %1, 0x1fffffff, %1\n\tv_alignbit_b32 %2, %2, %4, 7\n\tv_and_b32_e32 %3, 0x1fffffff, %3\n\t")
                   : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : "v"(x7));
    if (K == 8)  // independent v_addc_co_u32 with vcc (carry chains of fp_add)
      asm volatile(R8("v_add_co_u32_e32 %0, vcc, %0, %4\n\tv_addc_co_u32_e32 %1, vcc, %1, %4, vcc\n\tv_addc_co_u32_e32 %2, vcc, %2, %4, vcc\n\tv_addc_co_u32_e32 %3, vcc, %3, %4, vcc\n\t")
                   : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : "v"(x7) : "vcc");
    if (K == 9)  // 8 independent plain v_add_u32
      asm volatile(R8("v_add_u32_e32 %0, %0, %4\n\tv_add_u32_e32 %1, %1, %4\n\tv_add_u32_e32 %2, %2, %4\n\tv_add_u32_e32 %3, %3, %4\n\t")
                   : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : "v"(x7));
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 64 + threadIdx.x] = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7 ^ (uint32_t)(y0 ^ y1 ^ y2 ^ y3);
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

static double median_cycles(uint64_t* h, int n) {
  // median of per-wave cycle counts (simple nth selection)
  for (int i = 1; i < n; ++i)
    for (int j = i; j > 0 && h[j - 1] > h[j]; --j) {
      uint64_t t = h[j];
      h[j] = h[j - 1];
      h[j - 1] = t;
    }
  return (double)h[n / 2];
}

int main(int argc, char** argv) {
  const int iters = 200;
  const int maxw = 4;
  const int blocks_max = 1024 * maxw;
  uint32_t *d_in, *d_out;
  uint64_t* d_cyc;
  uint32_t h_in[64 * 24];
  for (int i = 0; i < 64 * 24; ++i) h_in[i] = (uint32_t)(0x9E3779B9u * (i + 1)) ^ (uint32_t)(i * 7919);
  for (int l = 0; l < 64; ++l) {  // keep operands < 2^383 (weakly reduced range of the new routines)
    h_in[l * 24 + 11] &= 0x0fffffff;
    h_in[l * 24 + 23] &= 0x0fffffff;
  }
  if (hipMalloc(&d_in, sizeof(h_in)) || hipMalloc(&d_out, (size_t)blocks_max * 64 * 48) ||
      hipMalloc(&d_cyc, (size_t)blocks_max * 8))
    return 1;
  (void)hipMemcpy(d_in, h_in, sizeof(h_in), hipMemcpyHostToDevice);
  uint64_t* h_cyc = (uint64_t*)malloc((size_t)blocks_max * 8);
  uint32_t* h_out = (uint32_t*)malloc((size_t)blocks_max * 64 * 48);
  const char* names[PROBE_NVAR] = PROBE_NAMES;
  FILE* fo = fopen(argc > 1 ? argv[1] : "gpurun_out/prod_probe_out.txt", "w");
  for (int v = 0; v < PROBE_NVAR; ++v) {
    for (int w = 1; w <= maxw; w *= 2) {
      const int blocks = 1024 * w;
      for (int rep = 0; rep < 2; ++rep) {
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        (void)hipEventRecord(e0);
        switch (v) {
#define LV(K) case K: hipLaunchKernelGGL(k_prod<K>, dim3(blocks), dim3(64), 0, 0, d_in, d_out, d_cyc, iters); break;
          LV(0) LV(1) LV(2) LV(3) LV(4) LV(5) LV(6)
        }
        (void)hipEventRecord(e1);
        if (hipEventSynchronize(e1) != hipSuccess) return 2;
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        (void)hipMemcpy(h_cyc, d_cyc, (size_t)blocks * 8, hipMemcpyDeviceToHost);
        const double med = median_cycles(h_cyc, blocks);
        if (rep == 1) {
          const double gps = (double)blocks * 64 * iters / (ms * 1e-3) / 1e9;
          printf("%-44s waves/SIMD %d: %8.1f cyc/product/wave (s_memtime median), %7.3f ms, %6.1f G products/s\n",
                 names[v], w, med / iters, ms, gps);
        }
      }
    }
    (void)hipMemcpy(h_out, d_out, 64 * 48, hipMemcpyDeviceToHost);
    fprintf(fo, "variant %d iters %d\n", v, iters);
    for (int l = 0; l < 4; ++l) {
      for (int i = 0; i < 12; ++i) fprintf(fo, "%08x ", h_out[l * 12 + i]);
      fprintf(fo, "\n");
    }
  }
  fclose(fo);
  const char* inames[10] = {"mad dep chain, rotating sdst", "mad 2 chains (vcc)", "mad 4 chains, rotating sdst", "mad+addc(vcc) pairs",
                            "v_lshrrev_b64 x4 indep", "v_lshl_add_u64 x4 (dep ring)", "v_mul_lo_u32 x4 indep",
                            "alignbit/and x4 indep", "add_co/addc_co carry chain", "v_add_u32 x4 indep"};
  for (int k = 0; k < 10; ++k) {
    for (int w = 1; w <= 4; w *= 4) {
      const int blocks = 1024 * w;
      for (int rep = 0; rep < 2; ++rep) {
        switch (k) {
#define L(K) case K: hipLaunchKernelGGL(k_ins<K>, dim3(blocks), dim3(64), 0, 0, d_out, d_cyc, 100); break;
          L(0) L(1) L(2) L(3) L(4) L(5) L(6) L(7) L(8) L(9)
        }
        if (hipDeviceSynchronize() != hipSuccess) return 3;
      }
      (void)hipMemcpy(h_cyc, d_cyc, (size_t)blocks * 8, hipMemcpyDeviceToHost);
      const double med = median_cycles(h_cyc, blocks);
      printf("%-30s waves/SIMD %d: %6.2f cycles per instruction per wave\n", inames[k], w, med / (100.0 * 32));
    }
  }
  return 0;
}
