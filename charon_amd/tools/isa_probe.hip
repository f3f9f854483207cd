// Microbenchmark (round 6): issue cost at one wave per SIMD of the instructions the product routines' remaining
// overhead is made of (tools/gen_fp_asm.py _comba and the final subtraction), cycles per wave64 instruction.
// Hard-coded registers, 128 instructions per loop iteration; s_memtime around the loop.
//   hipcc --offload-arch=gfx950 -O3 -o isa_probe isa_probe.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#define X4(S) S S S S
#define X32(S) X4(X4(S)) X4(X4(S))
#define CL "v0","v1","v2","v3","v4","v5","v6","v7","v8","v9","v10","v11","v12","v13","v14","v15","v16","v17", \
  "v18","v19","v20","v21","v22","v23","s40","s41","s42","s43","s44","s45","s46","s47","vcc"
template <int K>
__global__ void __launch_bounds__(64) k(uint64_t* cyc, int iters) {
  asm volatile("v_mov_b32 v0, 3\n\tv_mov_b32 v1, 5\n\tv_mov_b32 v4, 7\n\tv_mov_b32 v5, 9\n\tv_mov_b32 v8, 11\n\t"
               "v_mov_b32 v9, 13\n\tv_mov_b32 v12, 17\n\tv_mov_b32 v13, 19\n\tv_mov_b32 v16, 23\n\tv_mov_b32 v20, 29\n\t"
               "s_mov_b32 s44, 31\n\ts_mov_b32 s45, 37\n\ts_mov_b32 s46, 41\n\ts_mov_b32 s47, 43" ::: CL);
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    if (K == 0)  // v_mul_lo_u32, 4 independent destinations
      asm volatile(X32("v_mul_lo_u32 v2, v0, s44\n\tv_mul_lo_u32 v3, v1, s44\n\tv_mul_lo_u32 v6, v4, s44\n\t"
                       "v_mul_lo_u32 v7, v5, s44\n\t") ::: CL);
    if (K == 1)  // v_mul_lo_u32, one dependent chain
      asm volatile(X32("v_mul_lo_u32 v2, v2, s44\n\tv_mul_lo_u32 v2, v2, s44\n\tv_mul_lo_u32 v2, v2, s44\n\t"
                       "v_mul_lo_u32 v2, v2, s44\n\t") ::: CL);
    if (K == 2)  // v_mad_u64_u32 into a pair as a 32-bit product (lo word), independent
      asm volatile(X32("v_mad_u64_u32 v[2:3], s[40:41], v0, s44, 0\n\tv_mad_u64_u32 v[6:7], s[40:41], v1, s44, 0\n\t"
                       "v_mad_u64_u32 v[10:11], s[40:41], v4, s44, 0\n\tv_mad_u64_u32 v[14:15], s[40:41], v5, s44, 0\n\t") ::: CL);
    if (K == 3)  // v_mov_b64 from an SGPR pair
      asm volatile(X32("v_mov_b64 v[2:3], s[44:45]\n\tv_mov_b64 v[6:7], s[46:47]\n\tv_mov_b64 v[10:11], s[44:45]\n\t"
                       "v_mov_b64 v[14:15], s[46:47]\n\t") ::: CL);
    if (K == 4)  // v_mov_b32 from an SGPR
      asm volatile(X32("v_mov_b32 v2, s44\n\tv_mov_b32 v3, s45\n\tv_mov_b32 v6, s46\n\tv_mov_b32 v7, s47\n\t") ::: CL);
    if (K == 5)  // the product's mad + addc pairs on one accumulator
      asm volatile(X32("v_mad_u64_u32 v[2:3], vcc, v0, v1, v[2:3]\n\tv_addc_co_u32_e32 v23, vcc, 0, v23, vcc\n\t"
                       "v_mad_u64_u32 v[2:3], vcc, v4, v5, v[2:3]\n\tv_addc_co_u32_e32 v23, vcc, 0, v23, vcc\n\t") ::: CL);
    if (K == 6)  // carry-free mads back to back on one accumulator (the elided column heads)
      asm volatile(X32("v_mad_u64_u32 v[2:3], vcc, v0, v1, v[2:3]\n\tv_mad_u64_u32 v[2:3], vcc, v4, v5, v[2:3]\n\t"
                       "v_mad_u64_u32 v[2:3], vcc, v8, v9, v[2:3]\n\tv_mad_u64_u32 v[2:3], vcc, v12, v13, v[2:3]\n\t") ::: CL);
    if (K == 7)  // v_bfi_b32
      asm volatile(X32("v_bfi_b32 v2, v0, v1, v2\n\tv_bfi_b32 v3, v0, v4, v3\n\tv_bfi_b32 v6, v0, v5, v6\n\t"
                       "v_bfi_b32 v7, v0, v8, v7\n\t") ::: CL);
    if (K == 8)  // v_sub_co / v_subb_co chain (the final subtraction)
      asm volatile(X32("v_sub_co_u32_e32 v2, vcc, v0, v1\n\tv_subb_co_u32_e32 v3, vcc, v4, v5, vcc\n\t"
                       "v_subb_co_u32_e32 v6, vcc, v8, v9, vcc\n\tv_subb_co_u32_e32 v7, vcc, v12, v13, vcc\n\t") ::: CL);
    if (K == 9)  // v_pk_mov_b32 from one SGPR pair (two limbs per instruction)
      asm volatile(X32("v_pk_mov_b32 v[2:3], s[44:45], s[44:45] op_sel:[0,1]\n\t"
                       "v_pk_mov_b32 v[6:7], s[46:47], s[46:47] op_sel:[0,1]\n\t"
                       "v_pk_mov_b32 v[10:11], s[44:45], s[44:45] op_sel:[0,1]\n\t"
                       "v_pk_mov_b32 v[14:15], s[46:47], s[46:47] op_sel:[0,1]\n\t") ::: CL);
    if (K == 10)  // the column shift: mad, addc, then v_mov of the high word (the carried value)
      asm volatile(X32("v_mad_u64_u32 v[2:3], vcc, v0, v1, v[4:5]\n\tv_addc_co_u32_e64 v5, vcc, 0, 0, vcc\n\t"
                       "v_mov_b32 v4, v3\n\tv_mad_u64_u32 v[2:3], vcc, v8, v9, v[4:5]\n\t") ::: CL);
    if (K == 11)  // v_mov_b32 VGPR -> VGPR (baseline)
      asm volatile(X32("v_mov_b32 v2, v0\n\tv_mov_b32 v3, v1\n\tv_mov_b32 v6, v4\n\tv_mov_b32 v7, v5\n\t") ::: CL);
    if (K == 12)  // SALU only
      asm volatile(X32("s_mov_b32 s40, 0x1a0111ea\n\ts_mov_b32 s41, 0x397fe69a\n\ts_mov_b32 s42, 0x4b1ba7b6\n\t"
                       "s_mov_b32 s43, 0x434bacd7\n\t") ::: CL);
    if (K == 13)  // VALU and SALU alternating (64 + 64 per iteration): does a scalar move take a slot of its own?
      asm volatile(X32("v_add_u32_e32 v2, v0, v2\n\ts_mov_b32 s40, 0x1a0111ea\n\tv_add_u32_e32 v3, v1, v3\n\t"
                       "s_mov_b32 s41, 0x397fe69a\n\t") ::: CL);
    if (K == 14)  // mads with s_mov between (the routine head: p into SGPRs next to the first column)
      asm volatile(X32("v_mad_u64_u32 v[2:3], vcc, v0, v1, v[2:3]\n\ts_mov_b32 s40, 0x1a0111ea\n\t"
                       "v_mad_u64_u32 v[6:7], vcc, v4, v5, v[6:7]\n\ts_mov_b32 s41, 0x397fe69a\n\t") ::: CL);
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
int main() {
  const char* names[15] = {"v_mul_lo_u32 4 dests", "v_mul_lo_u32 dependent", "v_mad_u64_u32 as mul (pair)",
                           "v_mov_b64 from SGPR pair", "v_mov_b32 from SGPR", "mad + addc (product column)",
                           "mad back to back (carry-free)", "v_bfi_b32", "v_sub_co/v_subb_co chain",
                           "v_pk_mov_b32 from SGPR pair", "mad,addc,mov shift", "v_mov_b32 v->v", "s_mov_b32 (SALU only)",
                           "v_add / s_mov alternating", "v_mad / s_mov alternating"};
  uint64_t* d;
  if (hipMalloc(&d, 4096 * 8) != hipSuccess) return 2;
  static uint64_t h[4096];
  for (int kk = 0; kk < 15; ++kk)
    for (int w = 1; w <= 2; w *= 2) {
      const int blocks = 1024 * w;
      for (int rep = 0; rep < 2; ++rep) {
        switch (kk) {
#define L(K) case K: hipLaunchKernelGGL(k<K>, dim3(blocks), dim3(64), 0, 0, d, 50); break;
          L(0) L(1) L(2) L(3) L(4) L(5) L(6) L(7) L(8) L(9) L(10) L(11) L(12) L(13) L(14)
        }
        if (hipDeviceSynchronize() != hipSuccess) return 3;
      }
      if (hipMemcpy(h, d, blocks * 8, hipMemcpyDeviceToHost) != hipSuccess) return 4;
      uint64_t lo = h[0];
      double sum = 0;
      for (int i = 0; i < blocks; ++i) { sum += h[i]; if (h[i] < lo) lo = h[i]; }
      printf("%-32s waves/SIMD %d: %5.2f cyc/instr/wave (mean), %5.2f (min)\n", names[kk], w, sum / blocks / (50.0 * 128),
             lo / (50.0 * 128));
    }
  return 0;
}
