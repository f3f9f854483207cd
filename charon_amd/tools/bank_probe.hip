// Microbenchmark: VGPR bank placement of v_mad_u64_u32 operands on gfx950 (profiles/r02_prod_probe.txt).
// 4 independent accumulator chains, 128 mads per loop iteration, hard-coded registers.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#define X4(S) S S S S
#define X32(S) X4(X4(S)) X4(X4(S))
#define CL "v0","v1","v2","v3","v4","v5","v6","v7","v8","v9","v10","v11","v12","v13","v14","v15","v16","v17", \
  "v18","v19","v20","v21","v22","v23","s40","s41","s42","s43","s44","s45","s46","s47"
template <int K>
__global__ void __launch_bounds__(64) k(uint64_t* cyc, int iters) {
  asm volatile("v_mov_b32 v0, 3\n\tv_mov_b32 v1, 5\n\tv_mov_b32 v4, 7\n\tv_mov_b32 v5, 9\n\tv_mov_b32 v8, 11\n\t"
               "v_mov_b32 v9, 13\n\tv_mov_b32 v12, 17\n\tv_mov_b32 v13, 19\n\tv_mov_b32 v16, 23\n\tv_mov_b32 v20, 29\n\t"
               "s_mov_b32 s44, 31" ::: CL);
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    if (K == 0)  // banks: a 0, b 1, c 2/3 -- distinct
      asm volatile(X32("v_mad_u64_u32 v[2:3], s[40:41], v0, v1, v[2:3]\n\tv_mad_u64_u32 v[6:7], s[42:43], v4, v5, v[6:7]\n\t"
                       "v_mad_u64_u32 v[10:11], s[40:41], v8, v9, v[10:11]\n\tv_mad_u64_u32 v[14:15], s[42:43], v12, v13, v[14:15]\n\t") ::: CL);
    if (K == 1)  // a, b same bank (0), c 2/3
      asm volatile(X32("v_mad_u64_u32 v[2:3], s[40:41], v0, v4, v[2:3]\n\tv_mad_u64_u32 v[6:7], s[42:43], v8, v12, v[6:7]\n\t"
                       "v_mad_u64_u32 v[10:11], s[40:41], v16, v20, v[10:11]\n\tv_mad_u64_u32 v[14:15], s[42:43], v0, v8, v[14:15]\n\t") ::: CL);
    if (K == 2)  // a bank 0, b bank 1, c 0/1 (a and c.lo share bank 0, b and c.hi bank 1)
      asm volatile(X32("v_mad_u64_u32 v[16:17], s[40:41], v0, v1, v[16:17]\n\tv_mad_u64_u32 v[20:21], s[42:43], v4, v5, v[20:21]\n\t"
                       "v_mad_u64_u32 v[16:17], s[40:41], v8, v9, v[16:17]\n\tv_mad_u64_u32 v[20:21], s[42:43], v12, v13, v[20:21]\n\t") ::: CL);
    if (K == 3)  // a, b, c.lo all bank 0
      asm volatile(X32("v_mad_u64_u32 v[16:17], s[40:41], v0, v4, v[16:17]\n\tv_mad_u64_u32 v[20:21], s[42:43], v8, v12, v[20:21]\n\t"
                       "v_mad_u64_u32 v[16:17], s[40:41], v0, v8, v[16:17]\n\tv_mad_u64_u32 v[20:21], s[42:43], v4, v12, v[20:21]\n\t") ::: CL);
    if (K == 4)  // SGPR b, a bank 0, c 2/3
      asm volatile(X32("v_mad_u64_u32 v[2:3], s[40:41], v0, s44, v[2:3]\n\tv_mad_u64_u32 v[6:7], s[42:43], v4, s44, v[6:7]\n\t"
                       "v_mad_u64_u32 v[10:11], s[40:41], v8, s44, v[10:11]\n\tv_mad_u64_u32 v[14:15], s[42:43], v12, s44, v[14:15]\n\t") ::: CL);
    if (K == 5)  // 2 chains only, distinct banks (a 0, b 1, c 2/3)
      asm volatile(X32("v_mad_u64_u32 v[2:3], s[40:41], v0, v1, v[2:3]\n\tv_mad_u64_u32 v[6:7], s[42:43], v4, v5, v[6:7]\n\t"
                       "v_mad_u64_u32 v[2:3], s[40:41], v8, v9, v[2:3]\n\tv_mad_u64_u32 v[6:7], s[42:43], v12, v13, v[6:7]\n\t") ::: CL);
    if (K == 6)  // 1 chain, distinct banks
      asm volatile(X32("v_mad_u64_u32 v[2:3], s[40:41], v0, v1, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[42:43], v4, v5, v[2:3]\n\t"
                       "v_mad_u64_u32 v[2:3], s[40:41], v8, v9, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[42:43], v12, v13, v[2:3]\n\t") ::: CL);
    if (K == 7)  // v_add_u32 x 128 (baseline for loop overhead), independent
      asm volatile(X32("v_add_u32_e32 v2, v0, v2\n\tv_add_u32_e32 v3, v1, v3\n\tv_add_u32_e32 v6, v4, v6\n\tv_add_u32_e32 v7, v5, v7\n\t") ::: CL);
    if (K == 8)  // v_addc carry chain with vcc (add-with-carry)
      asm volatile(X32("v_add_co_u32_e32 v2, vcc, v0, v2\n\tv_addc_co_u32_e32 v3, vcc, v1, v3, vcc\n\tv_addc_co_u32_e32 v6, vcc, v4, v6, vcc\n\tv_addc_co_u32_e32 v7, vcc, v5, v7, vcc\n\t") ::: CL, "vcc");
    if (K == 9)  // v_cndmask with vcc
      asm volatile(X32("v_cndmask_b32_e32 v2, v0, v2, vcc\n\tv_cndmask_b32_e32 v3, v1, v3, vcc\n\tv_cndmask_b32_e32 v6, v4, v6, vcc\n\tv_cndmask_b32_e32 v7, v5, v7, vcc\n\t") ::: CL, "vcc");
    if (K == 10)  // v_mov_b32
      asm volatile(X32("v_mov_b32 v2, v0\n\tv_mov_b32 v3, v1\n\tv_mov_b32 v6, v4\n\tv_mov_b32 v7, v5\n\t") ::: CL);
    if (K == 11)  // v_lshrrev_b64 independent
      asm volatile(X32("v_lshrrev_b64 v[2:3], 29, v[2:3]\n\tv_lshrrev_b64 v[6:7], 29, v[6:7]\n\tv_lshrrev_b64 v[10:11], 29, v[10:11]\n\tv_lshrrev_b64 v[14:15], 29, v[14:15]\n\t") ::: CL);
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
int main() {
  const char* names[12] = {"mad 4ch banks a0 b1 c23", "mad 4ch a,b same bank", "mad 2ch a&c.lo bank0, b&c.hi bank1",
                           "mad 2ch a,b,c.lo bank0", "mad 4ch SGPR b", "mad 2ch distinct banks", "mad 1ch distinct banks",
                           "v_add_u32", "add_co/addc_co(vcc)", "v_cndmask(vcc)", "v_mov_b32", "v_lshrrev_b64 4ch"};
  uint64_t* d;
  (void)hipMalloc(&d, 4096 * 8);
  uint64_t h[4096];
  for (int kk = 0; kk < 12; ++kk)
    for (int w = 1; w <= 4; w *= 2) {
      const int blocks = 1024 * w;
      for (int rep = 0; rep < 2; ++rep) {
        switch (kk) {
#define L(K) case K: hipLaunchKernelGGL(k<K>, dim3(blocks), dim3(64), 0, 0, d, 50); break;
          L(0) L(1) L(2) L(3) L(4) L(5) L(6) L(7) L(8) L(9) L(10) L(11)
        }
        if (hipDeviceSynchronize() != hipSuccess) return 2;
      }
      (void)hipMemcpy(h, d, blocks * 8, hipMemcpyDeviceToHost);
      uint64_t lo = h[0];
      double sum = 0;
      for (int i = 0; i < blocks; ++i) { sum += h[i]; if (h[i] < lo) lo = h[i]; }
      printf("%-36s waves/SIMD %d: %5.2f cyc/instr/wave (mean), %5.2f (min)\n", names[kk], w, sum / blocks / (50.0 * 128),
             lo / (50.0 * 128));
    }
  return 0;
}
