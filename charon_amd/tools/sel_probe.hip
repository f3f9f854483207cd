// Microbenchmark: lane-select forms on gfx950 (profiles/r02_prod_probe.txt): v_cndmask with VCC / SGPR-pair
// masks vs v_bfi_b32 with a VGPR mask, and whole 12-limb modular-add sequences.  One wave per SIMD.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#define X4(S) S S S S
#define X32(S) X4(X4(S)) X4(X4(S))
#define CL "v0","v1","v2","v3","v4","v5","v6","v7","v8","v9","v10","v11","v12","v13","v14","v15","v16","v17", \
  "v18","v19","v20","v21","v22","v23","v24","v25","v26","v27","v28","v29","v30","v31","v32","v33","v34","v35", \
  "v36","v37","v38","v39","v40","v41","v42","v43","v44","v45","v46","v47","v48","v49","s40","s41","s42","s43","vcc"
// 12-limb add a(v0..11) + b(v12..23) -> s(v24..35), minus p(v36..47) -> d(v12..23), select by borrow
#define ADDCH "v_add_co_u32_e32 v24, vcc, v0, v12\n\tv_addc_co_u32_e32 v25, vcc, v1, v13, vcc\n\tv_addc_co_u32_e32 v26, vcc, v2, v14, vcc\n\tv_addc_co_u32_e32 v27, vcc, v3, v15, vcc\n\tv_addc_co_u32_e32 v28, vcc, v4, v16, vcc\n\tv_addc_co_u32_e32 v29, vcc, v5, v17, vcc\n\tv_addc_co_u32_e32 v30, vcc, v6, v18, vcc\n\tv_addc_co_u32_e32 v31, vcc, v7, v19, vcc\n\tv_addc_co_u32_e32 v32, vcc, v8, v20, vcc\n\tv_addc_co_u32_e32 v33, vcc, v9, v21, vcc\n\tv_addc_co_u32_e32 v34, vcc, v10, v22, vcc\n\tv_addc_co_u32_e32 v35, vcc, v11, v23, vcc\n\t"
#define SUBCH "v_sub_co_u32_e32 v12, vcc, v24, v36\n\tv_subb_co_u32_e32 v13, vcc, v25, v37, vcc\n\tv_subb_co_u32_e32 v14, vcc, v26, v38, vcc\n\tv_subb_co_u32_e32 v15, vcc, v27, v39, vcc\n\tv_subb_co_u32_e32 v16, vcc, v28, v40, vcc\n\tv_subb_co_u32_e32 v17, vcc, v29, v41, vcc\n\tv_subb_co_u32_e32 v18, vcc, v30, v42, vcc\n\tv_subb_co_u32_e32 v19, vcc, v31, v43, vcc\n\tv_subb_co_u32_e32 v20, vcc, v32, v44, vcc\n\tv_subb_co_u32_e32 v21, vcc, v33, v45, vcc\n\tv_subb_co_u32_e32 v22, vcc, v34, v46, vcc\n\tv_subb_co_u32_e32 v23, vcc, v35, v47, vcc\n\t"
#define SEL_CND "v_cndmask_b32_e32 v0, v12, v24, vcc\n\tv_cndmask_b32_e32 v1, v13, v25, vcc\n\tv_cndmask_b32_e32 v2, v14, v26, vcc\n\tv_cndmask_b32_e32 v3, v15, v27, vcc\n\tv_cndmask_b32_e32 v4, v16, v28, vcc\n\tv_cndmask_b32_e32 v5, v17, v29, vcc\n\tv_cndmask_b32_e32 v6, v18, v30, vcc\n\tv_cndmask_b32_e32 v7, v19, v31, vcc\n\tv_cndmask_b32_e32 v8, v20, v32, vcc\n\tv_cndmask_b32_e32 v9, v21, v33, vcc\n\tv_cndmask_b32_e32 v10, v22, v34, vcc\n\tv_cndmask_b32_e32 v11, v23, v35, vcc\n\t"
#define SEL_BFI "v_subb_co_u32_e64 v48, s[42:43], 0, 0, vcc\n\tv_bfi_b32 v0, v48, v24, v12\n\tv_bfi_b32 v1, v48, v25, v13\n\tv_bfi_b32 v2, v48, v26, v14\n\tv_bfi_b32 v3, v48, v27, v15\n\tv_bfi_b32 v4, v48, v28, v16\n\tv_bfi_b32 v5, v48, v29, v17\n\tv_bfi_b32 v6, v48, v30, v18\n\tv_bfi_b32 v7, v48, v31, v19\n\tv_bfi_b32 v8, v48, v32, v20\n\tv_bfi_b32 v9, v48, v33, v21\n\tv_bfi_b32 v10, v48, v34, v22\n\tv_bfi_b32 v11, v48, v35, v23\n\t"
template <int K>
__global__ void __launch_bounds__(64) k(uint64_t* cyc, int iters) {
  asm volatile("v_mov_b32 v48, 0\n\tv_mov_b32 v49, -1\n\ts_mov_b64 s[40:41], 0\n\ts_mov_b64 vcc, 0" ::: CL);
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    if (K == 0) asm volatile(X32("v_cndmask_b32_e32 v2, v0, v2, vcc\n\tv_cndmask_b32_e32 v3, v1, v3, vcc\n\tv_cndmask_b32_e32 v6, v4, v6, vcc\n\tv_cndmask_b32_e32 v7, v5, v7, vcc\n\t") ::: CL);
    if (K == 1) asm volatile(X32("v_cndmask_b32_e64 v2, v0, v2, s[40:41]\n\tv_cndmask_b32_e64 v3, v1, v3, s[40:41]\n\tv_cndmask_b32_e64 v6, v4, v6, s[40:41]\n\tv_cndmask_b32_e64 v7, v5, v7, s[40:41]\n\t") ::: CL);
    if (K == 2) asm volatile(X32("v_bfi_b32 v2, v48, v0, v2\n\tv_bfi_b32 v3, v48, v1, v3\n\tv_bfi_b32 v6, v48, v4, v6\n\tv_bfi_b32 v7, v48, v5, v7\n\t") ::: CL);
    if (K == 3) asm volatile(X32("v_cndmask_b32_e64 v2, v0, v2, vcc\n\tv_cndmask_b32_e64 v3, v1, v3, vcc\n\tv_cndmask_b32_e64 v6, v4, v6, vcc\n\tv_cndmask_b32_e64 v7, v5, v7, vcc\n\t") ::: CL);
    if (K == 4) asm volatile(X4(ADDCH SUBCH SEL_CND) ::: CL);   // 36 instructions x 4
    if (K == 5) asm volatile(X4(ADDCH SUBCH SEL_BFI) ::: CL);   // 37 instructions x 4
    if (K == 6) asm volatile(X4(ADDCH SUBCH) X4("v_mov_b32 v0, v12\n\tv_mov_b32 v1, v13\n\tv_mov_b32 v2, v14\n\t") ::: CL);
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
int main() {
  const char* names[7] = {"v_cndmask_e32 vcc x128", "v_cndmask_e64 s[40:41] x128", "v_bfi_b32 vgpr-mask x128",
                          "v_cndmask_e64 vcc x128", "fp_add 12: addc+subb+cndmask (x4)", "fp_add 12: addc+subb+bfi (x4)",
                          "addc+subb chains only (x4) +12 mov"};
  const double per[7] = {128, 128, 128, 128, 4, 4, 4};
  uint64_t* d;
  (void)hipMalloc(&d, 1024 * 8);
  uint64_t h[1024];
  for (int kk = 0; kk < 7; ++kk) {
    for (int rep = 0; rep < 2; ++rep) {
      switch (kk) {
#define L(K) case K: hipLaunchKernelGGL(k<K>, dim3(1024), dim3(64), 0, 0, d, 50); break;
        L(0) L(1) L(2) L(3) L(4) L(5) L(6)
      }
      if (hipDeviceSynchronize() != hipSuccess) return 2;
    }
    (void)hipMemcpy(h, d, 1024 * 8, hipMemcpyDeviceToHost);
    double sum = 0;
    for (int i = 0; i < 1024; ++i) sum += h[i];
    printf("%-40s 1 wave/SIMD: %7.2f cycles per %s\n", names[kk], sum / 1024 / (50.0 * per[kk]),
           per[kk] == 128 ? "instruction" : "12-limb sequence");
  }
  return 0;
}
