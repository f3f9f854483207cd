// Test-only GPU library (tests/native/libgpu_units.so): device entry points into single building blocks of the
// kernels, for -m gpu tests that compare them with the host build (tests/native/host_ops.cpp) and the oracle.
// Not part of the product (charon_amd/libhipbls.so); loaded only by tests/test_gpu_units.py.
//
//   gu_final_exp        final_exponentiation (pairing.h), one lane per element
//   gu_final_exp_split  final_exponentiation_split (lg2.h), a lane pair per element: lanes 2i, 2i+1 hold the
//                       halves c0 | c1 of element i.  Covers the lane-pair Karabina fallback (fp2_is_zero(pre[5]) ->
//                       fp12h_exp_xabs with DPP exchanges), reached when a saved compressed power has z2 = z3 = 0,
//                       e.g. for the identity and for Fp2 elements (ADVICE r02, lg2.h:263).
//   gu_exp_xabs_split   fp12h_exp (Karabina, Granger-Scott when degenerate) on a split value (no easy part): the raw a^|x| of the pair.
//   gu_quad             final_exponentiation_quad / fp12q_exp_xabs (lg2.h), a lane quad per element, the
//                       value in full on all four lanes; each lane's result is returned, so the test sees that the four
//                       agree.  Fp2 elements and the identity take the quad's degenerate branch (Granger-Scott).
// Elements cross the ABI as 12 big-endian 48-byte Fp coefficients (c0.c0.c0 .. c1.c2.c1), canonical, not Montgomery.
#include <hip/hip_runtime.h>

#include "kernels.h"

using namespace bls;

namespace {

__device__ void fp_in_be(fp& a, const uint8_t* b) {
  fp_plain_from_be48(a, b);
  fp_to_mont(a, a);
}
__device__ void fp_out_be(uint8_t* o, const fp& a) {
  fp t;
  fp_from_mont(t, a);
  fp_plain_to_be48(o, t);
}
__device__ void f12_in(fp12& f, const uint8_t* in) {
  fp* c = &f.c0.c0.c0;
  for (int i = 0; i < 12; ++i) fp_in_be(c[i], in + 48 * i);
}
__device__ void f12_out(uint8_t* out, const fp12& f) {
  const fp* c = &f.c0.c0.c0;
  for (int i = 0; i < 12; ++i) fp_out_be(out + 48 * i, c[i]);
}

__global__ void __launch_bounds__(64) k_gu_final_exp(const uint8_t* in, uint8_t* out, uint64_t n) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  fp12 f, r;
  f12_in(f, in + 576 * i);
  final_exponentiation(r, f);
  f12_out(out + 576 * i, r);
}

// op 0: final_exponentiation_split; op 1: fp12h_exp (Karabina); op 2: fp12h_exp_xabs (Granger-Scott, the fallback)
__global__ void __launch_bounds__(64) k_gu_split(const uint8_t* in, uint8_t* out, uint64_t n, int op) {
  const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  const uint64_t i = t >> 1;
  // pair-uniform exit: both lanes of a pair leave together (n counts pairs)
  if (i >= n) return;
  const uint32_t m = (t & 1) ? ~0u : 0u;
  fp12 f;
  f12_in(f, in + 576 * i);
  const fp6 h = sel(m, f.c1, f.c0);
  fp6 r;
  if (op == 0)
    final_exponentiation_split(r, h, m);
  else if (op == 1)
    fp12h_exp(r, h, m);  // Karabina, degenerate inputs through the Granger-Scott fallback
  else
    fp12h_exp_xabs(r, h, m);
  fp12 full;
  fp12h_gather(full, r, m);
  if (!m) f12_out(out + 576 * i, full);
}

// op 0: final_exponentiation_quad; op 1: fp12q_exp_xabs.  out holds 4 results per element (lanes 0..3).
__global__ void __launch_bounds__(64) k_gu_quad(const uint8_t* in, uint8_t* out, uint64_t n, int op) {
  const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  const uint64_t i = t >> 2;
  if (i >= n) return;  // quad-uniform
  const quad_m qm((int)(t & 3));
  fp12 f, r;
  f12_in(f, in + 576 * i);
  if (op == 0)
    final_exponentiation_quad(r, f, qm);
  else
    fp12q_exp_xabs(r, f, qm);
  f12_out(out + 576 * t, r);
}

int check(hipError_t e) { return e == hipSuccess ? 0 : 1; }

int run_quad(const uint8_t* in, uint8_t* out, uint64_t n, int op) {
  uint8_t *din = nullptr, *dout = nullptr;
  if (check(hipMalloc(&din, 576 * n)) || check(hipMalloc(&dout, 4 * 576 * n))) return 1;
  int rc = check(hipMemcpy(din, in, 576 * n, hipMemcpyHostToDevice));
  if (!rc) {
    hipLaunchKernelGGL(k_gu_quad, dim3((unsigned)((4 * n + 63) / 64)), dim3(64), 0, 0, din, dout, n, op);
    rc = check(hipGetLastError()) || check(hipDeviceSynchronize()) ||
         check(hipMemcpy(out, dout, 4 * 576 * n, hipMemcpyDeviceToHost));
  }
  (void)hipFree(din);
  (void)hipFree(dout);
  return rc;
}

int run(unsigned lanes, const uint8_t* in, uint8_t* out, uint64_t n, int extra_op, bool split) {
  uint8_t *din = nullptr, *dout = nullptr;
  if (check(hipMalloc(&din, 576 * n)) || check(hipMalloc(&dout, 576 * n))) return 1;
  int rc = check(hipMemcpy(din, in, 576 * n, hipMemcpyHostToDevice));
  if (!rc) {
    const unsigned grid = (lanes + 63) / 64;
    if (split)
      hipLaunchKernelGGL(k_gu_split, dim3(grid), dim3(64), 0, 0, din, dout, n, extra_op);
    else
      hipLaunchKernelGGL(k_gu_final_exp, dim3(grid), dim3(64), 0, 0, din, dout, n);
    rc = check(hipGetLastError()) || check(hipDeviceSynchronize()) ||
         check(hipMemcpy(out, dout, 576 * n, hipMemcpyDeviceToHost));
  }
  (void)hipFree(din);
  (void)hipFree(dout);
  return rc;
}

}  // namespace

extern "C" {
int gu_final_exp(const uint8_t* in, uint8_t* out, uint64_t n) {
  return n ? run((unsigned)n, in, out, n, 0, false) : 0;
}
int gu_final_exp_split(const uint8_t* in, uint8_t* out, uint64_t n) {
  return n ? run((unsigned)(2 * n), in, out, n, 0, true) : 0;
}
int gu_exp_xabs_split(const uint8_t* in, uint8_t* out, uint64_t n, int karabina) {
  return n ? run((unsigned)(2 * n), in, out, n, karabina ? 1 : 2, true) : 0;
}
int gu_quad(const uint8_t* in, uint8_t* out, uint64_t n, int op) { return n ? run_quad(in, out, n, op) : 0; }
}
