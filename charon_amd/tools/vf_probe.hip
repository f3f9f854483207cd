// k_verify_fused alone, for compile-only experiments on its register allocation (charon_amd/tools/vf_static.py): the
// same lane body as the product kernel (kernels.h), built with the product's flags plus the -D / -mllvm options under
// test, then disassembled and summarized (scratch instructions in the Miller loop, VGPR / AGPR use, private segment).
#include <hip/hip_runtime.h>

#include "ops.h"

using namespace bls;

constexpr int kBlock = 64;

__global__ void __launch_bounds__(kBlock) k_verify_fused(const uint8_t* __restrict__ pks,
                                                         const uint8_t* __restrict__ msgs,
                                                         const uint64_t* __restrict__ offs,
                                                         const uint8_t* __restrict__ sigs, uint64_t n,
                                                         int32_t* __restrict__ status) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t o0 = offs[i], o1 = offs[i + 1];
  __shared__ u32x4 s_f12_[36 * kBlock];
  const f12l<kBlock> F{(BLS_LDS u32x4*)&s_f12_[threadIdx.x]};
  status[i] = op_verify_l_kernel(pks + 48 * i, msgs + o0, (uint32_t)(o1 - o0), sigs + 96 * i, F);
}
