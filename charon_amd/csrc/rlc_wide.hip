// The RLC item and hash stages (rlc.h stages 1 and 2, rlcb.h stage 1) in a translation unit of their own, compiled
// for BLS_WIDE_WAVES (default two) waves per SIMD.
//
// Why a unit of its own: their launches hold more than the chip's 1,024 wave slots (C4/C5: 16,384 item waves, 2,048
// hash waves), none uses LDS, and a second wave per SIMD fills the first one's scratch and dependency waits. The
// occupancy attribute only reaches 256 registers per wave if every out-of-line callee is held to it as well; in
// hipbls.hip the callees (decompression, subgroup tests, scalar multiplications, hash_to_G2) are shared with the
// one-wave pairing kernels, so the attribute alone left these kernels at one wave (354 registers). Here the kernel
// headers are compiled with `bls` renamed to bls_wide: the callees are this unit's own copies, and the compiler holds
// them to the kernels' 256 registers.
//
// Same functions, same canonical values as the one-wave build: the RLC bitmaps are checked against per-item Verify
// and the oracle (tests/test_gpu_configs.py, tests/test_gpu_rlc*.py, test_gpu_r05.py).
// The kernels have C linkage so that hipbls.hip, which declares them with its own (layout-identical) bls::rlc_seed,
// can launch them.
#define bls bls_wide
#include <hip/hip_runtime.h>

#include "rlcb.h"

#ifndef BLS_WIDE_WAVES
#define BLS_WIDE_WAVES 2
#endif
#if BLS_WIDE_WAVES > 1
#define BLS_WIDE_ATTR __attribute__((amdgpu_waves_per_eu(BLS_WIDE_WAVES, BLS_WIDE_WAVES)))
#else
#define BLS_WIDE_ATTR
#endif

using bls::rlc_seed;
constexpr int kWideBlock = 64;  // hipbls.hip kBlock

// Stage 1: one lane per item -> status (final or RLC_PENDING), [r_i] pk_i and [r_i] sig_i in SoA.
// pks == nullptr: public keys come from the resident pubshare table (key_idx, T, tcode, tab).
extern "C" __global__ void __launch_bounds__(kWideBlock) BLS_WIDE_ATTR
k_rlc_items(uint64_t i0, uint64_t i1, const uint8_t* __restrict__ pks, const uint8_t* __restrict__ sigs,
            const uint32_t* __restrict__ msg_idx, uint64_t n, uint64_t n_msgs, rlc_seed seed,
            uint32_t* __restrict__ rpk, uint32_t* __restrict__ rsig, int32_t* __restrict__ status,
            const uint32_t* __restrict__ key_idx, uint64_t T, const int32_t* __restrict__ tcode,
            const uint32_t* __restrict__ tab) {
  const uint64_t i = i0 + blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (i < i1) bls::rlc_items_lane(i, pks, sigs, msg_idx, n, n_msgs, seed, rpk, rsig, status, key_idx, T, tcode, tab);
}

// Stage 2: one lane per message to hash -> H(m) in affine SoA (48 words) at its table column.  mlist lists the
// messages to hash (the H(m)-cache misses); nullptr = messages 0 .. n_hash-1.
extern "C" __global__ void __launch_bounds__(kWideBlock) BLS_WIDE_ATTR
k_rlc_hash(const uint8_t* __restrict__ msgs, const uint64_t* __restrict__ offs, uint64_t n_hash,
           const uint32_t* __restrict__ mlist, uint32_t* __restrict__ H, uint64_t hstride,
           const uint32_t* __restrict__ hslot) {
  const uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (j < n_hash) bls::rlc_hash_lane(mlist ? (uint64_t)mlist[j] : j, msgs, offs, H, hstride, hslot);
}

// The batch-wide check's stage 1 (rlcb.h): decode, subgroup tests and the scalars, points into the MSM inputs.
extern "C" __global__ void __launch_bounds__(kWideBlock) BLS_WIDE_ATTR
k_rlcb_items(uint64_t n, const uint8_t* __restrict__ pks, const uint8_t* __restrict__ sigs,
             const uint32_t* __restrict__ msg_idx, uint64_t n_msgs, rlc_seed seed, uint32_t* __restrict__ rpk,
             uint32_t* __restrict__ pts, uint32_t* __restrict__ sc, int32_t* __restrict__ status,
             const uint32_t* __restrict__ key_idx, uint64_t T, const int32_t* __restrict__ tcode,
             const uint32_t* __restrict__ tab, const uint32_t* __restrict__ g1pos, uint32_t* __restrict__ gpts,
             uint32_t* __restrict__ gsc) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (i < n)
    bls::rlcb_items_lane(i, pks, sigs, msg_idx, n, n_msgs, seed, rpk, pts, sc, status, key_idx, T, tcode, tab, g1pos,
                         gpts, gsc);
}
