// The drop-in n = 1 path's pairing check on SIXTEEN lanes per item (round 5; VERDICT r04 item 4, p50 <= 10 ms).
// verify_lat.hip's octet check (lg2.h lq4_verify in the split-Fp2 build: a quad of lanes, each Fp2 product split
// across the twins l and l ^ 4) compiled a third time with BLS_HEX: each item's octet state is held twice, on lanes
// 0-7 and 8-15 of its group of sixteen, and the two copies share the work of the steps on the check's critical path
// (lg2.h, BLS_HEX):
//   * every Fp6 product (the split Miller loop's Fp12 squaring, the quad final exponentiation's Fp12 products): the
//     low half forms Karatsuba's three diagonal products, the high half the three cross products (fp6_mul_hx);
//   * the compressed squarings of the final exponentiation's five exponentiations by |x|: their two rounds of Fp2
//     squarings become one (the low half squares z2 | z3 | z4 | z5, the high half z2 + z3 | z4 + z5).
// One DPP row_ror:8 per dword exchanges the halves.  Same formulas, same canonical values: the statuses equal the
// octet check's and the oracle's (tests/test_gpu_lg2.py, tests/test_gpu_r05.py).  A batch of at most four items
// (one workgroup) takes it; the prep stays the octet one (k_verify_prep8, its SoA workspace is the input here).
// Everything here lives in namespace bls_hex (the kernel headers are included with `bls` renamed).
#define BLS_FP2_PAIR 1
#define BLS_HEX 1
#ifdef BLS_HEX_FAV_WIDE  // fav_wide.hip: this file compiled again for FastAggregateVerify's check alone
#define bls bls_hexw
#else
#define bls bls_hex
#endif
#include <hip/hip_runtime.h>

#include "race.h"

#include "lg2.h"

namespace bls {

constexpr int kHexBlock = 64;

#ifndef BLS_HEX_FAV_WIDE
// Stage 2 on sixteen lanes per item (k_verify_pair_lq8's body: the status from the decode codes in herumi's order,
// then lq4_verify on lanes q = t & 3 with their twins and their second copies).  Replicas race as in verify_lat.hip
// (race word race[3]).
__global__ void __launch_bounds__(kHexBlock) k_verify_pair_lq16(const uint32_t* __restrict__ ws, uint64_t n,
                                                                int32_t* __restrict__ status, uint32_t replicas,
                                                                uint32_t* __restrict__ race, uint32_t epoch) {
  bls_race::init(replicas > 1 ? race + 3 : nullptr, epoch);
  const uint64_t t = (blockIdx.x / replicas) * (uint64_t)blockDim.x + threadIdx.x;
  const uint64_t i = t >> 4;
  if (i >= n) return;  // the same on all sixteen lanes
  const int32_t* codes = (const int32_t*)(ws + 120 * n);
  const int dp = codes[2 * i], ds = codes[2 * i + 1];
  const bool lead = (t & 15) == 0;
  g2a sig;
  if (ds == DEC_OK) soa_load<48>(&sig.x.c0.v[0], ws + 72 * n, n, i);
  int st = RLC_PENDING;
  if (dp == DEC_BAD)
    st = HIPBLS_ERR_PUBKEY;
  else if (ds == DEC_BAD)
    st = HIPBLS_ERR_SIGNATURE;
  else if (dp == DEC_INF || ds == DEC_INF)
    st = verify_inf_status(ds, sig);  // KeyValidate / e(pk, H) != 1
  if (st != RLC_PENDING) {
    if (lead) status[i] = st;
    return;
  }
  g1a pk;
  g2a hm;
  soa_load<24>(&pk.x.v[0], ws, n, i);
  soa_load<48>(&hm.x.c0.v[0], ws + 24 * n, n, i);
  st = lq4_verify(pk, hm, sig, (int)(t & 3));
  if (lead) status[i] = st;
  bls_race::finish();
}

#else
// FastAggregateVerify's check at two waves per SIMD (BLS_FAV_WAVES, default two): a batch call that fills every SIMD
// with two 256-register waves (the RLC item stage, rlc_wide.hip) otherwise starves this 512-register wave until that
// stage ends -- a full SIMD frees only when both of its waves end together (C5's overlapped sync-committee check).
#ifndef BLS_FAV_WAVES
#define BLS_FAV_WAVES 2
#endif
#if BLS_FAV_WAVES > 1
#define BLS_FAV_ATTR __attribute__((amdgpu_waves_per_eu(BLS_FAV_WAVES, BLS_FAV_WAVES)))
#endif
// FastAggregateVerify's check for a few groups (tbls/herumi.go:315-339), one workgroup per group g over the keys
// [goff[g], goff[g + 1]) that verify_lat.hip k_fav_prep8 decoded: the 64 lanes sum them (strided mixed additions, then
// an LDS tree, as kernels.h k_fav_batch), then lanes 0-15 run lq4_verify on the aggregate key in the sixteen-lane
// layout.  Status order as k_fav_batch: the signature's error first (its encoding, or G2 membership, which comes from
// lq4_verify's Miller loop, so the check runs whenever the signature decoded, with -g1 standing in for a key sum that
// cannot be used), then a key's encoding error, then "verification failed" (also for an empty key list, an infinity
// key or signature, a key sum at infinity).
#endif  // BLS_HEX_FAV_WIDE: k_verify_pair_lq16 here, k_fav_pair_lq16 in fav_wide.hip
#ifdef BLS_HEX_FAV_WIDE
#ifndef BLS_FAV_ATTR
#define BLS_FAV_ATTR
#endif
__global__ void __launch_bounds__(kHexBlock) BLS_FAV_ATTR k_fav_pair_lq16(const uint32_t* __restrict__ pts,
                                                             const int32_t* __restrict__ kcode, uint64_t nkeys,
                                                             const uint64_t* __restrict__ goff,
                                                             const uint32_t* __restrict__ ws, uint64_t G,
                                                             int32_t* __restrict__ status) {
  __shared__ uint32_t red[kHexBlock * 36];
  __shared__ int sh_bad, sh_inf;
  bls_race::init(nullptr, 0u);
  const uint64_t g = blockIdx.x;
  const int tid = threadIdx.x;
  const uint64_t k0 = goff[g], k1 = goff[g + 1];
  if (tid == 0) {
    sh_bad = 0;
    sh_inf = 0;
  }
  __syncthreads();
  {
    g1j acc;
    jac_set_inf(acc);
    int bad = 0, inf = 0;
    for (uint64_t k = k0 + tid; k < k1; k += kHexBlock) {
      const int c = kcode[k];
      if (c == DEC_BAD) {
        bad = 1;
      } else if (c == DEC_INF) {
        inf = 1;
      } else {
        g1a a;
        soa_load<24>(&a.x.v[0], pts, nkeys, k);
        jac_add_aff(acc, acc, a);
      }
    }
    if (bad) atomicOr(&sh_bad, 1);
    if (inf) atomicOr(&sh_inf, 1);
    for (int w = 0; w < 36; ++w) red[w * kHexBlock + tid] = (&acc.x.v[0])[w];
  }
  __syncthreads();
  for (int half = kHexBlock / 2; half >= 1; half >>= 1) {  // every thread reaches every barrier
    if (tid < half) {
      g1j x, y;
      for (int w = 0; w < 36; ++w) {
        (&x.x.v[0])[w] = red[w * kHexBlock + tid];
        (&y.x.v[0])[w] = red[w * kHexBlock + tid + half];
      }
      jac_add(x, x, y);
      for (int w = 0; w < 36; ++w) red[w * kHexBlock + tid] = (&x.x.v[0])[w];
    }
    __syncthreads();
  }
  if (tid >= 16) return;  // lanes 0-15: the check, every branch below on shared values only
  const int ds = ((const int32_t*)(ws + 120 * G))[2 * g + 1];
  g1j sum;
  for (int w = 0; w < 36; ++w) (&sum.x.v[0])[w] = red[w * kHexBlock];
  const bool sum_ok = !sh_bad && !sh_inf && k1 > k0 && !jac_is_inf(sum);
  int chk = HIPBLS_OK;
  if (ds == DEC_OK) {
    g1a pk;
    if (sum_ok) {
      jac_to_aff(pk, sum);
    } else {
      pk.x = G1_GEN_X;
      pk.y = G1_NEG_GEN_Y;
    }
    g2a hm, sig;
    soa_load<48>(&hm.x.c0.v[0], ws + 24 * G, G, g);
    soa_load<48>(&sig.x.c0.v[0], ws + 72 * G, G, g);
    chk = lq4_verify(pk, hm, sig, tid & 3);
  }
  int st;
  if (ds == DEC_BAD || chk == HIPBLS_ERR_SIGNATURE)
    st = HIPBLS_ERR_SIGNATURE;
  else if (sh_bad)
    st = HIPBLS_ERR_PUBKEY;
  else if (!sum_ok || ds == DEC_INF)
    st = HIPBLS_ERR_VERIFY;  // KeyValidate rejects the identity key; the empty set is false
  else
    st = chk;
  if (tid == 0) status[g] = st;
}

#endif
}  // namespace bls
