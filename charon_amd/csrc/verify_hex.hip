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
#define bls bls_hex
#include <hip/hip_runtime.h>

#include "race.h"

#include "lg2.h"

namespace bls {

constexpr int kHexBlock = 64;

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

}  // namespace bls
