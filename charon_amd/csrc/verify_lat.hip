// The drop-in latency path: tbls.Verify for batches far below one wave of work per SIMD (the unpatched callers'
// n = 1 calls, /root/reference/core/parsigex/parsigex.go:86-91 and core/validatorapi/validatorapi.go:246-283), on
// EIGHT lanes per item (VERDICT r03 "Next round" 8).  This translation unit is the lane-quad Verify of kernels.h
// (k_verify_prep + k_verify_pair_lq4, lg2.h lq4_verify) compiled with BLS_FP2_PAIR: every Fp2 product and square is
// split across lanes l and l ^ 4 (field.h fp2p_*, tower.h), so the quad's lanes 0-3 and their twins 4-7 hold the
// same values and each does half of every Fp2 product.  Same formulas, same statuses; ~half the latency of the
// Fp2-bound chains (hash to G2, the Miller loops, the final exponentiation).
//
// Everything here lives in namespace bls_fp2p (the kernel headers are included with `bls` renamed), so its inline
// functions never meet the main translation unit's on the host side; hipbls.hip declares and launches the two kernels.
#define BLS_FP2_PAIR 1
#define bls bls_fp2p
#include <hip/hip_runtime.h>

#include "lg2.h"

namespace bls {

constexpr int kOctBlock = 64;

// Stage 1, eight lanes per item (t >> 3): the first ceil(8n / 64) workgroups decode + check pk and sig (herumi's
// order, k_verify_prep's statuses), the rest hash the messages (lanes 0/1 of each quad split the two SSWU maps,
// lg2.h hash_to_g2_pair; lanes 2/3 repeat them).  ws: pk (24 x n), H(m) (48 x n), sig (48 x n), SoA.
__global__ void __launch_bounds__(kOctBlock) k_verify_prep8(const uint8_t* __restrict__ pks,
                                                            const uint8_t* __restrict__ msgs,
                                                            const uint64_t* __restrict__ offs,
                                                            const uint8_t* __restrict__ sigs, uint64_t n,
                                                            uint32_t* __restrict__ ws, int32_t* __restrict__ status) {
  const uint64_t nb = (8 * n + kOctBlock - 1) / kOctBlock;
  const bool hash_role = blockIdx.x >= nb;  // uniform per workgroup
  const uint64_t t = (blockIdx.x - (hash_role ? nb : 0)) * (uint64_t)blockDim.x + threadIdx.x;
  const uint64_t i = t >> 3;
  if (i >= n) return;  // the same on all eight lanes
  const bool lead = (t & 7) == 0;
  if (hash_role) {
    const uint32_t m = (t & 1) ? ~0u : 0u;
    const uint64_t o0 = offs[i], o1 = offs[i + 1];
    g2j hj;
    hash_to_g2_pair(hj, msgs + o0, (uint32_t)(o1 - o0), DST_POP, 43, m);
    g2a hm;
    jac_to_aff(hm, hj);
    if (lead) soa_store<48>(ws + 24 * n, n, i, &hm.x.c0.v[0]);
    return;
  }
  g1a pk;
  g2a sig;
  int st = RLC_PENDING;
  const int dp = g1_decompress(pk, pks + 48 * i, true);
  if (dp == DEC_BAD) {
    st = HIPBLS_ERR_PUBKEY;
  } else {
    const int ds = g2_decompress(sig, sigs + 96 * i, false);  // G2 membership: from the signature's Miller loop
    if (ds == DEC_BAD)
      st = HIPBLS_ERR_SIGNATURE;
    else if (dp == DEC_INF || ds == DEC_INF)
      st = verify_inf_status(ds, sig);
  }
  if (lead) {
    if (st == RLC_PENDING) {
      soa_store<24>(ws, n, i, &pk.x.v[0]);
      soa_store<48>(ws + 72 * n, n, i, &sig.x.c0.v[0]);
    }
    status[i] = st;
  }
}

// Stage 2, eight lanes per item: lq4_verify on lanes 0-3 (q = t & 3) and, as their Fp2 twins, on 4-7.
__global__ void __launch_bounds__(kOctBlock) k_verify_pair_lq8(const uint32_t* __restrict__ ws, uint64_t n,
                                                               int32_t* __restrict__ status) {
  const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  const uint64_t i = t >> 3;
  if (i >= n || status[i] != RLC_PENDING) return;  // the same on all eight lanes
  g1a pk;
  g2a hm, sig;
  soa_load<24>(&pk.x.v[0], ws, n, i);
  soa_load<48>(&hm.x.c0.v[0], ws + 24 * n, n, i);
  soa_load<48>(&sig.x.c0.v[0], ws + 72 * n, n, i);
  const int st = lq4_verify(pk, hm, sig, (int)(t & 3));
  if ((t & 7) == 0) status[i] = st;
}

}  // namespace bls
