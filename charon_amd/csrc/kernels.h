// hipbls kernels (gfx950): one lane (or one workgroup) per item; the lane bodies live in ops.h / rlc.h so the
// same arithmetic is compiled for the host tests.  Included once, by hipbls.hip (the C-ABI host runtime).
#pragma once
#include <hip/hip_runtime.h>

#include "lg2.h"
#include "ops.h"
#include "rlc.h"
#include "rlcb.h"

using namespace bls;

// ============================================================================ kernels
namespace {

#ifndef BLS_VERIFY_LDS
#define BLS_VERIFY_LDS 1
#endif
constexpr int kBlock = 64;
// This lane's Miller-loop accumulator in LDS (pairing_lds.h): 36 KiB per one-wave workgroup, so the four one-wave
// workgroups a CU holds at this register count use 144 of its 160 KiB.  Every single-lane pairing check declares it.
#define BLS_LANE_F12(F)                      \
  __shared__ u32x4 s_f12_[36 * kBlock];      \
  const f12l<kBlock> F { (BLS_LDS u32x4*)&s_f12_[threadIdx.x] }  // one wave per workgroup: these kernels are register-bound, not LDS-bound

__global__ void __launch_bounds__(kBlock) k_verify_fused(const uint8_t* __restrict__ pks,
                                                         const uint8_t* __restrict__ msgs,
                                                         const uint64_t* __restrict__ offs,
                                                         const uint8_t* __restrict__ sigs, uint64_t n,
                                                         int32_t* __restrict__ status) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t o0 = offs[i], o1 = offs[i + 1];
#if BLS_VERIFY_LDS
  BLS_LANE_F12(F);
  status[i] = op_verify_l_kernel(pks + 48 * i, msgs + o0, (uint32_t)(o1 - o0), sigs + 96 * i, F);
#else
  status[i] = op_verify(pks + 48 * i, msgs + o0, (uint32_t)(o1 - o0), sigs + 96 * i);
#endif
}

// ---------------------------------------------------------------- lane-pair Verify (lg2.h)
// Stage 1, two waves per 64 items: the first grid_for(n) blocks decode + check pk and sig and set the status (final or
// RLC_PENDING), the next grid_for(n) blocks hash the messages.  The roles are per workgroup (kBlock = one wave), so
// the two run side by side on different SIMDs and the stage's latency is the hash alone, not hash + decode (the
// batches that take lane pairs leave SIMDs free).  Every message is hashed, whatever its item's status.  The points
// go to SoA (pk 24 words, H(m) 48, sig 48 per item: `ws` holds 120 words x n).  Status order is op_verify's.
// pair_hash: the hash workgroups are 2 grid_for(n) and a lane pair hashes each message (small batches, where the
// extra waves still find idle SIMDs).
__global__ void __launch_bounds__(kBlock) k_verify_prep(const uint8_t* __restrict__ pks,
                                                        const uint8_t* __restrict__ msgs,
                                                        const uint64_t* __restrict__ offs,
                                                        const uint8_t* __restrict__ sigs, uint64_t n,
                                                        uint32_t* __restrict__ ws, int32_t* __restrict__ status,
                                                        int pair_hash) {
  const uint64_t nb = (n + kBlock - 1) / kBlock;
  const bool hash_role = blockIdx.x >= nb;  // uniform per workgroup
  if (hash_role && pair_hash) {  // lanes 2i, 2i+1 hash item i together (lg2.h hash_to_g2_pair)
    const uint64_t t = (blockIdx.x - nb) * (uint64_t)blockDim.x + threadIdx.x;
    const uint64_t i = t >> 1;
    if (i >= n) return;  // same on both lanes of the pair
    const uint32_t m = (t & 1) ? ~0u : 0u;
    const uint64_t o0 = offs[i], o1 = offs[i + 1];
    g2j hj;
    hash_to_g2_pair(hj, msgs + o0, (uint32_t)(o1 - o0), DST_POP, 43, m);
    if (!m) {
      g2a hm;
      jac_to_aff(hm, hj);
      soa_store<48>(ws + 24 * n, n, i, &hm.x.c0.v[0]);
    }
    return;
  }
  const uint64_t i = (blockIdx.x - (hash_role ? nb : 0)) * (uint64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (hash_role) {
    const uint64_t o0 = offs[i], o1 = offs[i + 1];
    g2j hj;
    hash_to_g2(hj, msgs + o0, (uint32_t)(o1 - o0), DST_POP, 43);
    g2a hm;
    jac_to_aff(hm, hj);
    soa_store<48>(ws + 24 * n, n, i, &hm.x.c0.v[0]);
    return;
  }
  g1a pk;
  g2a sig;
  int st = RLC_PENDING;
  const int dp = g1_decompress(pk, pks + 48 * i, true);
  if (dp == DEC_BAD) {
    st = HIPBLS_ERR_PUBKEY;
  } else {
    const int ds = g2_decompress(sig, sigs + 96 * i, false);  // G2 membership: from the pair's Miller loop
    if (ds == DEC_BAD)
      st = HIPBLS_ERR_SIGNATURE;
    else if (dp == DEC_INF || ds == DEC_INF)
      st = verify_inf_status(ds, sig);  // KeyValidate / e(pk,H) != 1
  }
  if (st == RLC_PENDING) {
    soa_store<24>(ws, n, i, &pk.x.v[0]);
    soa_store<48>(ws + 72 * n, n, i, &sig.x.c0.v[0]);
  }
  status[i] = st;
}

// Stage 2, lanes 2i and 2i+1 per item: e(pk, H(m)) * e(-g1, sig) == 1 with the two Miller loops side by side
// and the final exponentiation split across the pair.  The odd lane's loop runs over the signature, so its final T
// = [|x|] sig also decides the signature's G2 membership (pairing.h g2_subgroup_from_miller; the prep stage skipped
// the separate check): a signature outside G2 is herumi's deserialization error, whatever the pairing says.
__global__ void __launch_bounds__(kBlock) k_verify_pair_lg2(const uint32_t* __restrict__ ws, uint64_t n,
                                                            int32_t* __restrict__ status) {
  const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  const uint64_t i = t >> 1;
  const uint32_t m = (t & 1) ? ~0u : 0u;
  if (i >= n || status[i] != RLC_PENDING) return;  // same decision on both lanes of the pair
  g1a P[1];
  g2a Q[1];
  if (!m) {
    soa_load<24>(&P[0].x.v[0], ws, n, i);
    soa_load<48>(&Q[0].x.c0.v[0], ws + 24 * n, n, i);
  } else {
    P[0].x = G1_GEN_X;
    P[0].y = G1_NEG_GEN_Y;
    soa_load<48>(&Q[0].x.c0.v[0], ws + 72 * n, n, i);
  }
  fp12 f;
  g2j T;
  miller_loop_multi<1>(f, P, Q, 1, &T);
  const uint32_t in_g2 = g2_subgroup_from_miller(T, Q[0]) ? 1u : 0u;  // meaningful on the odd lane
  const uint32_t other = pair_swap(in_g2);  // both lanes of the pair take part in the exchange
  const uint32_t sig_in_g2 = m ? in_g2 : other;
  const bool ok = lg2_finish(f, m);
  if (!m) status[i] = !sig_in_g2 ? HIPBLS_ERR_SIGNATURE : (ok ? HIPBLS_OK : HIPBLS_ERR_VERIFY);
}

// Stage 2 on a lane quad per item (lg2.h lq4_verify): lanes 4i, 4i+1 split e(pk, H(m))'s Miller loop, lanes 4i+2,
// 4i+3 e(-g1, sig)'s, then the split final exponentiation.  Same statuses as k_verify_pair_lg2.
__device__ __forceinline__ void verify_pair_lq4_lane(uint64_t t, const uint32_t* __restrict__ ws, uint64_t n,
                                                     int32_t* __restrict__ status) {
  const uint64_t i = t >> 2;
  const int q = (int)(t & 3);
  if (i >= n || status[i] != RLC_PENDING) return;  // same decision on all four lanes of the quad
  g1a pk;
  g2a hm, sig;
  soa_load<24>(&pk.x.v[0], ws, n, i);
  soa_load<48>(&hm.x.c0.v[0], ws + 24 * n, n, i);
  soa_load<48>(&sig.x.c0.v[0], ws + 72 * n, n, i);
  const int st = lq4_verify(pk, hm, sig, q);
  if (q == 0) status[i] = st;
}
__global__ void __launch_bounds__(kBlock) k_verify_pair_lq4(const uint32_t* __restrict__ ws, uint64_t n,
                                                            int32_t* __restrict__ status) {
  verify_pair_lq4_lane(blockIdx.x * (uint64_t)blockDim.x + threadIdx.x, ws, n, status);
}

__global__ void __launch_bounds__(kBlock) k_sign(const uint8_t* __restrict__ sks, const uint8_t* __restrict__ msgs,
                                                 const uint64_t* __restrict__ offs, uint64_t n,
                                                 uint8_t* __restrict__ out, int32_t* __restrict__ status) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t o0 = offs[i], o1 = offs[i + 1];
  uint8_t sig[96];
  const int st = op_sign(sig, sks + 32 * i, msgs + o0, (uint32_t)(o1 - o0));
  for (int k = 0; k < 96; ++k) out[96 * i + k] = st == HIPBLS_OK ? sig[k] : (uint8_t)0;
  status[i] = st;
}

__global__ void __launch_bounds__(kBlock) k_sk_to_pk(const uint8_t* __restrict__ sks, uint64_t n,
                                                     uint8_t* __restrict__ out, int32_t* __restrict__ status) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t pk[48];
  const int st = op_sk_to_pk(pk, sks + 32 * i);
  for (int k = 0; k < 48; ++k) out[48 * i + k] = st == HIPBLS_OK ? pk[k] : (uint8_t)0;
  status[i] = st;
}

// ThresholdAggregate, stage 1: one lane per partial signature k.  Finds its group by binary search
// over group_offsets, decodes + subgroup-checks sig_k, computes lambda_k(0) from the group's ids and
// writes lambda_k * sig_k (Jacobian, limb-major SoA: 36 words x n_partials) plus a per-partial code.
#ifndef BLS_TAGG_WAVES
#define BLS_TAGG_WAVES 1
#endif
__device__ __forceinline__ void tagg_scale_lane(uint64_t k, const uint8_t* __restrict__ sigs,
                                                const int64_t* __restrict__ ids, const uint64_t* __restrict__ goffs,
                                                uint64_t n_groups, uint64_t n_parts, uint32_t* __restrict__ pts,
                                                int32_t* __restrict__ pstat) {
  if (k >= n_parts) return;
  uint64_t lo = 0, hi = n_groups;  // find g with goffs[g] <= k < goffs[g+1]
  while (hi - lo > 1) {
    const uint64_t mid = (lo + hi) / 2;
    if (goffs[mid] <= k)
      lo = mid;
    else
      hi = mid;
  }
  const uint64_t g0 = goffs[lo], g1 = goffs[lo + 1];
  const int t = (int)(g1 - g0);
  const int me = (int)(k - g0);
  g2j acc;
  jac_set_inf(acc);
  int st = HIPBLS_OK;
  // ids must be non-zero and distinct within the group (herumi Recover fails otherwise).  As Fr elements
  // (idx mod r, fr_from_i64) two int64 ids are equal only when equal as integers: |a - b| < 2^64 < r.
  for (int a = 0; a < t; ++a) {
    if (ids[g0 + a] == 0) st = HIPBLS_ERR_COMBINE;
    for (int b = a + 1; b < t; ++b)
      if (ids[g0 + a] == ids[g0 + b]) st = HIPBLS_ERR_COMBINE;
  }
  g2a s;
  int64_t c;
  uint64_t L;
  // small ids: the subgroup test and c_k sig_k share one doubling chain (ops.h g2_subgroup_and_mul_i64)
  const bool small = st == HIPBLS_OK && lagrange_small(ids + g0, t, me, c, L);
  int ds = g2_decompress(s, sigs + 96 * k, !small);
  if (small && ds == DEC_OK) {
    g2j sj;
    jac_from_aff(sj, s);
    if (!g2_subgroup_and_mul_i64(acc, sj, c)) {
      ds = DEC_BAD;
      jac_set_inf(acc);
    }
  }
  if (ds == DEC_BAD) st = HIPBLS_ERR_SIGNATURE;
  if (st == HIPBLS_OK && ds == DEC_OK && !small) {
    g2j sj;
    jac_from_aff(sj, s);
    tagg_scale_point(acc, sj, ids + g0, t, me);  // lambda_k sig_k (field path)
  }
  const uint32_t* src = &acc.x.c0.v[0];
  for (int w = 0; w < 72; ++w) pts[(uint64_t)w * n_parts + k] = src[w];
  pstat[k] = st;
}
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(BLS_TAGG_WAVES, BLS_TAGG_WAVES)))
k_tagg_scale(const uint8_t* __restrict__ sigs, const int64_t* __restrict__ ids, const uint64_t* __restrict__ goffs,
             uint64_t n_groups, uint64_t n_parts, uint32_t* __restrict__ pts, int32_t* __restrict__ pstat) {
  tagg_scale_lane(blockIdx.x * (uint64_t)blockDim.x + threadIdx.x, sigs, ids, goffs, n_groups, n_parts, pts, pstat);
}

// ThresholdAggregate, stage 2: one lane per group sums its scaled partials, multiplies the sum by L^-1 on the
// small-integer path (ops.h lagrange_small), and compresses.
__global__ void __launch_bounds__(kBlock) k_tagg_sum(const uint32_t* __restrict__ pts,
                                                     const int32_t* __restrict__ pstat,
                                                     const int64_t* __restrict__ ids,
                                                     const uint64_t* __restrict__ goffs, uint64_t n_groups,
                                                     uint64_t n_parts, uint8_t* __restrict__ out,
                                                     int32_t* __restrict__ status) {
  const uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (g >= n_groups) return;
  const uint64_t g0 = goffs[g], g1 = goffs[g + 1];
  int st = g1 > g0 ? HIPBLS_OK : HIPBLS_ERR_COMBINE;
  // the reference reports the first deserialization failure before any combine failure
  for (uint64_t k = g0; k < g1; ++k)
    if (pstat[k] == HIPBLS_ERR_SIGNATURE) st = HIPBLS_ERR_SIGNATURE;
  if (st == HIPBLS_OK)
    for (uint64_t k = g0; k < g1; ++k)
      if (pstat[k] != HIPBLS_OK) st = pstat[k];
  g2j acc;
  jac_set_inf(acc);
  if (st == HIPBLS_OK) {
    for (uint64_t k = g0; k < g1; ++k) {
      g2j p;
      uint32_t* dst = &p.x.c0.v[0];
      for (int w = 0; w < 72; ++w) dst[w] = pts[(uint64_t)w * n_parts + k];
      jac_add(acc, acc, p);
    }
    tagg_unscale(acc, ids + g0, (int)(g1 - g0));
  }
  uint8_t sig[96];
  g2_compress(sig, acc);
  for (int b = 0; b < 96; ++b) out[96 * g + b] = st == HIPBLS_OK ? sig[b] : (uint8_t)0;
  status[g] = st;
}

// ---------------------------------------------------------------- sigagg: aggregate + Verify in one call
// core/sigagg/sigagg.go:138-159 threshold-aggregates each validator's partials and verifies the aggregate
// against the validator's root pubkey.  hipbls_threshold_aggregate_verify_batch fuses the two:
//   * the key side (k_tv_prep_pk) decodes the root key, scales it by the group's L (ops.h tagg_group_L) and hashes the
//     message, beside the aggregation;
//   * k_tagg_sum_s sums the scaled partials into S and hands S straight to the pairing check, which tests
//     e([L] pk, H(m)) == e(g1, S) -- the same verdict as e(pk, H(m)) == e(g1, [L^-1] S);
//   * k_tagg_unscale runs beside the pairing check: sigma = [L^-1] S, compressed into the 96-byte output.
// The aggregate is never decompressed or subgroup-checked again (it is in G2 by construction).
// ws: the lane-pair Verify layout (pk 24 words, H(m) 48, sig 48; SoA over the groups).

// Stage 2 of ThresholdAggregate for the fused call: per group, the status (as k_tagg_sum) and S = the sum of the
// scaled partials, left affine in ws (sig slot) with agg_inf[g] = 1 when it is the point at infinity (or the group
// failed).
__global__ void __launch_bounds__(kBlock) k_tagg_sum_s(const uint32_t* __restrict__ pts,
                                                       const int32_t* __restrict__ pstat,
                                                       const uint64_t* __restrict__ goffs, uint64_t n_groups,
                                                       uint64_t n_parts, int32_t* __restrict__ status,
                                                       uint32_t* __restrict__ ws, int32_t* __restrict__ agg_inf) {
  const uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (g >= n_groups) return;
  const uint64_t g0 = goffs[g], g1 = goffs[g + 1];
  int st = g1 > g0 ? HIPBLS_OK : HIPBLS_ERR_COMBINE;
  for (uint64_t k = g0; k < g1; ++k)
    if (pstat[k] == HIPBLS_ERR_SIGNATURE) st = HIPBLS_ERR_SIGNATURE;
  if (st == HIPBLS_OK)
    for (uint64_t k = g0; k < g1; ++k)
      if (pstat[k] != HIPBLS_OK) st = pstat[k];
  g2j acc;
  jac_set_inf(acc);
  if (st == HIPBLS_OK) {
    for (uint64_t k = g0; k < g1; ++k) {
      g2j p;
      soa_load<72>(&p.x.c0.v[0], pts, n_parts, k);
      g2j x = acc, y;
      jac_add(y, x, p);
      acc = y;
    }
  }
  status[g] = st;
  const bool inf = jac_is_inf(acc);
  g2a a;
  if (inf) {
    fp2_set_zero(a.x);
    fp2_set_zero(a.y);
  } else {
    jac_to_aff(a, acc);
  }
  soa_store<48>(ws + 72 * n_groups, n_groups, g, &a.x.c0.v[0]);
  agg_inf[g] = inf ? 1 : 0;
}

// Stage 3 (beside the pairing check): sigma = [L^-1] S on the small-integer path (S itself otherwise), compressed.
// The output bytes equal k_tagg_sum's: the encoding of sigma for a group that combined, zeros otherwise.
__device__ __forceinline__ void tagg_unscale_lane(uint64_t g, const int64_t* __restrict__ ids,
                                                  const uint64_t* __restrict__ goffs, uint64_t n_groups,
                                                  const uint32_t* __restrict__ ws, const int32_t* __restrict__ agg_inf,
                                                  const int32_t* __restrict__ status, uint8_t* __restrict__ out) {
  if (g >= n_groups) return;
  const int st = status[g];
  g2j acc;
  jac_set_inf(acc);
  if (st == HIPBLS_OK && !agg_inf[g]) {
    g2a a;
    soa_load<48>(&a.x.c0.v[0], ws + 72 * n_groups, n_groups, g);
    jac_from_aff(acc, a);
    const uint64_t g0 = goffs[g], g1 = goffs[g + 1];
    tagg_unscale(acc, ids + g0, (int)(g1 - g0));
  }
  uint8_t sig[96];
  g2_compress(sig, acc);
  for (int b = 0; b < 96; ++b) out[96 * g + b] = st == HIPBLS_OK ? sig[b] : (uint8_t)0;
}
__global__ void __launch_bounds__(kBlock) k_tagg_unscale(const int64_t* __restrict__ ids,
                                                         const uint64_t* __restrict__ goffs, uint64_t n_groups,
                                                         const uint32_t* __restrict__ ws,
                                                         const int32_t* __restrict__ agg_inf,
                                                         const int32_t* __restrict__ status, uint8_t* __restrict__ out) {
  tagg_unscale_lane(blockIdx.x * (uint64_t)blockDim.x + threadIdx.x, ids, goffs, n_groups, ws, agg_inf, status, out);
}

// Verify prep of the key side (one lane per group, beside the aggregation): decode + subgroup-check the
// validator's root pubkey, scale it by the group's L, hash its message; vstatus = ERR_PUBKEY / ERR_VERIFY (identity
// key) or pending.
__global__ void __launch_bounds__(kBlock) k_tv_prep_pk(const uint8_t* __restrict__ pks, const uint8_t* __restrict__ msgs,
                                                       const uint64_t* __restrict__ offs, uint64_t n,
                                                       const int64_t* __restrict__ ids,
                                                       const uint64_t* __restrict__ goffs,
                                                       uint32_t* __restrict__ ws, int32_t* __restrict__ vstatus) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  g1a pk;
  const int dp = g1_decompress(pk, pks + 48 * i, true);
  int st = RLC_PENDING;
  if (dp == DEC_BAD)
    st = HIPBLS_ERR_PUBKEY;
  else if (dp == DEC_INF)
    st = HIPBLS_ERR_VERIFY;
  if (st == RLC_PENDING) {
    const uint64_t g0 = goffs[i], g1 = goffs[i + 1];
    g1_scale_affine(pk, tagg_group_L(ids + g0, (int)(g1 - g0)));
    const uint64_t o0 = offs[i], o1 = offs[i + 1];
    g2j hj;
    hash_to_g2(hj, msgs + o0, (uint32_t)(o1 - o0), DST_POP, 43);
    g2a hm;
    jac_to_aff(hm, hj);
    soa_store<24>(ws, n, i, &pk.x.v[0]);
    soa_store<48>(ws + 24 * n, n, i, &hm.x.c0.v[0]);
  }
  vstatus[i] = st;
}

// k_tv_prep_pk with the roles split per workgroup, as k_verify_prep: the first grid_for(n) blocks decode and scale
// the keys (status, pk), the next 2 grid_for(n) blocks hash the messages on lane pairs (lg2.h hash_to_g2_pair), so the
// key decode runs beside the hash and each hash takes about half the latency.  Every message is hashed.
__device__ __forceinline__ void tv_prep_pk2_block(uint64_t blk, const uint8_t* __restrict__ pks,
                                                  const uint8_t* __restrict__ msgs, const uint64_t* __restrict__ offs,
                                                  uint64_t n, const int64_t* __restrict__ ids,
                                                  const uint64_t* __restrict__ goffs, uint32_t* __restrict__ ws,
                                                  int32_t* __restrict__ vstatus) {
  const uint64_t nb = (n + kBlock - 1) / kBlock;
  if (blk >= nb) {  // uniform per workgroup
    const uint64_t t = (blk - nb) * (uint64_t)blockDim.x + threadIdx.x;
    const uint64_t i = t >> 1;
    if (i >= n) return;  // same on both lanes of the pair
    const uint32_t m = (t & 1) ? ~0u : 0u;
    const uint64_t o0 = offs[i], o1 = offs[i + 1];
    g2j hj;
    hash_to_g2_pair(hj, msgs + o0, (uint32_t)(o1 - o0), DST_POP, 43, m);
    if (!m) {
      g2a hm;
      jac_to_aff(hm, hj);
      soa_store<48>(ws + 24 * n, n, i, &hm.x.c0.v[0]);
    }
    return;
  }
  const uint64_t i = blk * (uint64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  g1a pk;
  const int dp = g1_decompress(pk, pks + 48 * i, true);
  int st = RLC_PENDING;
  if (dp == DEC_BAD)
    st = HIPBLS_ERR_PUBKEY;
  else if (dp == DEC_INF)
    st = HIPBLS_ERR_VERIFY;
  if (st == RLC_PENDING) {
    const uint64_t g0 = goffs[i], g1 = goffs[i + 1];
    g1_scale_affine(pk, tagg_group_L(ids + g0, (int)(g1 - g0)));
    soa_store<24>(ws, n, i, &pk.x.v[0]);
  }
  vstatus[i] = st;
}
__global__ void __launch_bounds__(kBlock) k_tv_prep_pk2(const uint8_t* __restrict__ pks,
                                                        const uint8_t* __restrict__ msgs,
                                                        const uint64_t* __restrict__ offs, uint64_t n,
                                                        const int64_t* __restrict__ ids,
                                                        const uint64_t* __restrict__ goffs,
                                                        uint32_t* __restrict__ ws, int32_t* __restrict__ vstatus) {
  tv_prep_pk2_block(blockIdx.x, pks, msgs, offs, n, ids, goffs, ws, vstatus);
}

// sigagg in one call, phase A as ONE launch (roles per workgroup, uniform): workgroups [0, 3 grid_for(n)) are
// k_tv_prep_pk2's (key decode + [L] pk, then the lane-pair hashes), the rest k_tagg_scale's (one lane per partial).
// The prep's workgroups come first so they take their wave slots before the scaling's; with the check and the
// unscale also one launch (k_tv_check_unscale), a sigagg call is three kernels on the caller's stream and needs no
// sub-streams, so calls on different streams overlap (the next call's phase A in the check's idle SIMDs).
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(BLS_TAGG_WAVES, BLS_TAGG_WAVES)))
k_tv_phase_a(const uint8_t* __restrict__ pks, const uint8_t* __restrict__ msgs, const uint64_t* __restrict__ offs,
             uint64_t n, const int64_t* __restrict__ ids, const uint64_t* __restrict__ goffs,
             uint32_t* __restrict__ ws, int32_t* __restrict__ vstatus, const uint8_t* __restrict__ sigs,
             uint64_t n_parts, uint32_t* __restrict__ pts, int32_t* __restrict__ pstat) {
  const uint64_t nprep = 3 * ((n + kBlock - 1) / kBlock);
  if (blockIdx.x < nprep) {
    tv_prep_pk2_block(blockIdx.x, pks, msgs, offs, n, ids, goffs, ws, vstatus);
    return;
  }
  tagg_scale_lane((blockIdx.x - nprep) * (uint64_t)blockDim.x + threadIdx.x, sigs, ids, goffs, n, n_parts, pts,
                  pstat);
}

// Join: a group whose aggregation failed reports that status for its Verify too; otherwise the key's status
// stands (Verify checks the key first), and an aggregate at infinity is "signature not verified".
__global__ void __launch_bounds__(kBlock) k_tv_join(uint64_t n, const int32_t* __restrict__ astatus,
                                                    const int32_t* __restrict__ agg_inf, int32_t* __restrict__ vstatus) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (astatus[i] != HIPBLS_OK)
    vstatus[i] = astatus[i];
  else if (vstatus[i] == RLC_PENDING && agg_inf[i])
    vstatus[i] = HIPBLS_ERR_VERIFY;
}

// sigagg's pairing check on lane quads beside [L^-1] S (roles per workgroup, uniform): workgroups [0, grid_for(4 n))
// run k_verify_pair_lq4's lanes, the rest k_tagg_unscale's.  Both only read ws.
__global__ void __launch_bounds__(kBlock) k_tv_check_unscale(const uint32_t* __restrict__ ws, uint64_t n,
                                                             int32_t* __restrict__ vstatus,
                                                             const int64_t* __restrict__ ids,
                                                             const uint64_t* __restrict__ goffs,
                                                             const int32_t* __restrict__ agg_inf,
                                                             const int32_t* __restrict__ astatus,
                                                             uint8_t* __restrict__ out) {
  const uint64_t nq = (4 * n + kBlock - 1) / kBlock;
  if (blockIdx.x < nq) {
    verify_pair_lq4_lane(blockIdx.x * (uint64_t)blockDim.x + threadIdx.x, ws, n, vstatus);
    return;
  }
  tagg_unscale_lane((blockIdx.x - nq) * (uint64_t)blockDim.x + threadIdx.x, ids, goffs, n, ws, agg_inf, astatus, out);
}

// One lane per item on the lane-pair Verify layout (for batches too large for lane pairs).
__global__ void __launch_bounds__(kBlock) k_verify_pair_single(const uint32_t* __restrict__ ws, uint64_t n,
                                                               int32_t* __restrict__ status) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (i >= n || status[i] != RLC_PENDING) return;
  g1a pk;
  g2a hm, sig;
  soa_load<24>(&pk.x.v[0], ws, n, i);
  soa_load<48>(&hm.x.c0.v[0], ws + 24 * n, n, i);
  soa_load<48>(&sig.x.c0.v[0], ws + 72 * n, n, i);
  BLS_LANE_F12(F);
  status[i] = pairing_check_verify_l(pk, hm, sig, F) ? HIPBLS_OK : HIPBLS_ERR_VERIFY;
}

// G1 decode of many public keys (FastAggregateVerify): affine SoA (24 words) + code per key
__global__ void __launch_bounds__(kBlock) k_g1_decode(const uint8_t* __restrict__ pks, uint64_t n,
                                                      uint32_t* __restrict__ pts, int32_t* __restrict__ code) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  g1a a;
  const int st = g1_decompress(a, pks + 48 * i, true);
  const uint32_t* src = &a.x.v[0];
  for (int w = 0; w < 24; ++w) pts[(uint64_t)w * n + i] = st == DEC_OK ? src[w] : 0u;
  code[i] = st;
}

// FastAggregateVerify (tbls/herumi.go:315-339), one workgroup of two waves per group g over keys
// [goff[g], goff[g+1]) decoded by k_g1_decode: wave 0 sums the keys (strided, then an LDS tree),
// wave 1 meanwhile decodes the signature and hashes the message; lane 0 then runs the pairing.
// Status order follows the reference: signature decode error, then key decode error, then
// "signature verification failed" (also for an empty key list, an infinity key or signature).
constexpr int kFavBlock = 128;
__global__ void __launch_bounds__(kFavBlock) k_fav_batch(const uint32_t* __restrict__ pts,
                                                         const int32_t* __restrict__ code, uint64_t nkeys,
                                                         const uint64_t* __restrict__ goff,
                                                         const uint8_t* __restrict__ sigs,
                                                         const uint8_t* __restrict__ msgs,
                                                         const uint64_t* __restrict__ moffs,
                                                         int32_t* __restrict__ status) {
  __shared__ uint32_t red[64 * 36];
  __shared__ uint32_t sh_sig[48], sh_hm[48];
  __shared__ int sh_ds, sh_bad, sh_inf;
  const uint64_t g = blockIdx.x;
  const uint64_t k0 = goff[g], k1 = goff[g + 1];
  const int tid = threadIdx.x;
  if (tid == 0) {
    sh_bad = 0;
    sh_inf = 0;
  }
  __syncthreads();
  if (tid < 64) {
    g1j acc;
    jac_set_inf(acc);
    int bad = 0, inf = 0;
    for (uint64_t k = k0 + tid; k < k1; k += 64) {
      const int c = code[k];
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
    for (int w = 0; w < 36; ++w) red[w * 64 + tid] = (&acc.x.v[0])[w];
  } else if (tid == 64) {
    g2a sg;
    const int ds = g2_decompress(sg, sigs + 96 * g, true);
    sh_ds = ds;
    g2a hm;
    if (ds == DEC_OK) {
      g2j hj;
      const uint64_t o0 = moffs[g], o1 = moffs[g + 1];
      hash_to_g2(hj, msgs + o0, (uint32_t)(o1 - o0), DST_POP, 43);
      jac_to_aff(hm, hj);
    } else {
      fp2_set_zero(sg.x);
      fp2_set_zero(sg.y);
      hm = sg;
    }
    for (int w = 0; w < 48; ++w) {
      sh_sig[w] = (&sg.x.c0.v[0])[w];
      sh_hm[w] = (&hm.x.c0.v[0])[w];
    }
  }
  __syncthreads();
  for (int half = 32; half >= 1; half >>= 1) {  // every thread reaches every barrier
    if (tid < half) {
      g1j x, y;
      for (int w = 0; w < 36; ++w) {
        (&x.x.v[0])[w] = red[w * 64 + tid];
        (&y.x.v[0])[w] = red[w * 64 + tid + half];
      }
      jac_add(x, x, y);
      for (int w = 0; w < 36; ++w) red[w * 64 + tid] = (&x.x.v[0])[w];
    }
    __syncthreads();
  }
  // lanes 0 and 1 finish as a pair (lg2.h): e(pk, H(m)) on lane 0 and e(-g1, sig) on lane 1, split final
  // exponentiation; every branch below depends on shared values only, so the pair stays together
  if (tid >= 2) return;
  const uint32_t lm = tid ? ~0u : 0u;
  int st;
  if (sh_ds == DEC_BAD) {
    st = HIPBLS_ERR_SIGNATURE;
  } else if (sh_bad) {
    st = HIPBLS_ERR_PUBKEY;
  } else if (k1 == k0 || sh_ds == DEC_INF || sh_inf) {
    st = HIPBLS_ERR_VERIFY;  // KeyValidate rejects the identity key; empty set is false [ext]
  } else {
    g1j sum;
    for (int w = 0; w < 36; ++w) (&sum.x.v[0])[w] = red[w * 64];
    if (jac_is_inf(sum)) {
      st = HIPBLS_ERR_VERIFY;
    } else {
      g1a pk;
      jac_to_aff(pk, sum);
      g2a sg, hm;
      for (int w = 0; w < 48; ++w) {
        (&sg.x.c0.v[0])[w] = sh_sig[w];
        (&hm.x.c0.v[0])[w] = sh_hm[w];
      }
      const bool ok = pairing_check_lg2<1>(2, lm, [&](int k, g1a& P, g2a& Q) {
        if (k == 0) {
          P = pk;
          Q = hm;
        } else {
          P.x = G1_GEN_X;
          P.y = G1_NEG_GEN_Y;
          Q = sg;
        }
      });
      st = ok ? HIPBLS_OK : HIPBLS_ERR_VERIFY;
    }
  }
  if (tid == 0) status[g] = st;
}

// Aggregate (tbls/herumi.go:220-242): sum of n signatures in G2.  Stage 1 decodes every signature in parallel
// (k_g2_decode: affine SoA + DEC_* code), stage 2 sums: each workgroup of kSumBlock lanes folds a strided
// slice and reduces it through an LDS tree to one Jacobian partial; stage 3 (one workgroup) sums the partials
// the same way and compresses.  herumi fails on the first signature that does not deserialize; every other
// outcome -- including n = 0, where sig.Aggregate leaves the zero point -- serializes the sum, so the empty
// aggregate is the infinity encoding 0xc0 || 0^95 with no error.
constexpr int kSumBlock = 256;
__global__ void __launch_bounds__(kBlock) k_g2_decode(const uint8_t* __restrict__ sigs, uint64_t n,
                                                      uint32_t* __restrict__ pts, int32_t* __restrict__ code) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  g2a a;
  const int st = g2_decompress(a, sigs + 96 * i, true);
  const uint32_t* src = &a.x.c0.v[0];
  for (int w = 0; w < 48; ++w) pts[(uint64_t)w * n + i] = st == DEC_OK ? src[w] : 0u;
  code[i] = st;
}

// LDS tree over kSumBlock Jacobian points; every thread reaches every barrier.  Returns the sum in thread 0.
__device__ void g2_block_tree_sum(g2j& acc, uint32_t* red) {
  const int tid = threadIdx.x;
  for (int w = 0; w < 72; ++w) red[w * kSumBlock + tid] = (&acc.x.c0.v[0])[w];
  __syncthreads();
  for (int half = kSumBlock / 2; half >= 1; half >>= 1) {
    if (tid < half) {
      g2j x, y;
      for (int w = 0; w < 72; ++w) {
        (&x.x.c0.v[0])[w] = red[w * kSumBlock + tid];
        (&y.x.c0.v[0])[w] = red[w * kSumBlock + tid + half];
      }
      jac_add(x, x, y);
      for (int w = 0; w < 72; ++w) red[w * kSumBlock + tid] = (&x.x.c0.v[0])[w];
    }
    __syncthreads();
  }
  for (int w = 0; w < 72; ++w) (&acc.x.c0.v[0])[w] = red[w * kSumBlock];
}

// Stage 2: workgroup b folds points b, b + stride, ... (stride = gridDim.x * kSumBlock) into partial b
// (Jacobian, 72 words, SoA over the grid); bad[0] |= 1 when any code is DEC_BAD.
__global__ void __launch_bounds__(kSumBlock) k_g2_sum_partial(const uint32_t* __restrict__ pts,
                                                              const int32_t* __restrict__ code, uint64_t n,
                                                              uint32_t* __restrict__ part, int32_t* __restrict__ bad) {
  __shared__ uint32_t red[72 * kSumBlock];
  g2j acc;
  jac_set_inf(acc);
  int my_bad = 0;
  const uint64_t stride = (uint64_t)gridDim.x * kSumBlock;
  for (uint64_t i = blockIdx.x * (uint64_t)kSumBlock + threadIdx.x; i < n; i += stride) {
    const int c = code[i];
    if (c == DEC_BAD) {
      my_bad = 1;
    } else if (c == DEC_OK) {
      g2a a;
      soa_load<48>(&a.x.c0.v[0], pts, n, i);
      jac_add_aff(acc, acc, a);
    }
  }
  if (my_bad) atomicOr(bad, 1);
  g2_block_tree_sum(acc, red);
  if (threadIdx.x == 0) soa_store<72>(part, gridDim.x, blockIdx.x, &acc.x.c0.v[0]);
}

// Stage 3: one workgroup sums the np partials and writes the 96-byte encoding + status.
__global__ void __launch_bounds__(kSumBlock) k_g2_sum_final(const uint32_t* __restrict__ part, uint64_t np,
                                                            const int32_t* __restrict__ bad, uint8_t* __restrict__ out,
                                                            int32_t* __restrict__ status) {
  __shared__ uint32_t red[72 * kSumBlock];
  g2j acc;
  jac_set_inf(acc);
  for (uint64_t i = threadIdx.x; i < np; i += kSumBlock) {
    g2j p;
    soa_load<72>(&p.x.c0.v[0], part, np, i);
    jac_add(acc, acc, p);
  }
  g2_block_tree_sum(acc, red);
  if (threadIdx.x != 0) return;
  if (*bad) {
    for (int b = 0; b < 96; ++b) out[b] = 0;
    *status = HIPBLS_ERR_SIGNATURE;
    return;
  }
  uint8_t sig[96];
  g2_compress(sig, acc);
  for (int b = 0; b < 96; ++b) out[b] = sig[b];
  *status = HIPBLS_OK;
}

// Shamir shares: lane i-1 evaluates share_i = sum_j poly_j i^j (Horner over Fr)
__global__ void __launch_bounds__(kBlock) k_threshold_split(const uint8_t* __restrict__ secret, const uint8_t* __restrict__ tail,
                                  uint32_t total, uint32_t threshold, uint8_t* __restrict__ out,
                                  int32_t* __restrict__ status) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  fr coef, acc, x, r2;
  for (int w = 0; w < 8; ++w) r2.v[w] = FR_R2[w];
  fr_from_u32(x, i + 1);
  bool ok = true;
  for (int w = 0; w < 8; ++w) acc.v[w] = 0;
  for (int j = (int)threshold - 1; j >= 0; --j) {
    const uint8_t* c = j == 0 ? secret : tail + 32 * (j - 1);
    if (!fr_plain_from_be32(coef, c)) ok = false;
    fr_mul(coef, coef, r2);  // to Montgomery
    fr_mul(acc, acc, x);
    fr_add(acc, acc, coef);
  }
  fr plain;
  fr_to_plain(plain, acc);
  for (int w = 0; w < 8; ++w)
    for (int b = 0; b < 4; ++b) out[32 * i + 31 - 4 * w - b] = ok ? (uint8_t)(plain.v[w] >> (8 * b)) : (uint8_t)0;
  if (i == 0) *status = ok ? HIPBLS_OK : HIPBLS_ERR_SECRET;
}

__global__ void __launch_bounds__(kBlock) k_recover_secret(const uint8_t* __restrict__ shares, const int64_t* __restrict__ ids, uint32_t n,
                                 uint8_t* __restrict__ out, int32_t* __restrict__ status) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  int st = n > 0 ? HIPBLS_OK : HIPBLS_ERR_COMBINE;
  for (uint32_t a = 0; a < n; ++a) {
    if (ids[a] == 0) st = HIPBLS_ERR_COMBINE;
    for (uint32_t b = a + 1; b < n; ++b)
      if (ids[a] == ids[b]) st = HIPBLS_ERR_COMBINE;
  }
  fr acc, r2;
  for (int w = 0; w < 8; ++w) {
    acc.v[w] = 0;
    r2.v[w] = FR_R2[w];
  }
  for (uint32_t k = 0; k < n && st == HIPBLS_OK; ++k) {
    fr s, lam;
    if (!fr_plain_from_be32(s, shares + 32 * k)) {
      st = HIPBLS_ERR_SECRET;
      break;
    }
    lagrange_at_zero(lam, ids, (int)n, (int)k);  // plain
    fr_mul(lam, lam, r2);
    fr_mul(s, s, r2);
    fr_mul(s, s, lam);
    fr_add(acc, acc, s);
  }
  fr plain;
  fr_to_plain(plain, acc);
  for (int w = 0; w < 8; ++w)
    for (int b = 0; b < 4; ++b)
      out[31 - 4 * w - b] = st == HIPBLS_OK ? (uint8_t)(plain.v[w] >> (8 * b)) : (uint8_t)0;
  *status = st;
}


// ---------------------------------------------------------------- RLC BatchVerify (rlc.h)
// The four stages run per sub-batch (a contiguous, window-aligned item range) so that several
// sub-batches' stages overlap on separate streams (launch_rlc).
// Stages 1 and 2 (k_rlc_items, k_rlc_hash) and the batch-wide check's stage 1 (k_rlcb_items) live in rlc_wide.hip:
// their own translation unit, compiled for two waves per SIMD.
// Stage 3: one lane per window of RLC_W items -> one multi-pairing check.  The items a failed window
// leaves pending are appended to this sub-batch's fallback list (one atomic per failed window), so
// stage 4 runs on a dense list instead of waking a wave for every scattered pending item.
// Windows from wdirect on (the launches' partial last waves, when those would start another round of waves on a full
// device: hipbls.hip launch_rlc) skip the check and send their pending items straight to stage 4, recorded as
// win_fail[w] = -(items sent) so the statistics count them as re-checked items, not failed windows.
__global__ void __launch_bounds__(kBlock) k_rlc_window(uint64_t w0, uint64_t w1, uint64_t n,
                                                       const uint32_t* __restrict__ msg_idx,
                                                       const uint32_t* __restrict__ rpk,
                                                       const uint32_t* __restrict__ rsig,
                                                       const uint32_t* __restrict__ H, uint64_t hstride,
                                                       const uint32_t* __restrict__ hslot,
                                                       int32_t* __restrict__ status, int32_t* __restrict__ win_fail,
                                                       uint32_t* __restrict__ list, uint32_t* __restrict__ list_len,
                                                       uint64_t wdirect) {
  const uint64_t w = w0 + blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (w >= w1) return;
  const uint64_t i1 = w * RLC_W + RLC_W < n ? w * RLC_W + RLC_W : n;
  int left;
  if (w >= wdirect) {
    left = 0;
    for (uint64_t i = w * RLC_W; i < i1; ++i) left += status[i] == RLC_PENDING ? 1 : 0;
    win_fail[w] = -left;
  } else {
    BLS_LANE_F12(F);
    left = rlc_window_lane(F, w, n, msg_idx, rpk, rsig, H, hstride, hslot, status, win_fail);
  }
  if (left == 0) return;
  uint32_t at = atomicAdd(list_len, (uint32_t)left);
  for (uint64_t i = w * RLC_W; i < i1; ++i)
    if (status[i] == RLC_PENDING) list[at++] = (uint32_t)i;
}

// Stage 3 on lane pairs (lg2.h rlc_window_lg2): lanes 2v and 2v+1 share window w0 + v; the even lane records
// the verdict.
__global__ void __launch_bounds__(kBlock) k_rlc_window_lg2(uint64_t w0, uint64_t w1, uint64_t n,
                                                           const uint32_t* __restrict__ msg_idx,
                                                           const uint32_t* __restrict__ rpk,
                                                           const uint32_t* __restrict__ rsig,
                                                           const uint32_t* __restrict__ H, uint64_t hstride,
                                                           const uint32_t* __restrict__ hslot,
                                                           int32_t* __restrict__ status, int32_t* __restrict__ win_fail,
                                                           uint32_t* __restrict__ list, uint32_t* __restrict__ list_len) {
  const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  const uint64_t w = w0 + (t >> 1);
  const uint32_t m = (t & 1) ? ~0u : 0u;
  if (w >= w1) return;
  const uint64_t i0 = w * RLC_W;
  const uint64_t i1 = i0 + RLC_W < n ? i0 + RLC_W : n;
  auto load_pk = [&](g1j& q, uint64_t i) { soa_load<36>(&q.x.v[0], rpk, n, i); };
  auto load_sig = [&](g2j& q, uint64_t i) { soa_load<72>(&q.x.c0.v[0], rsig, n, i); };
  auto load_h = [&](g2a& q, uint32_t mi) { soa_load<48>(&q.x.c0.v[0], H, hstride, h_col(hslot, mi)); };
  const bool ok = rlc_window_lg2(i0, i1, status, msg_idx, load_pk, load_sig, load_h, m);
  if (m) return;
  int left = 0;
  for (uint64_t i = i0; i < i1; ++i)
    if (status[i] == RLC_PENDING) {
      if (ok)
        status[i] = HIPBLS_OK;
      else
        ++left;
    }
  win_fail[w] = left;
  if (left == 0) return;
  uint32_t at = atomicAdd(list_len, (uint32_t)left);
  for (uint64_t i = i0; i < i1; ++i)
    if (status[i] == RLC_PENDING) list[at++] = (uint32_t)i;
}

// Stage 4: items of failed windows (dense list) are checked one by one (rlc_fallback_lane).
// Stage 4 over the list of failed-window items: the bare 2-pair check per item.  The list length is known only on
// the device, so the host launches both layouts (one lane per item here, a lane pair per item below) and each kernel
// takes the lists on its side of pair_upto: pairs halve a check's latency while the list leaves lanes idle, one lane
// per item wins once pairs would need a second round of waves.  Same verdicts either way.
__global__ void __launch_bounds__(kBlock) k_rlc_fallback(const uint32_t* __restrict__ list,
                                                         const uint32_t* __restrict__ list_len, uint64_t cap,
                                                         const uint8_t* __restrict__ pks, const uint8_t* __restrict__ sigs,
                                                         const uint32_t* __restrict__ msg_idx,
                                                         const uint32_t* __restrict__ H, uint64_t hstride,
                                                         const uint32_t* __restrict__ hslot,
                                                         int32_t* __restrict__ status,
                                                         const uint32_t* __restrict__ key_idx, uint64_t T,
                                                         const uint32_t* __restrict__ tab, uint64_t pair_upto,
                                                         const uint32_t* __restrict__ rpk,
                                                         const uint32_t* __restrict__ rsig, uint64_t n) {
  const uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  const uint64_t len = *list_len;
  if (len <= pair_upto) return;  // k_rlc_fallback_lg2 takes short lists
  if (j >= len || j >= cap) return;
  BLS_LANE_F12(F);
  rlc_fallback_lane(F, list[j], pks, sigs, msg_idx, H, hstride, hslot, status, key_idx, T, tab, rpk, rsig, n);
}

// The lane-pair layout (lg2.h): the even lane decodes the key and takes e(pk, H(m)), the odd lane decodes the
// signature and takes e(-g1, sig); the final exponentiation is split.
__global__ void __launch_bounds__(kBlock) k_rlc_fallback_lg2(const uint32_t* __restrict__ list,
                                                             const uint32_t* __restrict__ list_len, uint64_t cap,
                                                             const uint8_t* __restrict__ pks,
                                                             const uint8_t* __restrict__ sigs,
                                                             const uint32_t* __restrict__ msg_idx,
                                                             const uint32_t* __restrict__ H, uint64_t hstride,
                                                             const uint32_t* __restrict__ hslot,
                                                             int32_t* __restrict__ status,
                                                             const uint32_t* __restrict__ key_idx, uint64_t T,
                                                             const uint32_t* __restrict__ tab, uint64_t pair_upto,
                                                             const uint32_t* __restrict__ rpk,
                                                             const uint32_t* __restrict__ rsig, uint64_t n) {
  const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  const uint64_t j = t >> 1;
  const uint32_t m = (t & 1) ? ~0u : 0u;
  const uint64_t len = *list_len;
  if (len > pair_upto) return;  // a long list fills the GPU one lane per item (k_rlc_fallback)
  if (j >= len || j >= cap) return;
  const uint64_t i = list[j];
  if (status[i] != RLC_PENDING) return;
  g1a spk;
  g2a ssig;
  const bool scaled = rlc_scaled_pair(spk, ssig, rpk, rsig, n, i);  // the same decision on both lanes
  const bool ok = pairing_check_lg2<1>(2, m, [&](int k, g1a& P, g2a& Q) {
    if (k == 0) {
      if (scaled)
        P = spk;
      else if (pks)
        g1_decompress(P, pks + 48 * i, false);
      else
        soa_load<24>(&P.x.v[0], tab, T, key_idx[i]);
      soa_load<48>(&Q.x.c0.v[0], H, hstride, h_col(hslot, msg_idx[i]));
    } else {
      P.x = G1_GEN_X;
      P.y = G1_NEG_GEN_Y;
      if (scaled)
        Q = ssig;
      else
        g2_decompress(Q, sigs + 96 * i, false);
    }
  });
  if (!m) status[i] = ok ? HIPBLS_OK : HIPBLS_ERR_VERIFY;
}

// ---------------------------------------------------------------- batch-wide RLC check (rlcb.h)
// Stage 1 (k_rlcb_items): rlc_wide.hip.

// ---------------------------------------------------------------- the G1 MSM per large message (g1msm.h)
__global__ void __launch_bounds__(256) k_g1m_count(uint64_t n, const uint32_t* __restrict__ msg_idx, uint64_t n_msgs,
                                                   uint32_t* __restrict__ cnt) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (i < n && msg_idx[i] < n_msgs) atomicAdd(&cnt[msg_idx[i]], 1u);
}

// g1msm.h g1m_plan_serial as one workgroup: each thread a contiguous range of messages, an LDS scan of the ranges'
// (large messages, slots) counts, then the same assignments in message order.
constexpr int kPlanThreads = 1024;
__global__ void __launch_bounds__(kPlanThreads) k_g1m_plan(const uint32_t* __restrict__ cnt, uint64_t n_msgs,
                                                           uint32_t min, uint32_t* __restrict__ lid,
                                                           uint32_t* __restrict__ lmsg, uint32_t* __restrict__ soff,
                                                           uint32_t* __restrict__ meta) {
  __shared__ uint32_t s_nl[kPlanThreads], s_tot[kPlanThreads];
  const int t = threadIdx.x;
  const uint64_t span = (n_msgs + kPlanThreads - 1) / kPlanThreads;
  const uint64_t m0 = t * span, m1 = m0 + span < n_msgs ? m0 + span : n_msgs;
  uint32_t nl = 0, tot = 0;
  for (uint64_t m = m0; m < m1; ++m)
    if (cnt[m] >= min) {
      ++nl;
      tot += cnt[m];
    }
  s_nl[t] = nl;
  s_tot[t] = tot;
  __syncthreads();
  if (t == 0) {  // serial exclusive scan of 1,024 pairs
    uint32_t a = 0, b = 0;
    for (int k = 0; k < kPlanThreads; ++k) {
      const uint32_t x = s_nl[k], y = s_tot[k];
      s_nl[k] = a;
      s_tot[k] = b;
      a += x;
      b += y;
    }
    soff[a] = b;
    meta[0] = a;
    meta[1] = b;
  }
  __syncthreads();
  nl = s_nl[t];
  tot = s_tot[t];
  for (uint64_t m = m0; m < m1; ++m) {
    if (cnt[m] >= min) {
      lid[m] = nl;
      lmsg[nl] = (uint32_t)m;
      soff[nl] = tot;
      ++nl;
      tot += cnt[m];
    } else {
      lid[m] = G1M_NONE;
    }
  }
}

__global__ void __launch_bounds__(256) k_g1m_rank(uint64_t n, const uint32_t* __restrict__ msg_idx, uint64_t n_msgs,
                                                  const uint32_t* __restrict__ lid, const uint32_t* __restrict__ soff,
                                                  uint32_t* __restrict__ cursor, uint32_t* __restrict__ pos,
                                                  uint32_t* __restrict__ slot_l) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (i < n) g1m_rank_lane(i, msg_idx, n_msgs, lid, soff, cursor, pos, slot_l);
}

__global__ void __launch_bounds__(256) k_g1m_hist(uint64_t nslots, const uint32_t* __restrict__ meta,
                                                  const uint32_t* __restrict__ gsc, const uint32_t* __restrict__ slot_l,
                                                  uint32_t* __restrict__ bcnt) {
  const uint64_t s = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (s < nslots) g1m_hist_lane(s, meta, gsc, slot_l, bcnt);
}

__global__ void __launch_bounds__(256) k_g1m_scatter(uint64_t nslots, const uint32_t* __restrict__ meta,
                                                     const uint32_t* __restrict__ gsc,
                                                     const uint32_t* __restrict__ slot_l, uint32_t* __restrict__ bcur,
                                                     uint32_t* __restrict__ list) {
  const uint64_t s = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (s < nslots) g1m_scatter_lane(s, meta, gsc, slot_l, bcur, list);
}

__global__ void __launch_bounds__(kBlock) k_g1m_run(uint64_t nrun, const uint32_t* __restrict__ meta,
                                                    const uint32_t* __restrict__ boff, const uint32_t* __restrict__ list,
                                                    const uint32_t* __restrict__ gpts, uint64_t n,
                                                    uint32_t* __restrict__ B, uint32_t* __restrict__ P) {
  const uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (r < nrun) g1m_run_lane(r, meta, boff, list, gpts, n, B, P);
}

__global__ void __launch_bounds__(kBlock) k_g1m_fix(uint64_t nb, const uint32_t* __restrict__ meta,
                                                    const uint32_t* __restrict__ boff, uint32_t* __restrict__ B,
                                                    const uint32_t* __restrict__ P) {
  const uint64_t b = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (b < nb) g1m_fix_lane(b, meta, boff, B, P);
}

__global__ void __launch_bounds__(kBlock) k_g1m_fold(uint64_t nq, const uint32_t* __restrict__ meta,
                                                     const uint32_t* __restrict__ B, uint32_t* __restrict__ Wv) {
  const uint64_t q = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (q < nq) g1m_fold_lane(q, meta, B, Wv);
}


// ---- exclusive scan of n u32 counts (the G1 MSM's buckets): block sums, one-workgroup scan of them, block scans
constexpr int kScanBlk = 1024;
__global__ void __launch_bounds__(kScanBlk) k_scan_part(const uint32_t* __restrict__ in, uint64_t n,
                                                        uint32_t* __restrict__ part) {
  __shared__ uint32_t red[kScanBlk];
  const uint64_t i = blockIdx.x * (uint64_t)kScanBlk + threadIdx.x;
  red[threadIdx.x] = i < n ? in[i] : 0u;
  __syncthreads();
  for (int h = kScanBlk / 2; h > 0; h >>= 1) {
    if ((int)threadIdx.x < h) red[threadIdx.x] += red[threadIdx.x + h];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}
__global__ void __launch_bounds__(kScanBlk) k_scan_top(uint32_t* __restrict__ part, uint64_t nparts) {
  __shared__ uint32_t s[kScanBlk];
  const uint64_t span = (nparts + kScanBlk - 1) / kScanBlk;
  const uint64_t p0 = threadIdx.x * span, p1 = p0 + span < nparts ? p0 + span : nparts;
  uint32_t sum = 0;
  for (uint64_t p = p0; p < p1; ++p) sum += part[p];
  s[threadIdx.x] = sum;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t a = 0;
    for (int k = 0; k < kScanBlk; ++k) {
      const uint32_t x = s[k];
      s[k] = a;
      a += x;
    }
    part[nparts] = a;
  }
  __syncthreads();
  uint32_t a = s[threadIdx.x];
  for (uint64_t p = p0; p < p1; ++p) {
    const uint32_t x = part[p];
    part[p] = a;
    a += x;
  }
}
// out[i] = exclusive prefix (and cur[i] a copy); out[n] = the total
__global__ void __launch_bounds__(kScanBlk) k_scan_apply(const uint32_t* __restrict__ in, uint64_t n,
                                                         const uint32_t* __restrict__ part, uint64_t nparts,
                                                         uint32_t* __restrict__ out, uint32_t* __restrict__ cur) {
  __shared__ uint32_t s[kScanBlk];
  const uint64_t i = blockIdx.x * (uint64_t)kScanBlk + threadIdx.x;
  const uint32_t v = i < n ? in[i] : 0u;
  s[threadIdx.x] = v;
  __syncthreads();
  for (int d = 1; d < kScanBlk; d <<= 1) {  // Hillis-Steele inclusive scan
    const uint32_t x = (int)threadIdx.x >= d ? s[threadIdx.x - d] : 0u;
    __syncthreads();
    s[threadIdx.x] += x;
    __syncthreads();
  }
  if (i < n) {
    const uint32_t e = part[blockIdx.x] + s[threadIdx.x] - v;
    out[i] = e;
    cur[i] = e;
  }
  if (i == 0) out[n] = part[nparts];
}

__global__ void __launch_bounds__(256) k_msm_hist(uint64_t npts, const uint32_t* __restrict__ sc,
                                                  uint32_t* __restrict__ cnt) {
  const uint64_t p = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (p < npts) msm_hist_lane(p, sc, cnt);
}

// Exclusive scan of the MSM_WINDOWS x MSM_NB digit counts: one workgroup of 1024 threads, 512 per window, each
// owning 128 consecutive buckets.  off gets MSM_NB + 1 entries per window (the last is the window's total), cursor
// the same offsets as the scatter's write positions.
constexpr int kScanThreads = 1024;
__global__ void __launch_bounds__(kScanThreads) k_msm_scan(const uint32_t* __restrict__ cnt, uint32_t* __restrict__ off,
                                                           uint32_t* __restrict__ cursor) {
  constexpr int per_w = kScanThreads / MSM_WINDOWS;            // threads per window
  constexpr uint32_t span = MSM_NB / per_w;                    // buckets per thread
  __shared__ uint32_t part[kScanThreads];
  const int t = threadIdx.x;
  const int w = t / per_w;
  const uint32_t j0 = (uint32_t)(t % per_w) * span;
  uint32_t sum = 0;
  for (uint32_t k = 0; k < span; ++k) sum += cnt[w * MSM_NB + j0 + k];
  part[t] = sum;
  __syncthreads();
  if (t % per_w == 0) {  // serial scan of this window's 512 partial sums
    uint32_t acc = 0;
    for (int k = 0; k < per_w; ++k) {
      const uint32_t v = part[t + k];
      part[t + k] = acc;
      acc += v;
    }
    off[w * (MSM_NB + 1) + MSM_NB] = acc;
  }
  __syncthreads();
  uint32_t acc = part[t];
  for (uint32_t k = 0; k < span; ++k) {
    off[w * (MSM_NB + 1) + j0 + k] = acc;
    cursor[w * MSM_NB + j0 + k] = acc;
    acc += cnt[w * MSM_NB + j0 + k];
  }
}

__global__ void __launch_bounds__(256) k_msm_scatter(uint64_t npts, const uint32_t* __restrict__ sc,
                                                     uint32_t* __restrict__ cursor, uint32_t* __restrict__ list) {
  const uint64_t p = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (p < npts) msm_scatter_lane(p, sc, cursor, list, npts);
}

// Bucket sums: run lanes (MSM_RUN list entries each, rlcb.h msm_run_lane), then one lane per bucket for the buckets
// the runs cut (msm_fix_lane).
__global__ void __launch_bounds__(kBlock) k_msm_run(const uint32_t* __restrict__ off, const uint32_t* __restrict__ list,
                                                    uint64_t npts, const uint32_t* __restrict__ pts,
                                                    uint32_t* __restrict__ B, uint32_t* __restrict__ P, uint64_t lpw) {
  const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (t < (uint64_t)MSM_WINDOWS * lpw) msm_run_lane((uint32_t)(t / lpw), t % lpw, off, list, npts, pts, B, P, lpw);
}

__global__ void __launch_bounds__(kBlock) k_msm_fix(const uint32_t* __restrict__ off, uint32_t* __restrict__ B,
                                                    const uint32_t* __restrict__ P, uint64_t lpw) {
  const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (t < (uint64_t)MSM_WINDOWS * MSM_NB) msm_fix_lane((uint32_t)(t / MSM_NB), (uint32_t)(t % MSM_NB), off, B, P, lpw);
}

__global__ void __launch_bounds__(kBlock) k_msm_segment(const uint32_t* __restrict__ B, uint32_t* __restrict__ Sg) {
  const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (t < (uint64_t)MSM_WINDOWS * MSM_NSEG) msm_segment_lane((uint32_t)(t / MSM_NSEG), (uint32_t)(t % MSM_NSEG), B, Sg);
}

// Window sums in two steps, both latency-bound: MSM_WG workgroups per window each fold a strided share of the window's
// MSM_NSEG segment results (MSM_NSEG / (MSM_WG kSumBlock) additions per thread, then the LDS tree of g2_block_tree_sum)
// into Wp[w MSM_WG + b]; k_msm_wsum adds each window's MSM_WG partials into W[w] (72 contiguous words).
__global__ void __launch_bounds__(kSumBlock) k_msm_window(const uint32_t* __restrict__ Sg, uint32_t* __restrict__ Wp) {
  __shared__ uint32_t red[72 * kSumBlock];
  const uint32_t w = blockIdx.x / MSM_WG, b = blockIdx.x % MSM_WG;
  g2j acc;
  jac_set_inf(acc);
  for (uint32_t s = b * kSumBlock + threadIdx.x; s < MSM_NSEG; s += MSM_WG * kSumBlock) {
    g2j p;
    soa_load<72>(&p.x.c0.v[0], Sg, (uint64_t)MSM_WINDOWS * MSM_NSEG, (uint64_t)w * MSM_NSEG + s);
    g2j x = acc, y;
    jac_add_body(y, x, p);
    acc = y;
  }
  g2_block_tree_sum(acc, red);
  if (threadIdx.x == 0)
    for (int k = 0; k < 72; ++k) Wp[72 * blockIdx.x + k] = (&acc.x.c0.v[0])[k];
}

// One wave per window: lanes 0..MSM_WG-1 hold the partials, a log2(MSM_WG)-level tree through LDS.
__global__ void __launch_bounds__(64) k_msm_wsum(const uint32_t* __restrict__ Wp, uint32_t* __restrict__ W) {
  __shared__ uint32_t red[72 * MSM_WG];
  const uint32_t w = blockIdx.x, t = threadIdx.x;
  if (t < MSM_WG)
    for (int k = 0; k < 72; ++k) red[k * MSM_WG + t] = Wp[72 * (w * MSM_WG + t) + k];
  __syncthreads();
  for (int half = MSM_WG / 2; half >= 1; half >>= 1) {
    if (t < (uint32_t)half) {
      g2j x, y, z;
      for (int k = 0; k < 72; ++k) {
        (&x.x.c0.v[0])[k] = red[k * MSM_WG + t];
        (&y.x.c0.v[0])[k] = red[k * MSM_WG + t + half];
      }
      jac_add(z, x, y);
      for (int k = 0; k < 72; ++k) red[k * MSM_WG + t] = (&z.x.c0.v[0])[k];
    }
    __syncthreads();
  }
  if (t == 0)
    for (int k = 0; k < 72; ++k) W[72 * w + k] = red[k * MSM_WG];
}

// Stage 3: one lane per chunk, n_chunks lanes exactly (rlcb.h rlcb_chunk_count).  The (-g1, S) Miller value is NOT an
// extra lane here: at the bench's 1M items 65,536 chunks were exactly one wave per SIMD (four 36-KiB-LDS workgroups
// per CU) and one lane more made a 1,025th workgroup -- a second round of waves (profiles/r04: 41 ms for 28 ms of
// chunk work).  k_rlcb_sfactor8 (verify_lat.hip) computes it on the SIMD rlcb_chunk_count leaves free.
__global__ void __launch_bounds__(kBlock) k_rlcb_chunks(uint64_t n, const int32_t* __restrict__ status,
                                                        const uint32_t* __restrict__ msg_idx,
                                                        const uint32_t* __restrict__ rpk,
                                                        const uint32_t* __restrict__ H, uint64_t hstride,
                                                        const uint32_t* __restrict__ hslot, uint32_t* __restrict__ F,
                                                        uint64_t n_chunks, uint64_t fstride) {
  const uint64_t c = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  BLS_LANE_F12(Lf);
  if (c < n_chunks) rlcb_chunk_lane(Lf, c, n, status, msg_idx, rpk, H, hstride, hslot, F, n_chunks, fstride);
}

// Product of F's columns 64 at a time: workgroup g (one wave) multiplies columns [64 g, 64 g + 64) by a binary tree
// through LDS -- one Fp12 product of latency per level, six levels -- and lane 0 writes column g of Fout (missing
// columns count as 1).  65,472 chunk values take three launches and 16 products of latency, where fan-in-4 levels
// took eight launches and 24 (profiles/r04: 8 x 0.36 ms).
__global__ void __launch_bounds__(kBlock) k_fp12_prod64(const uint32_t* __restrict__ Fin, uint64_t nin,
                                                        uint32_t* __restrict__ Fout, uint64_t nout) {
  static_assert(kBlock == 64, "one wave per workgroup");
  __shared__ uint32_t s_x[144 * kBlock];
  const uint32_t lane = threadIdx.x;
  const uint64_t col = blockIdx.x * (uint64_t)kBlock + lane;
  fp12 acc;
  if (col < nin)
    soa_load<144>(&acc.c0.c0.c0.v[0], Fin, nin, col);
  else
    fp12_set_one(acc);
  for (uint32_t st = 1; st < (uint32_t)kBlock; st <<= 1) {
    for (int k = 0; k < 144; ++k) s_x[k * kBlock + lane] = (&acc.c0.c0.c0.v[0])[k];
    __syncthreads();
    if ((lane & (2 * st - 1)) == 0) {
      fp12 o;
      for (int k = 0; k < 144; ++k) (&o.c0.c0.c0.v[0])[k] = s_x[k * kBlock + lane + st];
      fp12 x = acc;
      fp12_mul(acc, x, o);
    }
    __syncthreads();
  }
  if (lane == 0) soa_store<144>(Fout, nout, blockIdx.x, &acc.c0.c0.c0.v[0]);
}



__global__ void __launch_bounds__(kBlock) k_rlcb_mark(uint64_t n, const int32_t* __restrict__ flag,
                                                      int32_t* __restrict__ status, const uint32_t* __restrict__ pts,
                                                      const uint32_t* __restrict__ sc, uint32_t* __restrict__ rsig,
                                                      const uint32_t* __restrict__ g1pos,
                                                      const uint32_t* __restrict__ gpts,
                                                      const uint32_t* __restrict__ gsc, uint32_t* __restrict__ rpk) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (i < n) rlcb_mark_lane(i, n, flag[0] != 0, status, pts, sc, rsig, g1pos, gpts, gsc, rpk);
}

// ---------------------------------------------------------------- resident pubshare table
// Load: one lane per pubshare -> decode + subgroup test once (app/app.go:343-381 builds the same set
// from the cluster lock at startup), keeping the affine key and [x] pk for the RLC scalars.
__global__ void __launch_bounds__(kBlock) k_pubtab_load(const uint8_t* __restrict__ pks, uint64_t T,
                                                        int32_t* __restrict__ code, uint32_t* __restrict__ tab,
                                                        int32_t* __restrict__ status) {
  const uint64_t k = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (k < T) status[k] = pubtab_load_lane(k, pks, T, code, tab);
}

// tbls.Verify with the key from the table: key_idx[i] >= T -> HIPBLS_ERR_ARG for that item.
__global__ void __launch_bounds__(kBlock) k_verify_keys(const uint32_t* __restrict__ key_idx, uint64_t T,
                                                        const int32_t* __restrict__ code,
                                                        const uint32_t* __restrict__ tab,
                                                        const uint8_t* __restrict__ msgs,
                                                        const uint64_t* __restrict__ offs,
                                                        const uint8_t* __restrict__ sigs, uint64_t n,
                                                        int32_t* __restrict__ status) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t k = key_idx[i];
  if (k >= T) {
    status[i] = HIPBLS_ERR_ARG;
    return;
  }
  g1a pk;
  g1j xpk;
  const int dp = pubtab_get(pk, xpk, k, T, code, tab);
  const uint64_t o0 = offs[i], o1 = offs[i + 1];
  BLS_LANE_F12(F);
  status[i] = op_verify_decoded_pk(dp, pk, msgs + o0, (uint32_t)(o1 - o0), sigs + 96 * i, F);
}

// ---------------------------------------------------------------- signing roots
// eth2util/signing.GetDataRoot (/root/reference/eth2util/signing/signing.go:57-69): the signing root is the SSZ
// hash_tree_root of SigningData{ObjectRoot, Domain}, two 32-byte leaves, i.e. SHA-256(object_root || domain).
// One lane per item writes the 32-byte message and its offset for the verify kernel.
__global__ void __launch_bounds__(kBlock) k_signing_roots(const uint8_t* __restrict__ roots,
                                                          const uint8_t* __restrict__ domains, uint64_t n,
                                                          uint8_t* __restrict__ out, uint64_t* __restrict__ offs) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (i > n) return;
  offs[i] = 32 * i;
  if (i == n) return;
  uint32_t w[16];
  for (int k = 0; k < 8; ++k) {
    const uint8_t* r = roots + 32 * i + 4 * k;
    const uint8_t* d = domains + 32 * i + 4 * k;
    w[k] = (uint32_t)r[0] << 24 | (uint32_t)r[1] << 16 | (uint32_t)r[2] << 8 | r[3];
    w[8 + k] = (uint32_t)d[0] << 24 | (uint32_t)d[1] << 16 | (uint32_t)d[2] << 8 | d[3];
  }
  sha256_state st;
  sha256_init(st);
  sha256_compress(st, w);
  for (int k = 0; k < 16; ++k) w[k] = 0;
  w[0] = 0x80000000u;
  w[15] = 512;
  sha256_compress(st, w);
  for (int k = 0; k < 8; ++k)
    for (int b = 0; b < 4; ++b) out[32 * i + 4 * k + b] = (uint8_t)(st.h[k] >> (24 - 8 * b));
}

// eth2util/signing.Verify rejects an all-zero signature before tbls.Verify (signing.go:99-102): that item's
// status becomes HIPBLS_ERR_ZERO_SIG whatever the pairing said.
__global__ void __launch_bounds__(kBlock) k_zero_sig_status(const uint8_t* __restrict__ sigs, uint64_t n,
                                                            int32_t* __restrict__ status) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t acc = 0;
  for (int b = 0; b < 96; ++b) acc |= sigs[96 * i + b];
  if (acc == 0) status[i] = HIPBLS_ERR_ZERO_SIG;
}

}  // namespace
