// hipbls: kernels + C-ABI host entry points (include/hipbls.h) for gfx950.
//
// Execution model: one process per GPU; within a process one context per device holding a HIP
// stream, reusable device workspaces and a mutex (the C-ABI is called concurrently from many
// goroutines in charon, tbls/tbls.go:79-141).  Host-buffer entry points copy in, launch, copy out
// and synchronize; *_device entry points only enqueue.
#include <hip/hip_runtime.h>

#include <atomic>
#include <map>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "ops.h"
#include "rlc.h"

using namespace bls;

// ============================================================================ kernels
namespace {

constexpr int kBlock = 64;  // one wave per workgroup: these kernels are register-bound, not LDS-bound

__global__ void __launch_bounds__(kBlock) k_verify_fused(const uint8_t* __restrict__ pks,
                                                         const uint8_t* __restrict__ msgs,
                                                         const uint64_t* __restrict__ offs,
                                                         const uint8_t* __restrict__ sigs, uint64_t n,
                                                         int32_t* __restrict__ status) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t o0 = offs[i], o1 = offs[i + 1];
  status[i] = op_verify(pks + 48 * i, msgs + o0, (uint32_t)(o1 - o0), sigs + 96 * i);
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
__global__ void __launch_bounds__(kBlock) k_tagg_scale(const uint8_t* __restrict__ sigs,
                                                       const uint32_t* __restrict__ ids,
                                                       const uint64_t* __restrict__ goffs, uint64_t n_groups,
                                                       uint64_t n_parts, uint32_t* __restrict__ pts,
                                                       int32_t* __restrict__ pstat) {
  const uint64_t k = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
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
  // ids must be non-zero and distinct within the group (herumi Recover fails otherwise)
  for (int a = 0; a < t; ++a) {
    if (ids[g0 + a] == 0) st = HIPBLS_ERR_COMBINE;
    for (int b = a + 1; b < t; ++b)
      if (ids[g0 + a] == ids[g0 + b]) st = HIPBLS_ERR_COMBINE;
  }
  g2a s;
  const int ds = g2_decompress(s, sigs + 96 * k, true);
  if (ds == DEC_BAD) st = HIPBLS_ERR_SIGNATURE;
  if (st == HIPBLS_OK && ds == DEC_OK) {
    fr lam;
    lagrange_at_zero(lam, ids + g0, t, me);
    g2j sj;
    jac_from_aff(sj, s);
    g2_mul_glv4(acc, sj, lam.v);
  }
  const uint32_t* src = &acc.x.c0.v[0];
  for (int w = 0; w < 72; ++w) pts[(uint64_t)w * n_parts + k] = src[w];
  pstat[k] = st;
}

// ThresholdAggregate, stage 2: one lane per group sums its scaled partials and compresses.
__global__ void __launch_bounds__(kBlock) k_tagg_sum(const uint32_t* __restrict__ pts,
                                                     const int32_t* __restrict__ pstat,
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
  }
  uint8_t sig[96];
  g2_compress(sig, acc);
  for (int b = 0; b < 96; ++b) out[96 * g + b] = st == HIPBLS_OK ? sig[b] : (uint8_t)0;
  status[g] = st;
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
  if (tid != 0) return;
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
      st = pairing_check_verify(pk, hm, sg) ? HIPBLS_OK : HIPBLS_ERR_VERIFY;
    }
  }
  status[g] = st;
}

__global__ void __launch_bounds__(kBlock) k_aggregate(const uint8_t* __restrict__ sigs, uint64_t n, uint8_t* __restrict__ out,
                            int32_t* __restrict__ status) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  if (n == 0) {
    *status = HIPBLS_ERR_COMBINE;
    return;
  }
  g2j acc;
  jac_set_inf(acc);
  for (uint64_t i = 0; i < n; ++i) {
    g2a s;
    const int ds = g2_decompress(s, sigs + 96 * i, true);
    if (ds == DEC_BAD) {
      *status = HIPBLS_ERR_SIGNATURE;
      return;
    }
    if (ds == DEC_OK) jac_add_aff(acc, acc, s);
  }
  g2_compress(out, acc);
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

__global__ void __launch_bounds__(kBlock) k_recover_secret(const uint8_t* __restrict__ shares, const uint32_t* __restrict__ ids, uint32_t n,
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
// Stage 1: one lane per item -> status (final or RLC_PENDING), [r_i] pk_i and [r_i] sig_i in SoA.
// pks == nullptr: public keys come from the resident pubshare table (key_idx, T, tcode, tab).
__global__ void __launch_bounds__(kBlock) k_rlc_items(uint64_t i0, uint64_t i1, const uint8_t* __restrict__ pks,
                                                      const uint8_t* __restrict__ sigs,
                                                      const uint32_t* __restrict__ msg_idx, uint64_t n,
                                                      uint64_t n_msgs, rlc_seed seed, uint32_t* __restrict__ rpk,
                                                      uint32_t* __restrict__ rsig, int32_t* __restrict__ status,
                                                      const uint32_t* __restrict__ key_idx, uint64_t T,
                                                      const int32_t* __restrict__ tcode,
                                                      const uint32_t* __restrict__ tab) {
  const uint64_t i = i0 + blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (i < i1) rlc_items_lane(i, pks, sigs, msg_idx, n, n_msgs, seed, rpk, rsig, status, key_idx, T, tcode, tab);
}

// Stage 2: one lane per distinct message -> H(m) in affine SoA (48 words).
__global__ void __launch_bounds__(kBlock) k_rlc_hash(const uint8_t* __restrict__ msgs, const uint64_t* __restrict__ offs,
                                                     uint64_t n_msgs, uint32_t* __restrict__ H) {
  const uint64_t m = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (m < n_msgs) rlc_hash_lane(m, msgs, offs, n_msgs, H);
}

// Stage 3: one lane per window of RLC_W items -> one multi-pairing check.  The items a failed window
// leaves pending are appended to this sub-batch's fallback list (one atomic per failed window), so
// stage 4 runs on a dense list instead of waking a wave for every scattered pending item.
__global__ void __launch_bounds__(kBlock) k_rlc_window(uint64_t w0, uint64_t w1, uint64_t n,
                                                       const uint32_t* __restrict__ msg_idx,
                                                       const uint32_t* __restrict__ rpk,
                                                       const uint32_t* __restrict__ rsig,
                                                       const uint32_t* __restrict__ H, uint64_t n_msgs,
                                                       int32_t* __restrict__ status, int32_t* __restrict__ win_fail,
                                                       uint32_t* __restrict__ list, uint32_t* __restrict__ list_len) {
  const uint64_t w = w0 + blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (w >= w1) return;
  const int left = rlc_window_lane(w, n, msg_idx, rpk, rsig, H, n_msgs, status, win_fail);
  if (left == 0) return;
  uint32_t at = atomicAdd(list_len, (uint32_t)left);
  const uint64_t i1 = w * RLC_W + RLC_W < n ? w * RLC_W + RLC_W : n;
  for (uint64_t i = w * RLC_W; i < i1; ++i)
    if (status[i] == RLC_PENDING) list[at++] = (uint32_t)i;
}

// Stage 4: items of failed windows (dense list) are checked one by one (rlc_fallback_lane).
__global__ void __launch_bounds__(kBlock) k_rlc_fallback(const uint32_t* __restrict__ list,
                                                         const uint32_t* __restrict__ list_len, uint64_t cap,
                                                         const uint8_t* __restrict__ pks, const uint8_t* __restrict__ sigs,
                                                         const uint32_t* __restrict__ msg_idx,
                                                         const uint32_t* __restrict__ H, uint64_t n_msgs,
                                                         int32_t* __restrict__ status,
                                                         const uint32_t* __restrict__ key_idx, uint64_t T,
                                                         const uint32_t* __restrict__ tab) {
  const uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  const uint64_t len = *list_len;
  if (j >= len || j >= cap) return;
  rlc_fallback_lane(list[j], pks, sigs, msg_idx, H, n_msgs, status, key_idx, T, tab);
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
  status[i] = op_verify_decoded_pk(dp, pk, msgs + o0, (uint32_t)(o1 - o0), sigs + 96 * i);
}

// ============================================================================ host runtime
thread_local std::string g_last_error;

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t n) {
    if (n <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    const size_t want = n < 4096 ? 4096 : n + n / 4;
    hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess) cap = want;
    return e;
  }
};

struct TimingSlot {
  std::vector<std::pair<hipEvent_t, hipEvent_t>> pending;
  double total_ms = 0;
  uint64_t launches = 0;
};

struct Context {
  int device = -1;
  hipStream_t stream = nullptr;
  std::mutex mu;
  DevBuf b_pk, b_msg, b_off, b_sig, b_st, b_out, b_ids, b_pts, b_pst, b_aux;
  DevBuf r_pk, r_sig, r_h, r_win, r_midx, r_list, r_cnt;  // RLC BatchVerify workspaces
  DevBuf t_code, t_tab, b_kidx;                            // resident pubshare table + key indices
  uint64_t t_size = 0;
  // RLC sub-batches in flight.  The process gets GPU_MAX_HW_QUEUES = 4 hardware queues, shared by
  // the caller's stream (which also hashes the messages), the library stream and these; a kernel
  // trace (profiles/r01_rlc_trace.txt) showed a third sub-stream landing on an occupied queue and
  // serializing behind it, so two sub-batches.
  static constexpr int kSub = 2;
  hipStream_t sub[kSub] = {};
  hipEvent_t ev_fork = nullptr, ev_hash = nullptr, ev_join[kSub] = {};
  uint64_t r_windows = 0;                  // window count of the last RLC call (hipbls_rlc_stats)
  std::map<std::string, TimingSlot> timing;  // per kernel name: HIP events on the launch stream
  bool timing_enabled = true;
};

Context g_ctx;
std::mutex g_init_mu;

int set_err(const char* what, hipError_t e) {
  g_last_error = std::string(what) + ": " + hipGetErrorString(e);
  return HIPBLS_ERR_DEVICE;
}

#define HIP_TRY(expr)                              \
  do {                                             \
    hipError_t _e = (expr);                        \
    if (_e != hipSuccess) return set_err(#expr, _e); \
  } while (0)

int ensure_init() {
  std::lock_guard<std::mutex> lk(g_init_mu);
  if (g_ctx.device >= 0) return HIPBLS_OK;
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess || ndev == 0) return set_err("hipGetDeviceCount (no GPU)", e == hipSuccess ? hipErrorNoDevice : e);
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  HIP_TRY(hipSetDevice(dev));
  HIP_TRY(hipStreamCreateWithFlags(&g_ctx.stream, hipStreamNonBlocking));
  g_ctx.device = dev;
  return HIPBLS_OK;
}

uint64_t grid_for(uint64_t n) { return (n + kBlock - 1) / kBlock; }

void drain_timing(TimingSlot& t) {
  for (auto& pr : t.pending) {
    float ms = 0;
    if (hipEventSynchronize(pr.second) == hipSuccess && hipEventElapsedTime(&ms, pr.first, pr.second) == hipSuccess) {
      t.total_ms += ms;
      t.launches += 1;
    }
    (void)hipEventDestroy(pr.first);
    (void)hipEventDestroy(pr.second);
  }
  t.pending.clear();
}

// Brackets one kernel launch with HIP events on its stream (bench.py roofline: the average
// duration per launch is read back through hipbls_kernel_timing).
template <class Launch>
int timed(const char* name, hipStream_t s, Launch launch) {
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (g_ctx.timing_enabled) {
    HIP_TRY(hipEventCreate(&e0));
    HIP_TRY(hipEventCreate(&e1));
    HIP_TRY(hipEventRecord(e0, s));
  }
  launch();
  HIP_TRY(hipGetLastError());
  if (g_ctx.timing_enabled) {
    HIP_TRY(hipEventRecord(e1, s));
    TimingSlot& t = g_ctx.timing[name];
    t.pending.emplace_back(e0, e1);
    if (t.pending.size() > 256) drain_timing(t);
  }
  return HIPBLS_OK;
}

int launch_verify(const uint8_t* d_pks, const uint8_t* d_msgs, const uint64_t* d_offs, const uint8_t* d_sigs,
                  uint64_t n, int32_t* d_status, hipStream_t s) {
  if (n == 0) return HIPBLS_OK;
  return timed("verify", s, [&] {
    hipLaunchKernelGGL(k_verify_fused, dim3((unsigned)grid_for(n)), dim3(kBlock), 0, s, d_pks, d_msgs, d_offs, d_sigs,
                       n, d_status);
  });
}

int ensure_rlc_streams() {
  Context& c = g_ctx;
  if (c.ev_fork) return HIPBLS_OK;
  for (int k = 0; k < Context::kSub; ++k) HIP_TRY(hipStreamCreateWithFlags(&c.sub[k], hipStreamNonBlocking));
  HIP_TRY(hipEventCreateWithFlags(&c.ev_hash, hipEventDisableTiming));
  for (int k = 0; k < Context::kSub; ++k) HIP_TRY(hipEventCreateWithFlags(&c.ev_join[k], hipEventDisableTiming));
  HIP_TRY(hipEventCreateWithFlags(&c.ev_fork, hipEventDisableTiming));
  return HIPBLS_OK;
}

// RLC BatchVerify: the batch is cut into up to kSub window-aligned sub-batches, each running
// items -> window -> fallback on its own stream, while the distinct messages are hashed on the
// caller's stream; windows wait only for the hash.  Every stage is latency-bound on its own (one lane per item
// at one wave per SIMD), so overlapping the sub-batches' stages is what fills the CUs.  The caller's
// stream `s` forks into the sub-streams and joins back, so the call stays stream-ordered.
int launch_rlc(const uint8_t* d_pks, const uint8_t* d_sigs, const uint32_t* d_midx, uint64_t n, const uint8_t* d_msgs,
               const uint64_t* d_offs, uint64_t n_msgs, const uint8_t* seed32, int32_t* d_status, hipStream_t s,
               const uint32_t* d_kidx = nullptr) {
  Context& c = g_ctx;
  // d_pks == nullptr: keys from the resident table
  const uint64_t T = c.t_size;
  const int32_t* tcode = (const int32_t*)c.t_code.p;
  const uint32_t* tab = (const uint32_t*)c.t_tab.p;
  c.r_windows = 0;
  if (n == 0) return HIPBLS_OK;
  if (n > 0xffffffffull) return HIPBLS_ERR_ARG;  // fallback list holds 32-bit item indices
  int rc = ensure_rlc_streams();
  if (rc) return rc;
  rlc_seed seed;
  for (int k = 0; k < 8; ++k)
    seed.w[k] = (uint32_t)seed32[4 * k] << 24 | (uint32_t)seed32[4 * k + 1] << 16 | (uint32_t)seed32[4 * k + 2] << 8 |
                (uint32_t)seed32[4 * k + 3];
  const uint64_t n_win = (n + RLC_W - 1) / RLC_W;
  HIP_TRY(c.r_pk.ensure(n * 36 * 4));
  HIP_TRY(c.r_sig.ensure(n * 72 * 4));
  HIP_TRY(c.r_h.ensure((n_msgs ? n_msgs : 1) * 48 * 4));
  HIP_TRY(c.r_win.ensure(n_win * 4));
  HIP_TRY(c.r_list.ensure(n * 4));
  HIP_TRY(c.r_cnt.ensure(Context::kSub * 4));
  uint32_t* rpk = (uint32_t*)c.r_pk.p;
  uint32_t* rsig = (uint32_t*)c.r_sig.p;
  uint32_t* H = (uint32_t*)c.r_h.p;
  int32_t* win = (int32_t*)c.r_win.p;
  uint32_t* list = (uint32_t*)c.r_list.p;
  uint32_t* cnt = (uint32_t*)c.r_cnt.p;
  // sub-batches of whole windows; small batches stay in one
  const uint64_t min_win = 2048;
  int nsub = (int)((n_win + min_win - 1) / min_win);
  if (nsub > Context::kSub) nsub = Context::kSub;
  if (nsub < 1) nsub = 1;
  const uint64_t win_per = (n_win + nsub - 1) / nsub;

  HIP_TRY(hipMemsetAsync(cnt, 0, Context::kSub * 4, s));
  HIP_TRY(hipEventRecord(c.ev_fork, s));
  hipStream_t hs = s;
  if (n_msgs) {
    rc = timed("rlc_hash", hs, [&] {
      hipLaunchKernelGGL(k_rlc_hash, dim3((unsigned)grid_for(n_msgs)), dim3(kBlock), 0, hs, d_msgs, d_offs, n_msgs, H);
    });
    if (rc) return rc;
  }
  HIP_TRY(hipEventRecord(c.ev_hash, hs));
  for (int k = 0; k < nsub; ++k) {
    hipStream_t ss = c.sub[k];
    const uint64_t w0 = win_per * k, w1 = w0 + win_per < n_win ? w0 + win_per : n_win;
    if (w0 >= w1) continue;
    const uint64_t i0 = w0 * RLC_W, i1 = w1 * RLC_W < n ? w1 * RLC_W : n;
    HIP_TRY(hipStreamWaitEvent(ss, c.ev_fork, 0));
    rc = timed("rlc_items", ss, [&] {
      hipLaunchKernelGGL(k_rlc_items, dim3((unsigned)grid_for(i1 - i0)), dim3(kBlock), 0, ss, i0, i1, d_pks, d_sigs,
                         d_midx, n, n_msgs, seed, rpk, rsig, d_status, d_kidx, T, tcode, tab);
    });
    if (rc) return rc;
    HIP_TRY(hipStreamWaitEvent(ss, c.ev_hash, 0));
    rc = timed("rlc_window", ss, [&] {
      hipLaunchKernelGGL(k_rlc_window, dim3((unsigned)grid_for(w1 - w0)), dim3(kBlock), 0, ss, w0, w1, n, d_midx,
                         (const uint32_t*)rpk, (const uint32_t*)rsig, (const uint32_t*)H, n_msgs, d_status, win,
                         list + i0, cnt + k);
    });
    if (rc) return rc;
    // the list length is only known on the device: launch for the worst case, idle lanes exit
    rc = timed("rlc_fallback", ss, [&] {
      hipLaunchKernelGGL(k_rlc_fallback, dim3((unsigned)grid_for(i1 - i0)), dim3(kBlock), 0, ss,
                         (const uint32_t*)(list + i0), (const uint32_t*)(cnt + k), i1 - i0, d_pks, d_sigs, d_midx,
                         (const uint32_t*)H, n_msgs, d_status, d_kidx, T, tab);
    });
    if (rc) return rc;
    HIP_TRY(hipEventRecord(c.ev_join[k], ss));
    HIP_TRY(hipStreamWaitEvent(s, c.ev_join[k], 0));
  }
  c.r_windows = n_win;
  return HIPBLS_OK;
}

int launch_tagg(const uint8_t* d_sigs, const uint32_t* d_ids, const uint64_t* d_goffs, uint64_t n_groups,
                uint64_t n_parts, uint8_t* d_out, int32_t* d_status, hipStream_t s) {
  if (n_groups == 0) return HIPBLS_OK;
  HIP_TRY(g_ctx.b_pts.ensure((n_parts ? n_parts : 1) * 72 * 4));
  HIP_TRY(g_ctx.b_pst.ensure((n_parts ? n_parts : 1) * 4));
  if (n_parts)
    hipLaunchKernelGGL(k_tagg_scale, dim3((unsigned)grid_for(n_parts)), dim3(kBlock), 0, s, d_sigs, d_ids, d_goffs,
                       n_groups, n_parts, (uint32_t*)g_ctx.b_pts.p, (int32_t*)g_ctx.b_pst.p);
  hipLaunchKernelGGL(k_tagg_sum, dim3((unsigned)grid_for(n_groups)), dim3(kBlock), 0, s,
                     (const uint32_t*)g_ctx.b_pts.p, (const int32_t*)g_ctx.b_pst.p, d_goffs, n_groups, n_parts,
                     d_out, d_status);
  HIP_TRY(hipGetLastError());
  return HIPBLS_OK;
}

bool mul_overflows(uint64_t a, uint64_t b) { return b != 0 && a > UINT64_MAX / b; }

}  // namespace

// ============================================================================ C-ABI
extern "C" {

int hipbls_abi_version(void) { return HIPBLS_ABI_VERSION; }

int hipbls_init(int device) {
  std::lock_guard<std::mutex> lk(g_init_mu);
  if (g_ctx.device >= 0) return g_ctx.device == device || device < 0 ? HIPBLS_OK : HIPBLS_ERR_ARG;
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess || ndev == 0) return set_err("hipGetDeviceCount (no GPU)", e == hipSuccess ? hipErrorNoDevice : e);
  if (device < 0) device = 0;
  if (device >= ndev) {
    g_last_error = "device index out of range";
    return HIPBLS_ERR_ARG;
  }
  HIP_TRY(hipSetDevice(device));
  HIP_TRY(hipStreamCreateWithFlags(&g_ctx.stream, hipStreamNonBlocking));
  g_ctx.device = device;
  return HIPBLS_OK;
}

int hipbls_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

const char* hipbls_last_error(void) { return g_last_error.c_str(); }

int hipbls_verify_batch(const uint8_t* pks, const uint8_t* msgs, const uint64_t* msg_offsets, const uint8_t* sigs,
                        uint64_t n, int32_t* status) {
  if (n == 0) return HIPBLS_OK;
  if (!pks || !msg_offsets || !sigs || !status || mul_overflows(n, 96)) return HIPBLS_ERR_ARG;
  const uint64_t msg_total = msg_offsets[n];
  if (msg_total && !msgs) return HIPBLS_ERR_ARG;
  for (uint64_t i = 0; i < n; ++i)
    if (msg_offsets[i + 1] < msg_offsets[i] || msg_offsets[i + 1] - msg_offsets[i] > 0xffffffffull)
      return HIPBLS_ERR_ARG;
  int rc = ensure_init();
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(g_ctx.mu);
  Context& c = g_ctx;
  HIP_TRY(c.b_pk.ensure(n * 48));
  HIP_TRY(c.b_sig.ensure(n * 96));
  HIP_TRY(c.b_msg.ensure(msg_total ? msg_total : 1));
  HIP_TRY(c.b_off.ensure((n + 1) * 8));
  HIP_TRY(c.b_st.ensure(n * 4));
  HIP_TRY(hipMemcpyAsync(c.b_pk.p, pks, n * 48, hipMemcpyHostToDevice, c.stream));
  HIP_TRY(hipMemcpyAsync(c.b_sig.p, sigs, n * 96, hipMemcpyHostToDevice, c.stream));
  if (msg_total) HIP_TRY(hipMemcpyAsync(c.b_msg.p, msgs, msg_total, hipMemcpyHostToDevice, c.stream));
  HIP_TRY(hipMemcpyAsync(c.b_off.p, msg_offsets, (n + 1) * 8, hipMemcpyHostToDevice, c.stream));
  rc = launch_verify((const uint8_t*)c.b_pk.p, (const uint8_t*)c.b_msg.p, (const uint64_t*)c.b_off.p,
                     (const uint8_t*)c.b_sig.p, n, (int32_t*)c.b_st.p, c.stream);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(status, c.b_st.p, n * 4, hipMemcpyDeviceToHost, c.stream));
  HIP_TRY(hipStreamSynchronize(c.stream));
  return HIPBLS_OK;
}

int hipbls_verify_batch_device(const uint8_t* d_pks, const uint8_t* d_msgs, const uint64_t* d_msg_offsets,
                               const uint8_t* d_sigs, uint64_t n, int32_t* d_status, void* stream) {
  int rc = ensure_init();
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(g_ctx.mu);
  return launch_verify(d_pks, d_msgs, d_msg_offsets, d_sigs, n, d_status,
                       stream ? (hipStream_t)stream : g_ctx.stream);
}

int hipbls_threshold_aggregate_batch(const uint8_t* sigs, const uint32_t* share_idx, const uint64_t* group_offsets,
                                     uint64_t n_groups, uint8_t* out_sigs, int32_t* status) {
  if (n_groups == 0) return HIPBLS_OK;
  if (!group_offsets || !out_sigs || !status) return HIPBLS_ERR_ARG;
  const uint64_t n_parts = group_offsets[n_groups] - group_offsets[0];
  if (group_offsets[0] != 0) return HIPBLS_ERR_ARG;
  for (uint64_t g = 0; g < n_groups; ++g)
    if (group_offsets[g + 1] < group_offsets[g]) return HIPBLS_ERR_ARG;
  if (n_parts && (!sigs || !share_idx)) return HIPBLS_ERR_ARG;
  int rc = ensure_init();
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(g_ctx.mu);
  Context& c = g_ctx;
  HIP_TRY(c.b_sig.ensure((n_parts ? n_parts : 1) * 96));
  HIP_TRY(c.b_ids.ensure((n_parts ? n_parts : 1) * 4));
  HIP_TRY(c.b_off.ensure((n_groups + 1) * 8));
  HIP_TRY(c.b_out.ensure(n_groups * 96));
  HIP_TRY(c.b_st.ensure(n_groups * 4));
  if (n_parts) {
    HIP_TRY(hipMemcpyAsync(c.b_sig.p, sigs, n_parts * 96, hipMemcpyHostToDevice, c.stream));
    HIP_TRY(hipMemcpyAsync(c.b_ids.p, share_idx, n_parts * 4, hipMemcpyHostToDevice, c.stream));
  }
  HIP_TRY(hipMemcpyAsync(c.b_off.p, group_offsets, (n_groups + 1) * 8, hipMemcpyHostToDevice, c.stream));
  rc = launch_tagg((const uint8_t*)c.b_sig.p, (const uint32_t*)c.b_ids.p, (const uint64_t*)c.b_off.p, n_groups,
                   n_parts, (uint8_t*)c.b_out.p, (int32_t*)c.b_st.p, c.stream);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(out_sigs, c.b_out.p, n_groups * 96, hipMemcpyDeviceToHost, c.stream));
  HIP_TRY(hipMemcpyAsync(status, c.b_st.p, n_groups * 4, hipMemcpyDeviceToHost, c.stream));
  HIP_TRY(hipStreamSynchronize(c.stream));
  return HIPBLS_OK;
}

int hipbls_threshold_aggregate_batch_device(const uint8_t* d_sigs, const uint32_t* d_share_idx,
                                            const uint64_t* d_group_offsets, uint64_t n_groups, uint8_t* d_out_sigs,
                                            int32_t* d_status, void* stream) {
  // the partial count is needed for the launch geometry: read the last offset (tiny D2H copy)
  if (n_groups == 0) return HIPBLS_OK;
  int rc = ensure_init();
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(g_ctx.mu);
  hipStream_t s = stream ? (hipStream_t)stream : g_ctx.stream;
  uint64_t n_parts = 0;
  HIP_TRY(hipMemcpyAsync(&n_parts, d_group_offsets + n_groups, 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  return launch_tagg(d_sigs, d_share_idx, d_group_offsets, n_groups, n_parts, d_out_sigs, d_status, s);
}

int hipbls_sign_batch(const uint8_t* sks, const uint8_t* msgs, const uint64_t* msg_offsets, uint64_t n,
                      uint8_t* out_sigs, int32_t* status) {
  if (n == 0) return HIPBLS_OK;
  if (!sks || !msg_offsets || !out_sigs || !status || mul_overflows(n, 96)) return HIPBLS_ERR_ARG;
  const uint64_t msg_total = msg_offsets[n];
  if (msg_total && !msgs) return HIPBLS_ERR_ARG;
  int rc = ensure_init();
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(g_ctx.mu);
  Context& c = g_ctx;
  HIP_TRY(c.b_pk.ensure(n * 32));
  HIP_TRY(c.b_msg.ensure(msg_total ? msg_total : 1));
  HIP_TRY(c.b_off.ensure((n + 1) * 8));
  HIP_TRY(c.b_out.ensure(n * 96));
  HIP_TRY(c.b_st.ensure(n * 4));
  HIP_TRY(hipMemcpyAsync(c.b_pk.p, sks, n * 32, hipMemcpyHostToDevice, c.stream));
  if (msg_total) HIP_TRY(hipMemcpyAsync(c.b_msg.p, msgs, msg_total, hipMemcpyHostToDevice, c.stream));
  HIP_TRY(hipMemcpyAsync(c.b_off.p, msg_offsets, (n + 1) * 8, hipMemcpyHostToDevice, c.stream));
  hipLaunchKernelGGL(k_sign, dim3((unsigned)grid_for(n)), dim3(kBlock), 0, c.stream, (const uint8_t*)c.b_pk.p,
                     (const uint8_t*)c.b_msg.p, (const uint64_t*)c.b_off.p, n, (uint8_t*)c.b_out.p,
                     (int32_t*)c.b_st.p);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(out_sigs, c.b_out.p, n * 96, hipMemcpyDeviceToHost, c.stream));
  HIP_TRY(hipMemcpyAsync(status, c.b_st.p, n * 4, hipMemcpyDeviceToHost, c.stream));
  HIP_TRY(hipStreamSynchronize(c.stream));
  return HIPBLS_OK;
}

int hipbls_sign_batch_device(const uint8_t* d_sks, const uint8_t* d_msgs, const uint64_t* d_msg_offsets, uint64_t n,
                             uint8_t* d_out_sigs, int32_t* d_status, void* stream) {
  if (n == 0) return HIPBLS_OK;
  int rc = ensure_init();
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(g_ctx.mu);
  hipStream_t s = stream ? (hipStream_t)stream : g_ctx.stream;
  hipLaunchKernelGGL(k_sign, dim3((unsigned)grid_for(n)), dim3(kBlock), 0, s, d_sks, d_msgs, d_msg_offsets, n,
                     d_out_sigs, d_status);
  HIP_TRY(hipGetLastError());
  return HIPBLS_OK;
}

int hipbls_secret_to_public_key_batch(const uint8_t* sks, uint64_t n, uint8_t* out_pks, int32_t* status) {
  if (n == 0) return HIPBLS_OK;
  if (!sks || !out_pks || !status || mul_overflows(n, 48)) return HIPBLS_ERR_ARG;
  int rc = ensure_init();
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(g_ctx.mu);
  Context& c = g_ctx;
  HIP_TRY(c.b_pk.ensure(n * 32));
  HIP_TRY(c.b_out.ensure(n * 48));
  HIP_TRY(c.b_st.ensure(n * 4));
  HIP_TRY(hipMemcpyAsync(c.b_pk.p, sks, n * 32, hipMemcpyHostToDevice, c.stream));
  hipLaunchKernelGGL(k_sk_to_pk, dim3((unsigned)grid_for(n)), dim3(kBlock), 0, c.stream, (const uint8_t*)c.b_pk.p, n,
                     (uint8_t*)c.b_out.p, (int32_t*)c.b_st.p);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(out_pks, c.b_out.p, n * 48, hipMemcpyDeviceToHost, c.stream));
  HIP_TRY(hipMemcpyAsync(status, c.b_st.p, n * 4, hipMemcpyDeviceToHost, c.stream));
  HIP_TRY(hipStreamSynchronize(c.stream));
  return HIPBLS_OK;
}

int hipbls_secret_to_public_key_batch_device(const uint8_t* d_sks, uint64_t n, uint8_t* d_out_pks, int32_t* d_status,
                                             void* stream) {
  if (n == 0) return HIPBLS_OK;
  int rc = ensure_init();
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(g_ctx.mu);
  hipStream_t s = stream ? (hipStream_t)stream : g_ctx.stream;
  hipLaunchKernelGGL(k_sk_to_pk, dim3((unsigned)grid_for(n)), dim3(kBlock), 0, s, d_sks, n, d_out_pks, d_status);
  HIP_TRY(hipGetLastError());
  return HIPBLS_OK;
}

int launch_fav(const uint8_t* d_pks, uint64_t nkeys, const uint64_t* d_goff, uint64_t n_groups, const uint8_t* d_sigs,
               const uint8_t* d_msgs, const uint64_t* d_moffs, int32_t* d_status, hipStream_t s) {
  Context& c = g_ctx;
  if (n_groups == 0) return HIPBLS_OK;
  HIP_TRY(c.b_pts.ensure((nkeys ? nkeys : 1) * 24 * 4));
  HIP_TRY(c.b_pst.ensure((nkeys ? nkeys : 1) * 4));
  if (nkeys)
    hipLaunchKernelGGL(k_g1_decode, dim3((unsigned)grid_for(nkeys)), dim3(kBlock), 0, s, d_pks, nkeys,
                       (uint32_t*)c.b_pts.p, (int32_t*)c.b_pst.p);
  return timed("fav", s, [&] {
    hipLaunchKernelGGL(k_fav_batch, dim3((unsigned)n_groups), dim3(kFavBlock), 0, s, (const uint32_t*)c.b_pts.p,
                       (const int32_t*)c.b_pst.p, nkeys, d_goff, d_sigs, d_msgs, d_moffs, d_status);
  });
}

int hipbls_verify_aggregate_batch(const uint8_t* pks, const uint64_t* key_offsets, uint64_t n_groups,
                                  const uint8_t* sigs, const uint8_t* msgs, const uint64_t* msg_offsets,
                                  int32_t* status) {
  if (n_groups == 0) return HIPBLS_OK;
  if (!key_offsets || !sigs || !msg_offsets || !status || key_offsets[0] != 0 || msg_offsets[0] != 0 ||
      mul_overflows(n_groups, 96))
    return HIPBLS_ERR_ARG;
  for (uint64_t g = 0; g < n_groups; ++g)
    if (key_offsets[g + 1] < key_offsets[g] || msg_offsets[g + 1] < msg_offsets[g] ||
        msg_offsets[g + 1] - msg_offsets[g] > 0xffffffffull)
      return HIPBLS_ERR_ARG;
  const uint64_t nkeys = key_offsets[n_groups], msg_total = msg_offsets[n_groups];
  if ((nkeys && !pks) || (msg_total && !msgs) || mul_overflows(nkeys, 96)) return HIPBLS_ERR_ARG;
  int rc = ensure_init();
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(g_ctx.mu);
  Context& c = g_ctx;
  HIP_TRY(c.b_pk.ensure((nkeys ? nkeys : 1) * 48));
  HIP_TRY(c.b_ids.ensure((n_groups + 1) * 8));
  HIP_TRY(c.b_sig.ensure(n_groups * 96));
  HIP_TRY(c.b_msg.ensure(msg_total ? msg_total : 1));
  HIP_TRY(c.b_off.ensure((n_groups + 1) * 8));
  HIP_TRY(c.b_st.ensure(n_groups * 4));
  if (nkeys) HIP_TRY(hipMemcpyAsync(c.b_pk.p, pks, nkeys * 48, hipMemcpyHostToDevice, c.stream));
  HIP_TRY(hipMemcpyAsync(c.b_ids.p, key_offsets, (n_groups + 1) * 8, hipMemcpyHostToDevice, c.stream));
  HIP_TRY(hipMemcpyAsync(c.b_sig.p, sigs, n_groups * 96, hipMemcpyHostToDevice, c.stream));
  if (msg_total) HIP_TRY(hipMemcpyAsync(c.b_msg.p, msgs, msg_total, hipMemcpyHostToDevice, c.stream));
  HIP_TRY(hipMemcpyAsync(c.b_off.p, msg_offsets, (n_groups + 1) * 8, hipMemcpyHostToDevice, c.stream));
  rc = launch_fav((const uint8_t*)c.b_pk.p, nkeys, (const uint64_t*)c.b_ids.p, n_groups, (const uint8_t*)c.b_sig.p,
                  (const uint8_t*)c.b_msg.p, (const uint64_t*)c.b_off.p, (int32_t*)c.b_st.p, c.stream);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(status, c.b_st.p, n_groups * 4, hipMemcpyDeviceToHost, c.stream));
  HIP_TRY(hipStreamSynchronize(c.stream));
  return HIPBLS_OK;
}

int hipbls_verify_aggregate_batch_device(const uint8_t* d_pks, uint64_t nkeys, const uint64_t* d_key_offsets,
                                         uint64_t n_groups, const uint8_t* d_sigs, const uint8_t* d_msgs,
                                         const uint64_t* d_msg_offsets, int32_t* d_status, void* stream) {
  if (n_groups == 0) return HIPBLS_OK;
  int rc = ensure_init();
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(g_ctx.mu);
  return launch_fav(d_pks, nkeys, d_key_offsets, n_groups, d_sigs, d_msgs, d_msg_offsets, d_status,
                    stream ? (hipStream_t)stream : g_ctx.stream);
}

int hipbls_verify_aggregate(const uint8_t* pks, uint64_t n, const uint8_t* sig, const uint8_t* msg, uint64_t msg_len,
                            int32_t* status) {
  if (!sig || !status || (n && !pks) || (msg_len && !msg) || mul_overflows(n, 48)) return HIPBLS_ERR_ARG;
  const uint64_t koff[2] = {0, n}, moff[2] = {0, msg_len};
  static const uint8_t empty = 0;
  return hipbls_verify_aggregate_batch(n ? pks : &empty, koff, 1, sig, msg_len ? msg : &empty, moff, status);
}

int hipbls_aggregate(const uint8_t* sigs, uint64_t n, uint8_t* out_sig, int32_t* status) {
  if (!out_sig || !status || (n && !sigs) || mul_overflows(n, 96)) return HIPBLS_ERR_ARG;
  int rc = ensure_init();
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(g_ctx.mu);
  Context& c = g_ctx;
  HIP_TRY(c.b_sig.ensure((n ? n : 1) * 96));
  HIP_TRY(c.b_out.ensure(96));
  HIP_TRY(c.b_st.ensure(4));
  if (n) HIP_TRY(hipMemcpyAsync(c.b_sig.p, sigs, n * 96, hipMemcpyHostToDevice, c.stream));
  hipLaunchKernelGGL(k_aggregate, dim3(1), dim3(kBlock), 0, c.stream, (const uint8_t*)c.b_sig.p, n,
                     (uint8_t*)c.b_out.p, (int32_t*)c.b_st.p);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(out_sig, c.b_out.p, 96, hipMemcpyDeviceToHost, c.stream));
  HIP_TRY(hipMemcpyAsync(status, c.b_st.p, 4, hipMemcpyDeviceToHost, c.stream));
  HIP_TRY(hipStreamSynchronize(c.stream));
  return HIPBLS_OK;
}

int hipbls_threshold_split(const uint8_t* secret, const uint8_t* poly_tail, uint32_t total, uint32_t threshold,
                           uint8_t* out_shares, int32_t* status) {
  if (!secret || !out_shares || !status || threshold == 0 || total == 0 || (threshold > 1 && !poly_tail))
    return HIPBLS_ERR_ARG;
  int rc = ensure_init();
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(g_ctx.mu);
  Context& c = g_ctx;
  HIP_TRY(c.b_aux.ensure(32 * (uint64_t)threshold));
  HIP_TRY(c.b_out.ensure(32 * (uint64_t)total));
  HIP_TRY(c.b_st.ensure(4));
  HIP_TRY(hipMemcpyAsync(c.b_aux.p, secret, 32, hipMemcpyHostToDevice, c.stream));
  if (threshold > 1)
    HIP_TRY(hipMemcpyAsync((uint8_t*)c.b_aux.p + 32, poly_tail, 32 * (uint64_t)(threshold - 1), hipMemcpyHostToDevice,
                           c.stream));
  hipLaunchKernelGGL(k_threshold_split, dim3((unsigned)grid_for(total)), dim3(kBlock), 0, c.stream,
                     (const uint8_t*)c.b_aux.p, (const uint8_t*)c.b_aux.p + 32, total, threshold, (uint8_t*)c.b_out.p,
                     (int32_t*)c.b_st.p);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(out_shares, c.b_out.p, 32 * (uint64_t)total, hipMemcpyDeviceToHost, c.stream));
  HIP_TRY(hipMemcpyAsync(status, c.b_st.p, 4, hipMemcpyDeviceToHost, c.stream));
  HIP_TRY(hipStreamSynchronize(c.stream));
  return HIPBLS_OK;
}

int hipbls_recover_secret(const uint8_t* shares, const uint32_t* ids, uint32_t n, uint8_t* out_secret,
                          int32_t* status) {
  if (!out_secret || !status || (n && (!shares || !ids))) return HIPBLS_ERR_ARG;
  int rc = ensure_init();
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(g_ctx.mu);
  Context& c = g_ctx;
  HIP_TRY(c.b_aux.ensure(32 * (uint64_t)(n ? n : 1)));
  HIP_TRY(c.b_ids.ensure(4 * (uint64_t)(n ? n : 1)));
  HIP_TRY(c.b_out.ensure(32));
  HIP_TRY(c.b_st.ensure(4));
  if (n) {
    HIP_TRY(hipMemcpyAsync(c.b_aux.p, shares, 32 * (uint64_t)n, hipMemcpyHostToDevice, c.stream));
    HIP_TRY(hipMemcpyAsync(c.b_ids.p, ids, 4 * (uint64_t)n, hipMemcpyHostToDevice, c.stream));
  }
  hipLaunchKernelGGL(k_recover_secret, dim3(1), dim3(kBlock), 0, c.stream, (const uint8_t*)c.b_aux.p,
                     (const uint32_t*)c.b_ids.p, n, (uint8_t*)c.b_out.p, (int32_t*)c.b_st.p);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(out_secret, c.b_out.p, 32, hipMemcpyDeviceToHost, c.stream));
  HIP_TRY(hipMemcpyAsync(status, c.b_st.p, 4, hipMemcpyDeviceToHost, c.stream));
  HIP_TRY(hipStreamSynchronize(c.stream));
  return HIPBLS_OK;
}

int hipbls_kernel_timing(const char* name, double* avg_ms, uint64_t* launches) {
  if (!name || !avg_ms || !launches) return HIPBLS_ERR_ARG;
  std::lock_guard<std::mutex> lk(g_ctx.mu);
  auto it = g_ctx.timing.find(name);
  if (it == g_ctx.timing.end()) {
    *launches = 0;
    *avg_ms = 0.0;
    return HIPBLS_OK;
  }
  TimingSlot& t = it->second;
  drain_timing(t);
  *launches = t.launches;
  *avg_ms = t.launches ? t.total_ms / t.launches : 0.0;
  return HIPBLS_OK;
}

int hipbls_kernel_timing_reset(void) {
  std::lock_guard<std::mutex> lk(g_ctx.mu);
  for (auto& kv : g_ctx.timing) {
    drain_timing(kv.second);
    kv.second.total_ms = 0;
    kv.second.launches = 0;
  }
  return HIPBLS_OK;
}

int hipbls_batch_verify_rlc(const uint8_t* pks, const uint8_t* sigs, const uint32_t* msg_idx, uint64_t n,
                            const uint8_t* msgs, const uint64_t* msg_offsets, uint64_t n_msgs, const uint8_t* seed32,
                            int32_t* status) {
  if (n == 0) return HIPBLS_OK;
  if (!pks || !sigs || !msg_idx || !msg_offsets || !seed32 || !status || mul_overflows(n, 288)) return HIPBLS_ERR_ARG;
  for (uint64_t i = 0; i < n; ++i)
    if (msg_idx[i] >= n_msgs) {
      g_last_error = "message index out of range";
      return HIPBLS_ERR_ARG;
    }
  for (uint64_t m = 0; m < n_msgs; ++m)
    if (msg_offsets[m + 1] < msg_offsets[m] || msg_offsets[m + 1] - msg_offsets[m] > 0xffffffffull)
      return HIPBLS_ERR_ARG;
  const uint64_t msg_total = msg_offsets[n_msgs];
  if (msg_total && !msgs) return HIPBLS_ERR_ARG;
  int rc = ensure_init();
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(g_ctx.mu);
  Context& c = g_ctx;
  HIP_TRY(c.b_pk.ensure(n * 48));
  HIP_TRY(c.b_sig.ensure(n * 96));
  HIP_TRY(c.r_midx.ensure(n * 4));
  HIP_TRY(c.b_msg.ensure(msg_total ? msg_total : 1));
  HIP_TRY(c.b_off.ensure((n_msgs + 1) * 8));
  HIP_TRY(c.b_st.ensure(n * 4));
  HIP_TRY(hipMemcpyAsync(c.b_pk.p, pks, n * 48, hipMemcpyHostToDevice, c.stream));
  HIP_TRY(hipMemcpyAsync(c.b_sig.p, sigs, n * 96, hipMemcpyHostToDevice, c.stream));
  HIP_TRY(hipMemcpyAsync(c.r_midx.p, msg_idx, n * 4, hipMemcpyHostToDevice, c.stream));
  if (msg_total) HIP_TRY(hipMemcpyAsync(c.b_msg.p, msgs, msg_total, hipMemcpyHostToDevice, c.stream));
  HIP_TRY(hipMemcpyAsync(c.b_off.p, msg_offsets, (n_msgs + 1) * 8, hipMemcpyHostToDevice, c.stream));
  rc = launch_rlc((const uint8_t*)c.b_pk.p, (const uint8_t*)c.b_sig.p, (const uint32_t*)c.r_midx.p, n,
                  (const uint8_t*)c.b_msg.p, (const uint64_t*)c.b_off.p, n_msgs, seed32, (int32_t*)c.b_st.p, c.stream);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(status, c.b_st.p, n * 4, hipMemcpyDeviceToHost, c.stream));
  HIP_TRY(hipStreamSynchronize(c.stream));
  return HIPBLS_OK;
}

int hipbls_batch_verify_rlc_device(const uint8_t* d_pks, const uint8_t* d_sigs, const uint32_t* d_msg_idx, uint64_t n,
                                   const uint8_t* d_msgs, const uint64_t* d_msg_offsets, uint64_t n_msgs,
                                   const uint8_t* seed32, int32_t* d_status, void* stream) {
  if (n == 0) return HIPBLS_OK;
  if (!seed32 || mul_overflows(n, 288)) return HIPBLS_ERR_ARG;
  int rc = ensure_init();
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(g_ctx.mu);
  return launch_rlc(d_pks, d_sigs, d_msg_idx, n, d_msgs, d_msg_offsets, n_msgs, seed32, d_status,
                    stream ? (hipStream_t)stream : g_ctx.stream);
}

int hipbls_pubshare_table_load(const uint8_t* pks, uint64_t n, int32_t* status) {
  if ((n && (!pks || !status)) || mul_overflows(n, 240) || n > 0xffffffffull) return HIPBLS_ERR_ARG;
  int rc = ensure_init();
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(g_ctx.mu);
  Context& c = g_ctx;
  HIP_TRY(hipStreamSynchronize(c.stream));
  HIP_TRY(hipDeviceSynchronize());  // no call may still read the old table
  c.t_size = 0;
  if (n == 0) return HIPBLS_OK;
  HIP_TRY(c.b_pk.ensure(n * 48));
  HIP_TRY(c.b_st.ensure(n * 4));
  HIP_TRY(c.t_code.ensure(n * 4));
  HIP_TRY(c.t_tab.ensure(n * PUBTAB_WORDS * 4));
  HIP_TRY(hipMemcpyAsync(c.b_pk.p, pks, n * 48, hipMemcpyHostToDevice, c.stream));
  hipLaunchKernelGGL(k_pubtab_load, dim3((unsigned)grid_for(n)), dim3(kBlock), 0, c.stream, (const uint8_t*)c.b_pk.p, n,
                     (int32_t*)c.t_code.p, (uint32_t*)c.t_tab.p, (int32_t*)c.b_st.p);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(status, c.b_st.p, n * 4, hipMemcpyDeviceToHost, c.stream));
  HIP_TRY(hipStreamSynchronize(c.stream));
  c.t_size = n;
  return HIPBLS_OK;
}

int hipbls_pubshare_table_size(uint64_t* n) {
  if (!n) return HIPBLS_ERR_ARG;
  std::lock_guard<std::mutex> lk(g_ctx.mu);
  *n = g_ctx.t_size;
  return HIPBLS_OK;
}

int hipbls_verify_batch_keys(const uint32_t* key_idx, const uint8_t* msgs, const uint64_t* msg_offsets,
                             const uint8_t* sigs, uint64_t n, int32_t* status) {
  if (n == 0) return HIPBLS_OK;
  if (!key_idx || !msg_offsets || !sigs || !status || mul_overflows(n, 96)) return HIPBLS_ERR_ARG;
  const uint64_t msg_total = msg_offsets[n];
  if (msg_total && !msgs) return HIPBLS_ERR_ARG;
  for (uint64_t i = 0; i < n; ++i)
    if (msg_offsets[i + 1] < msg_offsets[i] || msg_offsets[i + 1] - msg_offsets[i] > 0xffffffffull)
      return HIPBLS_ERR_ARG;
  int rc = ensure_init();
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(g_ctx.mu);
  Context& c = g_ctx;
  for (uint64_t i = 0; i < n; ++i)
    if (key_idx[i] >= c.t_size) {
      g_last_error = "key index outside the pubshare table";
      return HIPBLS_ERR_ARG;
    }
  HIP_TRY(c.b_kidx.ensure(n * 4));
  HIP_TRY(c.b_sig.ensure(n * 96));
  HIP_TRY(c.b_msg.ensure(msg_total ? msg_total : 1));
  HIP_TRY(c.b_off.ensure((n + 1) * 8));
  HIP_TRY(c.b_st.ensure(n * 4));
  HIP_TRY(hipMemcpyAsync(c.b_kidx.p, key_idx, n * 4, hipMemcpyHostToDevice, c.stream));
  HIP_TRY(hipMemcpyAsync(c.b_sig.p, sigs, n * 96, hipMemcpyHostToDevice, c.stream));
  if (msg_total) HIP_TRY(hipMemcpyAsync(c.b_msg.p, msgs, msg_total, hipMemcpyHostToDevice, c.stream));
  HIP_TRY(hipMemcpyAsync(c.b_off.p, msg_offsets, (n + 1) * 8, hipMemcpyHostToDevice, c.stream));
  rc = timed("verify_keys", c.stream, [&] {
    hipLaunchKernelGGL(k_verify_keys, dim3((unsigned)grid_for(n)), dim3(kBlock), 0, c.stream,
                       (const uint32_t*)c.b_kidx.p, c.t_size, (const int32_t*)c.t_code.p, (const uint32_t*)c.t_tab.p,
                       (const uint8_t*)c.b_msg.p, (const uint64_t*)c.b_off.p, (const uint8_t*)c.b_sig.p, n,
                       (int32_t*)c.b_st.p);
  });
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(status, c.b_st.p, n * 4, hipMemcpyDeviceToHost, c.stream));
  HIP_TRY(hipStreamSynchronize(c.stream));
  return HIPBLS_OK;
}

int hipbls_verify_batch_keys_device(const uint32_t* d_key_idx, const uint8_t* d_msgs, const uint64_t* d_msg_offsets,
                                    const uint8_t* d_sigs, uint64_t n, int32_t* d_status, void* stream) {
  if (n == 0) return HIPBLS_OK;
  int rc = ensure_init();
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(g_ctx.mu);
  Context& c = g_ctx;
  hipStream_t s = stream ? (hipStream_t)stream : c.stream;
  return timed("verify_keys", s, [&] {
    hipLaunchKernelGGL(k_verify_keys, dim3((unsigned)grid_for(n)), dim3(kBlock), 0, s, d_key_idx, c.t_size,
                       (const int32_t*)c.t_code.p, (const uint32_t*)c.t_tab.p, d_msgs, d_msg_offsets, d_sigs, n,
                       d_status);
  });
}

int hipbls_batch_verify_rlc_keys(const uint32_t* key_idx, const uint8_t* sigs, const uint32_t* msg_idx, uint64_t n,
                                 const uint8_t* msgs, const uint64_t* msg_offsets, uint64_t n_msgs,
                                 const uint8_t* seed32, int32_t* status) {
  if (n == 0) return HIPBLS_OK;
  if (!key_idx || !sigs || !msg_idx || !msg_offsets || !seed32 || !status || mul_overflows(n, 288))
    return HIPBLS_ERR_ARG;
  for (uint64_t i = 0; i < n; ++i)
    if (msg_idx[i] >= n_msgs) {
      g_last_error = "message index out of range";
      return HIPBLS_ERR_ARG;
    }
  for (uint64_t m = 0; m < n_msgs; ++m)
    if (msg_offsets[m + 1] < msg_offsets[m] || msg_offsets[m + 1] - msg_offsets[m] > 0xffffffffull)
      return HIPBLS_ERR_ARG;
  const uint64_t msg_total = msg_offsets[n_msgs];
  if (msg_total && !msgs) return HIPBLS_ERR_ARG;
  int rc = ensure_init();
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(g_ctx.mu);
  Context& c = g_ctx;
  for (uint64_t i = 0; i < n; ++i)
    if (key_idx[i] >= c.t_size) {
      g_last_error = "key index outside the pubshare table";
      return HIPBLS_ERR_ARG;
    }
  HIP_TRY(c.b_kidx.ensure(n * 4));
  HIP_TRY(c.b_sig.ensure(n * 96));
  HIP_TRY(c.r_midx.ensure(n * 4));
  HIP_TRY(c.b_msg.ensure(msg_total ? msg_total : 1));
  HIP_TRY(c.b_off.ensure((n_msgs + 1) * 8));
  HIP_TRY(c.b_st.ensure(n * 4));
  HIP_TRY(hipMemcpyAsync(c.b_kidx.p, key_idx, n * 4, hipMemcpyHostToDevice, c.stream));
  HIP_TRY(hipMemcpyAsync(c.b_sig.p, sigs, n * 96, hipMemcpyHostToDevice, c.stream));
  HIP_TRY(hipMemcpyAsync(c.r_midx.p, msg_idx, n * 4, hipMemcpyHostToDevice, c.stream));
  if (msg_total) HIP_TRY(hipMemcpyAsync(c.b_msg.p, msgs, msg_total, hipMemcpyHostToDevice, c.stream));
  HIP_TRY(hipMemcpyAsync(c.b_off.p, msg_offsets, (n_msgs + 1) * 8, hipMemcpyHostToDevice, c.stream));
  rc = launch_rlc(nullptr, (const uint8_t*)c.b_sig.p, (const uint32_t*)c.r_midx.p, n, (const uint8_t*)c.b_msg.p,
                  (const uint64_t*)c.b_off.p, n_msgs, seed32, (int32_t*)c.b_st.p, c.stream,
                  (const uint32_t*)c.b_kidx.p);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(status, c.b_st.p, n * 4, hipMemcpyDeviceToHost, c.stream));
  HIP_TRY(hipStreamSynchronize(c.stream));
  return HIPBLS_OK;
}

int hipbls_batch_verify_rlc_keys_device(const uint32_t* d_key_idx, const uint8_t* d_sigs, const uint32_t* d_msg_idx,
                                        uint64_t n, const uint8_t* d_msgs, const uint64_t* d_msg_offsets,
                                        uint64_t n_msgs, const uint8_t* seed32, int32_t* d_status, void* stream) {
  if (n == 0) return HIPBLS_OK;
  if (!seed32 || !d_key_idx || mul_overflows(n, 288)) return HIPBLS_ERR_ARG;
  int rc = ensure_init();
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(g_ctx.mu);
  return launch_rlc(nullptr, d_sigs, d_msg_idx, n, d_msgs, d_msg_offsets, n_msgs, seed32, d_status,
                    stream ? (hipStream_t)stream : g_ctx.stream, d_key_idx);
}

int hipbls_rlc_stats(uint64_t* windows, uint64_t* windows_failed, uint64_t* items_fallback) {
  if (!windows || !windows_failed || !items_fallback) return HIPBLS_ERR_ARG;
  std::lock_guard<std::mutex> lk(g_ctx.mu);
  Context& c = g_ctx;
  *windows = c.r_windows;
  *windows_failed = 0;
  *items_fallback = 0;
  if (c.r_windows == 0) return HIPBLS_OK;
  std::vector<int32_t> v(c.r_windows);
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(v.data(), c.r_win.p, v.size() * 4, hipMemcpyDeviceToHost));
  for (int32_t x : v)
    if (x > 0) {
      *windows_failed += 1;
      *items_fallback += (uint64_t)x;
    }
  return HIPBLS_OK;
}

}  // extern "C"
