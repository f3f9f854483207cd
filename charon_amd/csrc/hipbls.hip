// hipbls: kernels + C-ABI host entry points (include/hipbls.h) for gfx950.
//
// Execution model: one process per GPU; within a process one context per device holding a HIP
// stream, reusable device workspaces and a mutex (the C-ABI is called concurrently from many
// goroutines in charon, tbls/tbls.go:79-141).  Host-buffer entry points copy in, launch, copy out
// and synchronize; *_device entry points only enqueue.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "ops.h"

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
    jac_mul_limbs(acc, sj, lam.v, 8);
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

// FastAggregateVerify tail: one lane sums the decoded keys, hashes, pairs.
__global__ void __launch_bounds__(kBlock) k_fast_aggregate_verify_tail(const uint32_t* __restrict__ pts, const int32_t* __restrict__ code,
                                             uint64_t n, const uint8_t* __restrict__ sig,
                                             const uint8_t* __restrict__ msg, uint64_t msg_len,
                                             int32_t* __restrict__ status) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  g2a s;
  const int ds = g2_decompress(s, sig, true);
  if (ds == DEC_BAD) {
    *status = HIPBLS_ERR_SIGNATURE;
    return;
  }
  for (uint64_t i = 0; i < n; ++i)
    if (code[i] == DEC_BAD) {
      *status = HIPBLS_ERR_PUBKEY;
      return;
    }
  if (n == 0 || ds == DEC_INF) {
    *status = HIPBLS_ERR_VERIFY;
    return;
  }
  g1j acc;
  jac_set_inf(acc);
  for (uint64_t i = 0; i < n; ++i) {
    if (code[i] == DEC_INF) {
      *status = HIPBLS_ERR_VERIFY;  // KeyValidate rejects the identity key
      return;
    }
    g1a a;
    uint32_t* dst = &a.x.v[0];
    for (int w = 0; w < 24; ++w) dst[w] = pts[(uint64_t)w * n + i];
    jac_add_aff(acc, acc, a);
  }
  if (jac_is_inf(acc)) {
    *status = HIPBLS_ERR_VERIFY;
    return;
  }
  g1a pk;
  jac_to_aff(pk, acc);
  g2j hj;
  hash_to_g2(hj, msg, (uint32_t)msg_len, DST_POP, 43);
  g2a hm;
  jac_to_aff(hm, hj);
  *status = pairing_check_verify(pk, hm, s) ? HIPBLS_OK : HIPBLS_ERR_VERIFY;
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
  TimingSlot verify_timing;
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

int launch_verify(const uint8_t* d_pks, const uint8_t* d_msgs, const uint64_t* d_offs, const uint8_t* d_sigs,
                  uint64_t n, int32_t* d_status, hipStream_t s) {
  if (n == 0) return HIPBLS_OK;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (g_ctx.timing_enabled) {
    HIP_TRY(hipEventCreate(&e0));
    HIP_TRY(hipEventCreate(&e1));
    HIP_TRY(hipEventRecord(e0, s));
  }
  hipLaunchKernelGGL(k_verify_fused, dim3((unsigned)grid_for(n)), dim3(kBlock), 0, s, d_pks, d_msgs, d_offs, d_sigs,
                     n, d_status);
  HIP_TRY(hipGetLastError());
  if (g_ctx.timing_enabled) {
    HIP_TRY(hipEventRecord(e1, s));
    g_ctx.verify_timing.pending.emplace_back(e0, e1);
    if (g_ctx.verify_timing.pending.size() > 256) drain_timing(g_ctx.verify_timing);
  }
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

int hipbls_verify_aggregate(const uint8_t* pks, uint64_t n, const uint8_t* sig, const uint8_t* msg, uint64_t msg_len,
                            int32_t* status) {
  if (!sig || !status || (n && !pks) || (msg_len && !msg) || mul_overflows(n, 48)) return HIPBLS_ERR_ARG;
  int rc = ensure_init();
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(g_ctx.mu);
  Context& c = g_ctx;
  HIP_TRY(c.b_pk.ensure((n ? n : 1) * 48));
  HIP_TRY(c.b_sig.ensure(96));
  HIP_TRY(c.b_msg.ensure(msg_len ? msg_len : 1));
  HIP_TRY(c.b_pts.ensure((n ? n : 1) * 24 * 4));
  HIP_TRY(c.b_pst.ensure((n ? n : 1) * 4));
  HIP_TRY(c.b_st.ensure(4));
  if (n) HIP_TRY(hipMemcpyAsync(c.b_pk.p, pks, n * 48, hipMemcpyHostToDevice, c.stream));
  HIP_TRY(hipMemcpyAsync(c.b_sig.p, sig, 96, hipMemcpyHostToDevice, c.stream));
  if (msg_len) HIP_TRY(hipMemcpyAsync(c.b_msg.p, msg, msg_len, hipMemcpyHostToDevice, c.stream));
  if (n)
    hipLaunchKernelGGL(k_g1_decode, dim3((unsigned)grid_for(n)), dim3(kBlock), 0, c.stream, (const uint8_t*)c.b_pk.p,
                       n, (uint32_t*)c.b_pts.p, (int32_t*)c.b_pst.p);
  hipLaunchKernelGGL(k_fast_aggregate_verify_tail, dim3(1), dim3(kBlock), 0, c.stream, (const uint32_t*)c.b_pts.p,
                     (const int32_t*)c.b_pst.p, n, (const uint8_t*)c.b_sig.p, (const uint8_t*)c.b_msg.p, msg_len,
                     (int32_t*)c.b_st.p);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(status, c.b_st.p, 4, hipMemcpyDeviceToHost, c.stream));
  HIP_TRY(hipStreamSynchronize(c.stream));
  return HIPBLS_OK;
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
  if (std::strcmp(name, "verify") != 0) return HIPBLS_ERR_ARG;
  drain_timing(g_ctx.verify_timing);
  *launches = g_ctx.verify_timing.launches;
  *avg_ms = g_ctx.verify_timing.launches ? g_ctx.verify_timing.total_ms / g_ctx.verify_timing.launches : 0.0;
  return HIPBLS_OK;
}

int hipbls_kernel_timing_reset(void) {
  std::lock_guard<std::mutex> lk(g_ctx.mu);
  drain_timing(g_ctx.verify_timing);
  g_ctx.verify_timing.total_ms = 0;
  g_ctx.verify_timing.launches = 0;
  return HIPBLS_OK;
}

}  // extern "C"
