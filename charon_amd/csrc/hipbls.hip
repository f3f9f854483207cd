// hipbls: C-ABI host runtime (include/hipbls.h) over the gfx950 kernels in kernels.h.
//
// Execution model: one process per GPU (charon runs one node process; bench.py one rank per GPU).  The
// process has one device context: the device index, a library stream, reusable device workspaces and a
// mutex.  The C-ABI is called concurrently from many goroutines (tbls/tbls.go:79-141), and a goroutine can
// move between OS threads between two calls, so every entry point binds the context's device on the calling
// thread (hipSetDevice is per host thread in HIP) before it touches memory or streams.
//
//   * Host-buffer entry points copy in, launch, copy out and synchronize, holding the context lock.
//   * *_device entry points only enqueue on the caller's stream.  Calls that share a workspace are ordered on
//     the device: each waits for the previous workspace user's completion event (ws_done) before its first
//     kernel and records the event after its last, so two calls on different streams never see each other's
//     H(m) table, fallback list or partial sums.
//   * hipbls_verify / hipbls_verify_submit go through the submission queue (VerifyQueue): concurrent n = 1
//     calls from many threads are coalesced into one launch per batch; the queue's worker thread owns its own
//     stream and buffers, and no caller holds a lock while the GPU runs.
#include <hip/hip_runtime.h>

#include <array>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "kernels.h"

namespace {

// ============================================================================ device context
thread_local std::string g_last_error;

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t n) {
    if (n <= cap) return hipSuccess;
    if (p) (void)hipFree(p);  // hipFree waits for the device: no in-flight kernel still uses the old buffer
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

// Resident H(m) cache for signing roots: roots shared by a validator's t partials arrive in
// different calls (one parsigex message per peer, core/parsigex/parsigex.go:86-91, then sigagg,
// core/sigagg/sigagg.go:138-159), so each distinct root is hashed to G2 once and kept in HBM (affine, 48 words,
// SoA over the capacity).  FIFO replacement over a ring of slots; a hit whose slot this call is about to reuse
// is treated as a miss.
struct HCache {
  uint64_t cap = 0;  // 0 = disabled
  uint64_t ring = 0;
  std::unordered_map<std::string, uint32_t> map;
  std::vector<std::string> key_of;  // slot -> key ("" = empty)
  DevBuf table;
  uint64_t hits = 0, misses = 0;
};

struct Context {
  int device = -1;
  hipStream_t stream = nullptr;
  std::mutex mu;
  DevBuf b_pk, b_msg, b_off, b_sig, b_st, b_out, b_ids, b_pts, b_pst, b_aux, b_part, b_bad;
  DevBuf r_pk, r_sig, r_h, r_win, r_midx, r_list, r_cnt, r_slot, r_mlist;  // RLC BatchVerify workspaces
  DevBuf t_code, t_tab, b_kidx;                                            // resident pubshare table + key indices
  DevBuf v_ws;                                                             // lane-pair Verify points (SoA)
  uint64_t t_size = 0;
  // RLC sub-batches in flight.  The process gets GPU_MAX_HW_QUEUES = 4 hardware queues, shared by the caller's
  // stream (which also hashes the messages), the library stream and these; a kernel trace
  // (profiles/r01_rlc_trace.txt) showed a third sub-stream landing on an occupied queue and serializing behind
  // it, so two sub-batches.
  static constexpr int kSub = 2;
  hipStream_t sub[kSub] = {};
  hipEvent_t ev_fork = nullptr, ev_hash = nullptr, ev_join[kSub] = {};
  hipEvent_t ws_done = nullptr;  // last workspace user's completion (cross-stream ordering)
  uint64_t r_windows = 0;        // window count of the last RLC call (hipbls_rlc_stats)
  // batch-wide RLC check (rlcb.h): MSM inputs and stages, Miller values, verdict flag
  DevBuf m_pts, m_sc, m_cnt, m_off, m_cur, m_list, m_B, m_Sg, m_W, m_F, m_F2, m_FS, m_flag;
  // Verdicts come back through a ring of pinned slots, one per batch check in flight, so a launch only waits
  // on the host when kRlcbSlots checks are still unread (never in the enqueue-only *_device paths otherwise).
  static constexpr int kRlcbSlots = 8;
  int32_t* rlcb_host_flag = nullptr;  // pinned, kRlcbSlots verdicts
  hipEvent_t rlcb_ev[kRlcbSlots] = {};
  hipEvent_t rlcb_ev_items = nullptr, rlcb_ev_msm = nullptr;
  bool rlcb_pending[kRlcbSlots] = {};
  uint64_t rlcb_seq[kRlcbSlots] = {};  // launch order of the check in each slot
  uint64_t rlcb_next_seq = 0, rlcb_last_seq = 0;
  int rlcb_last = -1;                 // newest verdict read back: -1 none, 0 failed, 1 passed
  int rlcb_skipped = 0;               // AUTO: calls run windows-only since the last failed batch check
  uint64_t rlcb_attempted = 0, rlcb_passed = 0;
  HCache hcache;
  std::mutex tmu;                            // timing table (also used by the queue worker)
  std::map<std::string, TimingSlot> timing;  // per kernel name: HIP events on the launch stream
  std::atomic<bool> timing_enabled{false};
};

Context g_ctx;
std::mutex g_init_mu;

int set_err(const char* what, hipError_t e) {
  g_last_error = std::string(what) + ": " + hipGetErrorString(e);
  return HIPBLS_ERR_DEVICE;
}
int arg_err(const char* what) {
  g_last_error = what;
  return HIPBLS_ERR_ARG;
}

#define HIP_TRY(expr)                                \
  do {                                               \
    hipError_t _e = (expr);                          \
    if (_e != hipSuccess) return set_err(#expr, _e); \
  } while (0)

int init_locked(int device) {
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess || ndev == 0) return set_err("hipGetDeviceCount (no GPU)", e == hipSuccess ? hipErrorNoDevice : e);
  if (device < 0) HIP_TRY(hipGetDevice(&device));
  if (device >= ndev) return arg_err("device index out of range");
  HIP_TRY(hipSetDevice(device));
  HIP_TRY(hipStreamCreateWithFlags(&g_ctx.stream, hipStreamNonBlocking));
  HIP_TRY(hipEventCreateWithFlags(&g_ctx.ws_done, hipEventDisableTiming));
  const char* t = getenv("HIPBLS_TIMING");
  if (t && t[0] == '1') g_ctx.timing_enabled = true;
  g_ctx.device = device;
  return HIPBLS_OK;
}

// Binds the context's device on the calling thread (initializing on first use).
int bind_device() {
  if (g_ctx.device < 0) {
    std::lock_guard<std::mutex> lk(g_init_mu);
    if (g_ctx.device < 0) {
      const int rc = init_locked(-1);
      if (rc) return rc;
    }
  }
  HIP_TRY(hipSetDevice(g_ctx.device));
  return HIPBLS_OK;
}

// Entry-point prologue: device bound on this thread, context lock held for the scope.
#define ENTER()                                   \
  int _brc = bind_device();                       \
  if (_brc) return _brc;                          \
  std::lock_guard<std::mutex> _lk(g_ctx.mu)

hipStream_t pick(void* stream) { return stream ? (hipStream_t)stream : g_ctx.stream; }

// Workspace ordering: the call's stream waits for the previous workspace user, and publishes its own end.
int ws_begin(hipStream_t s) {
  HIP_TRY(hipStreamWaitEvent(s, g_ctx.ws_done, 0));
  return HIPBLS_OK;
}
int ws_end(hipStream_t s) {
  HIP_TRY(hipEventRecord(g_ctx.ws_done, s));
  return HIPBLS_OK;
}

uint64_t grid_for(uint64_t n) { return (n + kBlock - 1) / kBlock; }
// Verify batches up to this size hash each message on a lane pair in the prep stage (k_verify_prep pair_hash).
constexpr uint64_t kPairHashMaxVerify = 16384;

// wait = false: only events that have completed are folded in (never blocks a launch).
void drain_timing(TimingSlot& t, bool wait) {
  std::vector<std::pair<hipEvent_t, hipEvent_t>> keep;
  for (auto& pr : t.pending) {
    if (!wait && hipEventQuery(pr.second) != hipSuccess) {
      keep.push_back(pr);
      continue;
    }
    float ms = 0;
    if ((!wait || hipEventSynchronize(pr.second) == hipSuccess) &&
        hipEventElapsedTime(&ms, pr.first, pr.second) == hipSuccess) {
      t.total_ms += ms;
      t.launches += 1;
    }
    (void)hipEventDestroy(pr.first);
    (void)hipEventDestroy(pr.second);
  }
  t.pending.swap(keep);
}

// Brackets one kernel launch with HIP events on its stream when timing is enabled (bench.py roofline: the average
// duration per launch is read back through hipbls_kernel_timing).  Off by default: production launches create
// no events and never wait.
template <class Launch>
int timed(const char* name, hipStream_t s, Launch launch) {
  hipEvent_t e0 = nullptr, e1 = nullptr;
  const bool on = g_ctx.timing_enabled.load();
  if (on) {
    HIP_TRY(hipEventCreate(&e0));
    HIP_TRY(hipEventCreate(&e1));
    HIP_TRY(hipEventRecord(e0, s));
  }
  launch();
  HIP_TRY(hipGetLastError());
  if (on) {
    HIP_TRY(hipEventRecord(e1, s));
    std::lock_guard<std::mutex> lk(g_ctx.tmu);
    TimingSlot& t = g_ctx.timing[name];
    t.pending.emplace_back(e0, e1);
    if (t.pending.size() > 256) drain_timing(t, false);
  }
  return HIPBLS_OK;
}

// Pairing-check layout (hipbls_set_pair_mode): one lane per check (the fused kernels), or a lane pair per check
// (lg2.h: the two Miller loops side by side, split final exponentiation).  A pair halves a check's latency but
// uses two lanes, so it wins while the batch leaves lanes idle: one wave per SIMD is 64 x 1024 lanes on MI355X.
int initial_pair_mode() {
  const char* pm = getenv("HIPBLS_PAIR_MODE");
  if (pm && pm[0] >= '0' && pm[0] <= '2' && pm[1] == 0) return pm[0] - '0';
  return HIPBLS_PAIR_AUTO;
}
std::atomic<int> g_pair_mode{initial_pair_mode()};
// Crossovers measured on MI355X (profiles/r02_pair_sweep.txt): lane pairs win up to 32,768 Verify items (742k vs
// 634k verifies/s there) and lose from 49,152 (731k vs 919k).
constexpr uint64_t kLg2MaxVerify = 32768;    // auto: Verify batches up to this many items take lane pairs
constexpr uint64_t kLg2MaxWindows = 32768;   // auto: RLC sub-batches up to this many windows take lane pairs

bool use_pairs(uint64_t units, uint64_t auto_max) {
  const int mode = g_pair_mode.load();
  if (mode == HIPBLS_PAIR_SINGLE) return false;
  if (mode == HIPBLS_PAIR_LANES) return true;
  return units <= auto_max;
}

// Verify: fused (one lane per item) or prep + lane-pair check; `ws` is the caller's SoA workspace for the latter
// (120 words per item), so the library stream and the queue worker never share one.
int launch_verify(const uint8_t* d_pks, const uint8_t* d_msgs, const uint64_t* d_offs, const uint8_t* d_sigs,
                  uint64_t n, int32_t* d_status, hipStream_t s, DevBuf& ws) {
  if (n == 0) return HIPBLS_OK;
  if (!use_pairs(n, kLg2MaxVerify))
    return timed("verify", s, [&] {
      hipLaunchKernelGGL(k_verify_fused, dim3((unsigned)grid_for(n)), dim3(kBlock), 0, s, d_pks, d_msgs, d_offs,
                         d_sigs, n, d_status);
    });
  HIP_TRY(ws.ensure(n * 120 * 4));
  int rc = timed("verify_prep", s, [&] {
    const int pair_hash = n <= kPairHashMaxVerify ? 1 : 0;
    hipLaunchKernelGGL(k_verify_prep, dim3((unsigned)((pair_hash ? 3 : 2) * grid_for(n))), dim3(kBlock), 0, s, d_pks,
                       d_msgs, d_offs, d_sigs, n, (uint32_t*)ws.p, d_status, pair_hash);
  });
  if (rc) return rc;
  return timed("verify_pair_lg2", s, [&] {
    hipLaunchKernelGGL(k_verify_pair_lg2, dim3((unsigned)grid_for(2 * n)), dim3(kBlock), 0, s,
                       (const uint32_t*)ws.p, n, d_status);
  });
}

bool use_rlc_batch(uint64_t n);
int launch_rlc_batch(const uint8_t* d_pks, const uint8_t* d_sigs, const uint32_t* d_midx, uint64_t n,
                     const uint8_t* d_msgs, const uint64_t* d_offs, uint64_t n_msgs, const rlc_seed& seed,
                     int32_t* d_status, hipStream_t s, const uint32_t* d_kidx, uint32_t* d_H, uint64_t hstride,
                     const uint32_t* d_hslot, const uint32_t* d_mlist, uint64_t n_hash);

int ensure_rlc_streams() {
  Context& c = g_ctx;
  if (c.ev_fork) return HIPBLS_OK;
  for (int k = 0; k < Context::kSub; ++k) HIP_TRY(hipStreamCreateWithFlags(&c.sub[k], hipStreamNonBlocking));
  HIP_TRY(hipEventCreateWithFlags(&c.ev_hash, hipEventDisableTiming));
  for (int k = 0; k < Context::kSub; ++k) HIP_TRY(hipEventCreateWithFlags(&c.ev_join[k], hipEventDisableTiming));
  HIP_TRY(hipEventCreateWithFlags(&c.ev_fork, hipEventDisableTiming));
  return HIPBLS_OK;
}

// RLC BatchVerify: the batch is cut into up to kSub window-aligned sub-batches, each running items -> window ->
// fallback on its own stream, while the distinct messages are hashed on the caller's stream; windows wait only
// for the hash.  Every stage is latency-bound on its own (one lane per item at one wave per SIMD), so overlapping
// the sub-batches' stages is what fills the CUs.  The caller's stream `s` forks into the sub-streams and joins
// back, so the call stays stream-ordered.
// H table: H(m) of message m is at column hslot[m] (identity when hslot == nullptr) of an affine SoA table with
// `hstride` columns; k_rlc_hash fills the columns of the n_hash messages listed in mlist (all when nullptr).
int launch_rlc(const uint8_t* d_pks, const uint8_t* d_sigs, const uint32_t* d_midx, uint64_t n, const uint8_t* d_msgs,
               const uint64_t* d_offs, uint64_t n_msgs, const uint8_t* seed32, int32_t* d_status, hipStream_t s,
               const uint32_t* d_kidx = nullptr, uint32_t* d_H = nullptr, uint64_t hstride = 0,
               const uint32_t* d_hslot = nullptr, const uint32_t* d_mlist = nullptr, uint64_t n_hash = 0) {
  Context& c = g_ctx;
  // d_pks == nullptr: keys from the resident table
  const uint64_t T = c.t_size;
  const int32_t* tcode = (const int32_t*)c.t_code.p;
  const uint32_t* tab = (const uint32_t*)c.t_tab.p;
  c.r_windows = 0;
  if (n == 0) return HIPBLS_OK;
  if (n > 0xffffffffull) return arg_err("RLC batch larger than 2^32 items");  // fallback list holds 32-bit indices
  int rc = ensure_rlc_streams();
  if (rc) return rc;
  rlc_seed seed;
  for (int k = 0; k < 8; ++k)
    seed.w[k] = (uint32_t)seed32[4 * k] << 24 | (uint32_t)seed32[4 * k + 1] << 16 | (uint32_t)seed32[4 * k + 2] << 8 |
                (uint32_t)seed32[4 * k + 3];
  const uint64_t n_win = (n + RLC_W - 1) / RLC_W;
  HIP_TRY(c.r_pk.ensure(n * 36 * 4));
  HIP_TRY(c.r_sig.ensure(n * 72 * 4));
  if (!d_H) {  // per-call table, one column per message
    HIP_TRY(c.r_h.ensure((n_msgs ? n_msgs : 1) * 48 * 4));
    d_H = (uint32_t*)c.r_h.p;
    hstride = n_msgs;
    d_hslot = nullptr;
    d_mlist = nullptr;
    n_hash = n_msgs;
  }
  HIP_TRY(c.r_win.ensure(n_win * 4));
  HIP_TRY(c.r_list.ensure(n * 4));
  HIP_TRY(c.r_cnt.ensure(Context::kSub * 4));
  if (use_rlc_batch(n))
    return launch_rlc_batch(d_pks, d_sigs, d_midx, n, d_msgs, d_offs, n_msgs, seed, d_status, s, d_kidx, d_H, hstride,
                            d_hslot, d_mlist, n_hash);
  uint32_t* rpk = (uint32_t*)c.r_pk.p;
  uint32_t* rsig = (uint32_t*)c.r_sig.p;
  int32_t* win = (int32_t*)c.r_win.p;
  uint32_t* list = (uint32_t*)c.r_list.p;
  uint32_t* cnt = (uint32_t*)c.r_cnt.p;
  // sub-batches of whole windows; small batches stay in one
  const uint64_t min_win = 2048;
  int nsub = (int)((n_win + min_win - 1) / min_win);
  if (nsub > Context::kSub) nsub = Context::kSub;
  if (nsub < 1) nsub = 1;
  const uint64_t win_per = (n_win + nsub - 1) / nsub;

  rc = ws_begin(s);
  if (rc) return rc;
  HIP_TRY(hipMemsetAsync(cnt, 0, Context::kSub * 4, s));
  HIP_TRY(hipEventRecord(c.ev_fork, s));
  if (n_hash) {
    rc = timed("rlc_hash", s, [&] {
      hipLaunchKernelGGL(k_rlc_hash, dim3((unsigned)grid_for(n_hash)), dim3(kBlock), 0, s, d_msgs, d_offs, n_hash,
                         d_mlist, d_H, hstride, d_hslot);
    });
    if (rc) return rc;
  }
  HIP_TRY(hipEventRecord(c.ev_hash, s));
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
    if (use_pairs(w1 - w0, kLg2MaxWindows))
      rc = timed("rlc_window_lg2", ss, [&] {
        hipLaunchKernelGGL(k_rlc_window_lg2, dim3((unsigned)grid_for(2 * (w1 - w0))), dim3(kBlock), 0, ss, w0, w1, n,
                           d_midx, (const uint32_t*)rpk, (const uint32_t*)rsig, (const uint32_t*)d_H, hstride, d_hslot,
                           d_status, win, list + i0, cnt + k);
      });
    else
      rc = timed("rlc_window", ss, [&] {
        hipLaunchKernelGGL(k_rlc_window, dim3((unsigned)grid_for(w1 - w0)), dim3(kBlock), 0, ss, w0, w1, n, d_midx,
                           (const uint32_t*)rpk, (const uint32_t*)rsig, (const uint32_t*)d_H, hstride, d_hslot,
                           d_status, win, list + i0, cnt + k);
      });
    if (rc) return rc;
    // The list length is only known on the device: launch for the worst case, idle lanes exit.  The list is short
    // (failed windows only) and latency-bound, so lane pairs unless the caller forced single lanes.
    if (g_pair_mode.load() != HIPBLS_PAIR_SINGLE)
      rc = timed("rlc_fallback_lg2", ss, [&] {
        hipLaunchKernelGGL(k_rlc_fallback_lg2, dim3((unsigned)grid_for(2 * (i1 - i0))), dim3(kBlock), 0, ss,
                           (const uint32_t*)(list + i0), (const uint32_t*)(cnt + k), i1 - i0, d_pks, d_sigs, d_midx,
                           (const uint32_t*)d_H, hstride, d_hslot, d_status, d_kidx, T, tab);
      });
    else
      rc = timed("rlc_fallback", ss, [&] {
        hipLaunchKernelGGL(k_rlc_fallback, dim3((unsigned)grid_for(i1 - i0)), dim3(kBlock), 0, ss,
                           (const uint32_t*)(list + i0), (const uint32_t*)(cnt + k), i1 - i0, d_pks, d_sigs, d_midx,
                           (const uint32_t*)d_H, hstride, d_hslot, d_status, d_kidx, T, tab);
      });
    if (rc) return rc;
    HIP_TRY(hipEventRecord(c.ev_join[k], ss));
    HIP_TRY(hipStreamWaitEvent(s, c.ev_join[k], 0));
  }
  c.r_windows = n_win;
  return ws_end(s);
}

// ============================================================================ batch-wide RLC check (rlcb.h)
// Policy (hipbls_rlc_set_mode): WINDOWS = rlc.h only; BATCH = the batch-wide check first, windows for whatever it
// leaves pending; AUTO (default) = BATCH for batches of >= 1,024 items unless the last batch check failed, in
// which case the next 8 calls run windows only (a cluster that sends invalid partials keeps sending them; one
// whose batches pass keeps the cheap path).  The verdict comes back asynchronously (pinned copy + event), so the
// policy never blocks a launch.
std::atomic<int> g_rlc_mode{HIPBLS_RLC_AUTO};
constexpr uint64_t kRlcbMinItems = 1024;
constexpr int kRlcbBackoff = 8;

// Reads back every verdict whose copy has landed; with wait_slot >= 0 (or wait_all) blocks on that slot first.
void rlcb_poll(int wait_slot, bool wait_all = false) {
  Context& c = g_ctx;
  for (int k = 0; k < Context::kRlcbSlots; ++k) {
    if (!c.rlcb_pending[k]) continue;
    if (wait_all || k == wait_slot) {
      if (hipEventSynchronize(c.rlcb_ev[k]) != hipSuccess) continue;
    } else if (hipEventQuery(c.rlcb_ev[k]) != hipSuccess) {
      continue;
    }
    c.rlcb_pending[k] = false;
    const int v = c.rlcb_host_flag[k] ? 1 : 0;
    c.rlcb_passed += (uint64_t)v;
    if (c.rlcb_seq[k] >= c.rlcb_last_seq) {
      c.rlcb_last_seq = c.rlcb_seq[k];
      c.rlcb_last = v;
      if (!v) c.rlcb_skipped = 0;
    }
  }
}

bool use_rlc_batch(uint64_t n) {
  Context& c = g_ctx;
  const int mode = g_rlc_mode.load();
  if (mode == HIPBLS_RLC_WINDOWS) return false;
  if (mode == HIPBLS_RLC_BATCH) return true;
  rlcb_poll(-1);
  if (n < kRlcbMinItems) return false;
  if (c.rlcb_last == 0 && c.rlcb_skipped < kRlcbBackoff) {
    ++c.rlcb_skipped;
    return false;
  }
  return true;
}

// Stages 1-6 of rlcb.h on stream s, then the window/fallback stages of rlc.h for the items still pending (none
// when the batch check passed: those kernels then find nothing to do).  Shares launch_rlc's H(m) table setup.
int launch_rlc_batch(const uint8_t* d_pks, const uint8_t* d_sigs, const uint32_t* d_midx, uint64_t n,
                     const uint8_t* d_msgs, const uint64_t* d_offs, uint64_t n_msgs, const rlc_seed& seed,
                     int32_t* d_status, hipStream_t s, const uint32_t* d_kidx, uint32_t* d_H, uint64_t hstride,
                     const uint32_t* d_hslot, const uint32_t* d_mlist, uint64_t n_hash) {
  Context& c = g_ctx;
  const uint64_t T = c.t_size;
  const int32_t* tcode = (const int32_t*)c.t_code.p;
  const uint32_t* tab = (const uint32_t*)c.t_tab.p;
  const uint64_t npts = 2 * n;
  const uint64_t nch = (n + RLCB_C - 1) / RLCB_C;
  const uint64_t n_win = (n + RLC_W - 1) / RLC_W;
  if (!c.rlcb_host_flag) {
    HIP_TRY(hipHostMalloc((void**)&c.rlcb_host_flag, Context::kRlcbSlots * sizeof(int32_t), hipHostMallocDefault));
    for (int k = 0; k < Context::kRlcbSlots; ++k) HIP_TRY(hipEventCreateWithFlags(&c.rlcb_ev[k], hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&c.rlcb_ev_items, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&c.rlcb_ev_msm, hipEventDisableTiming));
  }
  int rc = ensure_rlc_streams();
  if (rc) return rc;
  const int slot = (int)(c.rlcb_next_seq % Context::kRlcbSlots);
  rlcb_poll(slot);  // only blocks when kRlcbSlots verdicts are still in flight
  HIP_TRY(c.m_pts.ensure(npts * 48 * 4));
  HIP_TRY(c.m_sc.ensure(npts * 4));
  HIP_TRY(c.m_cnt.ensure((uint64_t)MSM_WINDOWS * MSM_NB * 4));
  HIP_TRY(c.m_off.ensure((uint64_t)MSM_WINDOWS * (MSM_NB + 1) * 4));
  HIP_TRY(c.m_cur.ensure((uint64_t)MSM_WINDOWS * MSM_NB * 4));
  HIP_TRY(c.m_list.ensure((uint64_t)MSM_WINDOWS * npts * 4));
  HIP_TRY(c.m_B.ensure((uint64_t)MSM_WINDOWS * MSM_NB * 72 * 4));
  HIP_TRY(c.m_Sg.ensure((uint64_t)MSM_WINDOWS * MSM_NSEG * 72 * 4));
  HIP_TRY(c.m_W.ensure((uint64_t)MSM_WINDOWS * 72 * 4));
  HIP_TRY(c.m_F.ensure(nch * 144 * 4));
  HIP_TRY(c.m_F2.ensure(((nch + 15) / 16) * 144 * 4));
  HIP_TRY(c.m_FS.ensure(144 * 4));
  HIP_TRY(c.m_flag.ensure(4));
  uint32_t* rpk = (uint32_t*)c.r_pk.p;
  uint32_t* rsig = (uint32_t*)c.r_sig.p;
  uint32_t* pts = (uint32_t*)c.m_pts.p;
  uint32_t* sc = (uint32_t*)c.m_sc.p;
  int32_t* flag = (int32_t*)c.m_flag.p;
  // Streams: the caller's stream s hashes the messages; sub[0] runs items -> MSM -> the (-g1, S) Miller value;
  // sub[1] runs the chunk Miller loops and their product once the items and the hash are done; s joins both for
  // the verdict and the window stages.
  hipStream_t s0 = c.sub[0], s1 = c.sub[1];
  rc = ws_begin(s);
  if (rc) return rc;
  HIP_TRY(hipMemsetAsync(c.m_cnt.p, 0, (size_t)MSM_WINDOWS * MSM_NB * 4, s));
  HIP_TRY(hipMemsetAsync(c.r_cnt.p, 0, 4, s));
  HIP_TRY(hipEventRecord(c.ev_fork, s));
  if (n_hash) {
    rc = timed("rlc_hash", s, [&] {
      hipLaunchKernelGGL(k_rlc_hash, dim3((unsigned)grid_for(n_hash)), dim3(kBlock), 0, s, d_msgs, d_offs, n_hash,
                         d_mlist, d_H, hstride, d_hslot);
    });
    if (rc) return rc;
  }
  HIP_TRY(hipEventRecord(c.ev_hash, s));
  HIP_TRY(hipStreamWaitEvent(s0, c.ev_fork, 0));
  rc = timed("rlcb_items", s0, [&] {
    hipLaunchKernelGGL(k_rlcb_items, dim3((unsigned)grid_for(n)), dim3(kBlock), 0, s0, n, d_pks, d_sigs, d_midx, n_msgs,
                       seed, rpk, pts, sc, d_status, d_kidx, T, tcode, tab);
  });
  if (rc) return rc;
  HIP_TRY(hipEventRecord(c.rlcb_ev_items, s0));
  rc = timed("rlcb_msm", s0, [&] {
    hipStream_t s = s0;
    const unsigned g256 = (unsigned)((npts + 255) / 256);
    hipLaunchKernelGGL(k_msm_hist, dim3(g256), dim3(256), 0, s, npts, (const uint32_t*)sc, (uint32_t*)c.m_cnt.p);
    hipLaunchKernelGGL(k_msm_scan, dim3(1), dim3(kScanThreads), 0, s, (const uint32_t*)c.m_cnt.p, (uint32_t*)c.m_off.p,
                       (uint32_t*)c.m_cur.p);
    hipLaunchKernelGGL(k_msm_scatter, dim3(g256), dim3(256), 0, s, npts, (const uint32_t*)sc, (uint32_t*)c.m_cur.p,
                       (uint32_t*)c.m_list.p);
    hipLaunchKernelGGL(k_msm_bucket, dim3((unsigned)grid_for((uint64_t)MSM_WINDOWS * MSM_NB)), dim3(kBlock), 0, s,
                       (const uint32_t*)c.m_off.p, (const uint32_t*)c.m_list.p, npts, (const uint32_t*)pts,
                       (uint32_t*)c.m_B.p);
    hipLaunchKernelGGL(k_msm_segment, dim3((unsigned)grid_for((uint64_t)MSM_WINDOWS * MSM_NSEG)), dim3(kBlock), 0, s,
                       (const uint32_t*)c.m_B.p, (uint32_t*)c.m_Sg.p);
    hipLaunchKernelGGL(k_msm_window, dim3(MSM_WINDOWS), dim3(kSumBlock), 0, s, (const uint32_t*)c.m_Sg.p,
                       (uint32_t*)c.m_W.p);
  });
  if (rc) return rc;
  rc = timed("rlcb_sfactor", s0, [&] {
    hipLaunchKernelGGL(k_rlcb_sfactor, dim3(1), dim3(kBlock), 0, s0, (const uint32_t*)c.m_W.p, (uint32_t*)c.m_FS.p);
  });
  if (rc) return rc;
  HIP_TRY(hipEventRecord(c.rlcb_ev_msm, s0));
  HIP_TRY(hipStreamWaitEvent(s1, c.rlcb_ev_items, 0));
  HIP_TRY(hipStreamWaitEvent(s1, c.ev_hash, 0));
  rc = timed("rlcb_chunks", s1, [&] {
    hipLaunchKernelGGL(k_rlcb_chunks, dim3((unsigned)grid_for(nch)), dim3(kBlock), 0, s1, n, (const int32_t*)d_status,
                       d_midx, (const uint32_t*)rpk, (const uint32_t*)d_H, hstride, d_hslot, (uint32_t*)c.m_F.p, nch);
  });
  if (rc) return rc;
  uint32_t* src = (uint32_t*)c.m_F.p;
  uint32_t* dst = (uint32_t*)c.m_F2.p;
  uint64_t cur = nch;
  rc = timed("rlcb_product", s1, [&] {
    while (cur > 1) {
      const uint64_t nxt = (cur + 15) / 16;
      hipLaunchKernelGGL(k_fp12_prod, dim3((unsigned)grid_for(nxt)), dim3(kBlock), 0, s1, (const uint32_t*)src, cur,
                         dst, nxt, 16);
      uint32_t* t = src;
      src = dst;
      dst = t;
      cur = nxt;
    }
  });
  if (rc) return rc;
  HIP_TRY(hipEventRecord(c.ev_join[1], s1));
  HIP_TRY(hipStreamWaitEvent(s, c.rlcb_ev_msm, 0));
  HIP_TRY(hipStreamWaitEvent(s, c.ev_join[1], 0));
  rc = timed("rlcb_final", s, [&] {
    hipLaunchKernelGGL(k_rlcb_final, dim3(1), dim3(kBlock), 0, s, (const uint32_t*)src, (const uint32_t*)c.m_FS.p, flag);
  });
  if (rc) return rc;
  rc = timed("rlcb_mark", s, [&] {
    hipLaunchKernelGGL(k_rlcb_mark, dim3((unsigned)grid_for(n)), dim3(kBlock), 0, s, n, (const int32_t*)flag, d_status,
                       (const uint32_t*)pts, (const uint32_t*)sc, rsig);
  });
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(c.rlcb_host_flag + slot, flag, 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipEventRecord(c.rlcb_ev[slot], s));
  c.rlcb_pending[slot] = true;
  c.rlcb_seq[slot] = ++c.rlcb_next_seq;
  c.rlcb_attempted += 1;
  // window + fallback stages over whatever is still pending (nothing when the batch check passed)
  int32_t* win = (int32_t*)c.r_win.p;
  uint32_t* list = (uint32_t*)c.r_list.p;
  uint32_t* cnt = (uint32_t*)c.r_cnt.p;
  if (use_pairs(n_win, kLg2MaxWindows))
    rc = timed("rlc_window_lg2", s, [&] {
      hipLaunchKernelGGL(k_rlc_window_lg2, dim3((unsigned)grid_for(2 * n_win)), dim3(kBlock), 0, s, (uint64_t)0, n_win,
                         n, d_midx, (const uint32_t*)rpk, (const uint32_t*)rsig, (const uint32_t*)d_H, hstride, d_hslot,
                         d_status, win, list, cnt);
    });
  else
    rc = timed("rlc_window", s, [&] {
      hipLaunchKernelGGL(k_rlc_window, dim3((unsigned)grid_for(n_win)), dim3(kBlock), 0, s, (uint64_t)0, n_win, n,
                         d_midx, (const uint32_t*)rpk, (const uint32_t*)rsig, (const uint32_t*)d_H, hstride, d_hslot,
                         d_status, win, list, cnt);
    });
  if (rc) return rc;
  if (g_pair_mode.load() != HIPBLS_PAIR_SINGLE)
    rc = timed("rlc_fallback_lg2", s, [&] {
      hipLaunchKernelGGL(k_rlc_fallback_lg2, dim3((unsigned)grid_for(2 * n)), dim3(kBlock), 0, s,
                         (const uint32_t*)list, (const uint32_t*)cnt, n, d_pks, d_sigs, d_midx, (const uint32_t*)d_H,
                         hstride, d_hslot, d_status, d_kidx, T, tab);
    });
  else
    rc = timed("rlc_fallback", s, [&] {
      hipLaunchKernelGGL(k_rlc_fallback, dim3((unsigned)grid_for(n)), dim3(kBlock), 0, s, (const uint32_t*)list,
                         (const uint32_t*)cnt, n, d_pks, d_sigs, d_midx, (const uint32_t*)d_H, hstride, d_hslot,
                         d_status, d_kidx, T, tab);
    });
  if (rc) return rc;
  c.r_windows = n_win;
  return ws_end(s);
}

int launch_tagg(const uint8_t* d_sigs, const int64_t* d_ids, const uint64_t* d_goffs, uint64_t n_groups,
                uint64_t n_parts, uint8_t* d_out, int32_t* d_status, hipStream_t s) {
  if (n_groups == 0) return HIPBLS_OK;
  HIP_TRY(g_ctx.b_pts.ensure((n_parts ? n_parts : 1) * 72 * 4));
  HIP_TRY(g_ctx.b_pst.ensure((n_parts ? n_parts : 1) * 4));
  int rc = ws_begin(s);
  if (rc) return rc;
  if (n_parts) {
    rc = timed("tagg_scale", s, [&] {
      hipLaunchKernelGGL(k_tagg_scale, dim3((unsigned)grid_for(n_parts)), dim3(kBlock), 0, s, d_sigs, d_ids, d_goffs,
                         n_groups, n_parts, (uint32_t*)g_ctx.b_pts.p, (int32_t*)g_ctx.b_pst.p);
    });
    if (rc) return rc;
  }
  rc = timed("tagg_sum", s, [&] {
    hipLaunchKernelGGL(k_tagg_sum, dim3((unsigned)grid_for(n_groups)), dim3(kBlock), 0, s,
                       (const uint32_t*)g_ctx.b_pts.p, (const int32_t*)g_ctx.b_pst.p, d_goffs, n_groups, n_parts, d_out,
                       d_status);
  });
  if (rc) return rc;
  return ws_end(s);
}

// sigagg in one call: ThresholdAggregate on sub[0] while sub[1] decodes the validators' root keys and hashes their
// messages; the caller's stream joins both and runs the pairing checks on the aggregates (kernels.h, k_tagg_sum_v).
int launch_tagg_verify(const uint8_t* d_sigs, const int64_t* d_ids, const uint64_t* d_goffs, uint64_t n_groups,
                       uint64_t n_parts, const uint8_t* d_dvpks, const uint8_t* d_msgs, const uint64_t* d_moffs,
                       uint8_t* d_out, int32_t* d_astatus, int32_t* d_vstatus, hipStream_t s) {
  Context& c = g_ctx;
  if (n_groups == 0) return HIPBLS_OK;
  int rc = ensure_rlc_streams();
  if (rc) return rc;
  HIP_TRY(c.b_pts.ensure((n_parts ? n_parts : 1) * 72 * 4));
  HIP_TRY(c.b_pst.ensure((n_parts ? n_parts : 1) * 4));
  HIP_TRY(c.v_ws.ensure(n_groups * 120 * 4));
  HIP_TRY(c.b_aux.ensure(n_groups * 4));
  uint32_t* ws = (uint32_t*)c.v_ws.p;
  int32_t* agg_inf = (int32_t*)c.b_aux.p;
  hipStream_t s0 = c.sub[0], s1 = c.sub[1];
  rc = ws_begin(s);
  if (rc) return rc;
  HIP_TRY(hipEventRecord(c.ev_fork, s));
  HIP_TRY(hipStreamWaitEvent(s0, c.ev_fork, 0));
  HIP_TRY(hipStreamWaitEvent(s1, c.ev_fork, 0));
  if (n_parts) {
    rc = timed("tagg_scale", s0, [&] {
      hipLaunchKernelGGL(k_tagg_scale, dim3((unsigned)grid_for(n_parts)), dim3(kBlock), 0, s0, d_sigs, d_ids, d_goffs,
                         n_groups, n_parts, (uint32_t*)c.b_pts.p, (int32_t*)c.b_pst.p);
    });
    if (rc) return rc;
  }
  rc = timed("tagg_sum", s0, [&] {
    hipLaunchKernelGGL(k_tagg_sum_v, dim3((unsigned)grid_for(n_groups)), dim3(kBlock), 0, s0,
                       (const uint32_t*)c.b_pts.p, (const int32_t*)c.b_pst.p, d_goffs, n_groups, n_parts, d_out,
                       d_astatus, ws, agg_inf);
  });
  if (rc) return rc;
  HIP_TRY(hipEventRecord(c.ev_join[0], s0));
  rc = timed("tv_prep_pk", s1, [&] {
    hipLaunchKernelGGL(k_tv_prep_pk, dim3((unsigned)grid_for(n_groups)), dim3(kBlock), 0, s1, d_dvpks, d_msgs, d_moffs,
                       n_groups, ws, d_vstatus);
  });
  if (rc) return rc;
  HIP_TRY(hipEventRecord(c.ev_join[1], s1));
  HIP_TRY(hipStreamWaitEvent(s, c.ev_join[0], 0));
  HIP_TRY(hipStreamWaitEvent(s, c.ev_join[1], 0));
  hipLaunchKernelGGL(k_tv_join, dim3((unsigned)grid_for(n_groups)), dim3(kBlock), 0, s, n_groups,
                     (const int32_t*)d_astatus, (const int32_t*)agg_inf, d_vstatus);
  HIP_TRY(hipGetLastError());
  if (use_pairs(n_groups, kLg2MaxVerify))
    rc = timed("verify_pair_lg2", s, [&] {
      hipLaunchKernelGGL(k_verify_pair_lg2, dim3((unsigned)grid_for(2 * n_groups)), dim3(kBlock), 0, s,
                         (const uint32_t*)ws, n_groups, d_vstatus);
    });
  else
    rc = timed("verify_pair_single", s, [&] {
      hipLaunchKernelGGL(k_verify_pair_single, dim3((unsigned)grid_for(n_groups)), dim3(kBlock), 0, s,
                         (const uint32_t*)ws, n_groups, d_vstatus);
    });
  if (rc) return rc;
  return ws_end(s);
}

int launch_fav(const uint8_t* d_pks, uint64_t nkeys, const uint64_t* d_goff, uint64_t n_groups, const uint8_t* d_sigs,
               const uint8_t* d_msgs, const uint64_t* d_moffs, int32_t* d_status, hipStream_t s) {
  Context& c = g_ctx;
  if (n_groups == 0) return HIPBLS_OK;
  HIP_TRY(c.b_pts.ensure((nkeys ? nkeys : 1) * 24 * 4));
  HIP_TRY(c.b_pst.ensure((nkeys ? nkeys : 1) * 4));
  int rc = ws_begin(s);
  if (rc) return rc;
  if (nkeys)
    hipLaunchKernelGGL(k_g1_decode, dim3((unsigned)grid_for(nkeys)), dim3(kBlock), 0, s, d_pks, nkeys,
                       (uint32_t*)c.b_pts.p, (int32_t*)c.b_pst.p);
  rc = timed("fav", s, [&] {
    hipLaunchKernelGGL(k_fav_batch, dim3((unsigned)n_groups), dim3(kFavBlock), 0, s, (const uint32_t*)c.b_pts.p,
                       (const int32_t*)c.b_pst.p, nkeys, d_goff, d_sigs, d_msgs, d_moffs, d_status);
  });
  if (rc) return rc;
  return ws_end(s);
}

// Aggregate: decode in parallel, per-workgroup partial sums, one final workgroup (kernels.h).
int launch_aggregate(const uint8_t* d_sigs, uint64_t n, uint8_t* d_out, int32_t* d_status, hipStream_t s) {
  Context& c = g_ctx;
  const uint64_t per_wg = 8 * (uint64_t)kSumBlock;  // points folded per lane before the tree
  uint64_t nwg = (n + per_wg - 1) / per_wg;
  if (nwg < 1) nwg = 1;
  if (nwg > 1024) nwg = 1024;
  HIP_TRY(c.b_pts.ensure((n ? n : 1) * 48 * 4));
  HIP_TRY(c.b_pst.ensure((n ? n : 1) * 4));
  HIP_TRY(c.b_part.ensure(nwg * 72 * 4));
  HIP_TRY(c.b_bad.ensure(4));
  int rc = ws_begin(s);
  if (rc) return rc;
  HIP_TRY(hipMemsetAsync(c.b_bad.p, 0, 4, s));
  if (n)
    hipLaunchKernelGGL(k_g2_decode, dim3((unsigned)grid_for(n)), dim3(kBlock), 0, s, d_sigs, n, (uint32_t*)c.b_pts.p,
                       (int32_t*)c.b_pst.p);
  hipLaunchKernelGGL(k_g2_sum_partial, dim3((unsigned)nwg), dim3(kSumBlock), 0, s, (const uint32_t*)c.b_pts.p,
                     (const int32_t*)c.b_pst.p, n, (uint32_t*)c.b_part.p, (int32_t*)c.b_bad.p);
  hipLaunchKernelGGL(k_g2_sum_final, dim3(1), dim3(kSumBlock), 0, s, (const uint32_t*)c.b_part.p, nwg,
                     (const int32_t*)c.b_bad.p, d_out, d_status);
  HIP_TRY(hipGetLastError());
  return ws_end(s);
}

bool mul_overflows(uint64_t a, uint64_t b) { return b != 0 && a > UINT64_MAX / b; }

bool offsets_ok(const uint64_t* offs, uint64_t n) {
  if (offs[0] != 0) return false;
  for (uint64_t i = 0; i < n; ++i)
    if (offs[i + 1] < offs[i] || offs[i + 1] - offs[i] > 0xffffffffull) return false;
  return true;
}

// ============================================================================ submission queue
// Coalesces concurrent single-item Verify calls (tbls.Verify from parsigex / validatorapi / sigagg goroutines,
// core/parsigex/parsigex.go:86-91, core/validatorapi/validatorapi.go:246-283) into batched launches.  A batch
// is launched as soon as the worker is free and work is pending: while one batch runs on the GPU, arrivals
// accumulate into the next, so the batch size follows the offered load.  An idle worker waits gather_us for
// company before launching a small batch.  The worker owns its stream and buffers; callers block only on their
// own batch's completion, never on a lock held across GPU work.
struct VBatch {
  std::vector<uint8_t> pk, sig, msg;
  std::vector<uint64_t> off{0};
  std::vector<int32_t> status;
  int rc = HIPBLS_OK;
  bool done = false;
  uint64_t n() const { return off.size() - 1; }
};

struct VerifyQueue {
  std::mutex mu;
  std::condition_variable cv_work, cv_done;
  std::deque<std::shared_ptr<VBatch>> open;  // accepting (back) / waiting for the worker (front)
  std::unordered_map<uint64_t, std::pair<std::shared_ptr<VBatch>, uint32_t>> tickets;
  uint64_t next_ticket = 1;
  std::thread worker;
  bool started = false, stop = false;
  uint64_t max_batch = 65536;
  uint32_t gather_us = 200;
  uint64_t batches = 0, items = 0;
  hipStream_t stream = nullptr;
  DevBuf d_pk, d_sig, d_msg, d_off, d_st, d_ws;
};
VerifyQueue g_q;

int run_batch(VBatch& b) {
  VerifyQueue& q = g_q;
  const uint64_t n = b.n();
  b.status.assign(n, HIPBLS_ERR_DEVICE);
  HIP_TRY(q.d_pk.ensure(n * 48));
  HIP_TRY(q.d_sig.ensure(n * 96));
  HIP_TRY(q.d_msg.ensure(b.msg.size() ? b.msg.size() : 1));
  HIP_TRY(q.d_off.ensure((n + 1) * 8));
  HIP_TRY(q.d_st.ensure(n * 4));
  HIP_TRY(hipMemcpyAsync(q.d_pk.p, b.pk.data(), n * 48, hipMemcpyHostToDevice, q.stream));
  HIP_TRY(hipMemcpyAsync(q.d_sig.p, b.sig.data(), n * 96, hipMemcpyHostToDevice, q.stream));
  if (b.msg.size()) HIP_TRY(hipMemcpyAsync(q.d_msg.p, b.msg.data(), b.msg.size(), hipMemcpyHostToDevice, q.stream));
  HIP_TRY(hipMemcpyAsync(q.d_off.p, b.off.data(), (n + 1) * 8, hipMemcpyHostToDevice, q.stream));
  int rc = launch_verify((const uint8_t*)q.d_pk.p, (const uint8_t*)q.d_msg.p, (const uint64_t*)q.d_off.p,
                         (const uint8_t*)q.d_sig.p, n, (int32_t*)q.d_st.p, q.stream, q.d_ws);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(b.status.data(), q.d_st.p, n * 4, hipMemcpyDeviceToHost, q.stream));
  HIP_TRY(hipStreamSynchronize(q.stream));
  return HIPBLS_OK;
}

void queue_worker() {
  VerifyQueue& q = g_q;
  const bool dev_ok = hipSetDevice(g_ctx.device) == hipSuccess &&
                      hipStreamCreateWithFlags(&q.stream, hipStreamNonBlocking) == hipSuccess;
  std::unique_lock<std::mutex> lk(q.mu);
  for (;;) {
    q.cv_work.wait(lk, [&] { return q.stop || (!q.open.empty() && q.open.front()->n() > 0); });
    if (q.open.empty() || q.open.front()->n() == 0) break;  // stop requested and nothing pending
    if (q.gather_us && q.open.front()->n() < q.max_batch && !q.stop) {
      const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(q.gather_us);
      q.cv_work.wait_until(lk, until, [&] { return q.stop || q.open.front()->n() >= q.max_batch; });
    }
    std::shared_ptr<VBatch> b = q.open.front();
    q.open.pop_front();
    lk.unlock();
    const int rc = dev_ok ? run_batch(*b) : HIPBLS_ERR_DEVICE;
    lk.lock();
    b->rc = rc;
    b->done = true;
    q.batches += 1;
    q.items += b->n();
    q.cv_done.notify_all();
  }
}

void queue_shutdown() {
  {
    std::lock_guard<std::mutex> lk(g_q.mu);
    if (!g_q.started) return;
    g_q.stop = true;
  }
  g_q.cv_work.notify_all();
  if (g_q.worker.joinable()) g_q.worker.join();
  std::lock_guard<std::mutex> lk(g_q.mu);
  g_q.started = false;
  g_q.stop = false;
}

int queue_submit(const uint8_t* pk48, const uint8_t* msg, uint64_t msg_len, const uint8_t* sig96, uint64_t* ticket) {
  if (!pk48 || !sig96 || !ticket || (msg_len && !msg) || msg_len > 0xffffffffull) return arg_err("bad verify arguments");
  int rc = bind_device();
  if (rc) return rc;
  VerifyQueue& q = g_q;
  std::lock_guard<std::mutex> lk(q.mu);
  if (!q.started) {
    q.worker = std::thread(queue_worker);
    q.started = true;
    static bool hooked = false;
    if (!hooked) {
      hooked = true;
      atexit(queue_shutdown);  // drain the in-flight batch before the HIP runtime tears down
    }
  }
  if (q.open.empty() || q.open.back()->n() >= q.max_batch) q.open.push_back(std::make_shared<VBatch>());
  VBatch& b = *q.open.back();
  const uint32_t idx = (uint32_t)b.n();
  b.pk.insert(b.pk.end(), pk48, pk48 + 48);
  b.sig.insert(b.sig.end(), sig96, sig96 + 96);
  if (msg_len) b.msg.insert(b.msg.end(), msg, msg + msg_len);
  b.off.push_back(b.msg.size());
  const uint64_t t = q.next_ticket++;
  q.tickets.emplace(t, std::make_pair(q.open.back(), idx));
  *ticket = t;
  q.cv_work.notify_one();
  return HIPBLS_OK;
}

int queue_wait(uint64_t ticket, int32_t* status) {
  if (!status) return arg_err("null status");
  VerifyQueue& q = g_q;
  std::unique_lock<std::mutex> lk(q.mu);
  auto it = q.tickets.find(ticket);
  if (it == q.tickets.end()) return arg_err("unknown verify ticket");
  std::shared_ptr<VBatch> b = it->second.first;
  const uint32_t idx = it->second.second;
  q.tickets.erase(it);
  q.cv_done.wait(lk, [&] { return b->done; });
  if (b->rc) {
    g_last_error = "verify queue batch failed on the device";
    return b->rc;
  }
  *status = b->status[idx];
  return HIPBLS_OK;
}

// ============================================================================ H(m) cache
// Assigns cache columns for the n_msgs distinct messages of one call: fills slot[m] and the list of messages that
// must be hashed (misses).  Returns false (cache bypassed) when disabled or the call has more messages than slots.
bool hcache_assign(HCache& hc, const uint8_t* msgs, const uint64_t* offs, uint64_t n_msgs, std::vector<uint32_t>& slot,
                   std::vector<uint32_t>& miss) {
  if (hc.cap == 0 || n_msgs > hc.cap) return false;
  slot.assign(n_msgs, 0);
  miss.clear();
  std::vector<std::string> keys(n_msgs);
  std::vector<char> hit(n_msgs, 0);
  for (uint64_t m = 0; m < n_msgs; ++m) {
    keys[m].assign((const char*)msgs + offs[m], offs[m + 1] - offs[m]);
    auto it = hc.map.find(keys[m]);
    if (it != hc.map.end()) {
      slot[m] = (uint32_t)it->second;
      hit[m] = 1;
    }
  }
  // The misses take slots [ring, ring + k); a hit inside that range would be overwritten by this very call, so it
  // is demoted to a miss (which grows k): iterate to the fixed point.
  for (;;) {
    uint64_t k = 0;
    for (uint64_t m = 0; m < n_msgs; ++m) k += hit[m] ? 0 : 1;
    bool changed = false;
    for (uint64_t m = 0; m < n_msgs; ++m)
      if (hit[m] && (slot[m] + hc.cap - hc.ring) % hc.cap < k) {
        hit[m] = 0;
        changed = true;
      }
    if (!changed) break;
  }
  for (uint64_t m = 0; m < n_msgs; ++m) {
    if (hit[m]) {
      hc.hits += 1;
      continue;
    }
    // messages are distinct within a call (the caller's message table), so each miss takes its own slot
    const uint32_t s = (uint32_t)hc.ring;
    hc.ring = (hc.ring + 1) % hc.cap;
    if (!hc.key_of[s].empty()) hc.map.erase(hc.key_of[s]);
    hc.key_of[s] = keys[m];
    hc.map[keys[m]] = s;
    slot[m] = s;
    miss.push_back((uint32_t)m);
    hc.misses += 1;
  }
  return true;
}

// Host-buffer RLC body shared by the wire-format and key-table calls (context lock held).
int rlc_host(const uint8_t* pks, const uint32_t* key_idx, const uint8_t* sigs, const uint32_t* msg_idx, uint64_t n,
             const uint8_t* msgs, const uint64_t* msg_offsets, uint64_t n_msgs, const uint8_t* seed32, int32_t* status) {
  Context& c = g_ctx;
  const uint64_t msg_total = msg_offsets[n_msgs];
  if (pks) HIP_TRY(c.b_pk.ensure(n * 48));
  if (key_idx) HIP_TRY(c.b_kidx.ensure(n * 4));
  HIP_TRY(c.b_sig.ensure(n * 96));
  HIP_TRY(c.r_midx.ensure(n * 4));
  HIP_TRY(c.b_msg.ensure(msg_total ? msg_total : 1));
  HIP_TRY(c.b_off.ensure((n_msgs + 1) * 8));
  HIP_TRY(c.b_st.ensure(n * 4));
  if (pks) HIP_TRY(hipMemcpyAsync(c.b_pk.p, pks, n * 48, hipMemcpyHostToDevice, c.stream));
  if (key_idx) HIP_TRY(hipMemcpyAsync(c.b_kidx.p, key_idx, n * 4, hipMemcpyHostToDevice, c.stream));
  HIP_TRY(hipMemcpyAsync(c.b_sig.p, sigs, n * 96, hipMemcpyHostToDevice, c.stream));
  HIP_TRY(hipMemcpyAsync(c.r_midx.p, msg_idx, n * 4, hipMemcpyHostToDevice, c.stream));
  if (msg_total) HIP_TRY(hipMemcpyAsync(c.b_msg.p, msgs, msg_total, hipMemcpyHostToDevice, c.stream));
  HIP_TRY(hipMemcpyAsync(c.b_off.p, msg_offsets, (n_msgs + 1) * 8, hipMemcpyHostToDevice, c.stream));
  std::vector<uint32_t> slot, miss;
  uint32_t* dH = nullptr;
  const uint32_t *dslot = nullptr, *dmiss = nullptr;
  uint64_t stride = 0, n_hash = 0;
  if (hcache_assign(c.hcache, msgs, msg_offsets, n_msgs, slot, miss)) {
    HIP_TRY(c.r_slot.ensure((n_msgs ? n_msgs : 1) * 4));
    HIP_TRY(c.r_mlist.ensure((miss.size() ? miss.size() : 1) * 4));
    // the copies run on the library stream behind every earlier workspace user (ws_done)
    int rc = ws_begin(c.stream);
    if (rc) return rc;
    if (n_msgs) HIP_TRY(hipMemcpyAsync(c.r_slot.p, slot.data(), n_msgs * 4, hipMemcpyHostToDevice, c.stream));
    if (miss.size()) HIP_TRY(hipMemcpyAsync(c.r_mlist.p, miss.data(), miss.size() * 4, hipMemcpyHostToDevice, c.stream));
    dH = (uint32_t*)c.hcache.table.p;
    stride = c.hcache.cap;
    dslot = (const uint32_t*)c.r_slot.p;
    dmiss = (const uint32_t*)c.r_mlist.p;
    n_hash = miss.size();
  }
  int rc = launch_rlc(pks ? (const uint8_t*)c.b_pk.p : nullptr, (const uint8_t*)c.b_sig.p, (const uint32_t*)c.r_midx.p,
                      n, (const uint8_t*)c.b_msg.p, (const uint64_t*)c.b_off.p, n_msgs, seed32, (int32_t*)c.b_st.p,
                      c.stream, key_idx ? (const uint32_t*)c.b_kidx.p : nullptr, dH, stride, dslot, dmiss, n_hash);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(status, c.b_st.p, n * 4, hipMemcpyDeviceToHost, c.stream));
  HIP_TRY(hipStreamSynchronize(c.stream));
  return HIPBLS_OK;
}

}  // namespace

// ============================================================================ C-ABI
extern "C" {

int hipbls_abi_version(void) { return HIPBLS_ABI_VERSION; }

int hipbls_init(int device) {
  std::lock_guard<std::mutex> lk(g_init_mu);
  if (g_ctx.device >= 0) {
    if (device >= 0 && device != g_ctx.device) return arg_err("hipbls already bound to another device");
    HIP_TRY(hipSetDevice(g_ctx.device));
    return HIPBLS_OK;
  }
  return init_locked(device < 0 ? 0 : device);
}

int hipbls_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int hipbls_current_device(void) { return g_ctx.device; }

const char* hipbls_last_error(void) { return g_last_error.c_str(); }

int hipbls_set_timing(int enabled) {
  g_ctx.timing_enabled = enabled != 0;
  return HIPBLS_OK;
}

int hipbls_rlc_set_mode(int mode) {
  if (mode != HIPBLS_RLC_AUTO && mode != HIPBLS_RLC_WINDOWS && mode != HIPBLS_RLC_BATCH)
    return arg_err("unknown RLC mode");
  return g_rlc_mode.exchange(mode);
}

int hipbls_rlc_batch_stats(uint64_t* attempted, uint64_t* passed, int32_t* last) {
  if (!attempted || !passed || !last) return arg_err("null output");
  ENTER();
  rlcb_poll(-1, true);
  *attempted = g_ctx.rlcb_attempted;
  *passed = g_ctx.rlcb_passed;
  *last = g_ctx.rlcb_last;
  return HIPBLS_OK;
}

int hipbls_set_pair_mode(int mode) {
  if (mode != HIPBLS_PAIR_AUTO && mode != HIPBLS_PAIR_SINGLE && mode != HIPBLS_PAIR_LANES)
    return arg_err("unknown pair mode");
  return g_pair_mode.exchange(mode);
}

int hipbls_verify_batch(const uint8_t* pks, const uint8_t* msgs, const uint64_t* msg_offsets, const uint8_t* sigs,
                        uint64_t n, int32_t* status) {
  if (n == 0) return HIPBLS_OK;
  if (!pks || !msg_offsets || !sigs || !status || mul_overflows(n, 96)) return arg_err("bad verify arguments");
  if (!offsets_ok(msg_offsets, n)) return arg_err("bad message offsets");
  const uint64_t msg_total = msg_offsets[n];
  if (msg_total && !msgs) return arg_err("null messages");
  ENTER();
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
  int rc = ws_begin(c.stream);
  if (rc) return rc;
  rc = launch_verify((const uint8_t*)c.b_pk.p, (const uint8_t*)c.b_msg.p, (const uint64_t*)c.b_off.p,
                     (const uint8_t*)c.b_sig.p, n, (int32_t*)c.b_st.p, c.stream, c.v_ws);
  if (rc) return rc;
  rc = ws_end(c.stream);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(status, c.b_st.p, n * 4, hipMemcpyDeviceToHost, c.stream));
  HIP_TRY(hipStreamSynchronize(c.stream));
  return HIPBLS_OK;
}

int hipbls_verify_batch_device(const uint8_t* d_pks, const uint8_t* d_msgs, const uint64_t* d_msg_offsets,
                               const uint8_t* d_sigs, uint64_t n, int32_t* d_status, void* stream) {
  ENTER();
  const hipStream_t s = pick(stream);
  int rc = ws_begin(s);
  if (rc) return rc;
  rc = launch_verify(d_pks, d_msgs, d_msg_offsets, d_sigs, n, d_status, s, g_ctx.v_ws);
  if (rc) return rc;
  return ws_end(s);
}

int hipbls_verify(const uint8_t* pk48, const uint8_t* msg, uint64_t msg_len, const uint8_t* sig96, int32_t* status) {
  uint64_t t = 0;
  const int rc = queue_submit(pk48, msg, msg_len, sig96, &t);
  if (rc) return rc;
  return queue_wait(t, status);
}

int hipbls_verify_submit(const uint8_t* pk48, const uint8_t* msg, uint64_t msg_len, const uint8_t* sig96,
                         uint64_t* ticket) {
  return queue_submit(pk48, msg, msg_len, sig96, ticket);
}

int hipbls_verify_wait(uint64_t ticket, int32_t* status) { return queue_wait(ticket, status); }

int hipbls_queue_config(uint64_t max_batch, uint32_t gather_us) {
  if (max_batch == 0 || max_batch > (1ull << 24)) return arg_err("max_batch out of range");
  std::lock_guard<std::mutex> lk(g_q.mu);
  g_q.max_batch = max_batch;
  g_q.gather_us = gather_us;
  return HIPBLS_OK;
}

int hipbls_queue_stats(uint64_t* batches, uint64_t* items) {
  if (!batches || !items) return arg_err("null output");
  std::lock_guard<std::mutex> lk(g_q.mu);
  *batches = g_q.batches;
  *items = g_q.items;
  return HIPBLS_OK;
}

int hipbls_verify_signed_data_batch(const uint8_t* pks, const uint8_t* object_roots, const uint8_t* domains,
                                    const uint8_t* sigs, uint64_t n, int32_t* status) {
  if (n == 0) return HIPBLS_OK;
  if (!pks || !object_roots || !domains || !sigs || !status || mul_overflows(n, 96)) return arg_err("bad arguments");
  ENTER();
  Context& c = g_ctx;
  HIP_TRY(c.b_pk.ensure(n * 48));
  HIP_TRY(c.b_sig.ensure(n * 96));
  HIP_TRY(c.b_aux.ensure(n * 64));
  HIP_TRY(c.b_msg.ensure(n * 32));
  HIP_TRY(c.b_off.ensure((n + 1) * 8));
  HIP_TRY(c.b_st.ensure(n * 4));
  HIP_TRY(hipMemcpyAsync(c.b_pk.p, pks, n * 48, hipMemcpyHostToDevice, c.stream));
  HIP_TRY(hipMemcpyAsync(c.b_sig.p, sigs, n * 96, hipMemcpyHostToDevice, c.stream));
  HIP_TRY(hipMemcpyAsync(c.b_aux.p, object_roots, n * 32, hipMemcpyHostToDevice, c.stream));
  HIP_TRY(hipMemcpyAsync((uint8_t*)c.b_aux.p + n * 32, domains, n * 32, hipMemcpyHostToDevice, c.stream));
  hipLaunchKernelGGL(k_signing_roots, dim3((unsigned)grid_for(n)), dim3(kBlock), 0, c.stream, (const uint8_t*)c.b_aux.p,
                     (const uint8_t*)c.b_aux.p + n * 32, n, (uint8_t*)c.b_msg.p, (uint64_t*)c.b_off.p);
  HIP_TRY(hipGetLastError());
  int rc = ws_begin(c.stream);
  if (rc) return rc;
  rc = launch_verify((const uint8_t*)c.b_pk.p, (const uint8_t*)c.b_msg.p, (const uint64_t*)c.b_off.p,
                     (const uint8_t*)c.b_sig.p, n, (int32_t*)c.b_st.p, c.stream, c.v_ws);
  if (rc) return rc;
  rc = ws_end(c.stream);
  if (rc) return rc;
  hipLaunchKernelGGL(k_zero_sig_status, dim3((unsigned)grid_for(n)), dim3(kBlock), 0, c.stream,
                     (const uint8_t*)c.b_sig.p, n, (int32_t*)c.b_st.p);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(status, c.b_st.p, n * 4, hipMemcpyDeviceToHost, c.stream));
  HIP_TRY(hipStreamSynchronize(c.stream));
  return HIPBLS_OK;
}

int hipbls_threshold_aggregate_batch(const uint8_t* sigs, const int64_t* share_idx, const uint64_t* group_offsets,
                                     uint64_t n_groups, uint8_t* out_sigs, int32_t* status) {
  if (n_groups == 0) return HIPBLS_OK;
  if (!group_offsets || !out_sigs || !status || mul_overflows(n_groups, 96)) return arg_err("bad arguments");
  if (group_offsets[0] != 0) return arg_err("group_offsets[0] != 0");
  for (uint64_t g = 0; g < n_groups; ++g)
    if (group_offsets[g + 1] < group_offsets[g]) return arg_err("decreasing group offsets");
  const uint64_t n_parts = group_offsets[n_groups];
  if (n_parts && (!sigs || !share_idx)) return arg_err("null partials");
  if (mul_overflows(n_parts, 288)) return arg_err("too many partials");
  ENTER();
  Context& c = g_ctx;
  HIP_TRY(c.b_sig.ensure((n_parts ? n_parts : 1) * 96));
  HIP_TRY(c.b_ids.ensure((n_parts ? n_parts : 1) * 8));
  HIP_TRY(c.b_off.ensure((n_groups + 1) * 8));
  HIP_TRY(c.b_out.ensure(n_groups * 96));
  HIP_TRY(c.b_st.ensure(n_groups * 4));
  if (n_parts) {
    HIP_TRY(hipMemcpyAsync(c.b_sig.p, sigs, n_parts * 96, hipMemcpyHostToDevice, c.stream));
    HIP_TRY(hipMemcpyAsync(c.b_ids.p, share_idx, n_parts * 8, hipMemcpyHostToDevice, c.stream));
  }
  HIP_TRY(hipMemcpyAsync(c.b_off.p, group_offsets, (n_groups + 1) * 8, hipMemcpyHostToDevice, c.stream));
  int rc = launch_tagg((const uint8_t*)c.b_sig.p, (const int64_t*)c.b_ids.p, (const uint64_t*)c.b_off.p, n_groups,
                       n_parts, (uint8_t*)c.b_out.p, (int32_t*)c.b_st.p, c.stream);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(out_sigs, c.b_out.p, n_groups * 96, hipMemcpyDeviceToHost, c.stream));
  HIP_TRY(hipMemcpyAsync(status, c.b_st.p, n_groups * 4, hipMemcpyDeviceToHost, c.stream));
  HIP_TRY(hipStreamSynchronize(c.stream));
  return HIPBLS_OK;
}

int hipbls_threshold_aggregate_verify_batch(const uint8_t* sigs, const int64_t* share_idx,
                                            const uint64_t* group_offsets, uint64_t n_groups, const uint8_t* dv_pks,
                                            const uint8_t* msgs, const uint64_t* msg_offsets, uint8_t* out_sigs,
                                            int32_t* agg_status, int32_t* verify_status) {
  if (n_groups == 0) return HIPBLS_OK;
  if (!group_offsets || !dv_pks || !msg_offsets || !out_sigs || !agg_status || !verify_status ||
      mul_overflows(n_groups, 120 * 4))
    return arg_err("bad arguments");
  if (group_offsets[0] != 0) return arg_err("group_offsets[0] != 0");
  for (uint64_t g = 0; g < n_groups; ++g)
    if (group_offsets[g + 1] < group_offsets[g]) return arg_err("decreasing group offsets");
  if (!offsets_ok(msg_offsets, n_groups)) return arg_err("bad message offsets");
  const uint64_t n_parts = group_offsets[n_groups];
  const uint64_t msg_total = msg_offsets[n_groups];
  if (n_parts && (!sigs || !share_idx)) return arg_err("null partials");
  if (msg_total && !msgs) return arg_err("null messages");
  if (mul_overflows(n_parts, 288)) return arg_err("too many partials");
  ENTER();
  Context& c = g_ctx;
  HIP_TRY(c.b_sig.ensure((n_parts ? n_parts : 1) * 96));
  HIP_TRY(c.b_ids.ensure((n_parts ? n_parts : 1) * 8));
  HIP_TRY(c.b_off.ensure((n_groups + 1) * 8));
  HIP_TRY(c.b_pk.ensure(n_groups * 48));
  HIP_TRY(c.b_msg.ensure(msg_total ? msg_total : 1));
  HIP_TRY(c.b_kidx.ensure((n_groups + 1) * 8));  // message offsets
  HIP_TRY(c.b_out.ensure(n_groups * 96));
  HIP_TRY(c.b_st.ensure(n_groups * 8));          // aggregate statuses, then verify statuses
  if (n_parts) {
    HIP_TRY(hipMemcpyAsync(c.b_sig.p, sigs, n_parts * 96, hipMemcpyHostToDevice, c.stream));
    HIP_TRY(hipMemcpyAsync(c.b_ids.p, share_idx, n_parts * 8, hipMemcpyHostToDevice, c.stream));
  }
  HIP_TRY(hipMemcpyAsync(c.b_off.p, group_offsets, (n_groups + 1) * 8, hipMemcpyHostToDevice, c.stream));
  HIP_TRY(hipMemcpyAsync(c.b_pk.p, dv_pks, n_groups * 48, hipMemcpyHostToDevice, c.stream));
  if (msg_total) HIP_TRY(hipMemcpyAsync(c.b_msg.p, msgs, msg_total, hipMemcpyHostToDevice, c.stream));
  HIP_TRY(hipMemcpyAsync(c.b_kidx.p, msg_offsets, (n_groups + 1) * 8, hipMemcpyHostToDevice, c.stream));
  int32_t* ast = (int32_t*)c.b_st.p;
  int32_t* vst = ast + n_groups;
  int rc = launch_tagg_verify((const uint8_t*)c.b_sig.p, (const int64_t*)c.b_ids.p, (const uint64_t*)c.b_off.p,
                              n_groups, n_parts, (const uint8_t*)c.b_pk.p, (const uint8_t*)c.b_msg.p,
                              (const uint64_t*)c.b_kidx.p, (uint8_t*)c.b_out.p, ast, vst, c.stream);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(out_sigs, c.b_out.p, n_groups * 96, hipMemcpyDeviceToHost, c.stream));
  HIP_TRY(hipMemcpyAsync(agg_status, ast, n_groups * 4, hipMemcpyDeviceToHost, c.stream));
  HIP_TRY(hipMemcpyAsync(verify_status, vst, n_groups * 4, hipMemcpyDeviceToHost, c.stream));
  HIP_TRY(hipStreamSynchronize(c.stream));
  return HIPBLS_OK;
}

int hipbls_threshold_aggregate_verify_batch_device(const uint8_t* d_sigs, const int64_t* d_share_idx,
                                                   const uint64_t* d_group_offsets, uint64_t n_groups,
                                                   uint64_t n_parts, const uint8_t* d_dv_pks, const uint8_t* d_msgs,
                                                   const uint64_t* d_msg_offsets, uint8_t* d_out_sigs,
                                                   int32_t* d_agg_status, int32_t* d_verify_status, void* stream) {
  if (n_groups == 0) return HIPBLS_OK;
  if (mul_overflows(n_parts, 288) || mul_overflows(n_groups, 120 * 4)) return arg_err("too many items");
  ENTER();
  return launch_tagg_verify(d_sigs, d_share_idx, d_group_offsets, n_groups, n_parts, d_dv_pks, d_msgs, d_msg_offsets,
                            d_out_sigs, d_agg_status, d_verify_status, pick(stream));
}

int hipbls_threshold_aggregate_batch_device(const uint8_t* d_sigs, const int64_t* d_share_idx,
                                            const uint64_t* d_group_offsets, uint64_t n_groups, uint64_t n_parts,
                                            uint8_t* d_out_sigs, int32_t* d_status, void* stream) {
  if (n_groups == 0) return HIPBLS_OK;
  if (mul_overflows(n_parts, 288)) return arg_err("too many partials");
  ENTER();
  return launch_tagg(d_sigs, d_share_idx, d_group_offsets, n_groups, n_parts, d_out_sigs, d_status, pick(stream));
}

int hipbls_sign_batch(const uint8_t* sks, const uint8_t* msgs, const uint64_t* msg_offsets, uint64_t n,
                      uint8_t* out_sigs, int32_t* status) {
  if (n == 0) return HIPBLS_OK;
  if (!sks || !msg_offsets || !out_sigs || !status || mul_overflows(n, 96)) return arg_err("bad sign arguments");
  if (!offsets_ok(msg_offsets, n)) return arg_err("bad message offsets");
  const uint64_t msg_total = msg_offsets[n];
  if (msg_total && !msgs) return arg_err("null messages");
  ENTER();
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
  ENTER();
  hipLaunchKernelGGL(k_sign, dim3((unsigned)grid_for(n)), dim3(kBlock), 0, pick(stream), d_sks, d_msgs, d_msg_offsets,
                     n, d_out_sigs, d_status);
  HIP_TRY(hipGetLastError());
  return HIPBLS_OK;
}

int hipbls_secret_to_public_key_batch(const uint8_t* sks, uint64_t n, uint8_t* out_pks, int32_t* status) {
  if (n == 0) return HIPBLS_OK;
  if (!sks || !out_pks || !status || mul_overflows(n, 48)) return arg_err("bad arguments");
  ENTER();
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
  ENTER();
  hipLaunchKernelGGL(k_sk_to_pk, dim3((unsigned)grid_for(n)), dim3(kBlock), 0, pick(stream), d_sks, n, d_out_pks,
                     d_status);
  HIP_TRY(hipGetLastError());
  return HIPBLS_OK;
}

int hipbls_verify_aggregate_batch(const uint8_t* pks, const uint64_t* key_offsets, uint64_t n_groups,
                                  const uint8_t* sigs, const uint8_t* msgs, const uint64_t* msg_offsets,
                                  int32_t* status) {
  if (n_groups == 0) return HIPBLS_OK;
  if (!key_offsets || !sigs || !msg_offsets || !status || key_offsets[0] != 0 || mul_overflows(n_groups, 96))
    return arg_err("bad arguments");
  if (!offsets_ok(msg_offsets, n_groups)) return arg_err("bad message offsets");
  for (uint64_t g = 0; g < n_groups; ++g)
    if (key_offsets[g + 1] < key_offsets[g]) return arg_err("decreasing key offsets");
  const uint64_t nkeys = key_offsets[n_groups], msg_total = msg_offsets[n_groups];
  if ((nkeys && !pks) || (msg_total && !msgs) || mul_overflows(nkeys, 96)) return arg_err("bad arguments");
  ENTER();
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
  int rc = launch_fav((const uint8_t*)c.b_pk.p, nkeys, (const uint64_t*)c.b_ids.p, n_groups, (const uint8_t*)c.b_sig.p,
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
  ENTER();
  return launch_fav(d_pks, nkeys, d_key_offsets, n_groups, d_sigs, d_msgs, d_msg_offsets, d_status, pick(stream));
}

int hipbls_verify_aggregate(const uint8_t* pks, uint64_t n, const uint8_t* sig, const uint8_t* msg, uint64_t msg_len,
                            int32_t* status) {
  if (!sig || !status || (n && !pks) || (msg_len && !msg) || mul_overflows(n, 48) || msg_len > 0xffffffffull)
    return arg_err("bad arguments");
  const uint64_t koff[2] = {0, n}, moff[2] = {0, msg_len};
  static const uint8_t empty = 0;
  return hipbls_verify_aggregate_batch(n ? pks : &empty, koff, 1, sig, msg_len ? msg : &empty, moff, status);
}

int hipbls_aggregate(const uint8_t* sigs, uint64_t n, uint8_t* out_sig, int32_t* status) {
  if (!out_sig || !status || (n && !sigs) || mul_overflows(n, 192)) return arg_err("bad arguments");
  ENTER();
  Context& c = g_ctx;
  HIP_TRY(c.b_sig.ensure((n ? n : 1) * 96));
  HIP_TRY(c.b_out.ensure(96));
  HIP_TRY(c.b_st.ensure(4));
  if (n) HIP_TRY(hipMemcpyAsync(c.b_sig.p, sigs, n * 96, hipMemcpyHostToDevice, c.stream));
  int rc = launch_aggregate((const uint8_t*)c.b_sig.p, n, (uint8_t*)c.b_out.p, (int32_t*)c.b_st.p, c.stream);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(out_sig, c.b_out.p, 96, hipMemcpyDeviceToHost, c.stream));
  HIP_TRY(hipMemcpyAsync(status, c.b_st.p, 4, hipMemcpyDeviceToHost, c.stream));
  HIP_TRY(hipStreamSynchronize(c.stream));
  return HIPBLS_OK;
}

int hipbls_aggregate_device(const uint8_t* d_sigs, uint64_t n, uint8_t* d_out_sig, int32_t* d_status, void* stream) {
  if (mul_overflows(n, 192)) return arg_err("too many signatures");
  ENTER();
  return launch_aggregate(d_sigs, n, d_out_sig, d_status, pick(stream));
}

int hipbls_threshold_split(const uint8_t* secret, const uint8_t* poly_tail, uint32_t total, uint32_t threshold,
                           uint8_t* out_shares, int32_t* status) {
  if (!secret || !out_shares || !status || threshold == 0 || total == 0 || (threshold > 1 && !poly_tail))
    return arg_err("bad split arguments");
  ENTER();
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

int hipbls_recover_secret(const uint8_t* shares, const int64_t* ids, uint32_t n, uint8_t* out_secret,
                          int32_t* status) {
  if (!out_secret || !status || (n && (!shares || !ids))) return arg_err("bad recover arguments");
  ENTER();
  Context& c = g_ctx;
  HIP_TRY(c.b_aux.ensure(32 * (uint64_t)(n ? n : 1)));
  HIP_TRY(c.b_ids.ensure(8 * (uint64_t)(n ? n : 1)));
  HIP_TRY(c.b_out.ensure(32));
  HIP_TRY(c.b_st.ensure(4));
  if (n) {
    HIP_TRY(hipMemcpyAsync(c.b_aux.p, shares, 32 * (uint64_t)n, hipMemcpyHostToDevice, c.stream));
    HIP_TRY(hipMemcpyAsync(c.b_ids.p, ids, 8 * (uint64_t)n, hipMemcpyHostToDevice, c.stream));
  }
  hipLaunchKernelGGL(k_recover_secret, dim3(1), dim3(kBlock), 0, c.stream, (const uint8_t*)c.b_aux.p,
                     (const int64_t*)c.b_ids.p, n, (uint8_t*)c.b_out.p, (int32_t*)c.b_st.p);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(out_secret, c.b_out.p, 32, hipMemcpyDeviceToHost, c.stream));
  HIP_TRY(hipMemcpyAsync(status, c.b_st.p, 4, hipMemcpyDeviceToHost, c.stream));
  HIP_TRY(hipStreamSynchronize(c.stream));
  return HIPBLS_OK;
}

int hipbls_kernel_timing(const char* name, double* avg_ms, uint64_t* launches) {
  if (!name || !avg_ms || !launches) return arg_err("null argument");
  int rc = bind_device();
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(g_ctx.tmu);
  auto it = g_ctx.timing.find(name);
  if (it == g_ctx.timing.end()) {
    *launches = 0;
    *avg_ms = 0.0;
    return HIPBLS_OK;
  }
  TimingSlot& t = it->second;
  drain_timing(t, true);
  *launches = t.launches;
  *avg_ms = t.launches ? t.total_ms / t.launches : 0.0;
  return HIPBLS_OK;
}

int hipbls_kernel_timing_reset(void) {
  int rc = bind_device();
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(g_ctx.tmu);
  for (auto& kv : g_ctx.timing) {
    drain_timing(kv.second, true);
    kv.second.total_ms = 0;
    kv.second.launches = 0;
  }
  return HIPBLS_OK;
}

int hipbls_batch_verify_rlc(const uint8_t* pks, const uint8_t* sigs, const uint32_t* msg_idx, uint64_t n,
                            const uint8_t* msgs, const uint64_t* msg_offsets, uint64_t n_msgs, const uint8_t* seed32,
                            int32_t* status) {
  if (n == 0) return HIPBLS_OK;
  if (!pks || !sigs || !msg_idx || !msg_offsets || !seed32 || !status || mul_overflows(n, 288))
    return arg_err("bad RLC arguments");
  for (uint64_t i = 0; i < n; ++i)
    if (msg_idx[i] >= n_msgs) return arg_err("message index out of range");
  if (!offsets_ok(msg_offsets, n_msgs)) return arg_err("bad message offsets");
  if (msg_offsets[n_msgs] && !msgs) return arg_err("null messages");
  ENTER();
  return rlc_host(pks, nullptr, sigs, msg_idx, n, msgs, msg_offsets, n_msgs, seed32, status);
}

int hipbls_batch_verify_rlc_device(const uint8_t* d_pks, const uint8_t* d_sigs, const uint32_t* d_msg_idx, uint64_t n,
                                   const uint8_t* d_msgs, const uint64_t* d_msg_offsets, uint64_t n_msgs,
                                   const uint8_t* seed32, int32_t* d_status, void* stream) {
  if (n == 0) return HIPBLS_OK;
  if (!seed32 || mul_overflows(n, 288)) return arg_err("bad RLC arguments");
  ENTER();
  return launch_rlc(d_pks, d_sigs, d_msg_idx, n, d_msgs, d_msg_offsets, n_msgs, seed32, d_status, pick(stream));
}

int hipbls_hcache_config(uint64_t capacity) {
  if (capacity > (1ull << 24)) return arg_err("H(m) cache capacity above 2^24");
  ENTER();
  HCache& hc = g_ctx.hcache;
  HIP_TRY(hipDeviceSynchronize());  // no call may still read the old table
  hc.map.clear();
  hc.key_of.assign(capacity, std::string());
  hc.ring = 0;
  hc.hits = hc.misses = 0;
  hc.cap = capacity;
  if (capacity) HIP_TRY(hc.table.ensure(capacity * 48 * 4));
  return HIPBLS_OK;
}

int hipbls_hcache_stats(uint64_t* hits, uint64_t* misses, uint64_t* entries) {
  if (!hits || !misses || !entries) return arg_err("null output");
  std::lock_guard<std::mutex> lk(g_ctx.mu);
  *hits = g_ctx.hcache.hits;
  *misses = g_ctx.hcache.misses;
  *entries = g_ctx.hcache.map.size();
  return HIPBLS_OK;
}

int hipbls_pubshare_table_load(const uint8_t* pks, uint64_t n, int32_t* status) {
  if ((n && (!pks || !status)) || mul_overflows(n, 240) || n > 0xffffffffull) return arg_err("bad table arguments");
  ENTER();
  Context& c = g_ctx;
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
  if (!n) return arg_err("null output");
  std::lock_guard<std::mutex> lk(g_ctx.mu);
  *n = g_ctx.t_size;
  return HIPBLS_OK;
}

int hipbls_verify_batch_keys(const uint32_t* key_idx, const uint8_t* msgs, const uint64_t* msg_offsets,
                             const uint8_t* sigs, uint64_t n, int32_t* status) {
  if (n == 0) return HIPBLS_OK;
  if (!key_idx || !msg_offsets || !sigs || !status || mul_overflows(n, 96)) return arg_err("bad arguments");
  if (!offsets_ok(msg_offsets, n)) return arg_err("bad message offsets");
  const uint64_t msg_total = msg_offsets[n];
  if (msg_total && !msgs) return arg_err("null messages");
  ENTER();
  Context& c = g_ctx;
  for (uint64_t i = 0; i < n; ++i)
    if (key_idx[i] >= c.t_size) return arg_err("key index outside the pubshare table");
  HIP_TRY(c.b_kidx.ensure(n * 4));
  HIP_TRY(c.b_sig.ensure(n * 96));
  HIP_TRY(c.b_msg.ensure(msg_total ? msg_total : 1));
  HIP_TRY(c.b_off.ensure((n + 1) * 8));
  HIP_TRY(c.b_st.ensure(n * 4));
  HIP_TRY(hipMemcpyAsync(c.b_kidx.p, key_idx, n * 4, hipMemcpyHostToDevice, c.stream));
  HIP_TRY(hipMemcpyAsync(c.b_sig.p, sigs, n * 96, hipMemcpyHostToDevice, c.stream));
  if (msg_total) HIP_TRY(hipMemcpyAsync(c.b_msg.p, msgs, msg_total, hipMemcpyHostToDevice, c.stream));
  HIP_TRY(hipMemcpyAsync(c.b_off.p, msg_offsets, (n + 1) * 8, hipMemcpyHostToDevice, c.stream));
  int rc = timed("verify_keys", c.stream, [&] {
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
  ENTER();
  Context& c = g_ctx;
  hipStream_t s = pick(stream);
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
    return arg_err("bad RLC arguments");
  for (uint64_t i = 0; i < n; ++i)
    if (msg_idx[i] >= n_msgs) return arg_err("message index out of range");
  if (!offsets_ok(msg_offsets, n_msgs)) return arg_err("bad message offsets");
  if (msg_offsets[n_msgs] && !msgs) return arg_err("null messages");
  ENTER();
  for (uint64_t i = 0; i < n; ++i)
    if (key_idx[i] >= g_ctx.t_size) return arg_err("key index outside the pubshare table");
  return rlc_host(nullptr, key_idx, sigs, msg_idx, n, msgs, msg_offsets, n_msgs, seed32, status);
}

int hipbls_batch_verify_rlc_keys_device(const uint32_t* d_key_idx, const uint8_t* d_sigs, const uint32_t* d_msg_idx,
                                        uint64_t n, const uint8_t* d_msgs, const uint64_t* d_msg_offsets,
                                        uint64_t n_msgs, const uint8_t* seed32, int32_t* d_status, void* stream) {
  if (n == 0) return HIPBLS_OK;
  if (!seed32 || !d_key_idx || mul_overflows(n, 288)) return arg_err("bad RLC arguments");
  ENTER();
  return launch_rlc(nullptr, d_sigs, d_msg_idx, n, d_msgs, d_msg_offsets, n_msgs, seed32, d_status, pick(stream),
                    d_key_idx);
}

int hipbls_rlc_stats(uint64_t* windows, uint64_t* windows_failed, uint64_t* items_fallback) {
  if (!windows || !windows_failed || !items_fallback) return arg_err("null output");
  ENTER();
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
