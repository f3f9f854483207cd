// hipbls: C-ABI host runtime (include/hipbls.h) over the gfx950 kernels in kernels.h.
//
// Execution model: ONE process drives every GPU of the node.  charon is one Go process per node that wires every
// component through one global tbls implementation (/root/reference/app/app.go:127, tbls/tbls.go:11-14), so the
// library keeps one device context per GPU it was given (hipbls_init_devices; hipbls_init(d) is the one-device
// case).  A context owns its device index, a library stream, reusable device workspaces, the resident pubshare
// table, the H(m) cache, its submission-queue worker and a mutex.
//
//   * Host-buffer entry points split the batch into contiguous ranges (items, or whole validator groups / message
//     runs: SURVEY.md §8e shards by validator index) across the contexts, one host thread per range, and each
//     range copies in, launches, copies out and synchronizes on its own device under its own context lock.  The
//     results land directly in the caller's arrays; nothing crosses devices (no RCCL inside one process).  Small
//     batches stay on one context, picked round robin, so concurrent callers spread over the GPUs.
//   * *_device entry points run on the context of the device that owns the caller's memory and only enqueue.
//     Calls that share a workspace are ordered on the device: each waits for the previous workspace user's
//     completion event (ws_done) before its first kernel and records the event after its last.
//   * hipbls_verify / hipbls_verify_submit go through the submission queues: each item goes to the context its
//     message hashes to (all partials of one signing root, i.e. of one validator duty, meet on one GPU and share
//     one H(m)), where a worker thread coalesces concurrent n = 1 calls into batched launches.
//   * A goroutine can move between OS threads between two calls, and hipSetDevice is per host thread, so every
//     entry point binds its context's device on the calling thread before it touches memory or streams.
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <algorithm>
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

#include <sys/random.h>

#include "kernels.h"
#include "ranges.h"

// The RLC item and hash stages at two waves per SIMD (rlc_wide.hip: its own translation unit, C linkage).
extern "C" {
__global__ void k_rlc_items(uint64_t i0, uint64_t i1, const uint8_t* pks, const uint8_t* sigs, const uint32_t* msg_idx,
                            uint64_t n, uint64_t n_msgs, bls::rlc_seed seed, uint32_t* rpk, uint32_t* rsig,
                            int32_t* status, const uint32_t* key_idx, uint64_t T, const int32_t* tcode,
                            const uint32_t* tab);
__global__ void k_rlc_hash(const uint8_t* msgs, const uint64_t* offs, uint64_t n_hash, const uint32_t* mlist, uint32_t* H,
                           uint64_t hstride, const uint32_t* hslot);
__global__ void k_rlcb_items(uint64_t n, const uint8_t* pks, const uint8_t* sigs, const uint32_t* msg_idx,
                             uint64_t n_msgs, bls::rlc_seed seed, uint32_t* rpk, uint32_t* pts, uint32_t* sc,
                             int32_t* status, const uint32_t* key_idx, uint64_t T, const int32_t* tcode,
                             const uint32_t* tab, const uint32_t* g1pos, uint32_t* gpts, uint32_t* gsc);
}

// The eight-lane latency path (verify_lat.hip, its own translation unit: BLS_FP2_PAIR build in namespace bls_fp2p).
namespace bls_fp2p {
__global__ void k_verify_prep8(const uint8_t* pks, const uint8_t* msgs, const uint64_t* offs, const uint8_t* sigs,
                               uint64_t n, uint32_t* ws, int32_t* status, uint32_t replicas, uint32_t* race,
                               uint32_t epoch);
__global__ void k_verify_pair_lq8(const uint32_t* ws, uint64_t n, int32_t* status, uint32_t replicas, uint32_t* race,
                                  uint32_t epoch);
__global__ void k_rlcb_sfactor8(const uint32_t* W, uint32_t* Fs);
__global__ void k_rlcb_final8(const uint32_t* Ftot, const uint32_t* Fs, int32_t* flag);
__global__ void k_g1m_miller8(uint64_t nl_max, const uint32_t* meta, const uint32_t* lmsg, const uint32_t* Wv,
                              const uint32_t* H, uint64_t hstride, const uint32_t* hslot, uint32_t* F, uint64_t col0,
                              uint64_t fstride);
__global__ void k_fav_prep8(const uint8_t* pks, uint64_t nkeys, const uint8_t* sigs, const uint8_t* msgs,
                            const uint64_t* moffs, uint64_t G, uint32_t* pts, int32_t* kcode, uint32_t* ws);
}  // namespace bls_fp2p
// The sixteen-lane check for batches of at most four items (verify_hex.hip: BLS_FP2_PAIR + BLS_HEX, namespace bls_hex).
namespace bls_hex {
__global__ void k_verify_pair_lq16(const uint32_t* ws, uint64_t n, int32_t* status, uint32_t replicas, uint32_t* race,
                                   uint32_t epoch);

}  // namespace bls_hex
// FastAggregateVerify's check at two waves per SIMD (fav_wide.hip: verify_hex.hip again, namespace bls_hexw).
namespace bls_hexw {
__global__ void k_fav_pair_lq16(const uint32_t* pts, const int32_t* kcode, uint64_t nkeys, const uint64_t* goff,
                                const uint32_t* ws, uint64_t G, int32_t* status);
}  // namespace bls_hexw
namespace bls_fp2p {
// LDS the S-factor workgroup reserves at launch and never touches: the chunk kernel's 36 KiB per workgroup (four per
// CU), so a CU that hosts the S-factor wave takes at most three chunk waves and no SIMD runs two (a shared SIMD
// stretched the 1,023-wave chunk kernel by the S factor's run time: 34.9 -> 40.5 ms).
constexpr uint32_t kSfactorLds = 36 * 1024;
}  // namespace bls_fp2p

namespace {

// ============================================================================ device contexts
thread_local std::string g_last_error;

// Library streams per device: the library stream, the two fork sub-streams (RLC sub-batches, sigagg) and the
// submission queue's stream.  HIP maps a process's streams onto GPU_MAX_HW_QUEUES (4) hardware queues, and each
// hardware queue that runs these kernels sizes its scratch by the deepest private segment (charon_amd/codeobj.py
// PRIVATE_SEGMENT_BUDGET): four streams keep the library's own launches one hardware queue apiece.
constexpr int kStreamsPerDevice = 4;

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t n) {
    if (n <= cap) return hipSuccess;
    if (p) (void)hipFree(p);  // hipFree waits for the device: no in-flight kernel still uses the old buffer
    p = nullptr;
    cap = 0;
    // 256-byte multiples: a buffer's tail (the octet path's race words, launch_verify) stays naturally aligned
    const size_t want = ((n < 4096 ? 4096 : n + n / 4) + 255) & ~(size_t)255;
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

// One open or running batch of the submission queue.
struct VBatch {
  std::vector<uint8_t> pk, sig, msg;
  std::vector<uint64_t> off{0};
  std::vector<int32_t> status;
  int rc = HIPBLS_OK;
  bool done = false;
  uint64_t n() const { return off.size() - 1; }
};

// A wire-format batch in flight on the GPU: its own buffers, pinned status copy and completion event, so a second
// batch can be copied in and launched (behind the first, on the queue's stream) while the first one runs.
struct QSlot {
  hipStream_t stream = nullptr;
  hipEvent_t done_ev = nullptr;
  DevBuf d_pk, d_sig, d_msg, d_off, d_st, d_ws;
  int32_t* h_st = nullptr;  // pinned: the status copy is a real async D2H (a pageable one would block the worker)
  uint64_t h_cap = 0;
  std::shared_ptr<VBatch> b;
  int rc = HIPBLS_OK;
  std::chrono::steady_clock::time_point launched;
};

// Per-context submission queue (worker, streams and buffers of its own).
struct VerifyQueue {
  static constexpr int kSlots = 2;  // wire batches in flight at once
  std::mutex mu;
  std::condition_variable cv_work, cv_done;
  std::deque<std::shared_ptr<VBatch>> open;  // accepting (back) / waiting for the worker (front)
  std::unordered_map<uint64_t, std::pair<std::shared_ptr<VBatch>, uint32_t>> tickets;
  uint64_t next_ticket = 1;
  std::thread worker;
  bool started = false, stop = false;
  uint64_t batches = 0, items = 0, keyed = 0, overlapped = 0;
  uint64_t wakeups = 0;   // completion polls of the worker (hipbls_queue_worker_stats)
  double batch_us[26] = {};  // running estimate of a wire batch's launch-to-completion time, per log2(batch size)
  // running mean of the items per launched batch: below 1.5 the callers are serial (each waits for its own result
  // before the next call), so an idle worker launches at once instead of waiting gather_us for company that cannot
  // come; concurrent callers raise it (items that arrive while a batch runs coalesce into the next one) and turn the
  // gather window back on
  double batch_mean = 2.0;
  hipStream_t stream = nullptr;  // the keyed path's stream
  QSlot slot[kSlots];
  std::deque<int> inflight;  // slots in launch order
  DevBuf d_pk, d_sig, d_msg, d_off, d_kidx, d_midx, d_slot, d_mlist, d_rlc_st;
  // host staging of the keyed path (reused across batches)
  std::vector<uint32_t> kidx, midx, order, slotv, miss;
  std::vector<uint8_t> sig_sorted, umsg;
  std::vector<uint64_t> uoff;
  std::vector<int32_t> st_sorted;
};

struct Context {
  int device = -1;
  int slot = 0;  // index in the context list
  hipStream_t stream = nullptr;
  std::mutex mu;
  DevBuf b_pk, b_msg, b_off, b_sig, b_st, b_out, b_ids, b_pts, b_pst, b_aux, b_part, b_bad;
  DevBuf r_pk, r_sig, r_h, r_win, r_midx, r_list, r_cnt, r_slot, r_mlist;  // RLC BatchVerify workspaces
  DevBuf t_code, t_tab, b_kidx;                                            // resident pubshare table + key indices
  DevBuf f_ws;  // FastAggregateVerify on the octet / sixteen-lane layouts: per-group H(m), signature, codes
  DevBuf v_ws;                                                             // lane-pair Verify points (SoA)
  // sigagg in one call (launch_tagg_verify): two workspace sets used alternately, each with the completion event of
  // the call that last used it
  DevBuf tv_pts[2], tv_pst[2], tv_ws[2], tv_aux[2];
  // The host-buffer sigagg call (tagg_verify_host): two slots of input/output buffers, used alternately, each on its
  // own library sub-stream; a call holds its slot for its whole duration but the context lock only while it enqueues,
  // so the next caller's copies and phase A run beside this call's checks (the _device path's two-stream overlap,
  // reached from host buffers: two goroutines with consecutive duties).
  struct TvHostSlot {
    std::mutex mu;
    DevBuf sig, ids, off, pk, msg, moff, out, st;
    uint8_t* h_out = nullptr;  // pinned: the outputs come back by a real async D2H
    int32_t* h_st = nullptr;
    uint64_t h_groups = 0;
    hipEvent_t done = nullptr;
  } tvh[2];
  std::atomic<uint64_t> tvh_seq{0};
  hipEvent_t tv_done[2] = {}, tv_phase = nullptr;  // tv_phase: the last call's phase A (and S, statuses) done
  uint64_t tv_seq = 0;
  uint64_t t_size = 0;
  // pubshare bytes -> table index (host side), for the submission queue's keyed path
  std::unordered_map<std::string, uint32_t> t_index;
  // RLC sub-batches in flight.  The process gets GPU_MAX_HW_QUEUES = 4 hardware queues per device, shared by the
  // caller's stream (which also hashes the messages), the library stream and these; a kernel trace
  // (profiles/r01_rlc_trace.txt) showed a third sub-stream landing on an occupied queue and serializing behind
  // it, so two sub-batches.
  static constexpr int kSub = 2;
  hipStream_t sub[kSub] = {};
  hipEvent_t ev_fork = nullptr, ev_hash = nullptr, ev_join[kSub] = {};
  // Last workspace user's completion (cross-stream ordering), per workspace group: the general buffers (b_*, v_ws) and
  // the RLC ones (r_*, m_*, the H(m) cache), so an RLC batch and, say, a FastAggregateVerify on another stream (the C5
  // slot mix) overlap instead of queueing behind each other.  The two groups still SHARE the fork sub-streams
  // (sub[0], sub[1], the device's) and the fork/join events (ev_fork, ev_hash, ev_join): launch_rlc and
  // launch_rlc_batch issue every record/wait pair on those within one call under c.mu, which
  // is what makes the sharing safe.  sigagg in one call uses neither: its workspace sets (tv_*) carry their own events.
  hipEvent_t ws_done = nullptr, ws_done_rlc = nullptr;
  // A caller stream that would put the library's kernels on a hardware queue of its own (non-default priority, a CU
  // mask) is joined to the library stream instead (StreamJoin): these events carry the ordering.
  hipEvent_t ev_join_in = nullptr, ev_join_out = nullptr;
  int stream_prio = 0;                // the library streams' priority (the device default)
  std::vector<uint32_t> cu_mask;      // the library stream's CU mask (all CUs)
  uint64_t joined = 0;                // *_device calls run on the library stream for that reason
  uint64_t r_windows = 0;       // window count of this context's last RLC call (hipbls_rlc_stats)
  uint64_t r_call = 0;           // entry-point call that call belonged to
  // batch-wide RLC check (rlcb.h): MSM inputs and stages, Miller values, verdict flag
  DevBuf m_pts, m_sc, m_cnt, m_off, m_cur, m_list, m_B, m_P, m_Sg, m_Wp, m_W, m_F, m_F2, m_flag, m_Fs;
  DevBuf g1_ws;  // the G1 MSM per large message (g1msm.h), carved by G1mLayout; its Miller values go to m_F
  hipEvent_t rlcb_ev_sf = nullptr;  // the (-g1, S) Miller value is in m_Fs
  uint64_t slots = 0;               // waves in flight at one wave per SIMD: 4 x compute units (wave_slots)
  // Verdicts come back through a ring of pinned slots, one per batch check in flight, so a launch only waits
  // on the host when kRlcbSlots checks are still unread (never in the enqueue-only *_device paths otherwise).
  static constexpr int kRlcbSlots = 8;
  int32_t* rlcb_host_flag = nullptr;  // pinned, kRlcbSlots verdicts
  hipEvent_t rlcb_ev[kRlcbSlots] = {};
  hipEvent_t rlcb_ev_items = nullptr, rlcb_ev_msm = nullptr;
  bool rlcb_pending[kRlcbSlots] = {};
  uint64_t rlcb_seq[kRlcbSlots] = {};   // launch order of the check in each slot
  uint64_t rlcb_call[kRlcbSlots] = {};  // entry-point call of the check in each slot
  uint64_t rlcb_next_seq = 0, rlcb_last_seq = 0;
  int rlcb_last = -1;                   // newest verdict read back: -1 none, 0 failed, 1 passed
  uint64_t rlcb_last_call = 0;          // entry-point call of that verdict
  int rlcb_skipped = 0;                 // AUTO: calls run windows-only since the last failed batch check
  uint64_t rlcb_attempted = 0, rlcb_passed = 0;
  HCache hcache;
  std::mutex tmu;                            // timing table (also used by the queue worker)
  std::map<std::string, TimingSlot> timing;  // per kernel name: HIP events on the launch stream
  VerifyQueue q;
};

// The context list is written once, under g_init_mu, before g_nctx is published; contexts live for the process.
std::vector<Context*> g_ctxs;
std::map<int, int> g_streams_per_device;  // library streams created per device (written once at init)
std::atomic<int> g_nctx{0};
std::mutex g_init_mu;
std::atomic<bool> g_timing{false};
std::atomic<uint64_t> g_rr{0};        // round-robin context for single-range calls
std::atomic<uint64_t> g_call_seq{0};  // RLC entry-point calls (hipbls_rlc_stats / hipbls_rlc_batch_stats)
constexpr int kMaxContexts = 64;

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

int nctx() { return g_nctx.load(std::memory_order_acquire); }
Context& ctx(int k) { return *g_ctxs[k]; }

// ============================================================================ scratch
// Each hardware queue that dispatches a kernel holds a scratch block of (private segment per lane) x 64 lanes x 32
// wave slots per CU x CUs, rounded to 2 MiB: 520 MiB for 1,040 B/lane, 6,240 MiB for 12,480 B/lane
// (profiles/r05/r05_scratch_probe.txt, _layout.txt).  The blocks come from one region per device whose size is the
// agent's scratch limit (HSA_AMD_AGENT_INFO_SCRATCH_LIMIT_MAX: 32 GiB on MI355X), placed first-fit: a queue whose
// block must grow for a deeper kernel takes a new block and frees the old one, which leaves a hole.  Four queues grown
// in stages to 12,480 B/lane hold 24.4 GiB but leave at most 4.6 GiB contiguous of the 7.6 GiB free, so a fifth
// queue (a priority stream) asking for 6.1 GiB failed: HSA_STATUS_ERROR_OUT_OF_RESOURCES, a process abort (round 4).
// So the library (1) reserves each of its queues' blocks once at full size in stream order at init (contiguous, no
// holes: the rest of the region stays one block), (2) never launches on a stream that would give it a queue of its
// own (StreamJoin), and (3) refuses at init a device whose limit cannot hold its queues.
constexpr uint32_t kCuMaskWords = 16;  // 512 CUs
constexpr uint64_t kScratchAlign = 2ull << 20;
constexpr uint32_t kLaneBytes = 64;

struct Scratch {
  uint64_t per_lane = 0;   // deepest private segment of the library's kernels (bytes per lane)
  uint64_t per_queue = 0;  // the block one hardware queue holds for it
  uint64_t limit = 0;      // the device's scratch region (0: the runtime does not report one)
  uint32_t slots = 0;      // scratch wave slots per CU
  uint32_t cus = 0;
  uint32_t queues = 0;     // GPU_MAX_HW_QUEUES (HIP's normal-priority hardware queues per process)
  std::string deepest;
};
std::map<int, Scratch> g_scratch;      // per device, written once at init
std::atomic<bool> g_join_all{false};   // every *_device call runs on the library's streams (StreamJoin)

// Reserve kernels: a private segment of S bytes per lane (a volatile frame of S - 16 bytes; the frame adds 16), never
// touched when n == 0.  Launched once per library stream at init so each queue's block is allocated at full size.
template <int S>
__global__ void k_scratch_reserve(uint32_t* out, uint32_t n) {
  constexpr int W = (S - 16) / 4;
  volatile uint32_t frame[W];
  if (n) {
    frame[n % W] = n;
    out[threadIdx.x] = frame[(n * 7u) % W];
  }
}

struct KernelRef {
  const char* name;
  const void* fn;
};
#define KREF(k) {#k, reinterpret_cast<const void*>(&k)}
#define KREF8(k) {#k, reinterpret_cast<const void*>(&bls_fp2p::k)}
#define KREF16(k) {#k, reinterpret_cast<const void*>(&bls_hex::k)}
#define KREF16W(k) {#k, reinterpret_cast<const void*>(&bls_hexw::k)}
// Every kernel the library launches (tests/test_kernel_resources.py: the same set as both code objects hold, minus the
// reserve kernels).
const KernelRef kKernels[] = {
    KREF(k_fav_batch), KREF(k_fp12_prod64), KREF(k_g1_decode), KREF(k_g1m_count), KREF(k_g1m_fix), KREF(k_g1m_fold),
    KREF(k_g1m_hist), KREF(k_g1m_plan), KREF(k_g1m_rank), KREF(k_g1m_run), KREF(k_g1m_scatter), KREF(k_g2_decode),
    KREF(k_g2_sum_final), KREF(k_g2_sum_partial), KREF(k_msm_fix), KREF(k_msm_hist), KREF(k_msm_run), KREF(k_msm_scan),
    KREF(k_msm_scatter), KREF(k_msm_segment), KREF(k_msm_window), KREF(k_msm_wsum), KREF(k_pubtab_load),
    KREF(k_recover_secret), KREF(k_rlc_fallback), KREF(k_rlc_fallback_lg2), KREF(k_rlc_hash), KREF(k_rlc_items),
    KREF(k_rlc_window), KREF(k_rlc_window_lg2), KREF(k_rlcb_chunks), KREF(k_rlcb_items), KREF(k_rlcb_mark),
    KREF(k_scan_apply), KREF(k_scan_part), KREF(k_scan_top), KREF(k_sign), KREF(k_signing_roots), KREF(k_sk_to_pk),
    KREF(k_tagg_scale), KREF(k_tagg_sum), KREF(k_tagg_sum_s), KREF(k_tagg_unscale), KREF(k_threshold_split),
    KREF(k_tv_check_unscale), KREF(k_tv_join), KREF(k_tv_phase_a), KREF(k_tv_prep_pk), KREF(k_tv_prep_pk2),
    KREF(k_verify_fused), KREF(k_verify_keys), KREF(k_verify_pair_lg2), KREF(k_verify_pair_lq4),
    KREF(k_verify_pair_single), KREF(k_verify_prep), KREF(k_zero_sig_status), KREF8(k_g1m_miller8),
    KREF8(k_rlcb_final8), KREF8(k_rlcb_sfactor8), KREF8(k_verify_pair_lq8), KREF8(k_verify_prep8),
    KREF16(k_verify_pair_lq16), KREF8(k_fav_prep8), KREF16W(k_fav_pair_lq16),
};
#define RES(s) reinterpret_cast<const void*>(&k_scratch_reserve<s>)
// 8 KiB to the per-lane budget (charon_amd/codeobj.py PRIVATE_SEGMENT_BUDGET, 13,104 B) in 256-byte steps: at most
// 128 MiB of a queue's block beyond the deepest kernel's
const void* const kReserve[] = {
    RES(8192), RES(8448), RES(8704), RES(8960), RES(9216), RES(9472), RES(9728), RES(9984), RES(10240), RES(10496),
    RES(10752), RES(11008), RES(11264), RES(11520), RES(11776), RES(12032), RES(12288), RES(12544), RES(12800),
    RES(13056), RES(13104),
};
#undef RES
#undef KREF
#undef KREF8
#undef KREF16
#undef KREF16W

std::string kernel_names() {
  std::string s;
  for (const KernelRef& k : kKernels) {
    if (!s.empty()) s += ' ';
    s += k.name;
  }
  return s;
}

// The device's scratch region, from the HSA agent at the device's PCI location (0 when the runtime has no such query).
uint64_t scratch_limit(int device) {
  int bus = -1, dev = -1, dom = -1;
  if (hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, device) != hipSuccess ||
      hipDeviceGetAttribute(&dev, hipDeviceAttributePciDeviceId, device) != hipSuccess ||
      hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainId, device) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  struct Find {
    uint32_t bdf, dom;
    hsa_agent_t agent;
    bool found;
  } f{(uint32_t)((bus << 8) | (dev << 3)), (uint32_t)dom, {}, false};
  if (hsa_init() != HSA_STATUS_SUCCESS) return 0;  // HIP already holds the runtime open: this only adds a reference
  hsa_iterate_agents(
      [](hsa_agent_t a, void* p) -> hsa_status_t {
        Find& f = *(Find*)p;
        hsa_device_type_t t;
        uint32_t bdf = 0, dom = 0;
        if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS || t != HSA_DEVICE_TYPE_GPU)
          return HSA_STATUS_SUCCESS;
        if (hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf) != HSA_STATUS_SUCCESS ||
            hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DOMAIN, &dom) != HSA_STATUS_SUCCESS)
          return HSA_STATUS_SUCCESS;
        if ((bdf & ~7u) == f.bdf && dom == f.dom) {
          f.agent = a;
          f.found = true;
          return HSA_STATUS_INFO_BREAK;
        }
        return HSA_STATUS_SUCCESS;
      },
      &f);
  uint64_t lim = 0;
  if (!f.found ||
      hsa_agent_get_info(f.agent, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_SCRATCH_LIMIT_MAX, &lim) != HSA_STATUS_SUCCESS)
    lim = 0;
  return lim;
}

int scratch_budget(int device, Scratch& s) {
  s = Scratch();
  for (const KernelRef& k : kKernels) {
    hipFuncAttributes fa;
    HIP_TRY(hipFuncGetAttributes(&fa, k.fn));
    if ((uint64_t)fa.localSizeBytes > s.per_lane) {
      s.per_lane = fa.localSizeBytes;
      s.deepest = k.name;
    }
  }
  int threads = 0, warp = 0, cus = 0;
  HIP_TRY(hipDeviceGetAttribute(&threads, hipDeviceAttributeMaxThreadsPerMultiProcessor, device));
  HIP_TRY(hipDeviceGetAttribute(&warp, hipDeviceAttributeWarpSize, device));
  HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
  s.slots = warp > 0 ? (uint32_t)(threads / warp) : 32;
  s.cus = (uint32_t)cus;
  const uint64_t raw = s.per_lane * kLaneBytes * s.slots * s.cus;
  s.per_queue = (raw + kScratchAlign - 1) / kScratchAlign * kScratchAlign;
  const char* q = getenv("GPU_MAX_HW_QUEUES");
  s.queues = q && atoi(q) > 0 ? (uint32_t)atoi(q) : 4u;
  s.limit = scratch_limit(device);
  return HIPBLS_OK;
}

// One dispatch of the smallest reserve kernel at least as deep as the library's deepest kernel on each stream, in
// order, then a wait: each hardware queue takes its block now, at full size, next to the previous one.
int scratch_reserve(const hipStream_t* ss, int n, uint64_t per_lane) {
  const void* fn = nullptr;
  for (const void* r : kReserve) {
    hipFuncAttributes fa;
    HIP_TRY(hipFuncGetAttributes(&fa, r));
    if ((uint64_t)fa.localSizeBytes >= per_lane) {
      fn = r;
      break;
    }
  }
  if (!fn) {
    // deeper than the largest reserve kernel: the queues' blocks would grow on first use, the round-4 abort's
    // precondition, so refuse the device (the build budget, charon_amd/codeobj.py, keeps this from happening)
    g_last_error = "scratch: the deepest kernel needs " + std::to_string(per_lane) +
                   " B per lane, more than the largest reserve kernel";
    return HIPBLS_ERR_DEVICE;
  }
  void* args[2];
  uint32_t* none = nullptr;
  uint32_t zero = 0;
  args[0] = &none;
  args[1] = &zero;
  for (int k = 0; k < n; ++k) {
    HIP_TRY(hipLaunchKernel(fn, dim3(1), dim3(64), args, 0, ss[k]));
    HIP_TRY(hipStreamSynchronize(ss[k]));
  }
  return HIPBLS_OK;
}

int init_locked(const std::vector<int>& ids) {
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess || ndev == 0) return set_err("hipGetDeviceCount (no GPU)", e == hipSuccess ? hipErrorNoDevice : e);
  if (ids.empty() || ids.size() > (size_t)kMaxContexts) return arg_err("device list empty or longer than 64");
  for (int d : ids)
    if (d < 0 || d >= ndev) return arg_err("device index out of range");
  std::vector<Context*> made;
  std::map<int, std::array<hipStream_t, kStreamsPerDevice>> dev_streams;
  for (size_t k = 0; k < ids.size(); ++k) {
    Context* c = new Context();
    c->device = ids[k];
    c->slot = (int)k;
    HIP_TRY(hipSetDevice(c->device));
    // One set of library streams per DEVICE, shared by every context on it (streams only add ordering, and every
    // event a context records or waits on is its own): the library never holds more than kStreamsPerDevice streams
    // on a device, whatever the number of contexts.
    auto it = dev_streams.find(c->device);
    if (it == dev_streams.end()) {
      std::array<hipStream_t, kStreamsPerDevice> ss{};
      for (auto& x : ss) HIP_TRY(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
      it = dev_streams.emplace(c->device, ss).first;
    }
    c->stream = it->second[0];
    c->sub[0] = it->second[1];
    c->sub[1] = it->second[2];
    c->q.stream = it->second[3];
    HIP_TRY(hipEventCreateWithFlags(&c->ws_done, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&c->ws_done_rlc, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&c->ev_join_in, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&c->ev_join_out, hipEventDisableTiming));
    HIP_TRY(hipStreamGetPriority(c->stream, &c->stream_prio));
    c->cu_mask.assign(kCuMaskWords, 0);
    if (hipExtStreamGetCUMask(c->stream, kCuMaskWords, c->cu_mask.data()) != hipSuccess) {
      (void)hipGetLastError();
      c->cu_mask.clear();  // no CU-mask query on this runtime: only the priority decides
    }
    made.push_back(c);
  }
  // Scratch: refuse a device whose scratch limit cannot hold the library's own hardware queues at
  // its deepest kernel, and reserve each library queue's scratch once, at full size, in stream order.
  for (auto& kv : dev_streams) {
    HIP_TRY(hipSetDevice(kv.first));
    Scratch sb;
    int rc = scratch_budget(kv.first, sb);
    if (rc) return rc;
    if (sb.limit && (uint64_t)kStreamsPerDevice * sb.per_queue > sb.limit) {
      g_last_error = "scratch: " + std::to_string(kStreamsPerDevice) + " hardware queues x " +
                     std::to_string(sb.per_queue) + " B (" + std::to_string(sb.per_lane) + " B per lane, " + sb.deepest +
                     ") exceed device " + std::to_string(kv.first) + "'s scratch limit of " + std::to_string(sb.limit) +
                     " B";
      return HIPBLS_ERR_DEVICE;
    }
    // GPU_MAX_HW_QUEUES normal-priority queues that could all carry the library's kernels through callers' streams
    // must fit as well; otherwise every *_device call runs on the library's own streams (StreamJoin).
    if (sb.limit && (uint64_t)sb.queues * sb.per_queue > sb.limit) g_join_all = true;
    if (!sb.limit) {
      // no scratch limit to check against (no HSA query on this runtime): fail safe, and say so
      g_join_all = true;
      g_last_error = "scratch: device " + std::to_string(kv.first) +
                     " reports no scratch limit; every *_device call runs on the library's streams";
      fprintf(stderr, "hipbls: %s\n", g_last_error.c_str());
    }
    const char* rs = getenv("HIPBLS_SCRATCH_RESERVE");
    if (!(rs && rs[0] == '0')) {
      rc = scratch_reserve(kv.second.data(), kStreamsPerDevice, sb.per_lane);
      if (rc) return rc;
    }
    g_scratch[kv.first] = sb;
  }
  const char* t = getenv("HIPBLS_TIMING");
  if (t && t[0] == '1') g_timing = true;
  for (auto& kv : dev_streams) g_streams_per_device[kv.first] = (int)kv.second.size();
  g_ctxs = made;
  g_nctx.store((int)made.size(), std::memory_order_release);
  return HIPBLS_OK;
}

// HIPBLS_DEVICES = "all" | "0,2,5" picks the devices of a process that never calls hipbls_init*; otherwise the
// calling thread's current device.
int default_devices(std::vector<int>& ids) {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess) ndev = 0;
  const char* env = getenv("HIPBLS_DEVICES");
  if (env && env[0]) {
    if (!strcmp(env, "all")) {
      for (int d = 0; d < ndev; ++d) ids.push_back(d);
    } else {
      const char* p = env;
      while (*p) {
        char* end = nullptr;
        const long v = strtol(p, &end, 10);
        if (end == p) return arg_err("HIPBLS_DEVICES: expected 'all' or a comma-separated device list");
        ids.push_back((int)v);
        p = *end == ',' ? end + 1 : end;
        if (*end && *end != ',') return arg_err("HIPBLS_DEVICES: expected 'all' or a comma-separated device list");
      }
    }
    return HIPBLS_OK;
  }
  int d = 0;
  HIP_TRY(hipGetDevice(&d));
  ids.push_back(d);
  return HIPBLS_OK;
}

int ensure_init() {
  if (nctx()) return HIPBLS_OK;
  std::lock_guard<std::mutex> lk(g_init_mu);
  if (nctx()) return HIPBLS_OK;
  std::vector<int> ids;
  const int rc = default_devices(ids);
  if (rc) return rc;
  return init_locked(ids);
}

int bind(Context& c) {
  HIP_TRY(hipSetDevice(c.device));
  return HIPBLS_OK;
}

// Entry-point prologue for one context: device bound on this thread, context lock held for the scope.
#define ENTER_CTX(c)          \
  int _brc = bind(c);         \
  if (_brc) return _brc;      \
  std::lock_guard<std::mutex> _lk((c).mu)

#define ENSURE_INIT()              \
  do {                             \
    int _irc = ensure_init();      \
    if (_irc) return _irc;         \
  } while (0)

// The context of the device that owns a caller's device pointer (the *_device entry points): the first context on
// that device; the first context when the pointer is unknown to HIP.
Context& ctx_of(const void* p) {
  const int n = nctx();
  if (n > 1 && p) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) == hipSuccess)
      for (int k = 0; k < n; ++k)
        if (ctx(k).device == a.device) return ctx(k);
    (void)hipGetLastError();
  }
  return ctx(0);
}

// Whether a caller's stream shares the hardware queues the library's own streams hold: HIP spreads streams of the
// default priority without a CU mask over GPU_MAX_HW_QUEUES queues per process, and gives a priority stream (high or
// low) or a CU-masked one a queue of its own (profiles/r05/r05_scratch_probe.txt: a fifth normal stream took no new
// block, a high- and a low-priority stream each took one).
bool shares_library_queues(Context& c, hipStream_t st) {
  if (g_join_all.load()) return false;
  int prio = 0;
  if (hipStreamGetPriority(st, &prio) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  if (prio != c.stream_prio) return false;
  if (c.cu_mask.empty()) return true;
  uint32_t m[kCuMaskWords] = {};
  if (hipExtStreamGetCUMask(st, kCuMaskWords, m) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return std::equal(c.cu_mask.begin(), c.cu_mask.end(), m);
}

// The stream a *_device call launches on.  The caller's stream when it shares the library's hardware queues;
// otherwise the context's library stream, joined to the caller's both ways (the call starts after the caller's
// earlier work and the caller's later work waits for the call), so the library's kernels never make the process hold
// one more queue's scratch block.  Declared after ENTER_CTX: it runs under the context lock, and
// the destructor enqueues the join-back before the lock is released.
struct StreamJoin {
  Context& c;
  hipStream_t user = nullptr, s = nullptr;
  bool joined = false;
  StreamJoin(Context& cc, void* stream) : c(cc), user((hipStream_t)stream), s(stream ? (hipStream_t)stream : cc.stream) {}
  int begin() {
    if (!user || user == c.stream || shares_library_queues(c, user)) return HIPBLS_OK;
    HIP_TRY(hipEventRecord(c.ev_join_in, user));
    HIP_TRY(hipStreamWaitEvent(c.stream, c.ev_join_in, 0));
    s = c.stream;
    joined = true;
    c.joined += 1;
    return HIPBLS_OK;
  }
  ~StreamJoin() {
    if (joined && hipEventRecord(c.ev_join_out, c.stream) == hipSuccess) (void)hipStreamWaitEvent(user, c.ev_join_out, 0);
  }
};
#define ON_STREAM(c, stream, s)        \
  StreamJoin _sj((c), (stream));       \
  {                                    \
    const int _jrc = _sj.begin();      \
    if (_jrc) return _jrc;             \
  }                                    \
  const hipStream_t s = _sj.s

// Workspace ordering: the call's stream waits for the previous workspace user, and publishes its own end.
enum { WS_GEN = 0, WS_RLC = 1 };
int ws_begin(Context& c, hipStream_t s, int group = WS_GEN) {
  HIP_TRY(hipStreamWaitEvent(s, group == WS_RLC ? c.ws_done_rlc : c.ws_done, 0));
  return HIPBLS_OK;
}
int ws_end(Context& c, hipStream_t s, int group = WS_GEN) {
  HIP_TRY(hipEventRecord(group == WS_RLC ? c.ws_done_rlc : c.ws_done, s));
  return HIPBLS_OK;
}

// ============================================================================ splitting a batch across contexts
// plan_ranges: charon_amd/csrc/ranges.h (host-only, also built by the sanitizer test, tests/test_sanitizers.py).

// How many ranges a batch of n units gets: one per context, but never ranges below min_per units.
uint64_t parts_for(uint64_t n, uint64_t min_per) {
  const uint64_t k = (uint64_t)nctx();
  if (k <= 1 || n < 2 * min_per) return 1;
  const uint64_t p = n / min_per;
  return p < k ? p : k;
}

// Runs fn(context, lo, hi) for every range [bounds[j], bounds[j+1]): range j on context j, each on its own host
// thread (the first on the calling one), with the context's device bound and its lock held.  A single range runs on
// a round-robin context.  The first failing range's status and error text are returned.
template <class F>
int run_ranges(const std::vector<uint64_t>& b, F fn) {
  const size_t k = b.size() - 1;
  if (k == 1) {
    const int n = nctx();
    Context& c = n == 1 ? ctx(0) : ctx((int)(g_rr.fetch_add(1) % (uint64_t)n));
    ENTER_CTX(c);
    return fn(c, b[0], b[1]);
  }
  std::vector<int> rc(k, HIPBLS_OK);
  std::vector<std::string> err(k);
  auto one = [&](size_t j) {
    if (b[j] == b[j + 1]) return;
    Context& c = ctx((int)j);
    int r = bind(c);
    if (!r) {
      std::lock_guard<std::mutex> lk(c.mu);
      r = fn(c, b[j], b[j + 1]);
    }
    rc[j] = r;
    if (r) err[j] = g_last_error;
  };
  std::vector<std::thread> th;
  th.reserve(k - 1);
  for (size_t j = 1; j < k; ++j) th.emplace_back(one, j);
  one(0);
  for (auto& t : th) t.join();
  for (size_t j = 0; j < k; ++j)
    if (rc[j]) {
      g_last_error = err[j];
      return rc[j];
    }
  return HIPBLS_OK;
}

// run_ranges without the context lock: fn takes what it needs itself (tagg_verify_host).
template <class F>
int run_ranges_unlocked(const std::vector<uint64_t>& b, F fn) {
  const size_t k = b.size() - 1;
  if (k == 1) {
    const int n = nctx();
    Context& c = n == 1 ? ctx(0) : ctx((int)(g_rr.fetch_add(1) % (uint64_t)n));
    const int brc = bind(c);
    if (brc) return brc;
    return fn(c, b[0], b[1]);
  }
  std::vector<int> rc(k, HIPBLS_OK);
  std::vector<std::string> err(k);
  auto one = [&](size_t j) {
    if (b[j] == b[j + 1]) return;
    Context& c = ctx((int)j);
    int r = bind(c);
    if (!r) r = fn(c, b[j], b[j + 1]);
    rc[j] = r;
    if (r) err[j] = g_last_error;
  };
  std::vector<std::thread> th;
  th.reserve(k - 1);
  for (size_t j = 1; j < k; ++j) th.emplace_back(one, j);
  one(0);
  for (auto& t : th) t.join();
  for (size_t j = 0; j < k; ++j)
    if (rc[j]) {
      g_last_error = err[j];
      return rc[j];
    }
  return HIPBLS_OK;
}

// Runs fn(context) on every context (table loads, cache configuration), in parallel.
template <class F>
int run_all(F fn) {
  const int n = nctx();
  std::vector<uint64_t> b(n + 1);
  for (int k = 0; k <= n; ++k) b[k] = (uint64_t)k;
  if (n == 1) {
    ENTER_CTX(ctx(0));
    return fn(ctx(0));
  }
  return run_ranges(b, [&](Context& c, uint64_t, uint64_t) -> int { return fn(c); });
}

// Message offsets of items [lo, hi) relative to the range's first message byte.
const uint64_t* rebase(const uint64_t* offs, uint64_t lo, uint64_t hi, std::vector<uint64_t>& tmp) {
  if (offs[lo] == 0) return offs + lo;
  tmp.resize(hi - lo + 1);
  for (uint64_t i = lo; i <= hi; ++i) tmp[i - lo] = offs[i] - offs[lo];
  return tmp.data();
}

uint64_t grid_for(uint64_t n) { return (n + kBlock - 1) / kBlock; }

// Waves the device runs at once at one wave per SIMD (4 SIMDs per compute unit): a kernel of exactly a multiple of this
// many waves leaves nothing free for a kernel beside it (rlcb.h rlcb_chunk_count).
uint64_t wave_slots(Context& c) {
  if (!c.slots) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c.device) != hipSuccess || cus <= 0) cus = 256;
    c.slots = 4 * (uint64_t)cus;
  }
  return c.slots;
}
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
int timed(Context& c, const char* name, hipStream_t s, Launch launch) {
  hipEvent_t e0 = nullptr, e1 = nullptr;
  const bool on = g_timing.load();
  if (on) {
    HIP_TRY(hipEventCreate(&e0));
    HIP_TRY(hipEventCreate(&e1));
    HIP_TRY(hipEventRecord(e0, s));
  }
  launch();
  HIP_TRY(hipGetLastError());
  if (on) {
    HIP_TRY(hipEventRecord(e1, s));
    std::lock_guard<std::mutex> lk(c.tmu);
    TimingSlot& t = c.timing[name];
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
  if (pm && pm[0] >= '0' && pm[0] <= '4' && pm[1] == 0) return pm[0] - '0';
  return HIPBLS_PAIR_AUTO;
}
std::atomic<int> g_pair_mode{initial_pair_mode()};
// Crossovers measured on MI355X (profiles/r02_pair_sweep.txt): lane pairs win up to 32,768 Verify items (742k vs
// 634k verifies/s there) and lose from 49,152 (731k vs 919k).
constexpr uint64_t kLg2MaxVerify = 32768;    // auto: Verify batches up to this many items take lane pairs
constexpr uint64_t kLg2MaxWindows = 32768;   // auto: RLC sub-batches up to this many windows take lane pairs

#ifndef BLS_LQ4_MAX_VERIFY
#define BLS_LQ4_MAX_VERIFY 16384  // profiles/r03_pair_sweep_quads.txt: quads win up to 16,384 items (one round of waves)
#endif
constexpr uint64_t kLq4MaxVerify = BLS_LQ4_MAX_VERIFY;  // auto: Verify-shaped batches up to this many take quads

#ifndef BLS_LQ8_MAX_VERIFY
#define BLS_LQ8_MAX_VERIFY 4096  // scripts/latency_sweep.py: octets 14.1 vs quads 17.7 ms at 4,096, 19.5 vs 18.8 at 8,192
#endif
constexpr uint64_t kLq8MaxVerify = BLS_LQ8_MAX_VERIFY;  // auto: Verify batches up to this many take octets

// Replicas of a one-workgroup octet Verify (verify_lat.hip bls_race; HIPBLS_LAT_REPLICAS, 1 = off) and the epoch that
// names each raced launch in its race words.
uint32_t initial_lat_replicas() {
  const char* r = getenv("HIPBLS_LAT_REPLICAS");
  const int v = r ? atoi(r) : 8;
  return v < 1 ? 1u : (v > 32 ? 32u : (uint32_t)v);
}
std::atomic<uint32_t> g_lat_replicas{initial_lat_replicas()};
std::atomic<uint32_t> g_race_epoch{0};

bool use_pairs(uint64_t units, uint64_t auto_max) {
  const int mode = g_pair_mode.load();
  if (mode == HIPBLS_PAIR_SINGLE) return false;
  if (mode == HIPBLS_PAIR_LANES || mode == HIPBLS_PAIR_QUADS || mode == HIPBLS_PAIR_OCTETS) return true;
  return units <= auto_max;
}
bool use_quads(uint64_t n) {
  const int mode = g_pair_mode.load();
  if (mode == HIPBLS_PAIR_QUADS || mode == HIPBLS_PAIR_OCTETS) return true;
  return mode == HIPBLS_PAIR_AUTO && n <= kLq4MaxVerify;
}
// The octet path's check on sixteen lanes per item (verify_hex.hip) for batches of at most four items: AUTO only (the
// forced OCTETS mode keeps eight lanes, so the layout-parity tests compare the two), HIPBLS_LAT_HEX=0 turns it off.
constexpr uint64_t kLq16MaxVerify = 4;
bool initial_lat_hex() {
  const char* e = getenv("HIPBLS_LAT_HEX");
  return !(e && e[0] == '0');
}
const bool g_lat_hex = initial_lat_hex();
bool use_hex(uint64_t n) { return g_lat_hex && g_pair_mode.load() == HIPBLS_PAIR_AUTO && n <= kLq16MaxVerify; }
// Verify only (the drop-in latency path, verify_lat.hip); sigagg's check and the RLC stages keep quads / pairs.
bool use_octets(uint64_t n) {
  const int mode = g_pair_mode.load();
  if (mode == HIPBLS_PAIR_OCTETS) return true;
  return mode == HIPBLS_PAIR_AUTO && n <= kLq8MaxVerify;
}

// Verify: fused (one lane per item) or prep + lane-pair check; `ws` is the caller's SoA workspace for the latter
// (120 words per item), so the library stream and the queue worker never share one.
int launch_verify(Context& c, const uint8_t* d_pks, const uint8_t* d_msgs, const uint64_t* d_offs,
                  const uint8_t* d_sigs, uint64_t n, int32_t* d_status, hipStream_t s, DevBuf& ws) {
  if (n == 0) return HIPBLS_OK;
  if (!use_pairs(n, kLg2MaxVerify))
    return timed(c, "verify", s, [&] {
      hipLaunchKernelGGL(k_verify_fused, dim3((unsigned)grid_for(n)), dim3(kBlock), 0, s, d_pks, d_msgs, d_offs,
                         d_sigs, n, d_status);
    });
  // + two decode codes per item for the octet path, and the octet path's race words in the buffer's last 64 bytes (a
  // fixed place per allocation, 64-byte aligned since the capacity is a multiple of 256, beyond every batch's data;
  // zeroed when the buffer is allocated, then only ever written with a launch's epoch, so a stale word never equals a
  // new epoch)
  void* const before = ws.p;
  HIP_TRY(ws.ensure(n * 122 * 4 + 128));
  if (ws.p != before) HIP_TRY(hipMemsetAsync((uint8_t*)ws.p + ws.cap - 64, 0, 64, s));
  if (use_octets(n)) {
    const unsigned g8 = (unsigned)grid_for(8 * n);
    // A batch of one workgroup (<= 8 items: the drop-in n = 1 calls) races `lat_replicas` copies of it, one per XCD
    // (verify_lat.hip bls_race): the first copy to finish each stage wins.  Race words after the workspace.
    uint32_t* race = (uint32_t*)((uint8_t*)ws.p + ws.cap - 64);
    // (the race words must be naturally aligned: a misaligned word faults the device -- round 5, before capacities
    // were rounded to 256 bytes)
    const uint32_t reps = g8 == 1 && ((uintptr_t)race & 63) == 0 ? g_lat_replicas.load() : 1u;
    uint32_t epoch = reps > 1 ? g_race_epoch.fetch_add(1) + 1u : 0u;
    if (reps > 1 && epoch == 0) epoch = g_race_epoch.fetch_add(1) + 1u;  // 0 is a fresh word's value
    int rc = timed(c, "verify_prep8", s, [&] {  // three roles: key, signature, hash (verify_lat.hip)
      hipLaunchKernelGGL(bls_fp2p::k_verify_prep8, dim3(3 * g8 * reps), dim3(kBlock), 0, s, d_pks, d_msgs, d_offs,
                         d_sigs, n, (uint32_t*)ws.p, d_status, reps, race, epoch);
    });
    if (rc) return rc;
    return timed(c, use_hex(n) ? "verify_pair_lq16" : "verify_pair_lq8", s, [&] {
#if defined(BLS_LQ8_XCD_PROBE) && BLS_LQ8_XCD_PROBE
      hipLaunchKernelGGL(bls_fp2p::k_verify_pair_lq8, dim3(8 * g8), dim3(kBlock), 0, s, (const uint32_t*)ws.p, n,
                         d_status, 1u, race, 0u);  // experiment build: every workgroup once per XCD (verify_lat.hip)
#else
      if (use_hex(n))  // n <= 4: one workgroup of sixteen lanes per item, like g8 == 1
        hipLaunchKernelGGL(bls_hex::k_verify_pair_lq16, dim3(g8 * reps), dim3(kBlock), 0, s, (const uint32_t*)ws.p, n,
                           d_status, reps, race, epoch);
      else
        hipLaunchKernelGGL(bls_fp2p::k_verify_pair_lq8, dim3(g8 * reps), dim3(kBlock), 0, s, (const uint32_t*)ws.p, n,
                           d_status, reps, race, epoch);
#endif
    });
  }
  int rc = timed(c, "verify_prep", s, [&] {
    const int pair_hash = n <= kPairHashMaxVerify ? 1 : 0;
    hipLaunchKernelGGL(k_verify_prep, dim3((unsigned)((pair_hash ? 3 : 2) * grid_for(n))), dim3(kBlock), 0, s, d_pks,
                       d_msgs, d_offs, d_sigs, n, (uint32_t*)ws.p, d_status, pair_hash);
  });
  if (rc) return rc;
  if (use_quads(n))
    return timed(c, "verify_pair_lq4", s, [&] {
      hipLaunchKernelGGL(k_verify_pair_lq4, dim3((unsigned)grid_for(4 * n)), dim3(kBlock), 0, s,
                         (const uint32_t*)ws.p, n, d_status);
    });
  return timed(c, "verify_pair_lg2", s, [&] {
    hipLaunchKernelGGL(k_verify_pair_lg2, dim3((unsigned)grid_for(2 * n)), dim3(kBlock), 0, s,
                       (const uint32_t*)ws.p, n, d_status);
  });
}

bool use_rlc_batch(Context& c, uint64_t n);
int launch_rlc_batch(Context& c, const uint8_t* d_pks, const uint8_t* d_sigs, const uint32_t* d_midx, uint64_t n,
                     const uint8_t* d_msgs, const uint64_t* d_offs, uint64_t n_msgs, const rlc_seed& seed,
                     int32_t* d_status, hipStream_t s, const uint32_t* d_kidx, uint32_t* d_H, uint64_t hstride,
                     const uint32_t* d_hslot, const uint32_t* d_mlist, uint64_t n_hash);

int ensure_rlc_streams(Context& c) {  // the sub-streams are the device's (init_locked); the events are the context's
  if (c.ev_fork) return HIPBLS_OK;
  HIP_TRY(hipEventCreateWithFlags(&c.ev_hash, hipEventDisableTiming));
  for (int k = 0; k < Context::kSub; ++k) HIP_TRY(hipEventCreateWithFlags(&c.ev_join[k], hipEventDisableTiming));
  HIP_TRY(hipEventCreateWithFlags(&c.ev_fork, hipEventDisableTiming));
  return HIPBLS_OK;
}

rlc_seed parse_seed(const uint8_t* seed32) {
  rlc_seed seed;
  for (int k = 0; k < 8; ++k)
    seed.w[k] = (uint32_t)seed32[4 * k] << 24 | (uint32_t)seed32[4 * k + 1] << 16 | (uint32_t)seed32[4 * k + 2] << 8 |
                (uint32_t)seed32[4 * k + 3];
  return seed;
}

// RLC stage 4 over a device-side list of at most `cap` items (its length is only known on the device): AUTO launches
// both layouts and each kernel takes the lists on its side of the crossover -- lane pairs while the `concurrent`
// lists running side by side fit one round of waves (1024 waves x 64 lanes / 2 per item), one lane per item above.
// The pair kernel's grid covers only the lists it can take, so when it stands aside it costs a few hundred
// workgroups that exit at once.
constexpr uint64_t kLg2FallbackLanes = 32768;
int launch_fallback(Context& c, hipStream_t s, const uint32_t* list, const uint32_t* cnt, uint64_t cap,
                    uint64_t concurrent, const uint8_t* d_pks, const uint8_t* d_sigs, const uint32_t* d_midx,
                    const uint32_t* d_H, uint64_t hstride, const uint32_t* d_hslot, int32_t* d_status,
                    const uint32_t* d_kidx, uint64_t T, const uint32_t* tab, const uint32_t* rpk,
                    const uint32_t* rsig, uint64_t n) {
  const int mode = g_pair_mode.load();
  const uint64_t pair_upto = mode == HIPBLS_PAIR_SINGLE ? 0
                             : (mode == HIPBLS_PAIR_AUTO ? kLg2FallbackLanes / (concurrent ? concurrent : 1)
                                                         : ~(uint64_t)0);
  const uint64_t pairs = cap < pair_upto ? cap : pair_upto;
  int rc = HIPBLS_OK;
  if (pairs > 0)
    rc = timed(c, "rlc_fallback_lg2", s, [&] {
      hipLaunchKernelGGL(k_rlc_fallback_lg2, dim3((unsigned)grid_for(2 * pairs)), dim3(kBlock), 0, s, list, cnt, cap,
                         d_pks, d_sigs, d_midx, d_H, hstride, d_hslot, d_status, d_kidx, T, tab, pair_upto, rpk, rsig,
                         n);
    });
  if (rc) return rc;
  if (pair_upto < cap)
    rc = timed(c, "rlc_fallback", s, [&] {
      hipLaunchKernelGGL(k_rlc_fallback, dim3((unsigned)grid_for(cap)), dim3(kBlock), 0, s, list, cnt, cap, d_pks,
                         d_sigs, d_midx, d_H, hstride, d_hslot, d_status, d_kidx, T, tab, pair_upto, rpk, rsig, n);
    });
  return rc;
}

// RLC BatchVerify: the batch is cut into up to kSub window-aligned sub-batches, each running items -> window ->
// fallback on its own stream, while the distinct messages are hashed on the caller's stream; windows wait only
// for the hash.  Every stage is latency-bound on its own (one lane per item at one wave per SIMD), so overlapping
// the sub-batches' stages is what fills the CUs.  The caller's stream `s` forks into the sub-streams and joins
// back, so the call stays stream-ordered.
// H table: H(m) of message m is at column hslot[m] (identity when hslot == nullptr) of an affine SoA table with
// `hstride` columns; k_rlc_hash fills the columns of the n_hash messages listed in mlist (all when nullptr).
int launch_rlc(Context& c, const uint8_t* d_pks, const uint8_t* d_sigs, const uint32_t* d_midx, uint64_t n,
               const uint8_t* d_msgs, const uint64_t* d_offs, uint64_t n_msgs, const rlc_seed& seed,
               int32_t* d_status, hipStream_t s, uint64_t call, const uint32_t* d_kidx = nullptr,
               uint32_t* d_H = nullptr, uint64_t hstride = 0, const uint32_t* d_hslot = nullptr,
               const uint32_t* d_mlist = nullptr, uint64_t n_hash = 0) {
  // d_pks == nullptr: keys from the resident table
  const uint64_t T = c.t_size;
  const int32_t* tcode = (const int32_t*)c.t_code.p;
  const uint32_t* tab = (const uint32_t*)c.t_tab.p;
  c.r_windows = 0;
  c.r_call = call;
  if (n == 0) return HIPBLS_OK;
  if (n > 0xffffffffull) return arg_err("RLC batch larger than 2^32 items");  // fallback list holds 32-bit indices
  int rc = ensure_rlc_streams(c);
  if (rc) return rc;
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
  if (use_rlc_batch(c, n))
    return launch_rlc_batch(c, d_pks, d_sigs, d_midx, n, d_msgs, d_offs, n_msgs, seed, d_status, s, d_kidx, d_H,
                            hstride, d_hslot, d_mlist, n_hash);
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
  // The sub-batches' window launches run side by side at one lane per window.  When their partial last waves push the
  // total into one more round of waves than their full waves need (C5: 131,088 windows = 2 x 1,024.1 waves on 1,024
  // SIMDs, a third ~30 ms round for 16 windows), those windows' items go straight to the per-item checks instead
  // (k_rlc_window wdirect), which run in the fallback's tail.
  bool direct = false;
  {
    uint64_t full = 0, all = 0;
    for (int k = 0; k < nsub; ++k) {
      const uint64_t w0 = win_per * k, w1 = w0 + win_per < n_win ? w0 + win_per : n_win;
      if (w0 >= w1 || use_pairs(w1 - w0, kLg2MaxWindows)) continue;
      full += (w1 - w0) / kBlock;
      all += grid_for(w1 - w0);
    }
    const uint64_t S = wave_slots(c);
    direct = all > S && (full + S - 1) / S < (all + S - 1) / S;
  }

  rc = ws_begin(c, s, WS_RLC);
  if (rc) return rc;
  HIP_TRY(hipMemsetAsync(cnt, 0, Context::kSub * 4, s));
  HIP_TRY(hipEventRecord(c.ev_fork, s));
  if (n_hash) {
    rc = timed(c, "rlc_hash", s, [&] {
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
    rc = timed(c, "rlc_items", ss, [&] {
      hipLaunchKernelGGL(k_rlc_items, dim3((unsigned)grid_for(i1 - i0)), dim3(kBlock), 0, ss, i0, i1, d_pks, d_sigs,
                         d_midx, n, n_msgs, seed, rpk, rsig, d_status, d_kidx, T, tcode, tab);
    });
    if (rc) return rc;
    HIP_TRY(hipStreamWaitEvent(ss, c.ev_hash, 0));
    if (use_pairs(w1 - w0, kLg2MaxWindows))
      rc = timed(c, "rlc_window_lg2", ss, [&] {
        hipLaunchKernelGGL(k_rlc_window_lg2, dim3((unsigned)grid_for(2 * (w1 - w0))), dim3(kBlock), 0, ss, w0, w1, n,
                           d_midx, (const uint32_t*)rpk, (const uint32_t*)rsig, (const uint32_t*)d_H, hstride, d_hslot,
                           d_status, win, list + i0, cnt + k);
      });
    else
      rc = timed(c, "rlc_window", ss, [&] {
        const uint64_t wdirect = direct ? w0 + (w1 - w0) / kBlock * kBlock : w1;
        hipLaunchKernelGGL(k_rlc_window, dim3((unsigned)grid_for(w1 - w0)), dim3(kBlock), 0, ss, w0, w1, n, d_midx,
                           (const uint32_t*)rpk, (const uint32_t*)rsig, (const uint32_t*)d_H, hstride, d_hslot,
                           d_status, win, list + i0, cnt + k, wdirect);
      });
    if (rc) return rc;
    // The list length is only known on the device: launch for the worst case, idle lanes exit.  The list is short
    // (failed windows only) and latency-bound, so lane pairs unless the caller forced single lanes.  The last
    // sub-batch's list is the call's tail -- the other sub-batches' stages are done by then -- so with
    // HIPBLS_RLC_TAIL_PAIRS=1 it takes pairs up to the whole chip's lanes (the earlier ones share the chip with the
    // next sub-batch's windows); off by default until measured on its own.
    static const bool tail_pairs = getenv("HIPBLS_RLC_TAIL_PAIRS") && getenv("HIPBLS_RLC_TAIL_PAIRS")[0] == '1';
    rc = launch_fallback(c, ss, list + i0, cnt + k, i1 - i0, tail_pairs && k + 1 == nsub ? 1 : nsub, d_pks, d_sigs,
                         d_midx, d_H, hstride, d_hslot, d_status, d_kidx, T, tab, rpk, rsig, n);
    if (rc) return rc;
    HIP_TRY(hipEventRecord(c.ev_join[k], ss));
    HIP_TRY(hipStreamWaitEvent(s, c.ev_join[k], 0));
  }
  c.r_windows = n_win;
  return ws_end(c, s, WS_RLC);
}

// ============================================================================ batch-wide RLC check (rlcb.h)
// Policy (hipbls_rlc_set_mode): WINDOWS = rlc.h only; BATCH = the batch-wide check first, windows for whatever it
// leaves pending; AUTO (default) = BATCH for batches of >= 1,024 items unless the last batch check of this context
// failed, in which case its next 8 calls run windows only (a cluster that sends invalid partials keeps sending
// them; one whose batches pass keeps the cheap path).  The verdict comes back asynchronously (pinned copy +
// event), so the policy never blocks a launch.
std::atomic<int> g_rlc_mode{HIPBLS_RLC_AUTO};
// G1 MSM per message (g1msm.h, hipbls_rlc_set_g1_msm_min): messages with >= g_g1m_min items get one bucket-method
// sum instead of per-item [r_i] pk_i, when the batch averages >= kG1mAvg items per message (committee roots).
std::atomic<uint32_t> g_g1m_min{G1M_MIN};
constexpr uint64_t kG1mAvg = 8;

// The G1 MSM's workspace for n items over n_msgs messages, at most nl_max of them large; word offsets into one
// buffer (each region 64-word aligned).
struct G1mLayout {
  uint64_t nl_max = 0, nb = 0, nparts = 0;
  uint64_t nrun = 0;
  uint64_t cnt, lid, lmsg, soff, cur, meta, pos, slotl, pts, sc, bcnt, boff, bcur, list, B, P, Wv, part, words = 0;
  G1mLayout(uint64_t n, uint64_t n_msgs, uint64_t nl) : nl_max(nl) {
    nb = nl * G1M_NBL;
    nparts = (nb + kScanBlk - 1) / kScanBlk;
    nrun = nl ? g1m_run_lanes(n) : 0;
    auto take = [&](uint64_t w) {
      const uint64_t at = words;
      words += (w + 63) & ~(uint64_t)63;
      return at;
    };
    cnt = take(n_msgs);
    lid = take(n_msgs);
    lmsg = take(nl);
    soff = take(nl + 1);
    cur = take(nl);
    meta = take(2);
    pos = take(n);
    slotl = take(n);
    pts = take(60 * n);
    sc = take(2 * n);
    bcnt = take(nb);
    boff = take(nb + 1);
    bcur = take(nb);
    list = take(2 * (uint64_t)G1M_WIN * n);
    B = take(36 * nb);
    P = take(2 * 36 * nrun);
    Wv = take(36 * nl * G1M_NFOLD);
    part = take(nparts + 1);
  }
};
constexpr uint64_t kRlcbMinItems = 1024;
constexpr int kRlcbBackoff = 8;

// Reads back every verdict whose copy has landed; with wait_slot >= 0 (or wait_all) blocks on that slot first.
// A failed wait on wait_slot is an error: the slot is about to be reused and its verdict would be lost.
int rlcb_poll(Context& c, int wait_slot, bool wait_all = false) {
  for (int k = 0; k < Context::kRlcbSlots; ++k) {
    if (!c.rlcb_pending[k]) continue;
    if (wait_all || k == wait_slot) {
      const hipError_t e = hipEventSynchronize(c.rlcb_ev[k]);
      if (e != hipSuccess) return set_err("hipEventSynchronize (batch-check verdict)", e);
    } else if (hipEventQuery(c.rlcb_ev[k]) != hipSuccess) {
      continue;
    }
    c.rlcb_pending[k] = false;
    const int v = c.rlcb_host_flag[k] ? 1 : 0;
    c.rlcb_passed += (uint64_t)v;
    if (c.rlcb_seq[k] >= c.rlcb_last_seq) {
      c.rlcb_last_seq = c.rlcb_seq[k];
      c.rlcb_last = v;
      c.rlcb_last_call = c.rlcb_call[k];
      if (!v) c.rlcb_skipped = 0;
    }
  }
  return HIPBLS_OK;
}

bool use_rlc_batch(Context& c, uint64_t n) {
  const int mode = g_rlc_mode.load();
  if (mode == HIPBLS_RLC_WINDOWS) return false;
  if (mode == HIPBLS_RLC_BATCH) return true;
  (void)rlcb_poll(c, -1);
  if (n < kRlcbMinItems) return false;
  if (c.rlcb_last == 0 && c.rlcb_skipped < kRlcbBackoff) {
    ++c.rlcb_skipped;
    return false;
  }
  return true;
}

// Stages 1-6 of rlcb.h on stream s, then the window/fallback stages of rlc.h for the items still pending (none
// when the batch check passed: those kernels then find nothing to do).  Shares launch_rlc's H(m) table setup.
int launch_rlc_batch(Context& c, const uint8_t* d_pks, const uint8_t* d_sigs, const uint32_t* d_midx, uint64_t n,
                     const uint8_t* d_msgs, const uint64_t* d_offs, uint64_t n_msgs, const rlc_seed& seed,
                     int32_t* d_status, hipStream_t s, const uint32_t* d_kidx, uint32_t* d_H, uint64_t hstride,
                     const uint32_t* d_hslot, const uint32_t* d_mlist, uint64_t n_hash) {
  const uint64_t T = c.t_size;
  const int32_t* tcode = (const int32_t*)c.t_code.p;
  const uint32_t* tab = (const uint32_t*)c.t_tab.p;
  const uint64_t npts = 2 * n;
  const uint64_t nch = rlcb_chunk_count(n, wave_slots(c));
  const uint64_t n_win = (n + RLC_W - 1) / RLC_W;
  const uint32_t g1min = g_g1m_min.load();
  const bool g1 = g1min > 0 && n_msgs > 0 && n >= kG1mAvg * n_msgs && n >= g1min;
  const uint64_t nl_max = g1 ? std::min<uint64_t>(n_msgs, n / g1min) : 0;
  const uint64_t cols = nch + nl_max;  // product-tree columns: the chunks, then one per large message
  const G1mLayout gl(n, n_msgs, nl_max);
  if (!c.rlcb_host_flag) {
    HIP_TRY(hipHostMalloc((void**)&c.rlcb_host_flag, Context::kRlcbSlots * sizeof(int32_t), hipHostMallocDefault));
    for (int k = 0; k < Context::kRlcbSlots; ++k) HIP_TRY(hipEventCreateWithFlags(&c.rlcb_ev[k], hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&c.rlcb_ev_items, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&c.rlcb_ev_msm, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&c.rlcb_ev_sf, hipEventDisableTiming));
  }
  int rc = ensure_rlc_streams(c);
  if (rc) return rc;
  const int slot = (int)(c.rlcb_next_seq % Context::kRlcbSlots);
  rc = rlcb_poll(c, slot);  // only blocks when kRlcbSlots verdicts are still in flight
  if (rc) return rc;
  HIP_TRY(c.m_pts.ensure(npts * 48 * 4));
  HIP_TRY(c.m_sc.ensure(npts * 4));
  HIP_TRY(c.m_cnt.ensure((uint64_t)MSM_WINDOWS * MSM_NB * 4));
  HIP_TRY(c.m_off.ensure((uint64_t)MSM_WINDOWS * (MSM_NB + 1) * 4));
  HIP_TRY(c.m_cur.ensure((uint64_t)MSM_WINDOWS * MSM_NB * 4));
  HIP_TRY(c.m_list.ensure((uint64_t)MSM_WINDOWS * npts * 4));
  HIP_TRY(c.m_B.ensure((uint64_t)MSM_WINDOWS * MSM_NB * 72 * 4));
  const uint64_t lpw = msm_run_lanes(npts);  // bucket-run lanes per window
  HIP_TRY(c.m_P.ensure(2 * MSM_WINDOWS * lpw * 72 * 4));
  HIP_TRY(c.m_Sg.ensure((uint64_t)MSM_WINDOWS * MSM_NSEG * 72 * 4));
  HIP_TRY(c.m_Wp.ensure((uint64_t)MSM_WINDOWS * MSM_WG * 72 * 4));
  HIP_TRY(c.m_W.ensure((uint64_t)MSM_WINDOWS * 72 * 4));
  HIP_TRY(c.m_F.ensure(cols * 144 * 4));
  HIP_TRY(c.m_F2.ensure(((cols + kBlock - 1) / kBlock) * 144 * 4));
  if (g1) HIP_TRY(c.g1_ws.ensure(gl.words * 4));
  uint32_t* gw = (uint32_t*)c.g1_ws.p;
  auto G = [&](uint64_t off) { return g1 ? gw + off : nullptr; };
  HIP_TRY(c.m_flag.ensure(4));
  HIP_TRY(c.m_Fs.ensure(144 * 4));
  uint32_t* rpk = (uint32_t*)c.r_pk.p;
  uint32_t* rsig = (uint32_t*)c.r_sig.p;
  uint32_t* pts = (uint32_t*)c.m_pts.p;
  uint32_t* sc = (uint32_t*)c.m_sc.p;
  int32_t* flag = (int32_t*)c.m_flag.p;
  // Streams: the caller's stream s hashes the messages while sub[0] runs the items and then the G2 MSM's short
  // kernels; sub[1] runs the G1 MSM of the large messages beside the G2 MSM (both only need the items) and their
  // Miller values, then the chunk Miller loops and the product once the G2 MSM and the hash are done -- after the
  // MSM, because the chunk kernel holds every SIMD for its whole run and a short kernel queued behind it waits that
  // long (round 2: k_msm_scan 33 ms beside k_rlcb_chunks 37.7 ms).  sub[0] follows the G2 MSM with the (-g1, S)
  // Miller value; s joins for the verdict and the windows.
  hipStream_t s0 = c.sub[0], s1 = c.sub[1];
  rc = ws_begin(c, s, WS_RLC);
  if (rc) return rc;
  HIP_TRY(hipMemsetAsync(c.m_cnt.p, 0, (size_t)MSM_WINDOWS * MSM_NB * 4, s));
  HIP_TRY(hipMemsetAsync(c.r_cnt.p, 0, 4, s));
  HIP_TRY(hipEventRecord(c.ev_fork, s));
  if (n_hash) {
    rc = timed(c, "rlc_hash", s, [&] {
      hipLaunchKernelGGL(k_rlc_hash, dim3((unsigned)grid_for(n_hash)), dim3(kBlock), 0, s, d_msgs, d_offs, n_hash,
                         d_mlist, d_H, hstride, d_hslot);
    });
    if (rc) return rc;
  }
  HIP_TRY(hipEventRecord(c.ev_hash, s));
  HIP_TRY(hipStreamWaitEvent(s0, c.ev_fork, 0));
  const unsigned gn256 = (unsigned)((n + 255) / 256);
  if (g1) {  // which messages are large, and each of their items' slot (g1msm.h)
    HIP_TRY(hipMemsetAsync(G(gl.cnt), 0, n_msgs * 4, s0));
    HIP_TRY(hipMemsetAsync(G(gl.cur), 0, nl_max * 4, s0));
    HIP_TRY(hipMemsetAsync(G(gl.bcnt), 0, gl.nb * 4, s0));
    rc = timed(c, "rlcb_g1plan", s0, [&] {
      hipLaunchKernelGGL(k_g1m_count, dim3(gn256), dim3(256), 0, s0, n, d_midx, n_msgs, G(gl.cnt));
      hipLaunchKernelGGL(k_g1m_plan, dim3(1), dim3(kPlanThreads), 0, s0, (const uint32_t*)G(gl.cnt), n_msgs, g1min,
                         G(gl.lid), G(gl.lmsg), G(gl.soff), G(gl.meta));
      hipLaunchKernelGGL(k_g1m_rank, dim3(gn256), dim3(256), 0, s0, n, d_midx, n_msgs, (const uint32_t*)G(gl.lid),
                         (const uint32_t*)G(gl.soff), G(gl.cur), G(gl.pos), G(gl.slotl));
    });
    if (rc) return rc;
  }
  rc = timed(c, "rlcb_items", s0, [&] {
    hipLaunchKernelGGL(k_rlcb_items, dim3((unsigned)grid_for(n)), dim3(kBlock), 0, s0, n, d_pks, d_sigs, d_midx, n_msgs,
                       seed, rpk, pts, sc, d_status, d_kidx, T, tcode, tab, (const uint32_t*)G(gl.pos), G(gl.pts),
                       G(gl.sc));
  });
  if (rc) return rc;
  HIP_TRY(hipEventRecord(c.rlcb_ev_items, s0));
  rc = timed(c, "rlcb_msm", s0, [&] {
    hipStream_t s = s0;
    const unsigned g256 = (unsigned)((npts + 255) / 256);
    hipLaunchKernelGGL(k_msm_hist, dim3(g256), dim3(256), 0, s, npts, (const uint32_t*)sc, (uint32_t*)c.m_cnt.p);
    hipLaunchKernelGGL(k_msm_scan, dim3(1), dim3(kScanThreads), 0, s, (const uint32_t*)c.m_cnt.p, (uint32_t*)c.m_off.p,
                       (uint32_t*)c.m_cur.p);
    hipLaunchKernelGGL(k_msm_scatter, dim3(g256), dim3(256), 0, s, npts, (const uint32_t*)sc, (uint32_t*)c.m_cur.p,
                       (uint32_t*)c.m_list.p);
    hipLaunchKernelGGL(k_msm_run, dim3((unsigned)grid_for((uint64_t)MSM_WINDOWS * lpw)), dim3(kBlock), 0, s,
                       (const uint32_t*)c.m_off.p, (const uint32_t*)c.m_list.p, npts, (const uint32_t*)pts,
                       (uint32_t*)c.m_B.p, (uint32_t*)c.m_P.p, lpw);
    hipLaunchKernelGGL(k_msm_fix, dim3((unsigned)grid_for((uint64_t)MSM_WINDOWS * MSM_NB)), dim3(kBlock), 0, s,
                       (const uint32_t*)c.m_off.p, (uint32_t*)c.m_B.p, (const uint32_t*)c.m_P.p, lpw);
    hipLaunchKernelGGL(k_msm_segment, dim3((unsigned)grid_for((uint64_t)MSM_WINDOWS * MSM_NSEG)), dim3(kBlock), 0, s,
                       (const uint32_t*)c.m_B.p, (uint32_t*)c.m_Sg.p);
    hipLaunchKernelGGL(k_msm_window, dim3(MSM_WINDOWS * MSM_WG), dim3(kSumBlock), 0, s, (const uint32_t*)c.m_Sg.p,
                       (uint32_t*)c.m_Wp.p);
    hipLaunchKernelGGL(k_msm_wsum, dim3(MSM_WINDOWS), dim3(64), 0, s, (const uint32_t*)c.m_Wp.p, (uint32_t*)c.m_W.p);
  });
  if (rc) return rc;
  HIP_TRY(hipEventRecord(c.rlcb_ev_msm, s0));
  // (-g1, S) right behind the MSM on its own queue, beside the chunks on the SIMD rlcb_chunk_count leaves free.  (On
  // the caller's stream, released by the same event as the chunks, it made the 1,023-wave chunk kernel 4.5 ms slower:
  // scripts/ab_c4_chunks.sh.)
  rc = timed(c, "rlcb_sfactor", s0, [&] {
    hipLaunchKernelGGL(bls_fp2p::k_rlcb_sfactor8, dim3(1), dim3(kBlock), bls_fp2p::kSfactorLds, s0,
                       (const uint32_t*)c.m_W.p, (uint32_t*)c.m_Fs.p);
  });
  if (rc) return rc;
  HIP_TRY(hipEventRecord(c.rlcb_ev_sf, s0));
  if (g1) {  // the large messages' sums R_L and their Miller values, beside the G2 MSM
    HIP_TRY(hipStreamWaitEvent(s1, c.rlcb_ev_items, 0));
    rc = timed(c, "rlcb_g1sort", s1, [&] {
      hipLaunchKernelGGL(k_g1m_hist, dim3(gn256), dim3(256), 0, s1, n, (const uint32_t*)G(gl.meta),
                         (const uint32_t*)G(gl.sc), (const uint32_t*)G(gl.slotl), G(gl.bcnt));
      hipLaunchKernelGGL(k_scan_part, dim3((unsigned)gl.nparts), dim3(kScanBlk), 0, s1, (const uint32_t*)G(gl.bcnt),
                         gl.nb, G(gl.part));
      hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(kScanBlk), 0, s1, G(gl.part), gl.nparts);
      hipLaunchKernelGGL(k_scan_apply, dim3((unsigned)gl.nparts), dim3(kScanBlk), 0, s1, (const uint32_t*)G(gl.bcnt),
                         gl.nb, (const uint32_t*)G(gl.part), gl.nparts, G(gl.boff), G(gl.bcur));
      hipLaunchKernelGGL(k_g1m_scatter, dim3(gn256), dim3(256), 0, s1, n, (const uint32_t*)G(gl.meta),
                         (const uint32_t*)G(gl.sc), (const uint32_t*)G(gl.slotl), G(gl.bcur), G(gl.list));
    });
    if (rc) return rc;
    rc = timed(c, "rlcb_g1msm", s1, [&] {
      hipLaunchKernelGGL(k_g1m_run, dim3((unsigned)grid_for(gl.nrun)), dim3(kBlock), 0, s1, gl.nrun,
                         (const uint32_t*)G(gl.meta), (const uint32_t*)G(gl.boff), (const uint32_t*)G(gl.list),
                         (const uint32_t*)G(gl.pts), n, G(gl.B), G(gl.P));
      hipLaunchKernelGGL(k_g1m_fix, dim3((unsigned)grid_for(gl.nb)), dim3(kBlock), 0, s1, gl.nb,
                         (const uint32_t*)G(gl.meta), (const uint32_t*)G(gl.boff), G(gl.B), (const uint32_t*)G(gl.P));
      hipLaunchKernelGGL(k_g1m_fold, dim3((unsigned)grid_for(nl_max * G1M_NFOLD)), dim3(kBlock), 0, s1,
                         nl_max * G1M_NFOLD, (const uint32_t*)G(gl.meta), (const uint32_t*)G(gl.B), G(gl.Wv));
    });
    if (rc) return rc;
    HIP_TRY(hipStreamWaitEvent(s1, c.ev_hash, 0));
    rc = timed(c, "rlcb_g1miller", s1, [&] {
      hipLaunchKernelGGL(bls_fp2p::k_g1m_miller8, dim3((unsigned)grid_for(8 * nl_max)), dim3(kBlock), 0, s1, nl_max,
                         (const uint32_t*)G(gl.meta), (const uint32_t*)G(gl.lmsg), (const uint32_t*)G(gl.Wv),
                         (const uint32_t*)d_H, hstride, d_hslot, (uint32_t*)c.m_F.p, nch, cols);
    });
    if (rc) return rc;
  }
  HIP_TRY(hipStreamWaitEvent(s1, c.rlcb_ev_msm, 0));
  HIP_TRY(hipStreamWaitEvent(s1, c.ev_hash, 0));
  rc = timed(c, "rlcb_chunks", s1, [&] {
    hipLaunchKernelGGL(k_rlcb_chunks, dim3((unsigned)grid_for(nch)), dim3(kBlock), 0, s1, n, (const int32_t*)d_status,
                       d_midx, (const uint32_t*)rpk, (const uint32_t*)d_H, hstride, d_hslot, (uint32_t*)c.m_F.p, nch,
                       cols);
  });
  if (rc) return rc;
  uint32_t* src = (uint32_t*)c.m_F.p;
  uint32_t* dst = (uint32_t*)c.m_F2.p;
  uint64_t cur = cols;
  rc = timed(c, "rlcb_product", s1, [&] {
    while (cur > 1) {  // 64 columns per wave (k_fp12_prod64)
      const uint64_t nxt = (cur + kBlock - 1) / kBlock;
      hipLaunchKernelGGL(k_fp12_prod64, dim3((unsigned)nxt), dim3(kBlock), 0, s1, (const uint32_t*)src, cur, dst, nxt);
      uint32_t* t = src;
      src = dst;
      dst = t;
      cur = nxt;
    }
  });
  if (rc) return rc;
  HIP_TRY(hipEventRecord(c.ev_join[1], s1));
  HIP_TRY(hipStreamWaitEvent(s, c.ev_join[1], 0));
  HIP_TRY(hipStreamWaitEvent(s, c.rlcb_ev_sf, 0));
  rc = timed(c, "rlcb_final", s, [&] {
    hipLaunchKernelGGL(bls_fp2p::k_rlcb_final8, dim3(1), dim3(kBlock), 0, s, (const uint32_t*)src,
                       (const uint32_t*)c.m_Fs.p, flag);
  });
  if (rc) return rc;
  rc = timed(c, "rlcb_mark", s, [&] {
    hipLaunchKernelGGL(k_rlcb_mark, dim3((unsigned)grid_for(n)), dim3(kBlock), 0, s, n, (const int32_t*)flag, d_status,
                       (const uint32_t*)pts, (const uint32_t*)sc, rsig, (const uint32_t*)G(gl.pos),
                       (const uint32_t*)G(gl.pts), (const uint32_t*)G(gl.sc), rpk);
  });
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(c.rlcb_host_flag + slot, flag, 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipEventRecord(c.rlcb_ev[slot], s));
  c.rlcb_pending[slot] = true;
  c.rlcb_seq[slot] = ++c.rlcb_next_seq;
  c.rlcb_call[slot] = c.r_call;
  c.rlcb_attempted += 1;
  // window + fallback stages over whatever is still pending (nothing when the batch check passed)
  int32_t* win = (int32_t*)c.r_win.p;
  uint32_t* list = (uint32_t*)c.r_list.p;
  uint32_t* cnt = (uint32_t*)c.r_cnt.p;
  if (use_pairs(n_win, kLg2MaxWindows))
    rc = timed(c, "rlc_window_lg2", s, [&] {
      hipLaunchKernelGGL(k_rlc_window_lg2, dim3((unsigned)grid_for(2 * n_win)), dim3(kBlock), 0, s, (uint64_t)0, n_win,
                         n, d_midx, (const uint32_t*)rpk, (const uint32_t*)rsig, (const uint32_t*)d_H, hstride, d_hslot,
                         d_status, win, list, cnt);
    });
  else
    rc = timed(c, "rlc_window", s, [&] {
      // as in launch_rlc: a partial last wave that would start another round goes straight to the per-item checks
      const uint64_t S = wave_slots(c), full = n_win / kBlock, all = grid_for(n_win);
      const uint64_t wdirect = all > S && (full + S - 1) / S < (all + S - 1) / S ? full * kBlock : n_win;
      hipLaunchKernelGGL(k_rlc_window, dim3((unsigned)grid_for(n_win)), dim3(kBlock), 0, s, (uint64_t)0, n_win, n,
                         d_midx, (const uint32_t*)rpk, (const uint32_t*)rsig, (const uint32_t*)d_H, hstride, d_hslot,
                         d_status, win, list, cnt, wdirect);
    });
  if (rc) return rc;
  rc = launch_fallback(c, s, list, cnt, n, 1, d_pks, d_sigs, d_midx, d_H, hstride, d_hslot, d_status, d_kidx, T, tab,
                       (const uint32_t*)rpk, (const uint32_t*)rsig, n);
  if (rc) return rc;
  c.r_windows = n_win;
  return ws_end(c, s, WS_RLC);
}

int launch_tagg(Context& c, const uint8_t* d_sigs, const int64_t* d_ids, const uint64_t* d_goffs, uint64_t n_groups,
                uint64_t n_parts, uint8_t* d_out, int32_t* d_status, hipStream_t s) {
  if (n_groups == 0) return HIPBLS_OK;
  HIP_TRY(c.b_pts.ensure((n_parts ? n_parts : 1) * 72 * 4));
  HIP_TRY(c.b_pst.ensure((n_parts ? n_parts : 1) * 4));
  int rc = ws_begin(c, s);
  if (rc) return rc;
  if (n_parts) {
    rc = timed(c, "tagg_scale", s, [&] {
      hipLaunchKernelGGL(k_tagg_scale, dim3((unsigned)grid_for(n_parts)), dim3(kBlock), 0, s, d_sigs, d_ids, d_goffs,
                         n_groups, n_parts, (uint32_t*)c.b_pts.p, (int32_t*)c.b_pst.p);
    });
    if (rc) return rc;
  }
  rc = timed(c, "tagg_sum", s, [&] {
    hipLaunchKernelGGL(k_tagg_sum, dim3((unsigned)grid_for(n_groups)), dim3(kBlock), 0, s, (const uint32_t*)c.b_pts.p,
                       (const int32_t*)c.b_pst.p, d_ids, d_goffs, n_groups, n_parts, d_out, d_status);
  });
  if (rc) return rc;
  return ws_end(c, s);
}

// sigagg in one call, three kernels on the caller's stream (kernels.h): phase A (the root keys' decode, [L] pk and
// message hashes, beside the partials' decode + subgroup test + c_k sig_k: one launch, prep workgroups first), the
// sums S (k_tagg_sum_s) and the status join, then the pairing checks on S against [L] pk beside [L^-1] S and the
// 96-byte aggregates (k_tv_check_unscale).  No sub-streams: the workspace comes from one of two sets used
// alternately (each waits for the call two back that used it), so calls enqueued on different streams overlap --
// the next call's phase A runs in the SIMDs the quad check leaves idle.  Same statuses and bytes as before.
#ifndef BLS_TV_PAIR_HASH
#define BLS_TV_PAIR_HASH 1
#endif
int launch_tagg_verify(Context& c, const uint8_t* d_sigs, const int64_t* d_ids, const uint64_t* d_goffs,
                       uint64_t n_groups, uint64_t n_parts, const uint8_t* d_dvpks, const uint8_t* d_msgs,
                       const uint64_t* d_moffs, uint8_t* d_out, int32_t* d_astatus, int32_t* d_vstatus, hipStream_t s) {
  if (n_groups == 0) return HIPBLS_OK;
  const int p = (int)(c.tv_seq & 1);
  if (!c.tv_done[p]) HIP_TRY(hipEventCreateWithFlags(&c.tv_done[p], hipEventDisableTiming));
  HIP_TRY(c.tv_pts[p].ensure((n_parts ? n_parts : 1) * 72 * 4));
  HIP_TRY(c.tv_pst[p].ensure((n_parts ? n_parts : 1) * 4));
  HIP_TRY(c.tv_ws[p].ensure(n_groups * 120 * 4));
  HIP_TRY(c.tv_aux[p].ensure(n_groups * 4));
  ++c.tv_seq;
  uint32_t* ws = (uint32_t*)c.tv_ws[p].p;
  int32_t* agg_inf = (int32_t*)c.tv_aux[p].p;
  uint32_t* pts = (uint32_t*)c.tv_pts[p].p;
  int32_t* pst = (int32_t*)c.tv_pst[p].p;
  if (!c.tv_phase) HIP_TRY(hipEventCreateWithFlags(&c.tv_phase, hipEventDisableTiming));
  HIP_TRY(hipStreamWaitEvent(s, c.tv_done[p], 0));
  // From here on every exit records tv_done[p] (and tv_phase, if phase A's end was not recorded yet) on s: the call
  // two later reuses workspace set p and waits on tv_done[p], so a call that fails after enqueueing work must still
  // publish the end of what it enqueued, or the next user of the set could overwrite buffers its kernels still read.
  struct TvEnd {
    Context& c;
    hipStream_t s;
    int p;
    bool phase = false;
    ~TvEnd() {
      if (!phase) (void)hipEventRecord(c.tv_phase, s);
      (void)hipEventRecord(c.tv_done[p], s);
    }
  } tv_end{c, s, p};
  // Phase A after the previous call's phase A, whatever its stream: two calls' phase A would only share the same
  // wave slots, while this call's phase A beside the previous call's check fills the SIMDs that check leaves idle.
  HIP_TRY(hipStreamWaitEvent(s, c.tv_phase, 0));
  int rc = HIPBLS_OK;
  if (BLS_TV_PAIR_HASH && n_groups <= kPairHashMaxVerify) {
    const uint64_t nprep = 3 * grid_for(n_groups), nscale = n_parts ? grid_for(n_parts) : 0;
    rc = timed(c, "tv_phase_a", s, [&] {
      hipLaunchKernelGGL(k_tv_phase_a, dim3((unsigned)(nprep + nscale)), dim3(kBlock), 0, s, d_dvpks, d_msgs, d_moffs,
                         n_groups, d_ids, d_goffs, ws, d_vstatus, d_sigs, n_parts, pts, pst);
    });
  } else {
    rc = timed(c, "tv_prep_pk", s, [&] {
      hipLaunchKernelGGL(k_tv_prep_pk, dim3((unsigned)grid_for(n_groups)), dim3(kBlock), 0, s, d_dvpks, d_msgs,
                         d_moffs, n_groups, d_ids, d_goffs, ws, d_vstatus);
    });
    if (rc) return rc;
    if (n_parts)
      rc = timed(c, "tagg_scale", s, [&] {
        hipLaunchKernelGGL(k_tagg_scale, dim3((unsigned)grid_for(n_parts)), dim3(kBlock), 0, s, d_sigs, d_ids,
                           d_goffs, n_groups, n_parts, pts, pst);
      });
  }
  if (rc) return rc;
  rc = timed(c, "tagg_sum", s, [&] {
    hipLaunchKernelGGL(k_tagg_sum_s, dim3((unsigned)grid_for(n_groups)), dim3(kBlock), 0, s, (const uint32_t*)pts,
                       (const int32_t*)pst, d_goffs, n_groups, n_parts, d_astatus, ws, agg_inf);
  });
  if (rc) return rc;
  hipLaunchKernelGGL(k_tv_join, dim3((unsigned)grid_for(n_groups)), dim3(kBlock), 0, s, n_groups,
                     (const int32_t*)d_astatus, (const int32_t*)agg_inf, d_vstatus);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipEventRecord(c.tv_phase, s));
  tv_end.phase = true;
  if (use_quads(n_groups)) {
    rc = timed(c, "tv_check_unscale", s, [&] {
      hipLaunchKernelGGL(k_tv_check_unscale, dim3((unsigned)(grid_for(4 * n_groups) + grid_for(n_groups))),
                         dim3(kBlock), 0, s, (const uint32_t*)ws, n_groups, d_vstatus, d_ids, d_goffs,
                         (const int32_t*)agg_inf, (const int32_t*)d_astatus, d_out);
    });
  } else {
    if (use_pairs(n_groups, kLg2MaxVerify))
      rc = timed(c, "verify_pair_lg2", s, [&] {
        hipLaunchKernelGGL(k_verify_pair_lg2, dim3((unsigned)grid_for(2 * n_groups)), dim3(kBlock), 0, s,
                           (const uint32_t*)ws, n_groups, d_vstatus);
      });
    else
      rc = timed(c, "verify_pair_single", s, [&] {
        hipLaunchKernelGGL(k_verify_pair_single, dim3((unsigned)grid_for(n_groups)), dim3(kBlock), 0, s,
                           (const uint32_t*)ws, n_groups, d_vstatus);
      });
    if (rc) return rc;
    rc = timed(c, "tagg_unscale", s, [&] {
      hipLaunchKernelGGL(k_tagg_unscale, dim3((unsigned)grid_for(n_groups)), dim3(kBlock), 0, s, d_ids, d_goffs,
                         n_groups, (const uint32_t*)ws, (const int32_t*)agg_inf, (const int32_t*)d_astatus, d_out);
    });
  }
  return rc;  // tv_end records tv_done[p]
}

// A few groups (the sync committee's one aggregate per slot) take the drop-in path's layouts: keys, signatures and
// messages decoded / hashed on octets (verify_lat.hip k_fav_prep8), then the key sum and the sixteen-lane check per
// group (verify_hex.hip k_fav_pair_lq16), instead of k_fav_batch's one workgroup per group with its hash and pairing
// at one or two lanes' speed.  AUTO pair mode only, so PAIR_SINGLE / PAIR_LANES keep k_fav_batch for the layout-parity
// tests; HIPBLS_LAT_HEX=0 turns it off with the n = 1 check.
constexpr uint64_t kFavHexMaxGroups = 16;
bool use_fav_hex(uint64_t n_groups) {
  return g_lat_hex && g_pair_mode.load() == HIPBLS_PAIR_AUTO && n_groups <= kFavHexMaxGroups;
}

int launch_fav(Context& c, const uint8_t* d_pks, uint64_t nkeys, const uint64_t* d_goff, uint64_t n_groups,
               const uint8_t* d_sigs, const uint8_t* d_msgs, const uint64_t* d_moffs, int32_t* d_status,
               hipStream_t s) {
  if (n_groups == 0) return HIPBLS_OK;
  HIP_TRY(c.b_pts.ensure((nkeys ? nkeys : 1) * 24 * 4));
  HIP_TRY(c.b_pst.ensure((nkeys ? nkeys : 1) * 4));
  int rc = ws_begin(c, s);
  if (rc) return rc;
  if (use_fav_hex(n_groups)) {
    HIP_TRY(c.f_ws.ensure(n_groups * 122 * 4));
    // the kernel derives the same role boundaries from nkeys and n_groups
    const uint64_t nbk = (8 * nkeys + kBlock - 1) / kBlock, nbg = (8 * n_groups + kBlock - 1) / kBlock;
    rc = timed(c, "fav_prep8", s, [&] {
      hipLaunchKernelGGL(bls_fp2p::k_fav_prep8, dim3((unsigned)(nbk + 2 * nbg)), dim3(kBlock), 0, s, d_pks, nkeys,
                         d_sigs, d_msgs, d_moffs, n_groups, (uint32_t*)c.b_pts.p, (int32_t*)c.b_pst.p,
                         (uint32_t*)c.f_ws.p);
    });
    if (rc) return rc;
    rc = timed(c, "fav_lq16", s, [&] {
      hipLaunchKernelGGL(bls_hexw::k_fav_pair_lq16, dim3((unsigned)n_groups), dim3(kBlock), 0, s,
                         (const uint32_t*)c.b_pts.p, (const int32_t*)c.b_pst.p, nkeys, d_goff,
                         (const uint32_t*)c.f_ws.p, n_groups, d_status);
    });
    if (rc) return rc;
    return ws_end(c, s);
  }
  if (nkeys)
    hipLaunchKernelGGL(k_g1_decode, dim3((unsigned)grid_for(nkeys)), dim3(kBlock), 0, s, d_pks, nkeys,
                       (uint32_t*)c.b_pts.p, (int32_t*)c.b_pst.p);
  rc = timed(c, "fav", s, [&] {
    hipLaunchKernelGGL(k_fav_batch, dim3((unsigned)n_groups), dim3(kFavBlock), 0, s, (const uint32_t*)c.b_pts.p,
                       (const int32_t*)c.b_pst.p, nkeys, d_goff, d_sigs, d_msgs, d_moffs, d_status);
  });
  if (rc) return rc;
  return ws_end(c, s);
}

// Aggregate: decode in parallel, per-workgroup partial sums, one final workgroup (kernels.h).
int launch_aggregate(Context& c, const uint8_t* d_sigs, uint64_t n, uint8_t* d_out, int32_t* d_status, hipStream_t s) {
  const uint64_t per_wg = 8 * (uint64_t)kSumBlock;  // points folded per lane before the tree
  uint64_t nwg = (n + per_wg - 1) / per_wg;
  if (nwg < 1) nwg = 1;
  if (nwg > 1024) nwg = 1024;
  HIP_TRY(c.b_pts.ensure((n ? n : 1) * 48 * 4));
  HIP_TRY(c.b_pst.ensure((n ? n : 1) * 4));
  HIP_TRY(c.b_part.ensure(nwg * 72 * 4));
  HIP_TRY(c.b_bad.ensure(4));
  int rc = ws_begin(c, s);
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
  return ws_end(c, s);
}

bool mul_overflows(uint64_t a, uint64_t b) { return b != 0 && a > UINT64_MAX / b; }

bool offsets_ok(const uint64_t* offs, uint64_t n) {
  if (offs[0] != 0) return false;
  for (uint64_t i = 0; i < n; ++i)
    if (offs[i + 1] < offs[i] || offs[i + 1] - offs[i] > 0xffffffffull) return false;
  return true;
}

bool groups_ok(const uint64_t* goffs, uint64_t n_groups) {
  if (goffs[0] != 0) return false;
  for (uint64_t g = 0; g < n_groups; ++g)
    if (goffs[g + 1] < goffs[g]) return false;
  return true;
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

// Host-buffer RLC body shared by the wire-format and key-table calls, on one context (lock held), stream `s` with
// the given workspaces for the inputs.  The H(m) table is the context's cache when enabled, else per call.
struct RlcBufs {
  DevBuf *pk, *kidx, *sig, *midx, *msg, *off, *st, *slot, *mlist;
};
int rlc_host_on(Context& c, RlcBufs B, hipStream_t s, const uint8_t* pks, const uint32_t* key_idx, const uint8_t* sigs,
                const uint32_t* msg_idx, uint64_t n, const uint8_t* msgs, const uint64_t* msg_offsets, uint64_t n_msgs,
                const rlc_seed& seed, int32_t* status, uint64_t call) {
  const uint64_t msg_total = msg_offsets[n_msgs];
  if (pks) HIP_TRY(B.pk->ensure(n * 48));
  if (key_idx) HIP_TRY(B.kidx->ensure(n * 4));
  HIP_TRY(B.sig->ensure(n * 96));
  HIP_TRY(B.midx->ensure(n * 4));
  HIP_TRY(B.msg->ensure(msg_total ? msg_total : 1));
  HIP_TRY(B.off->ensure((n_msgs + 1) * 8));
  HIP_TRY(B.st->ensure(n * 4));
  if (pks) HIP_TRY(hipMemcpyAsync(B.pk->p, pks, n * 48, hipMemcpyHostToDevice, s));
  if (key_idx) HIP_TRY(hipMemcpyAsync(B.kidx->p, key_idx, n * 4, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(B.sig->p, sigs, n * 96, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(B.midx->p, msg_idx, n * 4, hipMemcpyHostToDevice, s));
  if (msg_total) HIP_TRY(hipMemcpyAsync(B.msg->p, msgs, msg_total, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(B.off->p, msg_offsets, (n_msgs + 1) * 8, hipMemcpyHostToDevice, s));
  std::vector<uint32_t> slot, miss;
  uint32_t* dH = nullptr;
  const uint32_t *dslot = nullptr, *dmiss = nullptr;
  uint64_t stride = 0, n_hash = 0;
  if (hcache_assign(c.hcache, msgs, msg_offsets, n_msgs, slot, miss)) {
    HIP_TRY(B.slot->ensure((n_msgs ? n_msgs : 1) * 4));
    HIP_TRY(B.mlist->ensure((miss.size() ? miss.size() : 1) * 4));
    // the copies run on s behind every earlier workspace user (ws_done): the slot table is per call
    int rc = ws_begin(c, s, WS_RLC);
    if (rc) return rc;
    if (n_msgs) HIP_TRY(hipMemcpyAsync(B.slot->p, slot.data(), n_msgs * 4, hipMemcpyHostToDevice, s));
    if (miss.size()) HIP_TRY(hipMemcpyAsync(B.mlist->p, miss.data(), miss.size() * 4, hipMemcpyHostToDevice, s));
    dH = (uint32_t*)c.hcache.table.p;
    stride = c.hcache.cap;
    dslot = (const uint32_t*)B.slot->p;
    dmiss = (const uint32_t*)B.mlist->p;
    n_hash = miss.size();
  }
  int rc = launch_rlc(c, pks ? (const uint8_t*)B.pk->p : nullptr, (const uint8_t*)B.sig->p, (const uint32_t*)B.midx->p,
                      n, (const uint8_t*)B.msg->p, (const uint64_t*)B.off->p, n_msgs, seed, (int32_t*)B.st->p, s, call,
                      key_idx ? (const uint32_t*)B.kidx->p : nullptr, dH, stride, dslot, dmiss, n_hash);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(status, B.st->p, n * 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  return HIPBLS_OK;
}

int rlc_host(Context& c, const uint8_t* pks, const uint32_t* key_idx, const uint8_t* sigs, const uint32_t* msg_idx,
             uint64_t n, const uint8_t* msgs, const uint64_t* msg_offsets, uint64_t n_msgs, const rlc_seed& seed,
             int32_t* status, uint64_t call) {
  RlcBufs B{&c.b_pk, &c.b_kidx, &c.b_sig, &c.r_midx, &c.b_msg, &c.b_off, &c.b_st, &c.r_slot, &c.r_mlist};
  return rlc_host_on(c, B, c.stream, pks, key_idx, sigs, msg_idx, n, msgs, msg_offsets, n_msgs, seed, status, call);
}

// An RLC call over items [lo, hi) of a larger batch: the range's own message table (the messages its items use,
// renumbered in first-use order) and its own scalars (the seed's last word is mixed with the range start, so two
// ranges never share scalar streams).
int rlc_range(Context& c, const uint8_t* pks, const uint32_t* key_idx, const uint8_t* sigs, const uint32_t* msg_idx,
              uint64_t lo, uint64_t hi, const uint8_t* msgs, const uint64_t* msg_offsets, uint64_t n_msgs,
              const uint8_t* seed32, int32_t* status, uint64_t call, bool whole) {
  rlc_seed seed = parse_seed(seed32);
  if (whole)
    return rlc_host(c, pks, key_idx, sigs, msg_idx, hi - lo, msgs, msg_offsets, n_msgs, seed, status, call);
  seed.w[7] ^= (uint32_t)lo;
  seed.w[6] ^= (uint32_t)(lo >> 32);
  const uint64_t n = hi - lo;
  std::vector<uint32_t> lmidx(n), remap;
  std::unordered_map<uint32_t, uint32_t> sparse;
  const bool dense = n_msgs <= 4 * n + 1024;
  if (dense) remap.assign(n_msgs, UINT32_MAX);
  std::vector<uint32_t> used;
  for (uint64_t i = 0; i < n; ++i) {
    const uint32_t m = msg_idx[lo + i];
    uint32_t l;
    if (dense) {
      if (remap[m] == UINT32_MAX) {
        remap[m] = (uint32_t)used.size();
        used.push_back(m);
      }
      l = remap[m];
    } else {
      auto it = sparse.find(m);
      if (it == sparse.end()) {
        it = sparse.emplace(m, (uint32_t)used.size()).first;
        used.push_back(m);
      }
      l = it->second;
    }
    lmidx[i] = l;
  }
  std::vector<uint64_t> loff(used.size() + 1);
  uint64_t tot = 0;
  for (size_t k = 0; k < used.size(); ++k) {
    loff[k] = tot;
    tot += msg_offsets[used[k] + 1] - msg_offsets[used[k]];
  }
  loff[used.size()] = tot;
  std::vector<uint8_t> lmsg(tot ? tot : 1);
  for (size_t k = 0; k < used.size(); ++k)
    memcpy(lmsg.data() + loff[k], msgs + msg_offsets[used[k]], loff[k + 1] - loff[k]);
  return rlc_host(c, pks ? pks + 48 * lo : nullptr, key_idx ? key_idx + lo : nullptr, sigs + 96 * lo, lmidx.data(), n,
                  lmsg.data(), loff.data(), used.size(), seed, status + lo, call);
}

// ============================================================================ submission queue
// Coalesces concurrent single-item Verify calls (tbls.Verify from parsigex / validatorapi / sigagg goroutines,
// core/parsigex/parsigex.go:86-91, core/validatorapi/validatorapi.go:246-283) into batched launches.  Each context
// has its own queue; an item goes to the context its message hashes to, so the t partials of one signing root meet
// on one device.  A batch is launched as soon as the worker is free and work is pending: while one batch runs on
// the GPU, arrivals accumulate into the next, so the batch size follows the offered load.  An idle worker waits
// gather_us for company before launching a small batch.  The worker owns its stream and buffers; callers block only
// on their own batch's completion, never on a lock held across GPU work.
//
// Keyed path: when every key of a batch is in the resident pubshare table (and the batch has at
// least kQueueKeyedMin items or the H(m) cache is enabled), the batch runs as an
// RLC BatchVerify with keys by table index (no decode or subgroup test per call, herumi.go:286-289 does both every
// time) over the batch's DISTINCT messages, through the context's H(m) cache: a root shared by a validator's t
// partials or by a committee is hashed once, and once across batches while it stays cached.  Statuses are exactly
// the per-item Verify's (rlc.h).  Batches with a key outside the table take the wire-format Verify.
std::atomic<uint64_t> g_q_max_batch{65536};
// 50 us: what an idle worker waits for company before launching a small batch; callers arriving while a batch runs
// coalesce into the next one regardless (two batches in flight).  Serial callers (the parsigex loop: a running mean
// below 1.5 items per batch, VerifyQueue::batch_mean) skip it.
std::atomic<uint32_t> g_q_gather_us{50};
constexpr uint64_t kQueueKeyedMin = 8;  // without the H(m) cache, batches below this take the lane-pair Verify

// Copies a wire-format batch in and launches it on slot k; the status comes back into the slot's pinned buffer and
// done_ev marks completion (wire_finish collects it).  Nothing here waits for the GPU.
int wire_launch(Context& c, QSlot& k, VBatch& b) {
  const uint64_t n = b.n();
  HIP_TRY(k.d_pk.ensure(n * 48));
  HIP_TRY(k.d_sig.ensure(n * 96));
  HIP_TRY(k.d_msg.ensure(b.msg.size() ? b.msg.size() : 1));
  HIP_TRY(k.d_off.ensure((n + 1) * 8));
  HIP_TRY(k.d_st.ensure(n * 4));
  if (k.h_cap < n) {
    if (k.h_st) HIP_TRY(hipHostFree(k.h_st));
    k.h_st = nullptr;
    k.h_cap = 0;
    HIP_TRY(hipHostMalloc((void**)&k.h_st, n * 4, hipHostMallocDefault));
    k.h_cap = n;
  }
  HIP_TRY(hipMemcpyAsync(k.d_pk.p, b.pk.data(), n * 48, hipMemcpyHostToDevice, k.stream));
  HIP_TRY(hipMemcpyAsync(k.d_sig.p, b.sig.data(), n * 96, hipMemcpyHostToDevice, k.stream));
  if (b.msg.size()) HIP_TRY(hipMemcpyAsync(k.d_msg.p, b.msg.data(), b.msg.size(), hipMemcpyHostToDevice, k.stream));
  HIP_TRY(hipMemcpyAsync(k.d_off.p, b.off.data(), (n + 1) * 8, hipMemcpyHostToDevice, k.stream));
  int rc = launch_verify(c, (const uint8_t*)k.d_pk.p, (const uint8_t*)k.d_msg.p, (const uint64_t*)k.d_off.p,
                         (const uint8_t*)k.d_sig.p, n, (int32_t*)k.d_st.p, k.stream, k.d_ws);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(k.h_st, k.d_st.p, n * 4, hipMemcpyDeviceToHost, k.stream));
  HIP_TRY(hipEventRecord(k.done_ev, k.stream));
  return HIPBLS_OK;
}

int wire_finish(QSlot& k) {
  if (k.rc) return k.rc;
  HIP_TRY(hipEventSynchronize(k.done_ev));
  memcpy(k.b->status.data(), k.h_st, k.b->n() * 4);
  return HIPBLS_OK;
}

// The keyed path, under the context lock (the table, the H(m) cache and the RLC workspaces are the context's).
// Items are ordered by message so each message's partials are adjacent (one Miller loop per run per window).
int run_batch_keyed(Context& c, VBatch& b) {
  VerifyQueue& q = c.q;
  const uint64_t n = b.n();
  // distinct messages in first-use order
  std::unordered_map<std::string, uint32_t> pos;
  std::vector<uint32_t> mid(n);
  q.umsg.clear();
  q.uoff.assign(1, 0);
  for (uint64_t i = 0; i < n; ++i) {
    std::string key((const char*)b.msg.data() + b.off[i], b.off[i + 1] - b.off[i]);
    auto it = pos.find(key);
    if (it == pos.end()) {
      it = pos.emplace(std::move(key), (uint32_t)(q.uoff.size() - 1)).first;
      q.umsg.insert(q.umsg.end(), b.msg.begin() + b.off[i], b.msg.begin() + b.off[i + 1]);
      q.uoff.push_back(q.umsg.size());
    }
    mid[i] = it->second;
  }
  const uint64_t n_msgs = q.uoff.size() - 1;
  // counting sort by message
  std::vector<uint64_t> start(n_msgs + 1, 0);
  for (uint64_t i = 0; i < n; ++i) start[mid[i] + 1] += 1;
  for (uint64_t m = 0; m < n_msgs; ++m) start[m + 1] += start[m];
  q.order.resize(n);
  for (uint64_t i = 0; i < n; ++i) q.order[start[mid[i]]++] = (uint32_t)i;
  q.kidx.resize(n);
  q.midx.resize(n);
  q.sig_sorted.resize(n * 96);
  for (uint64_t j = 0; j < n; ++j) {
    const uint32_t i = q.order[j];
    q.kidx[j] = c.t_index.at(std::string((const char*)b.pk.data() + 48 * i, 48));
    q.midx[j] = mid[i];
    memcpy(q.sig_sorted.data() + 96 * j, b.sig.data() + 96 * i, 96);
  }
  q.st_sorted.resize(n);
  uint8_t seed32[32];  // the RLC scalars must be unpredictable to whoever made the signatures: kernel CSPRNG
  if (getrandom(seed32, sizeof seed32, 0) != (ssize_t)sizeof seed32) return arg_err("getrandom failed");
  const rlc_seed seed = parse_seed(seed32);
  RlcBufs B{&q.d_pk, &q.d_kidx, &q.d_sig, &q.d_midx, &q.d_msg, &q.d_off, &q.d_rlc_st, &q.d_slot, &q.d_mlist};
  const int rc = rlc_host_on(c, B, q.stream, nullptr, q.kidx.data(), q.sig_sorted.data(), q.midx.data(), n,
                             q.umsg.data(), q.uoff.data(), n_msgs, seed, q.st_sorted.data(),
                             g_call_seq.fetch_add(1) + 1);
  if (rc) return rc;
  for (uint64_t j = 0; j < n; ++j) b.status[q.order[j]] = q.st_sorted[j];
  return HIPBLS_OK;
}

// The keyed path when every key of the batch is in the table (run here, synchronously); otherwise false.
bool try_keyed(Context& c, VBatch& b, int& rc) {
  const uint64_t n = b.n();
  std::lock_guard<std::mutex> lk(c.mu);
  // small batches take the lower-latency lane-pair Verify, unless the caller enabled the H(m) cache
  bool keyed = c.t_size > 0 && (n >= kQueueKeyedMin || c.hcache.cap > 0);
  uint64_t miss_at = n;
  for (uint64_t i = 0; keyed && i < n; ++i) {
    keyed = c.t_index.count(std::string((const char*)b.pk.data() + 48 * i, 48)) != 0;
    if (!keyed) miss_at = i;
  }
  static const bool dbg = getenv("HIPBLS_DEBUG_QUEUE") != nullptr;
  if (dbg)
    fprintf(stderr, "[hipbls queue] ctx %d batch n=%llu keyed=%d t_size=%llu cap=%llu miss_at=%llu\n", c.slot,
            (unsigned long long)n, (int)keyed, (unsigned long long)c.t_size, (unsigned long long)c.hcache.cap,
            (unsigned long long)miss_at);
  if (!keyed) return false;
  c.q.keyed += 1;
  rc = run_batch_keyed(c, b);
  return true;
}

// Marks a batch finished (under q.mu) and drops its inputs: a ticket that is never waited then holds only its
// status word, not the batch's keys, signatures and messages.
void batch_done(VerifyQueue& q, VBatch& b, int rc) {
  b.rc = rc;
  b.done = true;
  std::vector<uint8_t>().swap(b.pk);
  std::vector<uint8_t>().swap(b.sig);
  std::vector<uint8_t>().swap(b.msg);
  std::vector<uint64_t>(1, 0).swap(b.off);
  q.batches += 1;
  q.cv_done.notify_all();
}

// The worker: up to kSlots wire batches in flight (the next one is copied in and launched while the previous one
// runs, on its own stream), keyed batches run synchronously on the queue's stream.  An idle worker (nothing in
// flight) waits gather_us for company before launching a small batch.
int size_class(uint64_t n) {
  int k = 0;
  while (n > 1 && k < 25) {
    n >>= 1;
    ++k;
  }
  return k;
}

void queue_worker(Context* cp) {
  Context& c = *cp;
  VerifyQueue& q = c.q;
  bool dev_ok = hipSetDevice(c.device) == hipSuccess && q.stream != nullptr;  // the device's queue stream
  // Both slots run on the queue's one stream: the next batch's copies and kernels are enqueued behind the running
  // batch (no host round trip between them), and the queue occupies one hardware queue.  Every hardware queue that
  // runs these kernels holds a scratch allocation sized for ~17 KB per lane over the whole device; with a stream per
  // slot, the context's streams and the queue's together spread over all four of HIP's hardware queues and the
  // runtime's scratch pool ran out under 64 concurrent callers (HSA_STATUS_ERROR_OUT_OF_RESOURCES on a lane-quad
  // dispatch).
  for (int k = 0; dev_ok && k < VerifyQueue::kSlots; ++k) {
    q.slot[k].stream = q.stream;
    dev_ok = hipEventCreateWithFlags(&q.slot[k].done_ev, hipEventDisableTiming) == hipSuccess;
  }
  std::unique_lock<std::mutex> lk(q.mu);
  for (;;) {
    const bool pending = !q.open.empty() && q.open.front()->n() > 0;
    if (pending && (int)q.inflight.size() < VerifyQueue::kSlots) {
      const uint64_t max_batch = g_q_max_batch.load();
      const uint32_t gather_us = g_q_gather_us.load();
      if (q.inflight.empty() && gather_us && q.open.front()->n() < max_batch && !q.stop && q.batch_mean >= 1.5) {
        const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(gather_us);
        q.cv_work.wait_until(lk, until, [&] { return q.stop || q.open.front()->n() >= max_batch; });
      }
      std::shared_ptr<VBatch> b = q.open.front();
      q.open.pop_front();
      q.items += b->n();
      q.batch_mean = 0.75 * q.batch_mean + 0.25 * (double)b->n();
      lk.unlock();
      b->status.assign(b->n(), HIPBLS_ERR_DEVICE);
      int rc = HIPBLS_ERR_DEVICE;
      if (dev_ok && try_keyed(c, *b, rc)) {
        lk.lock();
        batch_done(q, *b, rc);
        continue;
      }
      int k = 0;
      while (q.slot[k].b) ++k;  // a free slot (inflight.size() < kSlots); only this thread touches slots
      QSlot& sl = q.slot[k];
      sl.b = b;
      sl.rc = dev_ok ? wire_launch(c, sl, *b) : HIPBLS_ERR_DEVICE;
      sl.launched = std::chrono::steady_clock::now();
      // A launch that failed after its first copy was queued never records done_ev, and batch_done frees the batch's
      // host vectors as soon as it is collected: drain the stream first so no queued copy reads freed memory.
      if (sl.rc != HIPBLS_OK && dev_ok) (void)hipStreamSynchronize(sl.stream);
      lk.lock();
      if (!q.inflight.empty()) q.overlapped += 1;
      q.inflight.push_back(k);
      continue;
    }
    if (!q.inflight.empty()) {  // collect the oldest batch in flight
      const int k = q.inflight.front();
      QSlot& sl = q.slot[k];
      q.wakeups += 1;
      const bool ready = sl.rc != HIPBLS_OK || hipEventQuery(sl.done_ev) != hipErrorNotReady;
      if (!ready && (int)q.inflight.size() < VerifyQueue::kSlots) {
        // A slot is free: wait for new work or the batch, whichever comes first (arrivals launch at once).  The
        // completion is polled every 20 us, but only from 85 % of the running estimate of a batch's time on: a
        // 12 ms n = 1 batch costs ~100 wakeups instead of ~600, at the same completion latency.
        const auto now = std::chrono::steady_clock::now();
        const auto due = sl.launched + std::chrono::microseconds((int64_t)(0.85 * q.batch_us[size_class(sl.b->n())]));
        const auto until = due > now + std::chrono::microseconds(20) ? due : now + std::chrono::microseconds(20);
        q.cv_work.wait_until(lk, until, [&] { return q.stop || (!q.open.empty() && q.open.front()->n() > 0); });
        continue;
      }
      if (sl.rc == HIPBLS_OK) {
        const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - sl.launched).count();
        double& e = q.batch_us[size_class(sl.b->n())];
        // The estimate follows a faster batch of the class at once and drifts up slowly: a measured time includes the
        // slack of a poll deferred past the batch's real end, so an average of those kept serial n = 1 callers late
        // for many batches after a change to a faster layout, fewer replicas or a race won early.
        e = (e <= 0 || us < e) ? us : e + 0.05 * (us - e);
      }
      lk.unlock();
      const int rc = wire_finish(sl);
      lk.lock();
      q.inflight.pop_front();
      // the next batch queued behind this one on the stream starts now: its estimate runs from here
      if (!q.inflight.empty()) {
        QSlot& nx = q.slot[q.inflight.front()];
        nx.launched = std::max(nx.launched, std::chrono::steady_clock::now());
      }
      std::shared_ptr<VBatch> b = std::move(sl.b);
      sl.b.reset();
      batch_done(q, *b, rc);
      continue;
    }
    if (q.stop) break;  // nothing pending, nothing in flight
    q.cv_work.wait(lk, [&] { return q.stop || (!q.open.empty() && q.open.front()->n() > 0); });
  }
}

void queue_shutdown() {
  const int n = nctx();
  for (int k = 0; k < n; ++k) {
    VerifyQueue& q = ctx(k).q;
    {
      std::lock_guard<std::mutex> lk(q.mu);
      if (!q.started) continue;
      q.stop = true;
    }
    q.cv_work.notify_all();
    if (q.worker.joinable()) q.worker.join();
    std::lock_guard<std::mutex> lk(q.mu);
    q.started = false;
    q.stop = false;
  }
}

uint32_t msg_hash(const uint8_t* msg, uint64_t len) {  // FNV-1a: the queue a message goes to
  uint32_t h = 2166136261u;
  for (uint64_t i = 0; i < len; ++i) h = (h ^ msg[i]) * 16777619u;
  return h;
}

int queue_submit(const uint8_t* pk48, const uint8_t* msg, uint64_t msg_len, const uint8_t* sig96, uint64_t* ticket) {
  if (!pk48 || !sig96 || !ticket || (msg_len && !msg) || msg_len > 0xffffffffull) return arg_err("bad verify arguments");
  ENSURE_INIT();
  const int n = nctx();
  Context& c = ctx(n == 1 ? 0 : (int)(msg_hash(msg, msg_len) % (uint32_t)n));
  int rc = bind(c);
  if (rc) return rc;
  VerifyQueue& q = c.q;
  std::lock_guard<std::mutex> lk(q.mu);
  if (!q.started) {
    q.worker = std::thread(queue_worker, &c);
    q.started = true;
    static std::once_flag hooked;
    std::call_once(hooked, [] { atexit(queue_shutdown); });  // drain in-flight batches before HIP tears down
  }
  const uint64_t max_batch = g_q_max_batch.load();
  if (q.open.empty() || q.open.back()->n() >= max_batch) q.open.push_back(std::make_shared<VBatch>());
  VBatch& b = *q.open.back();
  const uint32_t idx = (uint32_t)b.n();
  b.pk.insert(b.pk.end(), pk48, pk48 + 48);
  b.sig.insert(b.sig.end(), sig96, sig96 + 96);
  if (msg_len) b.msg.insert(b.msg.end(), msg, msg + msg_len);
  b.off.push_back(b.msg.size());
  const uint64_t t = q.next_ticket++ * kMaxContexts + (uint64_t)c.slot;  // the ticket names its queue
  q.tickets.emplace(t, std::make_pair(q.open.back(), idx));
  *ticket = t;
  q.cv_work.notify_one();
  return HIPBLS_OK;
}

int queue_wait(uint64_t ticket, int32_t* status) {
  if (!status) return arg_err("null status");
  const int n = nctx();
  const int k = (int)(ticket % kMaxContexts);
  if (k >= n) return arg_err("unknown verify ticket");
  VerifyQueue& q = ctx(k).q;
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

// ============================================================================ host-buffer bodies (one context)
int verify_host(Context& c, const uint8_t* pks, const uint8_t* msgs, const uint64_t* offs, const uint8_t* sigs,
                uint64_t n, int32_t* status) {
  const uint64_t msg_total = offs[n];
  HIP_TRY(c.b_pk.ensure(n * 48));
  HIP_TRY(c.b_sig.ensure(n * 96));
  HIP_TRY(c.b_msg.ensure(msg_total ? msg_total : 1));
  HIP_TRY(c.b_off.ensure((n + 1) * 8));
  HIP_TRY(c.b_st.ensure(n * 4));
  HIP_TRY(hipMemcpyAsync(c.b_pk.p, pks, n * 48, hipMemcpyHostToDevice, c.stream));
  HIP_TRY(hipMemcpyAsync(c.b_sig.p, sigs, n * 96, hipMemcpyHostToDevice, c.stream));
  if (msg_total) HIP_TRY(hipMemcpyAsync(c.b_msg.p, msgs, msg_total, hipMemcpyHostToDevice, c.stream));
  HIP_TRY(hipMemcpyAsync(c.b_off.p, offs, (n + 1) * 8, hipMemcpyHostToDevice, c.stream));
  int rc = ws_begin(c, c.stream);
  if (rc) return rc;
  rc = launch_verify(c, (const uint8_t*)c.b_pk.p, (const uint8_t*)c.b_msg.p, (const uint64_t*)c.b_off.p,
                     (const uint8_t*)c.b_sig.p, n, (int32_t*)c.b_st.p, c.stream, c.v_ws);
  if (rc) return rc;
  rc = ws_end(c, c.stream);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(status, c.b_st.p, n * 4, hipMemcpyDeviceToHost, c.stream));
  HIP_TRY(hipStreamSynchronize(c.stream));
  return HIPBLS_OK;
}

int signed_data_host(Context& c, const uint8_t* pks, const uint8_t* object_roots, const uint8_t* domains,
                     const uint8_t* sigs, uint64_t n, int32_t* status) {
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
  int rc = ws_begin(c, c.stream);
  if (rc) return rc;
  rc = launch_verify(c, (const uint8_t*)c.b_pk.p, (const uint8_t*)c.b_msg.p, (const uint64_t*)c.b_off.p,
                     (const uint8_t*)c.b_sig.p, n, (int32_t*)c.b_st.p, c.stream, c.v_ws);
  if (rc) return rc;
  rc = ws_end(c, c.stream);
  if (rc) return rc;
  hipLaunchKernelGGL(k_zero_sig_status, dim3((unsigned)grid_for(n)), dim3(kBlock), 0, c.stream,
                     (const uint8_t*)c.b_sig.p, n, (int32_t*)c.b_st.p);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(status, c.b_st.p, n * 4, hipMemcpyDeviceToHost, c.stream));
  HIP_TRY(hipStreamSynchronize(c.stream));
  return HIPBLS_OK;
}

int tagg_host(Context& c, const uint8_t* sigs, const int64_t* share_idx, const uint64_t* goffs, uint64_t n_groups,
              uint8_t* out_sigs, int32_t* status) {
  const uint64_t n_parts = goffs[n_groups];
  HIP_TRY(c.b_sig.ensure((n_parts ? n_parts : 1) * 96));
  HIP_TRY(c.b_ids.ensure((n_parts ? n_parts : 1) * 8));
  HIP_TRY(c.b_off.ensure((n_groups + 1) * 8));
  HIP_TRY(c.b_out.ensure(n_groups * 96));
  HIP_TRY(c.b_st.ensure(n_groups * 4));
  if (n_parts) {
    HIP_TRY(hipMemcpyAsync(c.b_sig.p, sigs, n_parts * 96, hipMemcpyHostToDevice, c.stream));
    HIP_TRY(hipMemcpyAsync(c.b_ids.p, share_idx, n_parts * 8, hipMemcpyHostToDevice, c.stream));
  }
  HIP_TRY(hipMemcpyAsync(c.b_off.p, goffs, (n_groups + 1) * 8, hipMemcpyHostToDevice, c.stream));
  int rc = launch_tagg(c, (const uint8_t*)c.b_sig.p, (const int64_t*)c.b_ids.p, (const uint64_t*)c.b_off.p, n_groups,
                       n_parts, (uint8_t*)c.b_out.p, (int32_t*)c.b_st.p, c.stream);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(out_sigs, c.b_out.p, n_groups * 96, hipMemcpyDeviceToHost, c.stream));
  HIP_TRY(hipMemcpyAsync(status, c.b_st.p, n_groups * 4, hipMemcpyDeviceToHost, c.stream));
  HIP_TRY(hipStreamSynchronize(c.stream));
  return HIPBLS_OK;
}

// Called WITHOUT the context lock (run_ranges_unlocked): it takes a host slot for the whole call and the context lock
// only to enqueue (copies in, the sigagg kernels, copies out into the slot's pinned buffers), then waits for the slot's
// completion event with no lock held.
int tagg_verify_host(Context& c, const uint8_t* sigs, const int64_t* share_idx, const uint64_t* goffs,
                     uint64_t n_groups, const uint8_t* dv_pks, const uint8_t* msgs, const uint64_t* moffs,
                     uint8_t* out_sigs, int32_t* agg_status, int32_t* verify_status) {
  const uint64_t n_parts = goffs[n_groups];
  const uint64_t msg_total = moffs[n_groups];
  const int p = (int)(c.tvh_seq.fetch_add(1) & 1);
  Context::TvHostSlot& h = c.tvh[p];
  std::lock_guard<std::mutex> slot_lock(h.mu);
  // The slot's pinned result buffers grow under the slot lock only, not the context lock: hipHostFree may wait for
  // the device, and the other slot's call must keep enqueueing meanwhile.  This slot's previous call has
  // completed (its event was waited on before the slot lock was released).
  if (h.h_groups < n_groups) {
    if (h.h_out) HIP_TRY(hipHostFree(h.h_out));
    if (h.h_st) HIP_TRY(hipHostFree(h.h_st));
    h.h_out = nullptr;
    h.h_st = nullptr;
    h.h_groups = 0;
    HIP_TRY(hipHostMalloc((void**)&h.h_out, n_groups * 96, hipHostMallocDefault));
    HIP_TRY(hipHostMalloc((void**)&h.h_st, n_groups * 8, hipHostMallocDefault));
    h.h_groups = n_groups;
  }
  {
    std::lock_guard<std::mutex> lk(c.mu);
    const hipStream_t s = c.sub[p];
    // Every early return below drains the slot's stream: nothing this call enqueued may still read the caller's host
    // arrays once it returns (a failing copy after the first one used to return without a wait).
    struct Drain {
      hipStream_t s;
      bool on;
      ~Drain() {
        if (on) (void)hipStreamSynchronize(s);
      }
    } drain{s, true};
    if (!h.done) HIP_TRY(hipEventCreateWithFlags(&h.done, hipEventDisableTiming));
    HIP_TRY(h.sig.ensure((n_parts ? n_parts : 1) * 96));
    HIP_TRY(h.ids.ensure((n_parts ? n_parts : 1) * 8));
    HIP_TRY(h.off.ensure((n_groups + 1) * 8));
    HIP_TRY(h.pk.ensure(n_groups * 48));
    HIP_TRY(h.msg.ensure(msg_total ? msg_total : 1));
    HIP_TRY(h.moff.ensure((n_groups + 1) * 8));
    HIP_TRY(h.out.ensure(n_groups * 96));
    HIP_TRY(h.st.ensure(n_groups * 8));  // aggregate statuses, then verify statuses
    if (n_parts) {
      HIP_TRY(hipMemcpyAsync(h.sig.p, sigs, n_parts * 96, hipMemcpyHostToDevice, s));
      HIP_TRY(hipMemcpyAsync(h.ids.p, share_idx, n_parts * 8, hipMemcpyHostToDevice, s));
    }
    HIP_TRY(hipMemcpyAsync(h.off.p, goffs, (n_groups + 1) * 8, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(h.pk.p, dv_pks, n_groups * 48, hipMemcpyHostToDevice, s));
    if (msg_total) HIP_TRY(hipMemcpyAsync(h.msg.p, msgs, msg_total, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(h.moff.p, moffs, (n_groups + 1) * 8, hipMemcpyHostToDevice, s));
    int32_t* ast = (int32_t*)h.st.p;
    int32_t* vst = ast + n_groups;
    const int rc = launch_tagg_verify(c, (const uint8_t*)h.sig.p, (const int64_t*)h.ids.p, (const uint64_t*)h.off.p,
                                      n_groups, n_parts, (const uint8_t*)h.pk.p, (const uint8_t*)h.msg.p,
                                      (const uint64_t*)h.moff.p, (uint8_t*)h.out.p, ast, vst, s);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(h.h_out, h.out.p, n_groups * 96, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(h.h_st, h.st.p, n_groups * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipEventRecord(h.done, s));
    drain.on = false;  // the wait below (no lock held) covers the enqueued work
  }
  HIP_TRY(hipEventSynchronize(h.done));
  memcpy(out_sigs, h.h_out, n_groups * 96);
  memcpy(agg_status, h.h_st, n_groups * 4);
  memcpy(verify_status, h.h_st + n_groups, n_groups * 4);
  return HIPBLS_OK;
}

int sign_host(Context& c, const uint8_t* sks, const uint8_t* msgs, const uint64_t* offs, uint64_t n, uint8_t* out_sigs,
              int32_t* status) {
  const uint64_t msg_total = offs[n];
  HIP_TRY(c.b_pk.ensure(n * 32));
  HIP_TRY(c.b_msg.ensure(msg_total ? msg_total : 1));
  HIP_TRY(c.b_off.ensure((n + 1) * 8));
  HIP_TRY(c.b_out.ensure(n * 96));
  HIP_TRY(c.b_st.ensure(n * 4));
  HIP_TRY(hipMemcpyAsync(c.b_pk.p, sks, n * 32, hipMemcpyHostToDevice, c.stream));
  if (msg_total) HIP_TRY(hipMemcpyAsync(c.b_msg.p, msgs, msg_total, hipMemcpyHostToDevice, c.stream));
  HIP_TRY(hipMemcpyAsync(c.b_off.p, offs, (n + 1) * 8, hipMemcpyHostToDevice, c.stream));
  hipLaunchKernelGGL(k_sign, dim3((unsigned)grid_for(n)), dim3(kBlock), 0, c.stream, (const uint8_t*)c.b_pk.p,
                     (const uint8_t*)c.b_msg.p, (const uint64_t*)c.b_off.p, n, (uint8_t*)c.b_out.p,
                     (int32_t*)c.b_st.p);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(out_sigs, c.b_out.p, n * 96, hipMemcpyDeviceToHost, c.stream));
  HIP_TRY(hipMemcpyAsync(status, c.b_st.p, n * 4, hipMemcpyDeviceToHost, c.stream));
  HIP_TRY(hipStreamSynchronize(c.stream));
  return HIPBLS_OK;
}

int sk_to_pk_host(Context& c, const uint8_t* sks, uint64_t n, uint8_t* out_pks, int32_t* status) {
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

int fav_host(Context& c, const uint8_t* pks, const uint64_t* koffs, uint64_t n_groups, const uint8_t* sigs,
             const uint8_t* msgs, const uint64_t* moffs, int32_t* status) {
  const uint64_t nkeys = koffs[n_groups], msg_total = moffs[n_groups];
  HIP_TRY(c.b_pk.ensure((nkeys ? nkeys : 1) * 48));
  HIP_TRY(c.b_ids.ensure((n_groups + 1) * 8));
  HIP_TRY(c.b_sig.ensure(n_groups * 96));
  HIP_TRY(c.b_msg.ensure(msg_total ? msg_total : 1));
  HIP_TRY(c.b_off.ensure((n_groups + 1) * 8));
  HIP_TRY(c.b_st.ensure(n_groups * 4));
  if (nkeys) HIP_TRY(hipMemcpyAsync(c.b_pk.p, pks, nkeys * 48, hipMemcpyHostToDevice, c.stream));
  HIP_TRY(hipMemcpyAsync(c.b_ids.p, koffs, (n_groups + 1) * 8, hipMemcpyHostToDevice, c.stream));
  HIP_TRY(hipMemcpyAsync(c.b_sig.p, sigs, n_groups * 96, hipMemcpyHostToDevice, c.stream));
  if (msg_total) HIP_TRY(hipMemcpyAsync(c.b_msg.p, msgs, msg_total, hipMemcpyHostToDevice, c.stream));
  HIP_TRY(hipMemcpyAsync(c.b_off.p, moffs, (n_groups + 1) * 8, hipMemcpyHostToDevice, c.stream));
  int rc = launch_fav(c, (const uint8_t*)c.b_pk.p, nkeys, (const uint64_t*)c.b_ids.p, n_groups,
                      (const uint8_t*)c.b_sig.p, (const uint8_t*)c.b_msg.p, (const uint64_t*)c.b_off.p,
                      (int32_t*)c.b_st.p, c.stream);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(status, c.b_st.p, n_groups * 4, hipMemcpyDeviceToHost, c.stream));
  HIP_TRY(hipStreamSynchronize(c.stream));
  return HIPBLS_OK;
}

int aggregate_host(Context& c, const uint8_t* sigs, uint64_t n, uint8_t* out_sig, int32_t* status) {
  HIP_TRY(c.b_sig.ensure((n ? n : 1) * 96));
  HIP_TRY(c.b_out.ensure(96));
  HIP_TRY(c.b_st.ensure(4));
  if (n) HIP_TRY(hipMemcpyAsync(c.b_sig.p, sigs, n * 96, hipMemcpyHostToDevice, c.stream));
  int rc = launch_aggregate(c, (const uint8_t*)c.b_sig.p, n, (uint8_t*)c.b_out.p, (int32_t*)c.b_st.p, c.stream);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(out_sig, c.b_out.p, 96, hipMemcpyDeviceToHost, c.stream));
  HIP_TRY(hipMemcpyAsync(status, c.b_st.p, 4, hipMemcpyDeviceToHost, c.stream));
  HIP_TRY(hipStreamSynchronize(c.stream));
  return HIPBLS_OK;
}

int verify_keys_host(Context& c, const uint32_t* key_idx, const uint8_t* msgs, const uint64_t* offs,
                     const uint8_t* sigs, uint64_t n, int32_t* status) {
  const uint64_t msg_total = offs[n];
  HIP_TRY(c.b_kidx.ensure(n * 4));
  HIP_TRY(c.b_sig.ensure(n * 96));
  HIP_TRY(c.b_msg.ensure(msg_total ? msg_total : 1));
  HIP_TRY(c.b_off.ensure((n + 1) * 8));
  HIP_TRY(c.b_st.ensure(n * 4));
  HIP_TRY(hipMemcpyAsync(c.b_kidx.p, key_idx, n * 4, hipMemcpyHostToDevice, c.stream));
  HIP_TRY(hipMemcpyAsync(c.b_sig.p, sigs, n * 96, hipMemcpyHostToDevice, c.stream));
  if (msg_total) HIP_TRY(hipMemcpyAsync(c.b_msg.p, msgs, msg_total, hipMemcpyHostToDevice, c.stream));
  HIP_TRY(hipMemcpyAsync(c.b_off.p, offs, (n + 1) * 8, hipMemcpyHostToDevice, c.stream));
  int rc = timed(c, "verify_keys", c.stream, [&] {
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

int table_load_host(Context& c, const uint8_t* pks, uint64_t n, int32_t* status) {
  HIP_TRY(hipDeviceSynchronize());  // no call may still read the old table
  c.t_size = 0;
  c.t_index.clear();
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
  c.t_index.reserve(n);
  for (uint64_t k = 0; k < n; ++k) c.t_index.emplace(std::string((const char*)pks + 48 * k, 48), (uint32_t)k);
  return HIPBLS_OK;
}

// herumi's Deserialize of n points (kind 1: 48-byte G1 public keys, kind 2: 96-byte G2 signatures): decode, on-curve
// and subgroup checks; status[i] = OK, or ERR_PUBKEY / ERR_SIGNATURE.
int deserialize_host(Context& c, const uint8_t* data, uint64_t n, int kind, int32_t* status) {
  const uint64_t w = kind == 1 ? 48 : 96;
  HIP_TRY(c.b_sig.ensure(n * w));
  HIP_TRY(c.b_pts.ensure(n * (w / 2) * 4));
  HIP_TRY(c.b_pst.ensure(n * 4));
  HIP_TRY(hipMemcpyAsync(c.b_sig.p, data, n * w, hipMemcpyHostToDevice, c.stream));
  int rc = ws_begin(c, c.stream);
  if (rc) return rc;
  if (kind == 1)
    hipLaunchKernelGGL(k_g1_decode, dim3((unsigned)grid_for(n)), dim3(kBlock), 0, c.stream, (const uint8_t*)c.b_sig.p,
                       n, (uint32_t*)c.b_pts.p, (int32_t*)c.b_pst.p);
  else
    hipLaunchKernelGGL(k_g2_decode, dim3((unsigned)grid_for(n)), dim3(kBlock), 0, c.stream, (const uint8_t*)c.b_sig.p,
                       n, (uint32_t*)c.b_pts.p, (int32_t*)c.b_pst.p);
  HIP_TRY(hipGetLastError());
  rc = ws_end(c, c.stream);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(status, c.b_pst.p, n * 4, hipMemcpyDeviceToHost, c.stream));
  HIP_TRY(hipStreamSynchronize(c.stream));
  const int32_t bad = kind == 1 ? HIPBLS_ERR_PUBKEY : HIPBLS_ERR_SIGNATURE;
  for (uint64_t i = 0; i < n; ++i) status[i] = status[i] == DEC_BAD ? bad : HIPBLS_OK;
  return HIPBLS_OK;
}

// Minimum units per range before a batch is split across devices (each range must still fill a GPU's SIMDs for a
// while; below this the call stays on one device and concurrent calls spread round robin).
constexpr uint64_t kSplitVerify = 4096;   // Verify items
constexpr uint64_t kSplitRlc = 16384;     // RLC items
constexpr uint64_t kSplitGroups = 1024;   // ThresholdAggregate groups
constexpr uint64_t kSplitSign = 4096;     // Sign / SecretToPublicKey items
constexpr uint64_t kSplitFav = 64;        // FastAggregateVerify groups
constexpr uint64_t kSplitAgg = 1 << 16;   // Aggregate signatures

}  // namespace

// ============================================================================ C-ABI
extern "C" {

int hipbls_abi_version(void) { return HIPBLS_ABI_VERSION; }

int hipbls_init_devices(const int32_t* ids, uint32_t n) {
  if (!ids || n == 0 || n > (uint32_t)kMaxContexts) return arg_err("device list empty or longer than 64");
  std::lock_guard<std::mutex> lk(g_init_mu);
  const int have = nctx();
  if (have) {
    bool same = have == (int)n;
    for (int k = 0; same && k < have; ++k) same = ctx(k).device == ids[k];
    if (!same) return arg_err("hipbls already bound to another device list");
    HIP_TRY(hipSetDevice(ctx(0).device));
    return HIPBLS_OK;
  }
  return init_locked(std::vector<int>(ids, ids + n));
}

int hipbls_init(int device) {
  {
    std::lock_guard<std::mutex> lk(g_init_mu);
    if (device < 0 && nctx()) {
      HIP_TRY(hipSetDevice(ctx(0).device));
      return HIPBLS_OK;
    }
  }
  const int32_t d = device < 0 ? 0 : device;
  return hipbls_init_devices(&d, 1);
}

int hipbls_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int hipbls_current_device(void) { return nctx() ? ctx(0).device : -1; }

int hipbls_device_streams(int device) {
  if (!nctx()) return 0;
  auto it = g_streams_per_device.find(device);
  return it == g_streams_per_device.end() ? 0 : it->second;
}

int hipbls_scratch_budget(int device, uint64_t* per_lane, uint64_t* per_queue, uint64_t* limit, uint32_t* queues) {
  if (!per_lane || !per_queue || !limit || !queues) return arg_err("null output");
  if (!nctx()) return arg_err("no context on that device");
  auto it = g_scratch.find(device);
  if (it == g_scratch.end()) return arg_err("no context on that device");
  *per_lane = it->second.per_lane;
  *per_queue = it->second.per_queue;
  *limit = it->second.limit;
  *queues = it->second.queues;
  return HIPBLS_OK;
}

int hipbls_stream_joins(uint64_t* calls) {
  if (!calls) return arg_err("null output");
  *calls = 0;
  const int n = nctx();
  for (int k = 0; k < n; ++k) {
    std::lock_guard<std::mutex> lk(ctx(k).mu);
    *calls += ctx(k).joined;
  }
  return HIPBLS_OK;
}

const char* hipbls_kernel_names(void) {
  static const std::string names = kernel_names();
  return names.c_str();
}

int hipbls_queue_worker_stats(uint64_t* wakeups, uint64_t* batches) {
  if (!wakeups || !batches) return arg_err("null output");
  *wakeups = *batches = 0;
  const int n = nctx();
  for (int k = 0; k < n; ++k) {
    VerifyQueue& q = ctx(k).q;
    std::lock_guard<std::mutex> lk(q.mu);
    *wakeups += q.wakeups;
    *batches += q.batches;
  }
  return HIPBLS_OK;
}

int hipbls_device_slots(int32_t* ids, uint32_t cap) {
  const int n = nctx();
  for (int k = 0; k < n && ids && (uint32_t)k < cap; ++k) ids[k] = ctx(k).device;
  return n;
}

int hipbls_plan_ranges(uint64_t n, uint32_t parts, const uint32_t* run_keys, uint64_t* bounds) {
  if (!bounds || parts == 0) return arg_err("bad plan arguments");
  const std::vector<uint64_t> b = plan_ranges(n, parts, run_keys);
  for (uint32_t k = 0; k <= parts; ++k) bounds[k] = k < b.size() ? b[k] : n;
  return HIPBLS_OK;
}

const char* hipbls_last_error(void) { return g_last_error.c_str(); }

// Build identity (charon_amd/build.py source_digest / flags_digest): a marker string the build script and the test,
// smoke and bench entry points read from the .so's bytes and compare with the shipped sources.
#ifndef HIPBLS_SRC_SHA
#define HIPBLS_SRC_SHA "none"
#endif
#ifndef HIPBLS_FLAGS_SHA
#define HIPBLS_FLAGS_SHA "none"
#endif
extern "C" __attribute__((used, visibility("default"))) const char hipbls_build_id_mark[] =
    "HIPBLS_BUILD_ID src=" HIPBLS_SRC_SHA " flags=" HIPBLS_FLAGS_SHA;
const char* hipbls_build_id(void) { return hipbls_build_id_mark + sizeof("HIPBLS_BUILD_ID ") - 1; }

int hipbls_set_timing(int enabled) {
  g_timing = enabled != 0;
  return HIPBLS_OK;
}

int hipbls_rlc_set_g1_msm_min(uint32_t min) { return (int)g_g1m_min.exchange(min); }

int hipbls_rlc_set_mode(int mode) {
  if (mode != HIPBLS_RLC_AUTO && mode != HIPBLS_RLC_WINDOWS && mode != HIPBLS_RLC_BATCH)
    return arg_err("unknown RLC mode");
  return g_rlc_mode.exchange(mode);
}

int hipbls_rlc_batch_stats(uint64_t* attempted, uint64_t* passed, int32_t* last) {
  if (!attempted || !passed || !last) return arg_err("null output");
  ENSURE_INIT();
  uint64_t a = 0, p = 0, newest = 0;
  const int n = nctx();
  for (int k = 0; k < n; ++k) {
    Context& c = ctx(k);
    ENTER_CTX(c);
    const int rc = rlcb_poll(c, -1, true);
    if (rc) return rc;
    a += c.rlcb_attempted;
    p += c.rlcb_passed;
    if (c.rlcb_last >= 0 && c.rlcb_last_call > newest) newest = c.rlcb_last_call;
  }
  // the newest call's verdict: failed if the check of any of its ranges failed
  int lst = -1;
  for (int k = 0; k < n; ++k) {
    Context& c = ctx(k);
    std::lock_guard<std::mutex> lk(c.mu);
    if (c.rlcb_last >= 0 && c.rlcb_last_call == newest) lst = lst < 0 ? c.rlcb_last : (lst & c.rlcb_last);
  }
  *attempted = a;
  *passed = p;
  *last = lst;
  return HIPBLS_OK;
}

int hipbls_set_latency_replicas(uint32_t replicas) {
  if (replicas < 1 || replicas > 32) return arg_err("latency replicas out of range (1-32)");
  return (int)g_lat_replicas.exchange(replicas);
}

int hipbls_set_pair_mode(int mode) {
  if (mode != HIPBLS_PAIR_AUTO && mode != HIPBLS_PAIR_SINGLE && mode != HIPBLS_PAIR_LANES && mode != HIPBLS_PAIR_QUADS &&
      mode != HIPBLS_PAIR_OCTETS)
    return arg_err("unknown pair mode");
  return g_pair_mode.exchange(mode);
}

int hipbls_verify_batch(const uint8_t* pks, const uint8_t* msgs, const uint64_t* msg_offsets, const uint8_t* sigs,
                        uint64_t n, int32_t* status) {
  if (n == 0) return HIPBLS_OK;
  if (!pks || !msg_offsets || !sigs || !status || mul_overflows(n, 96)) return arg_err("bad verify arguments");
  if (!offsets_ok(msg_offsets, n)) return arg_err("bad message offsets");
  if (msg_offsets[n] && !msgs) return arg_err("null messages");
  ENSURE_INIT();
  return run_ranges(plan_ranges(n, parts_for(n, kSplitVerify), nullptr), [&](Context& c, uint64_t lo, uint64_t hi) {
    std::vector<uint64_t> tmp;
    const uint64_t* offs = rebase(msg_offsets, lo, hi, tmp);
    return verify_host(c, pks + 48 * lo, msgs ? msgs + msg_offsets[lo] : msgs, offs, sigs + 96 * lo, hi - lo,
                       status + lo);
  });
}

int hipbls_verify_batch_device(const uint8_t* d_pks, const uint8_t* d_msgs, const uint64_t* d_msg_offsets,
                               const uint8_t* d_sigs, uint64_t n, int32_t* d_status, void* stream) {
  ENSURE_INIT();
  Context& c = ctx_of(d_status);
  ENTER_CTX(c);
  ON_STREAM(c, stream, s);
  int rc = ws_begin(c, s);
  if (rc) return rc;
  rc = launch_verify(c, d_pks, d_msgs, d_msg_offsets, d_sigs, n, d_status, s, c.v_ws);
  if (rc) return rc;
  return ws_end(c, s);
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
  g_q_max_batch = max_batch;
  g_q_gather_us = gather_us;
  return HIPBLS_OK;
}

int hipbls_queue_stats(uint64_t* batches, uint64_t* items) {
  if (!batches || !items) return arg_err("null output");
  *batches = 0;
  *items = 0;
  const int n = nctx();
  for (int k = 0; k < n; ++k) {
    VerifyQueue& q = ctx(k).q;
    std::lock_guard<std::mutex> lk(q.mu);
    *batches += q.batches;
    *items += q.items;
  }
  return HIPBLS_OK;
}

int hipbls_deserialize_status(const uint8_t* data, uint64_t n, int32_t kind, int32_t* status) {
  if (n == 0) return HIPBLS_OK;
  if (!data || !status || (kind != 1 && kind != 2) || mul_overflows(n, 192)) return arg_err("bad deserialize arguments");
  ENSURE_INIT();
  const uint64_t w = kind == 1 ? 48 : 96;
  return run_ranges(plan_ranges(n, parts_for(n, kSplitSign), nullptr), [&](Context& c, uint64_t lo, uint64_t hi) {
    return deserialize_host(c, data + w * lo, hi - lo, kind, status + lo);
  });
}

int hipbls_queue_keyed_batches(uint64_t* batches) {
  if (!batches) return arg_err("null output");
  *batches = 0;
  const int n = nctx();
  for (int k = 0; k < n; ++k) {
    Context& c = ctx(k);
    std::lock_guard<std::mutex> lk(c.mu);
    *batches += c.q.keyed;
  }
  return HIPBLS_OK;
}

int hipbls_verify_signed_data_batch(const uint8_t* pks, const uint8_t* object_roots, const uint8_t* domains,
                                    const uint8_t* sigs, uint64_t n, int32_t* status) {
  if (n == 0) return HIPBLS_OK;
  if (!pks || !object_roots || !domains || !sigs || !status || mul_overflows(n, 96)) return arg_err("bad arguments");
  ENSURE_INIT();
  return run_ranges(plan_ranges(n, parts_for(n, kSplitVerify), nullptr), [&](Context& c, uint64_t lo, uint64_t hi) {
    return signed_data_host(c, pks + 48 * lo, object_roots + 32 * lo, domains + 32 * lo, sigs + 96 * lo, hi - lo,
                            status + lo);
  });
}

// Group ranges: whole groups per device; partial offsets rebased to the range's first partial.
int hipbls_threshold_aggregate_batch(const uint8_t* sigs, const int64_t* share_idx, const uint64_t* group_offsets,
                                     uint64_t n_groups, uint8_t* out_sigs, int32_t* status) {
  if (n_groups == 0) return HIPBLS_OK;
  if (!group_offsets || !out_sigs || !status || mul_overflows(n_groups, 96)) return arg_err("bad arguments");
  if (!groups_ok(group_offsets, n_groups)) return arg_err("bad group offsets");
  const uint64_t n_parts = group_offsets[n_groups];
  if (n_parts && (!sigs || !share_idx)) return arg_err("null partials");
  if (mul_overflows(n_parts, 288)) return arg_err("too many partials");
  ENSURE_INIT();
  return run_ranges(plan_ranges(n_groups, parts_for(n_groups, kSplitGroups), nullptr),
                    [&](Context& c, uint64_t lo, uint64_t hi) {
                      std::vector<uint64_t> tmp;
                      const uint64_t p0 = group_offsets[lo];
                      return tagg_host(c, sigs ? sigs + 96 * p0 : sigs, share_idx ? share_idx + p0 : share_idx,
                                       rebase(group_offsets, lo, hi, tmp), hi - lo, out_sigs + 96 * lo, status + lo);
                    });
}

int hipbls_threshold_aggregate_verify_batch(const uint8_t* sigs, const int64_t* share_idx,
                                            const uint64_t* group_offsets, uint64_t n_groups, const uint8_t* dv_pks,
                                            const uint8_t* msgs, const uint64_t* msg_offsets, uint8_t* out_sigs,
                                            int32_t* agg_status, int32_t* verify_status) {
  if (n_groups == 0) return HIPBLS_OK;
  if (!group_offsets || !dv_pks || !msg_offsets || !out_sigs || !agg_status || !verify_status ||
      mul_overflows(n_groups, 120 * 4))
    return arg_err("bad arguments");
  if (!groups_ok(group_offsets, n_groups)) return arg_err("bad group offsets");
  if (!offsets_ok(msg_offsets, n_groups)) return arg_err("bad message offsets");
  const uint64_t n_parts = group_offsets[n_groups];
  if (n_parts && (!sigs || !share_idx)) return arg_err("null partials");
  if (msg_offsets[n_groups] && !msgs) return arg_err("null messages");
  if (mul_overflows(n_parts, 288)) return arg_err("too many partials");
  ENSURE_INIT();
  return run_ranges_unlocked(plan_ranges(n_groups, parts_for(n_groups, kSplitGroups), nullptr),
                    [&](Context& c, uint64_t lo, uint64_t hi) {
                      std::vector<uint64_t> tg, tm;
                      const uint64_t p0 = group_offsets[lo];
                      return tagg_verify_host(c, sigs ? sigs + 96 * p0 : sigs, share_idx ? share_idx + p0 : share_idx,
                                              rebase(group_offsets, lo, hi, tg), hi - lo, dv_pks + 48 * lo,
                                              msgs ? msgs + msg_offsets[lo] : msgs, rebase(msg_offsets, lo, hi, tm),
                                              out_sigs + 96 * lo, agg_status + lo, verify_status + lo);
                    });
}

int hipbls_threshold_aggregate_verify_batch_device(const uint8_t* d_sigs, const int64_t* d_share_idx,
                                                   const uint64_t* d_group_offsets, uint64_t n_groups,
                                                   uint64_t n_parts, const uint8_t* d_dv_pks, const uint8_t* d_msgs,
                                                   const uint64_t* d_msg_offsets, uint8_t* d_out_sigs,
                                                   int32_t* d_agg_status, int32_t* d_verify_status, void* stream) {
  if (n_groups == 0) return HIPBLS_OK;
  if (mul_overflows(n_parts, 288) || mul_overflows(n_groups, 120 * 4)) return arg_err("too many items");
  ENSURE_INIT();
  Context& c = ctx_of(d_agg_status);
  ENTER_CTX(c);
  ON_STREAM(c, stream, s);
  return launch_tagg_verify(c, d_sigs, d_share_idx, d_group_offsets, n_groups, n_parts, d_dv_pks, d_msgs,
                            d_msg_offsets, d_out_sigs, d_agg_status, d_verify_status, s);
}

int hipbls_threshold_aggregate_batch_device(const uint8_t* d_sigs, const int64_t* d_share_idx,
                                            const uint64_t* d_group_offsets, uint64_t n_groups, uint64_t n_parts,
                                            uint8_t* d_out_sigs, int32_t* d_status, void* stream) {
  if (n_groups == 0) return HIPBLS_OK;
  if (mul_overflows(n_parts, 288)) return arg_err("too many partials");
  ENSURE_INIT();
  Context& c = ctx_of(d_status);
  ENTER_CTX(c);
  ON_STREAM(c, stream, s);
  return launch_tagg(c, d_sigs, d_share_idx, d_group_offsets, n_groups, n_parts, d_out_sigs, d_status,
                     s);
}

int hipbls_sign_batch(const uint8_t* sks, const uint8_t* msgs, const uint64_t* msg_offsets, uint64_t n,
                      uint8_t* out_sigs, int32_t* status) {
  if (n == 0) return HIPBLS_OK;
  if (!sks || !msg_offsets || !out_sigs || !status || mul_overflows(n, 96)) return arg_err("bad sign arguments");
  if (!offsets_ok(msg_offsets, n)) return arg_err("bad message offsets");
  if (msg_offsets[n] && !msgs) return arg_err("null messages");
  ENSURE_INIT();
  return run_ranges(plan_ranges(n, parts_for(n, kSplitSign), nullptr), [&](Context& c, uint64_t lo, uint64_t hi) {
    std::vector<uint64_t> tmp;
    return sign_host(c, sks + 32 * lo, msgs ? msgs + msg_offsets[lo] : msgs, rebase(msg_offsets, lo, hi, tmp),
                     hi - lo, out_sigs + 96 * lo, status + lo);
  });
}

int hipbls_sign_batch_device(const uint8_t* d_sks, const uint8_t* d_msgs, const uint64_t* d_msg_offsets, uint64_t n,
                             uint8_t* d_out_sigs, int32_t* d_status, void* stream) {
  if (n == 0) return HIPBLS_OK;
  ENSURE_INIT();
  Context& c = ctx_of(d_status);
  ENTER_CTX(c);
  ON_STREAM(c, stream, s);
  hipLaunchKernelGGL(k_sign, dim3((unsigned)grid_for(n)), dim3(kBlock), 0, s, d_sks, d_msgs,
                     d_msg_offsets, n, d_out_sigs, d_status);
  HIP_TRY(hipGetLastError());
  return HIPBLS_OK;
}

int hipbls_secret_to_public_key_batch(const uint8_t* sks, uint64_t n, uint8_t* out_pks, int32_t* status) {
  if (n == 0) return HIPBLS_OK;
  if (!sks || !out_pks || !status || mul_overflows(n, 48)) return arg_err("bad arguments");
  ENSURE_INIT();
  return run_ranges(plan_ranges(n, parts_for(n, kSplitSign), nullptr), [&](Context& c, uint64_t lo, uint64_t hi) {
    return sk_to_pk_host(c, sks + 32 * lo, hi - lo, out_pks + 48 * lo, status + lo);
  });
}

int hipbls_secret_to_public_key_batch_device(const uint8_t* d_sks, uint64_t n, uint8_t* d_out_pks, int32_t* d_status,
                                             void* stream) {
  if (n == 0) return HIPBLS_OK;
  ENSURE_INIT();
  Context& c = ctx_of(d_status);
  ENTER_CTX(c);
  ON_STREAM(c, stream, s);
  hipLaunchKernelGGL(k_sk_to_pk, dim3((unsigned)grid_for(n)), dim3(kBlock), 0, s, d_sks, n, d_out_pks,
                     d_status);
  HIP_TRY(hipGetLastError());
  return HIPBLS_OK;
}

int hipbls_verify_aggregate_batch(const uint8_t* pks, const uint64_t* key_offsets, uint64_t n_groups,
                                  const uint8_t* sigs, const uint8_t* msgs, const uint64_t* msg_offsets,
                                  int32_t* status) {
  if (n_groups == 0) return HIPBLS_OK;
  if (!key_offsets || !sigs || !msg_offsets || !status || mul_overflows(n_groups, 96)) return arg_err("bad arguments");
  if (!groups_ok(key_offsets, n_groups)) return arg_err("bad key offsets");
  if (!offsets_ok(msg_offsets, n_groups)) return arg_err("bad message offsets");
  const uint64_t nkeys = key_offsets[n_groups], msg_total = msg_offsets[n_groups];
  if ((nkeys && !pks) || (msg_total && !msgs) || mul_overflows(nkeys, 96)) return arg_err("bad arguments");
  ENSURE_INIT();
  return run_ranges(plan_ranges(n_groups, parts_for(n_groups, kSplitFav), nullptr),
                    [&](Context& c, uint64_t lo, uint64_t hi) {
                      std::vector<uint64_t> tk, tm;
                      return fav_host(c, pks ? pks + 48 * key_offsets[lo] : pks, rebase(key_offsets, lo, hi, tk),
                                      hi - lo, sigs + 96 * lo, msgs ? msgs + msg_offsets[lo] : msgs,
                                      rebase(msg_offsets, lo, hi, tm), status + lo);
                    });
}

int hipbls_verify_aggregate_batch_device(const uint8_t* d_pks, uint64_t nkeys, const uint64_t* d_key_offsets,
                                         uint64_t n_groups, const uint8_t* d_sigs, const uint8_t* d_msgs,
                                         const uint64_t* d_msg_offsets, int32_t* d_status, void* stream) {
  if (n_groups == 0) return HIPBLS_OK;
  ENSURE_INIT();
  Context& c = ctx_of(d_status);
  ENTER_CTX(c);
  ON_STREAM(c, stream, s);
  return launch_fav(c, d_pks, nkeys, d_key_offsets, n_groups, d_sigs, d_msgs, d_msg_offsets, d_status,
                    s);
}

int hipbls_verify_aggregate(const uint8_t* pks, uint64_t n, const uint8_t* sig, const uint8_t* msg, uint64_t msg_len,
                            int32_t* status) {
  if (!sig || !status || (n && !pks) || (msg_len && !msg) || mul_overflows(n, 48) || msg_len > 0xffffffffull)
    return arg_err("bad arguments");
  const uint64_t koff[2] = {0, n}, moff[2] = {0, msg_len};
  static const uint8_t empty = 0;
  return hipbls_verify_aggregate_batch(n ? pks : &empty, koff, 1, sig, msg_len ? msg : &empty, moff, status);
}

// A large Aggregate is summed per device range; the ranges' 96-byte partial sums are then aggregated once more (a
// compressed sum decodes to the same point, so the total is the same G2 sum; a bad encoding anywhere fails).
int hipbls_aggregate(const uint8_t* sigs, uint64_t n, uint8_t* out_sig, int32_t* status) {
  if (!out_sig || !status || (n && !sigs) || mul_overflows(n, 192)) return arg_err("bad arguments");
  ENSURE_INIT();
  const std::vector<uint64_t> b = plan_ranges(n, parts_for(n, kSplitAgg), nullptr);
  const size_t k = b.size() - 1;
  if (k == 1)
    return run_ranges(b, [&](Context& c, uint64_t lo, uint64_t hi) {
      return aggregate_host(c, sigs + 96 * lo, hi - lo, out_sig, status);
    });
  std::vector<uint8_t> part(96 * k);
  std::vector<int32_t> pst(k, HIPBLS_OK);
  std::vector<char> filled(k, 0);
  int rc = run_ranges(b, [&](Context& c, uint64_t lo, uint64_t hi) {
    // the range's own index (the last bound <= lo: an empty range before it shares its start), not the context's
    const size_t j = (size_t)(std::upper_bound(b.begin(), b.end() - 1, lo) - b.begin()) - 1;
    filled[j] = 1;
    return aggregate_host(c, sigs + 96 * lo, hi - lo, part.data() + 96 * j, &pst[j]);
  });
  if (rc) return rc;
  std::vector<uint8_t> parts;  // the non-empty ranges' sums only (an empty range left 96 zero bytes, not a point)
  for (size_t j = 0; j < k; ++j) {
    if (!filled[j]) continue;
    if (pst[j] != HIPBLS_OK) {
      *status = pst[j];
      memset(out_sig, 0, 96);
      return HIPBLS_OK;
    }
    parts.insert(parts.end(), part.begin() + 96 * j, part.begin() + 96 * (j + 1));
  }
  Context& c0 = ctx(0);
  ENTER_CTX(c0);
  return aggregate_host(c0, parts.data(), parts.size() / 96, out_sig, status);
}

int hipbls_aggregate_device(const uint8_t* d_sigs, uint64_t n, uint8_t* d_out_sig, int32_t* d_status, void* stream) {
  if (mul_overflows(n, 192)) return arg_err("too many signatures");
  ENSURE_INIT();
  Context& c = ctx_of(d_status);
  ENTER_CTX(c);
  ON_STREAM(c, stream, s);
  return launch_aggregate(c, d_sigs, n, d_out_sig, d_status, s);
}

int hipbls_threshold_split(const uint8_t* secret, const uint8_t* poly_tail, uint32_t total, uint32_t threshold,
                           uint8_t* out_shares, int32_t* status) {
  if (!secret || !out_shares || !status || threshold == 0 || total == 0 || (threshold > 1 && !poly_tail))
    return arg_err("bad split arguments");
  ENSURE_INIT();
  Context& c = ctx(0);
  ENTER_CTX(c);
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
  ENSURE_INIT();
  Context& c = ctx(0);
  ENTER_CTX(c);
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
  ENSURE_INIT();
  double total = 0;
  uint64_t cnt = 0;
  const int n = nctx();
  for (int k = 0; k < n; ++k) {
    Context& c = ctx(k);
    int rc = bind(c);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(c.tmu);
    auto it = c.timing.find(name);
    if (it == c.timing.end()) continue;
    drain_timing(it->second, true);
    total += it->second.total_ms;
    cnt += it->second.launches;
  }
  *launches = cnt;
  *avg_ms = cnt ? total / cnt : 0.0;
  return HIPBLS_OK;
}

int hipbls_kernel_timing_reset(void) {
  ENSURE_INIT();
  const int n = nctx();
  for (int k = 0; k < n; ++k) {
    Context& c = ctx(k);
    int rc = bind(c);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(c.tmu);
    for (auto& kv : c.timing) {
      drain_timing(kv.second, true);
      kv.second.total_ms = 0;
      kv.second.launches = 0;
    }
  }
  return HIPBLS_OK;
}

// RLC ranges: whole message runs (a validator's partials) per device, each with its own message table and scalars.
int rlc_entry(const uint8_t* pks, const uint32_t* key_idx, const uint8_t* sigs, const uint32_t* msg_idx, uint64_t n,
              const uint8_t* msgs, const uint64_t* msg_offsets, uint64_t n_msgs, const uint8_t* seed32,
              int32_t* status) {
  const uint64_t call = g_call_seq.fetch_add(1) + 1;
  const std::vector<uint64_t> b = plan_ranges(n, parts_for(n, kSplitRlc), msg_idx);
  const bool whole = b.size() == 2;
  return run_ranges(b, [&](Context& c, uint64_t lo, uint64_t hi) {
    return rlc_range(c, pks, key_idx, sigs, msg_idx, lo, hi, msgs, msg_offsets, n_msgs, seed32, status, call, whole);
  });
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
  ENSURE_INIT();
  return rlc_entry(pks, nullptr, sigs, msg_idx, n, msgs, msg_offsets, n_msgs, seed32, status);
}

int hipbls_batch_verify_rlc_device(const uint8_t* d_pks, const uint8_t* d_sigs, const uint32_t* d_msg_idx, uint64_t n,
                                   const uint8_t* d_msgs, const uint64_t* d_msg_offsets, uint64_t n_msgs,
                                   const uint8_t* seed32, int32_t* d_status, void* stream) {
  if (n == 0) return HIPBLS_OK;
  if (!seed32 || mul_overflows(n, 288)) return arg_err("bad RLC arguments");
  ENSURE_INIT();
  Context& c = ctx_of(d_status);
  ENTER_CTX(c);
  ON_STREAM(c, stream, s);
  return launch_rlc(c, d_pks, d_sigs, d_msg_idx, n, d_msgs, d_msg_offsets, n_msgs, parse_seed(seed32), d_status,
                    s, g_call_seq.fetch_add(1) + 1);
}

int hipbls_hcache_config(uint64_t capacity) {
  if (capacity > (1ull << 24)) return arg_err("H(m) cache capacity above 2^24");
  ENSURE_INIT();
  return run_all([&](Context& c) -> int {
    HCache& hc = c.hcache;
    HIP_TRY(hipDeviceSynchronize());  // no call may still read the old table
    hc.map.clear();
    hc.key_of.assign(capacity, std::string());
    hc.ring = 0;
    hc.hits = hc.misses = 0;
    hc.cap = capacity;
    if (capacity) HIP_TRY(hc.table.ensure(capacity * 48 * 4));
    return HIPBLS_OK;
  });
}

int hipbls_hcache_stats(uint64_t* hits, uint64_t* misses, uint64_t* entries) {
  if (!hits || !misses || !entries) return arg_err("null output");
  *hits = *misses = *entries = 0;
  const int n = nctx();
  for (int k = 0; k < n; ++k) {
    Context& c = ctx(k);
    std::lock_guard<std::mutex> lk(c.mu);
    *hits += c.hcache.hits;
    *misses += c.hcache.misses;
    *entries += c.hcache.map.size();
  }
  return HIPBLS_OK;
}

// The table is replicated on every device (244 B per key: a whole cluster's pubshares fit many times over).
int hipbls_pubshare_table_load(const uint8_t* pks, uint64_t n, int32_t* status) {
  if ((n && (!pks || !status)) || mul_overflows(n, 240) || n > 0xffffffffull) return arg_err("bad table arguments");
  ENSURE_INIT();
  const int nc = nctx();
  std::vector<std::vector<int32_t>> st(nc, std::vector<int32_t>(n ? n : 1));
  int rc = run_all([&](Context& c) -> int { return table_load_host(c, pks, n, st[c.slot].data()); });
  if (rc) return rc;
  if (n) memcpy(status, st[0].data(), n * 4);
  return HIPBLS_OK;
}

int hipbls_pubshare_table_size(uint64_t* n) {
  if (!n) return arg_err("null output");
  ENSURE_INIT();
  Context& c = ctx(0);
  std::lock_guard<std::mutex> lk(c.mu);
  *n = c.t_size;
  return HIPBLS_OK;
}

int hipbls_verify_batch_keys(const uint32_t* key_idx, const uint8_t* msgs, const uint64_t* msg_offsets,
                             const uint8_t* sigs, uint64_t n, int32_t* status) {
  if (n == 0) return HIPBLS_OK;
  if (!key_idx || !msg_offsets || !sigs || !status || mul_overflows(n, 96)) return arg_err("bad arguments");
  if (!offsets_ok(msg_offsets, n)) return arg_err("bad message offsets");
  if (msg_offsets[n] && !msgs) return arg_err("null messages");
  ENSURE_INIT();
  uint64_t T = 0;
  {
    std::lock_guard<std::mutex> lk(ctx(0).mu);
    T = ctx(0).t_size;
  }
  for (uint64_t i = 0; i < n; ++i)
    if (key_idx[i] >= T) return arg_err("key index outside the pubshare table");
  return run_ranges(plan_ranges(n, parts_for(n, kSplitVerify), nullptr), [&](Context& c, uint64_t lo, uint64_t hi) {
    std::vector<uint64_t> tmp;
    return verify_keys_host(c, key_idx + lo, msgs ? msgs + msg_offsets[lo] : msgs, rebase(msg_offsets, lo, hi, tmp),
                            sigs + 96 * lo, hi - lo, status + lo);
  });
}

int hipbls_verify_batch_keys_device(const uint32_t* d_key_idx, const uint8_t* d_msgs, const uint64_t* d_msg_offsets,
                                    const uint8_t* d_sigs, uint64_t n, int32_t* d_status, void* stream) {
  if (n == 0) return HIPBLS_OK;
  ENSURE_INIT();
  Context& c = ctx_of(d_status);
  ENTER_CTX(c);
  ON_STREAM(c, stream, s);
  return timed(c, "verify_keys", s, [&] {
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
  ENSURE_INIT();
  uint64_t T = 0;
  {
    std::lock_guard<std::mutex> lk(ctx(0).mu);
    T = ctx(0).t_size;
  }
  for (uint64_t i = 0; i < n; ++i)
    if (key_idx[i] >= T) return arg_err("key index outside the pubshare table");
  return rlc_entry(nullptr, key_idx, sigs, msg_idx, n, msgs, msg_offsets, n_msgs, seed32, status);
}

int hipbls_batch_verify_rlc_keys_device(const uint32_t* d_key_idx, const uint8_t* d_sigs, const uint32_t* d_msg_idx,
                                        uint64_t n, const uint8_t* d_msgs, const uint64_t* d_msg_offsets,
                                        uint64_t n_msgs, const uint8_t* seed32, int32_t* d_status, void* stream) {
  if (n == 0) return HIPBLS_OK;
  if (!seed32 || !d_key_idx || mul_overflows(n, 288)) return arg_err("bad RLC arguments");
  ENSURE_INIT();
  Context& c = ctx_of(d_status);
  ENTER_CTX(c);
  ON_STREAM(c, stream, s);
  return launch_rlc(c, nullptr, d_sigs, d_msg_idx, n, d_msgs, d_msg_offsets, n_msgs, parse_seed(seed32), d_status,
                    s, g_call_seq.fetch_add(1) + 1, d_key_idx);
}

// Windows, failed windows and re-verified items of the newest RLC call, summed over the devices it ran on.
int hipbls_rlc_stats(uint64_t* windows, uint64_t* windows_failed, uint64_t* items_fallback) {
  if (!windows || !windows_failed || !items_fallback) return arg_err("null output");
  ENSURE_INIT();
  *windows = *windows_failed = *items_fallback = 0;
  const int n = nctx();
  uint64_t newest = 0;
  for (int k = 0; k < n; ++k) {
    std::lock_guard<std::mutex> lk(ctx(k).mu);
    if (ctx(k).r_call > newest) newest = ctx(k).r_call;
  }
  for (int k = 0; k < n; ++k) {
    Context& c = ctx(k);
    ENTER_CTX(c);
    if (c.r_call != newest || c.r_windows == 0) continue;
    std::vector<int32_t> v(c.r_windows);
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(v.data(), c.r_win.p, v.size() * 4, hipMemcpyDeviceToHost));
    *windows += c.r_windows;
    for (int32_t x : v)
      if (x > 0) {
        *windows_failed += 1;
        *items_fallback += (uint64_t)x;
      } else if (x < 0) {  // a window sent straight to the per-item checks (k_rlc_window wdirect)
        *items_fallback += (uint64_t)-x;
      }
  }
  return HIPBLS_OK;
}

}  // extern "C"
