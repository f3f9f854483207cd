/*
 * hipbls — MI355X (gfx950) BLS12-381 engine behind charon's tbls.Implementation.
 *
 * C-ABI only: plain pointers and sizes, no HIP or torch types.  All buffers are owned by the
 * caller; the library never keeps a caller pointer after a call returns (cgo pointer rules).
 * One process drives every GPU of the node (charon is one process per node: app/app.go:127 wires all components
 * through the one global tbls implementation, tbls/tbls.go:11-14): the library keeps a context per device it was
 * given (hipbls_init_devices) and splits every host-buffer batch into contiguous ranges -- whole validators /
 * message runs -- across them, writing each range's results straight into the caller's arrays.  Every entry point
 * is thread-safe and binds the right device on the calling thread (cgo goroutines move between OS threads).  Calls
 * that share a device workspace are ordered on the device even when they are issued on different streams.  A HIP
 * failure is reported as HIPBLS_ERR_DEVICE for the whole call and NEVER as a per-item "verified".
 *
 * Reference interface each entry point replaces (paths relative to the charon repository):
 *   hipbls_verify                      tbls.Implementation.Verify (one item, coalesced by the submission queue)
 *                                      tbls/tbls.go:53-55, tbls/herumi.go:285-301
 *   hipbls_verify_batch                tbls.Implementation.Verify            tbls/tbls.go:53-55, tbls/herumi.go:285-301
 *   hipbls_verify_signed_data_batch    eth2util/signing.Verify (signing root + zero-signature check + tbls.Verify)
 *                                      eth2util/signing/signing.go:57-69, 88-107
 *   hipbls_threshold_aggregate_batch   tbls.Implementation.ThresholdAggregate tbls/tbls.go:50-51, tbls/herumi.go:244-283
 *   hipbls_sign_batch                  tbls.Implementation.Sign              tbls/tbls.go:57-59, tbls/herumi.go:303-313
 *   hipbls_secret_to_public_key_batch  tbls.Implementation.SecretToPublicKey tbls/tbls.go:36-38, tbls/herumi.go:67-80
 *   hipbls_verify_aggregate[_batch]    tbls.Implementation.VerifyAggregate   tbls/tbls.go:61-63, tbls/herumi.go:315-339
 *   hipbls_aggregate                   tbls.Implementation.Aggregate         tbls/tbls.go:65-67, tbls/herumi.go:220-242
 *   hipbls_threshold_split             tbls.Implementation.ThresholdSplit[Insecure] tbls/tbls.go:40-47, tbls/herumi.go:84-181
 *   hipbls_recover_secret              tbls.Implementation.RecoverSecret     tbls/tbls.go:49, tbls/herumi.go:183-218
 *   hipbls_pubshare_table_load         the pubshare set charon builds from the cluster lock at startup
 *                                      (app/app.go:343-381, core/parsigex/parsigex.go:139-163 lookup)
 *   hipbls_verify_batch_keys           tbls.Verify with that pubshare (tbls/herumi.go:285-301)
 *   hipbls_batch_verify_rlc            many tbls.Verify calls at once: the per-item loops of
 *                                      core/parsigex/parsigex.go:139-163, core/validatorapi/validatorapi.go:246-283,
 *                                      core/sigagg/sigagg.go:138-159 (optional BatchVerifier extension)
 * Underneath, these replace herumi's cgo entry points blsVerify / blsSignatureRecover /
 * blsSign / blsGetPublicKey / blsFastAggregateVerify / blsAggregateSignature
 * (github.com/herumi/bls-eth-go-binary v1.32.1, imported at tbls/herumi.go:12).
 *
 * Wire formats (herumi ETH mode): secret key 32 bytes big-endian; public key 48-byte compressed G1;
 * signature 96-byte compressed G2 (x = c1 || c0), ZCash flag bits.
 */
#ifndef HIPBLS_H
#define HIPBLS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Per-item and per-call status codes.  1..5 map onto the reference's error strings. */
enum {
  HIPBLS_OK = 0,
  HIPBLS_ERR_PUBKEY = 1,    /* "cannot set compressed public key in Herumi format" */
  HIPBLS_ERR_SIGNATURE = 2, /* "cannot unmarshal signature into Herumi signature" */
  HIPBLS_ERR_VERIFY = 3,    /* "signature not verified" (Verify) / "signature verification failed" (VerifyAggregate) */
  HIPBLS_ERR_SECRET = 4,    /* "cannot unmarshal secret into Herumi secret key" / "cannot obtain public key from secret" */
  HIPBLS_ERR_COMBINE = 5,   /* "cannot combine signatures" (empty set, id 0, duplicate id) */
  HIPBLS_ERR_ZERO_SIG = 6,  /* eth2util/signing.Verify: "no signature found" (all-zero signature, signing.go:99-102) */
  HIPBLS_ERR_ARG = 16,      /* bad arguments (null pointer, size overflow) */
  HIPBLS_ERR_DEVICE = 17    /* HIP runtime failure; see hipbls_last_error() */
};

/* Library/ABI version (bumped on any signature change). */
#define HIPBLS_ABI_VERSION 12
int hipbls_abi_version(void);

/* Bind the library to the n devices ids[0..n) (n <= 64; a device may repeat: each entry is one context, e.g. to
 * test the range split on one GPU).  Host-buffer batches are split across them; each device holds its own copy of
 * the pubshare table and its own H(m) cache and submission queue.  Idempotent for the same list; a different list
 * after the first bind is HIPBLS_ERR_ARG.  Without any init call the first entry point binds the devices named by
 * the environment variable HIPBLS_DEVICES ("all" or "0,1,2") or else the calling thread's current device. */
int hipbls_init_devices(const int32_t* ids, uint32_t n);
/* hipbls_init_devices(&device, 1); device < 0: device 0, or the existing binding. */
int hipbls_init(int device);
/* Number of device contexts (0 before the first bind); their device ids in ids[0..min(n, cap)). */
int hipbls_device_slots(int32_t* ids, uint32_t cap);
/* The split planner the batch entry points use (no GPU needed): bounds[0] = 0 <= ... <= bounds[parts] = n, equal
 * shares; with run_keys (e.g. each item's message index) an inner bound moves forward to the next change of key, by
 * at most half a share, so a validator's partials stay on one device. */
int hipbls_plan_ranges(uint64_t n, uint32_t parts, const uint32_t* run_keys, uint64_t* bounds);
/* Number of visible HIP devices (0 when none). */
int hipbls_device_count(void);
/* Streams the library created on `device` (its library stream, two fork sub-streams and the submission queue's
 * stream), shared by every context bound to that device: at most 4 whatever the number of contexts, so the library's
 * launches never need more than GPU_MAX_HW_QUEUES hardware queues.  0 for a device without a context. */
int hipbls_device_streams(int device);
/* Scratch budget of `device`.  Each hardware queue that runs the library's kernels holds a scratch
 * block of per_lane (the deepest kernel's private segment) x 64 lanes x 32 wave slots x CUs, rounded to 2 MiB
 * (*per_queue); all of a process's queues on the device share one region of *limit bytes (the HSA agent's scratch
 * limit, 32 GiB on MI355X; 0 = not reported), and *queues is GPU_MAX_HW_QUEUES (HIP's normal-priority queues per
 * process).  The library holds 4 queues (hipbls_device_streams), reserves their blocks at init (HIPBLS_SCRATCH_RESERVE=0
 * skips it), refuses a device where they do not fit (hipbls_init* -> HIPBLS_ERR_DEVICE), and never launches on a
 * stream that would take another queue: a *_device call on a priority or CU-masked stream (or on any caller stream when
 * *queues blocks would not fit) runs on the library stream, ordered after the caller's stream and before its later
 * work (hipbls_stream_joins counts those calls).  So (*limit - 4 x *per_queue) is what other queues of the process
 * may still hold.  HIPBLS_ERR_ARG for a device without a context. */
int hipbls_scratch_budget(int device, uint64_t* per_lane, uint64_t* per_queue, uint64_t* limit, uint32_t* queues);
int hipbls_stream_joins(uint64_t* calls);
/* Space-separated names of every kernel the library can launch (no GPU needed; the scratch budget's kernel set). */
const char* hipbls_kernel_names(void);
/* Thread-local text of the last HIPBLS_ERR_DEVICE / HIPBLS_ERR_ARG (and, after an init on a runtime without a
 * scratch-limit query, the note that every *_device call runs on the library's streams). */
const char* hipbls_last_error(void);
/* "src=<sha256> flags=<sha256>": digests of the sources and compile flags the library was built from
 * (charon_amd/build.py); smoke(), the GPU test session and bench.py compare them with the shipped sources. */
const char* hipbls_build_id(void);
/* Device index the library is bound to (-1 before the first call). */
int hipbls_current_device(void);
/* Per-kernel HIP-event timing (hipbls_kernel_timing); off by default, or HIPBLS_TIMING=1 in the environment. */
int hipbls_set_timing(int enabled);
/* Pairing-check layout.  HIPBLS_PAIR_SINGLE: one lane per check.  HIPBLS_PAIR_LANES: a lane pair per check (the
 * two Miller loops side by side, the final exponentiation split across the pair; about half the latency, twice
 * the lanes).  HIPBLS_PAIR_QUADS: four lanes per Verify-shaped check (each Miller loop split across a lane pair,
 * the two pairs side by side; RLC windows keep lane pairs).  HIPBLS_PAIR_OCTETS: eight lanes per Verify (the quad
 * layout with every Fp2 product and square split across twin lanes, charon_amd/csrc/verify_lat.hip: the drop-in
 * n = 1 latency path; other checks as QUADS).  HIPBLS_PAIR_AUTO (default): the widest layout the batch leaves
 * lanes for (Verify: octets up to 4,096 items, quads up to the quad limit, then pairs up to 32,768 items; RLC
 * sub-batches up to 32,768 windows, every RLC fallback list and FastAggregateVerify on pairs).  Results are
 * identical in every mode.  Returns the previous mode, or HIPBLS_ERR_ARG for an unknown one.  The environment
 * variable HIPBLS_PAIR_MODE (0-4) sets the initial mode. */
enum { HIPBLS_PAIR_AUTO = 0, HIPBLS_PAIR_SINGLE = 1, HIPBLS_PAIR_LANES = 2, HIPBLS_PAIR_QUADS = 3,
       HIPBLS_PAIR_OCTETS = 4 };
int hipbls_set_pair_mode(int mode);
/* Replicas of a Verify batch of at most 8 items on octets (the drop-in n = 1 path): that many copies of its one
 * workgroup race, one per XCD, and the first to finish each stage wins (the others end early); the results are the
 * same.  A single wave's check time varies 7.2-9.8 ms with where it runs.  Default 8
 * (HIPBLS_LAT_REPLICAS); 1 turns it off.  Returns the previous value, HIPBLS_ERR_ARG outside 1-32. */
int hipbls_set_latency_replicas(uint32_t replicas);

/* ------------------------------------------------ single-item Verify through the submission queue ---- */
/* tbls.Verify for one item.  Concurrent callers (any thread) are coalesced into one kernel launch per batch:
 * while a batch runs on the GPU the next one fills, so the batch size follows the offered load; an idle queue
 * waits gather_us for company.  *status as hipbls_verify_batch.  The queue has its own stream and buffers and
 * no lock is held while the GPU runs. */
int hipbls_verify(const uint8_t* pk48, const uint8_t* msg, uint64_t msg_len, const uint8_t* sig96, int32_t* status);
/* Asynchronous form: submit returns a ticket; wait blocks until that item's batch completed (each ticket once). */
int hipbls_verify_submit(const uint8_t* pk48, const uint8_t* msg, uint64_t msg_len, const uint8_t* sig96,
                         uint64_t* ticket);
int hipbls_verify_wait(uint64_t ticket, int32_t* status);
/* Queue policy (defaults 65,536 items, 50 us) and counters (batches launched, items verified), summed over the
 * devices.  An item goes to the device its message hashes to, so the partials of one signing root meet in one
 * batch.  A batch of >= 8 items whose keys are all in the resident pubshare table runs as an RLC BatchVerify with
 * keys by index over its distinct messages, through the H(m) cache (statuses unchanged); the number of batches
 * that took this keyed path is hipbls_queue_keyed_batches. */
int hipbls_queue_config(uint64_t max_batch, uint32_t gather_us);
int hipbls_queue_stats(uint64_t* batches, uint64_t* items);
int hipbls_queue_keyed_batches(uint64_t* batches);
/* Completion polls of the queue workers (a batch in flight is polled every 20 us from 85 % of the running estimate
 * of its time on) and wire batches collected, summed over the devices. */
int hipbls_queue_worker_stats(uint64_t* wakeups, uint64_t* batches);

/* ---------------------------------------------------------------- batched, host buffers ---- */

/* Verify n items: item i is (pks[48 i..], msgs[msg_offsets[i] .. msg_offsets[i+1]), sigs[96 i..]).
 * status[i] = HIPBLS_OK | HIPBLS_ERR_PUBKEY | HIPBLS_ERR_SIGNATURE | HIPBLS_ERR_VERIFY,
 * exactly the outcome tbls.Herumi.Verify returns for that item. */
int hipbls_verify_batch(const uint8_t* pks, const uint8_t* msgs, const uint64_t* msg_offsets,
                        const uint8_t* sigs, uint64_t n, int32_t* status);

/* eth2util/signing.Verify for n items: the signing root SHA-256(object_root || domain) (SSZ SigningData) is
 * computed on the GPU from object_roots[32 i ..] and domains[32 i ..]; status[i] as hipbls_verify_batch, or
 * HIPBLS_ERR_ZERO_SIG for an all-zero signature. */
int hipbls_verify_signed_data_batch(const uint8_t* pks, const uint8_t* object_roots, const uint8_t* domains,
                                    const uint8_t* sigs, uint64_t n, int32_t* status);

/* ThresholdAggregate for n_groups sets: group g holds partials
 * sigs[96 k ..], share_idx[k] for k in [group_offsets[g], group_offsets[g+1]).
 * out_sigs[96 g ..] = sum_k lambda_k(0) * sig_k: Lagrange at 0 over the share indices taken as Fr elements the
 * way herumi parses strconv.Itoa(idx) (tbls/herumi.go:264-271): a signed Go int reduced mod r, so -k is r - k.
 * status[g] = HIPBLS_OK | HIPBLS_ERR_SIGNATURE | HIPBLS_ERR_COMBINE (empty set, id = 0, duplicate id). */
int hipbls_threshold_aggregate_batch(const uint8_t* sigs, const int64_t* share_idx,
                                     const uint64_t* group_offsets, uint64_t n_groups,
                                     uint8_t* out_sigs, int32_t* status);

/* Sign n messages: out_sigs[96 i ..] = sks[32 i ..] * H(msg_i).  status[i] = OK | ERR_SECRET. */
int hipbls_sign_batch(const uint8_t* sks, const uint8_t* msgs, const uint64_t* msg_offsets, uint64_t n,
                      uint8_t* out_sigs, int32_t* status);

/* out_pks[48 i ..] = sks[32 i ..] * g1.  status[i] = OK | ERR_SECRET (zero or >= r). */
int hipbls_secret_to_public_key_batch(const uint8_t* sks, uint64_t n, uint8_t* out_pks, int32_t* status);

/* FastAggregateVerify(pks[0..n), sig, msg).  *status = OK | ERR_PUBKEY | ERR_SIGNATURE | ERR_VERIFY. */
int hipbls_verify_aggregate(const uint8_t* pks, uint64_t n, const uint8_t* sig, const uint8_t* msg,
                            uint64_t msg_len, int32_t* status);

/* n_groups FastAggregateVerify calls in one launch: group g checks sigs[96 g ..] over message
 * msgs[msg_offsets[g] .. msg_offsets[g+1]) against the keys pks[48 k ..], k in
 * [key_offsets[g], key_offsets[g+1]).  status[g] as hipbls_verify_aggregate.  Sync-committee and
 * cluster-lock checks (cluster/lock.go:178,267) batch this way. */
int hipbls_verify_aggregate_batch(const uint8_t* pks, const uint64_t* key_offsets, uint64_t n_groups,
                                  const uint8_t* sigs, const uint8_t* msgs, const uint64_t* msg_offsets,
                                  int32_t* status);

/* herumi's Deserialize of n points, one status each: kind 1 = 48-byte public keys (OK | ERR_PUBKEY), kind 2 = 96-byte
 * signatures (OK | ERR_SIGNATURE); flags, x < p, on the curve, in the subgroup (the point at infinity deserializes).
 * The Go binding uses it to name the failing item in Aggregate / ThresholdAggregate errors, the
 * z.Int("signature_number", idx) field of tbls/herumi.go:229-233, 255-258. */
int hipbls_deserialize_status(const uint8_t* data, uint64_t n, int32_t kind, int32_t* status);

/* Plain G2 sum of n signatures (decoded in parallel, tree-summed).  *status = OK | ERR_SIGNATURE.  As herumi
 * (tbls/herumi.go:220-242), n == 0 is not an error: the sum is the point at infinity, 0xc0 || 0^95. */
int hipbls_aggregate(const uint8_t* sigs, uint64_t n, uint8_t* out_sig, int32_t* status);

/* Shamir split: share_i = secret + sum_j poly_tail[j] * i^(j+1) mod r, i = 1..total.
 * poly_tail holds threshold-1 secrets of 32 bytes (the reference draws them from a CSPRNG or an
 * insecure reader; the caller supplies them).  *status = OK | ERR_SECRET. */
int hipbls_threshold_split(const uint8_t* secret, const uint8_t* poly_tail, uint32_t total, uint32_t threshold,
                           uint8_t* out_shares, int32_t* status);

/* Lagrange recovery of the secret at 0 from n (id, share) pairs; ids as in ThresholdAggregate (int mod r).
 * *status = OK | ERR_SECRET | ERR_COMBINE. */
int hipbls_recover_secret(const uint8_t* shares, const int64_t* ids, uint32_t n, uint8_t* out_secret,
                          int32_t* status);

/* Random-linear-combination BatchVerify.  Item i is (pks[48 i..], message msg_idx[i], sigs[96 i..]);
 * message m is msgs[msg_offsets[m] .. msg_offsets[m+1]) (n_msgs distinct messages, each hashed once).
 * status[i] is exactly hipbls_verify_batch's (i.e. tbls.Verify's) outcome for the item: items are
 * decoded and subgroup-checked one by one, windows of consecutive items are checked with one
 * multi-pairing under 64-bit random scalars derived from seed32 (32 bytes the caller draws from a
 * CSPRNG), and the items of a window that fails are re-verified individually.  Items sharing a
 * message should be adjacent (e.g. all partials of one validator): each run of equal msg_idx inside
 * a window costs one Miller loop.  HIPBLS_ERR_ARG when a msg_idx is out of range. */
int hipbls_batch_verify_rlc(const uint8_t* pks, const uint8_t* sigs, const uint32_t* msg_idx, uint64_t n,
                            const uint8_t* msgs, const uint64_t* msg_offsets, uint64_t n_msgs, const uint8_t* seed32,
                            int32_t* status);
/* Resident pubshare table: decode + subgroup-check n public keys once and keep
 * them in HBM; replaces the previous table.  status[k] = OK | ERR_PUBKEY (an infinity key loads and
 * later verifies as ERR_VERIFY, like Verify).  The *_keys entry points name keys by table index and
 * return exactly what the wire-format calls return for the same key bytes. */
int hipbls_pubshare_table_load(const uint8_t* pks, uint64_t n, int32_t* status);
int hipbls_pubshare_table_size(uint64_t* n);
/* hipbls_verify_batch with pks[i] = table[key_idx[i]]; HIPBLS_ERR_ARG when an index is outside the table. */
int hipbls_verify_batch_keys(const uint32_t* key_idx, const uint8_t* msgs, const uint64_t* msg_offsets,
                             const uint8_t* sigs, uint64_t n, int32_t* status);
/* hipbls_batch_verify_rlc with pks[i] = table[key_idx[i]]. */
int hipbls_batch_verify_rlc_keys(const uint32_t* key_idx, const uint8_t* sigs, const uint32_t* msg_idx, uint64_t n,
                                 const uint8_t* msgs, const uint64_t* msg_offsets, uint64_t n_msgs,
                                 const uint8_t* seed32, int32_t* status);

/* Windows checked, windows that failed, and items re-verified one by one in the last RLC call
 * (synchronizes the device). */
int hipbls_rlc_stats(uint64_t* windows, uint64_t* windows_failed, uint64_t* items_fallback);
/* Batch-wide check (charon_amd/csrc/rlcb.h): one multi-pairing over the whole batch with a Pippenger MSM for
 * sum r_i sig_i, ahead of the windows.  It decides an all-valid batch alone; when it fails, the windows decide
 * item by item, so statuses never depend on the mode.  HIPBLS_RLC_AUTO (default): batch-wide first for batches of
 * >= 1,024 items unless the last batch-wide check failed (then 8 calls windows-only); HIPBLS_RLC_WINDOWS: windows
 * only; HIPBLS_RLC_BATCH: batch-wide first always.  Returns the previous mode or HIPBLS_ERR_ARG. */
enum { HIPBLS_RLC_AUTO = 0, HIPBLS_RLC_WINDOWS = 1, HIPBLS_RLC_BATCH = 2 };
int hipbls_rlc_set_mode(int mode);
/* The batch-wide check's G1 side for batches that average >= 8 items per message (committee roots): each message
 * with >= `min` items gets one Pippenger sum of [r_i] pk_i (charon_amd/csrc/g1msm.h) and one Miller loop, instead of
 * a scalar multiplication per item.  0 turns it off; default 64.  Statuses never depend on it.  Returns the previous
 * value. */
int hipbls_rlc_set_g1_msm_min(uint32_t min);
/* Batch-wide checks launched and passed since load, and the last verdict (-1 none, 0 failed, 1 passed); waits for
 * the last one in flight. */
int hipbls_rlc_batch_stats(uint64_t* attempted, uint64_t* passed, int32_t* last);

/* Resident H(m) cache used by the host-buffer RLC calls: each distinct message is hashed to G2
 * once and kept in HBM across calls (FIFO over `capacity` slots, 192 B each); 0 disables it (the default).
 * Statuses are unchanged by the cache. */
int hipbls_hcache_config(uint64_t capacity);
int hipbls_hcache_stats(uint64_t* hits, uint64_t* misses, uint64_t* entries);

/* ------------------------------------------- device-resident variants (inputs already in HBM) ---- */
/* Same semantics; every pointer is a device pointer; work is enqueued on `stream` (a hipStream_t,
 * NULL = the library's own non-blocking stream of that device, which is NOT ordered with the caller's default
 * stream: a caller that reads the results with other work must pass that work's stream) and the call returns
 * without synchronizing.  The call runs on the
 * device that owns the status array. */
int hipbls_verify_batch_device(const uint8_t* d_pks, const uint8_t* d_msgs, const uint64_t* d_msg_offsets,
                               const uint8_t* d_sigs, uint64_t n, int32_t* d_status, void* stream);
/* n_parts = group_offsets[n_groups], passed explicitly so the call never reads device memory.  The _device sigagg
 * call is three kernels on `stream`; calls enqueued on different streams overlap (two workspace sets, each call's
 * first kernel after the previous call's), so a caller with consecutive duties can keep two in flight. */
/* core/sigagg (sigagg.go:138-159) in one call: ThresholdAggregate of every group (as
 * hipbls_threshold_aggregate_batch: out_sigs, agg_status) and Verify(dv_pks[g], msg g, out_sigs[g]) of each
 * aggregate (verify_status, as hipbls_verify_batch).  A group whose aggregation failed reports its aggregation
 * status in verify_status too.  The key decode and hash run beside the aggregation, and the aggregate goes to the
 * pairing check without being decompressed again: the same verdicts as the two calls, in less time. */
int hipbls_threshold_aggregate_verify_batch(const uint8_t* sigs, const int64_t* share_idx,
                                            const uint64_t* group_offsets, uint64_t n_groups, const uint8_t* dv_pks,
                                            const uint8_t* msgs, const uint64_t* msg_offsets, uint8_t* out_sigs,
                                            int32_t* agg_status, int32_t* verify_status);
int hipbls_threshold_aggregate_verify_batch_device(const uint8_t* d_sigs, const int64_t* d_share_idx,
                                                   const uint64_t* d_group_offsets, uint64_t n_groups,
                                                   uint64_t n_parts, const uint8_t* d_dv_pks, const uint8_t* d_msgs,
                                                   const uint64_t* d_msg_offsets, uint8_t* d_out_sigs,
                                                   int32_t* d_agg_status, int32_t* d_verify_status, void* stream);
int hipbls_threshold_aggregate_batch_device(const uint8_t* d_sigs, const int64_t* d_share_idx,
                                            const uint64_t* d_group_offsets, uint64_t n_groups, uint64_t n_parts,
                                            uint8_t* d_out_sigs, int32_t* d_status, void* stream);
int hipbls_aggregate_device(const uint8_t* d_sigs, uint64_t n, uint8_t* d_out_sig, int32_t* d_status, void* stream);
int hipbls_sign_batch_device(const uint8_t* d_sks, const uint8_t* d_msgs, const uint64_t* d_msg_offsets,
                             uint64_t n, uint8_t* d_out_sigs, int32_t* d_status, void* stream);
int hipbls_secret_to_public_key_batch_device(const uint8_t* d_sks, uint64_t n, uint8_t* d_out_pks,
                                             int32_t* d_status, void* stream);

/* As hipbls_batch_verify_rlc; seed32 is a host pointer.  An out-of-range msg_idx[i] yields
 * status[i] = HIPBLS_ERR_ARG. */
int hipbls_batch_verify_rlc_device(const uint8_t* d_pks, const uint8_t* d_sigs, const uint32_t* d_msg_idx, uint64_t n,
                                   const uint8_t* d_msgs, const uint64_t* d_msg_offsets, uint64_t n_msgs,
                                   const uint8_t* seed32, int32_t* d_status, void* stream);

/* Device variant of hipbls_verify_aggregate_batch (nkeys = key_offsets[n_groups], passed explicitly). */
int hipbls_verify_aggregate_batch_device(const uint8_t* d_pks, uint64_t nkeys, const uint64_t* d_key_offsets,
                                         uint64_t n_groups, const uint8_t* d_sigs, const uint8_t* d_msgs,
                                         const uint64_t* d_msg_offsets, int32_t* d_status, void* stream);

/* Device variants of the *_keys calls: an out-of-range key or message index yields
 * status[i] = HIPBLS_ERR_ARG. */
int hipbls_verify_batch_keys_device(const uint32_t* d_key_idx, const uint8_t* d_msgs, const uint64_t* d_msg_offsets,
                                    const uint8_t* d_sigs, uint64_t n, int32_t* d_status, void* stream);
int hipbls_batch_verify_rlc_keys_device(const uint32_t* d_key_idx, const uint8_t* d_sigs, const uint32_t* d_msg_idx,
                                        uint64_t n, const uint8_t* d_msgs, const uint64_t* d_msg_offsets,
                                        uint64_t n_msgs, const uint8_t* seed32, int32_t* d_status, void* stream);

/* Average duration (ms) per launch of a kernel over the calls since the last reset, measured with HIP
 * events on the stream it runs on (bench.py roofline; enable with hipbls_set_timing).  Names: "verify"
 * (k_verify_fused), "verify_prep" + "verify_pair_lg2" (lane-pair Verify), "verify_keys", "rlc_items",
 * "rlc_hash", "rlc_window" / "rlc_window_lg2", "rlc_fallback" / "rlc_fallback_lg2", "tagg_scale", "tagg_sum",
 * "fav". */
int hipbls_kernel_timing(const char* name, double* avg_ms, uint64_t* launches);
int hipbls_kernel_timing_reset(void);

#ifdef __cplusplus
}
#endif

#endif /* HIPBLS_H */
