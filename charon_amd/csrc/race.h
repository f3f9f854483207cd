// Replica races for the n = 1 drop-in path (verify_lat.hip, verify_hex.hip): device-only, included before lg2.h so
// its polls (BLS_RACE_POLL) reach the pairing code.  Each translation unit that includes it gets its own copy (the
// LDS words are per kernel; nothing here has a host-side symbol).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

// ---------------------------------------------------------------- replica races (the n = 1 drop-in path)
// The octet check of one item takes 7.2 to 9.8 ms depending on where its single wave runs: eight copies of the same
// work in one launch, one per XCD, finished 7.2-9.8 ms apart with no XCD consistently fast
// (profiles/r05/r05_xcd_lq8.txt).  So a batch of at most 8 items runs as `replicas` copies of its workgroups; every
// copy computes the same result, polls its race word at coarse steps (BLS_RACE_POLL in lg2.h and below), and the
// first to finish sets the word to this launch's epoch, which ends the others.  The word lives in LDS per workgroup
// (nullptr: not raced); EVERY kernel of this translation unit sets it at entry, since LDS is not zero-initialized.
namespace {
namespace bls_race {
__shared__ uint32_t* s_word;
__shared__ uint32_t s_epoch;
__device__ __forceinline__ void init(uint32_t* word, uint32_t epoch) {
  s_word = word;
  s_epoch = epoch;
}
__device__ __forceinline__ uint32_t* word_u() {  // wave-uniform copy of the LDS pointer; nullptr unless 4-aligned
  const uint64_t w = (uint64_t)s_word;
  // readfirstlane returns int: each half goes through uint32_t, or a low half with bit 31 set (half of all buffer
  // addresses) sign-extends over the high half -- round 5's first race build read a wild address (an illegal access in
  // one run, a hung queue worker in the next)
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(w >> 32));
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)w);
  const uint64_t u = ((uint64_t)hi << 32) | lo;
  return (u & 3) ? nullptr : (uint32_t*)u;  // the words are race[0..3]: the launch checks race's 64-B alignment
}
// The word is written by a wave on another XCD: the poll is a `global_load_dword ... sc1` (past this CU's L1, served
// coherently across the XCDs' L2s) and the winner's store a write-through `global_store_dword ... sc1`
// (MI355X_MICROARCH.md, inter-workgroup visibility: flag polls by global/buffer sc1 loads, never flat; the generic
// pointer made __hip_atomic_load/store flat_ forms).  The second race build also asked each word for 64-byte alignment,
// which only race[0] has: no polled stage was raced, and every raced kernel took as long as its slowest copy
// (profiles/r05/race_trace_flat.json).
__device__ __forceinline__ void poll() {
  uint32_t* w = word_u();
  if (!w) return;
  uint32_t v;
  asm volatile("global_load_dword %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(w) : "memory");
  if ((uint32_t)__builtin_amdgcn_readfirstlane(v) == (uint32_t)__builtin_amdgcn_readfirstlane(s_epoch))
    asm volatile("s_endpgm");
}
// After this copy's results are stored: the race is won (the other copies end at their next poll).
__device__ __forceinline__ void finish() {
  uint32_t* w = word_u();
  if (w && threadIdx.x == 0) {
    const uint32_t e = s_epoch;
    asm volatile("s_waitcnt vmcnt(0)\n\tglobal_store_dword %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : : "v"(w), "v"(e)
                 : "memory");
  }
}
}  // namespace bls_race
}  // namespace
#define BLS_RACE_POLL() ::bls_race::poll()
