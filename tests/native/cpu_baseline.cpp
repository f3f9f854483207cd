// CPU baseline: the repo's C++ restatement of the path -- the same per-item
// operations the kernels run (charon_amd/csrc/ops.h), compiled for x86-64 at -O3 with a 6 x 64-bit Montgomery
// product -- timed on the host cores with one thread per core.  NOT herumi: herumi/mcl (x86 asm/JIT) is not in
// this image or on the GPU box and Go is absent.  TEST/BENCH INFRASTRUCTURE ONLY: bench.py's
// cpu_baseline leg calls it; the product library never does.
#define BLS_HOST_FAST_MUL 1
#include "../../charon_amd/csrc/ops.h"

#include <atomic>
#include <chrono>
#include <thread>
#include <vector>

using namespace bls;

namespace {
template <class F>
double run_parallel(uint64_t n, int threads, F body) {
  if (threads < 1) threads = 1;
  std::atomic<uint64_t> next{0};
  const auto t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> pool;
  for (int t = 0; t < threads; ++t)
    pool.emplace_back([&] {
      for (;;) {
        const uint64_t i = next.fetch_add(1);
        if (i >= n) break;
        body(i);
      }
    });
  for (auto& th : pool) th.join();
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}
}  // namespace

extern "C" {

// tbls.Verify for n items on `threads` threads; returns seconds.
double cb_verify_batch(const uint8_t* pks, const uint8_t* msgs, const uint64_t* offs, const uint8_t* sigs, uint64_t n,
                       int32_t* status, int threads) {
  return run_parallel(n, threads, [&](uint64_t i) {
    status[i] = op_verify(pks + 48 * i, msgs + offs[i], (uint32_t)(offs[i + 1] - offs[i]), sigs + 96 * i);
  });
}

// ThresholdAggregate per group (ids int64, Lagrange at 0 over Fr, GLS scalar products) on `threads` threads;
// returns seconds.  out[96 g ..], status[g] as hipbls_threshold_aggregate_batch.
double cb_threshold_aggregate_batch(const uint8_t* sigs, const int64_t* ids, const uint64_t* goffs, uint64_t n_groups,
                                    uint8_t* out, int32_t* status, int threads) {
  return run_parallel(n_groups, threads, [&](uint64_t g) {
    const uint64_t g0 = goffs[g], g1 = goffs[g + 1];
    uint8_t sig[96];
    const int st = op_threshold_aggregate(sig, sigs + 96 * g0, ids + g0, (int)(g1 - g0));
    for (int b = 0; b < 96; ++b) out[96 * g + b] = st == HIPBLS_OK ? sig[b] : 0;
    status[g] = st;
  });
}

}  // extern "C"
