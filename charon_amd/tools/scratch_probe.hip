// Scratch reservation per hardware queue on gfx950 (VERDICT r04 "Next round" item 1).
//
// Prints the agent's scratch limits (HSA_AMD_AGENT_INFO_SCRATCH_LIMIT_MAX / _CURRENT), then dispatches a kernel of
// known private segment on streams of normal priority and on one high-priority stream and reads the device's free
// memory (hipMemGetInfo) after each.  The deltas show which streams get a hardware queue of their own and how much
// scratch a queue reserves for a given private segment, so the round-4 abort (a 5th queue beside 4 that carry the
// library's kernels) can be computed instead of guessed.  Every dispatch is small in private segment (<= 4 KiB per
// lane) so the probe itself never approaches the limit.
//
//   hipcc --offload-arch=gfx950 -O2 -o scratch_probe scratch_probe.hip -L/opt/rocm/lib -lhsa-runtime64
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

template <int WORDS>
__global__ void k_stack(uint32_t* out, uint64_t* base, uint32_t salt) {
  volatile uint32_t buf[WORDS];  // dynamically indexed volatile array: lives in the private segment
  for (int i = (int)(threadIdx.x & 7); i < WORDS; i += 8) buf[i] = (uint32_t)i * salt;
  uint32_t s = 0;
  for (int i = 0; i < WORDS; i += 17) s += buf[(uint32_t)(i * salt + threadIdx.x) % WORDS];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  // the wave's scratch base (architected flat scratch: the queue's scratch block + this wave slot's offset), read
  // from the register the dispatcher set; written by lane 0 with a vector store
  uint32_t lo, hi;
  asm volatile("s_mov_b32 %0, flat_scratch_lo" : "=s"(lo));
  asm volatile("s_mov_b32 %0, flat_scratch_hi" : "=s"(hi));
  if (threadIdx.x == 0) base[blockIdx.x] = ((uint64_t)hi << 32) | lo;
}

static hsa_status_t first_gpu(hsa_agent_t a, void* data) {
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) == HSA_STATUS_SUCCESS && t == HSA_DEVICE_TYPE_GPU) {
    *(hsa_agent_t*)data = a;
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}

static size_t free_bytes() {
  size_t f = 0, t = 0;
  CK(hipMemGetInfo(&f, &t));
  return f;
}

template <int WORDS>
static void dispatch(const char* what, hipStream_t s, uint32_t* out, unsigned groups) {
  static uint64_t* d_base = nullptr;
  static std::vector<uint64_t> h_base;
  if (!d_base) CK(hipMalloc(&d_base, 65536 * 8));
  h_base.assign(groups, 0);
  hipFuncAttributes fa;
  CK(hipFuncGetAttributes(&fa, (const void*)k_stack<WORDS>));
  const size_t before = free_bytes();
  hipLaunchKernelGGL(k_stack<WORDS>, dim3(groups), dim3(64), 0, s, out, d_base, 3u);
  CK(hipGetLastError());
  CK(hipStreamSynchronize(s));
  const size_t after = free_bytes();
  CK(hipMemcpy(h_base.data(), d_base, (size_t)groups * 8, hipMemcpyDeviceToHost));
  uint64_t bmin = ~0ull, bmax = 0;
  for (uint64_t b : h_base) {
    bmin = b < bmin ? b : bmin;
    bmax = b > bmax ? b : bmax;
  }
  printf("{\"dispatch\": \"%s\", \"private_segment_B\": %zu, \"groups\": %u, \"free_delta_MiB\": %.1f, "
         "\"base_min\": \"0x%llx\", \"base_max\": \"0x%llx\", \"span_MiB\": %.1f}\n", what,
         (size_t)fa.localSizeBytes, groups, ((double)before - (double)after) / 1048576.0, (unsigned long long)bmin,
         (unsigned long long)bmax, (double)(bmax - bmin) / 1048576.0);
  fflush(stdout);
}

int main() {
  CK(hipSetDevice(0));
  CK(hipFree(nullptr));
  hsa_agent_t agent{};
  hsa_iterate_agents(first_gpu, &agent);
  uint64_t lim_max = 0, lim_cur = 0;
  uint32_t cus = 0;
  const hsa_status_t s1 = hsa_agent_get_info(agent, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_SCRATCH_LIMIT_MAX, &lim_max);
  const hsa_status_t s2 = hsa_agent_get_info(agent, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_SCRATCH_LIMIT_CURRENT, &lim_cur);
  hsa_agent_get_info(agent, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_COMPUTE_UNIT_COUNT, &cus);
  int lo = 0, hi = 0;
  CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
  size_t stack = 0;
  CK(hipDeviceGetLimit(&stack, hipLimitStackSize));
  const char* hwq = getenv("GPU_MAX_HW_QUEUES");
  printf("{\"scratch_limit_max_B\": %llu, \"st_max\": %d, \"scratch_limit_current_B\": %llu, \"st_cur\": %d, "
         "\"cus\": %u, \"prio_least\": %d, \"prio_greatest\": %d, \"hip_stack_limit_B\": %zu, \"GPU_MAX_HW_QUEUES\": "
         "\"%s\"}\n",
         (unsigned long long)lim_max, (int)s1, (unsigned long long)lim_cur, (int)s2, cus, lo, hi, stack,
         hwq ? hwq : "(unset)");
  fflush(stdout);

  const unsigned groups = 16 * 1024;  // 16,384 one-wave workgroups: more waves than the device can hold at once
  uint32_t* out = nullptr;
  CK(hipMalloc(&out, (size_t)groups * 64 * 4));

  hipStream_t ss[6];
  for (auto& s : ss) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  char name[64];
  if (getenv("PROBE_LAYOUT")) {
    // Allocation layout and the permanent/use-once split, within the library's own envelope (four queues at its
    // deepest kernel, 12,480 B per lane): block bases from the wave's flat-scratch register.
    dispatch<256>("q0 1KiB", ss[0], out, groups);
    dispatch<256>("q1 1KiB", ss[1], out, groups);
    dispatch<1024>("q0 4KiB (growth)", ss[0], out, groups);
    dispatch<256>("q2 1KiB", ss[2], out, groups);
    dispatch<3116>("q3 12.5KiB", ss[3], out, groups);
    dispatch<3116>("q1 12.5KiB", ss[1], out, groups);
    dispatch<3116>("q2 12.5KiB", ss[2], out, groups);
    dispatch<3116>("q0 12.5KiB (4 queues > 24 GiB)", ss[0], out, groups);
    dispatch<3116>("q0 12.5KiB again", ss[0], out, groups);
    dispatch<3116>("q3 12.5KiB again", ss[3], out, groups);
    dispatch<256>("q0 1KiB after", ss[0], out, groups);
    CK(hipDeviceSynchronize());
    printf("{\"done\": true}\n");
    return 0;
  }
  // 1 KiB per lane on six normal-priority streams: HIP maps them onto GPU_MAX_HW_QUEUES hardware queues
  for (int k = 0; k < 6; ++k) {
    snprintf(name, sizeof name, "1KiB stream %d (normal)", k);
    dispatch<256>(name, ss[k], out, groups);
  }
  // the same kernel again on stream 0: a queue that already holds enough scratch takes nothing more
  dispatch<256>("1KiB stream 0 again", ss[0], out, groups);
  // a small grid: does the reservation follow the dispatch's wave count?
  dispatch<512>("2KiB stream 0, 64 groups", ss[0], out, 64);
  // twice the private segment on stream 0: the queue's reservation grows
  dispatch<512>("2KiB stream 0", ss[0], out, groups);
  dispatch<1024>("4KiB stream 0", ss[0], out, groups);
  // a high-priority stream: its own hardware queue?
  hipStream_t hp;
  CK(hipStreamCreateWithPriority(&hp, hipStreamNonBlocking, hi));
  dispatch<256>("1KiB high-priority stream", hp, out, groups);
  hipStream_t lp;
  CK(hipStreamCreateWithPriority(&lp, hipStreamNonBlocking, lo));
  dispatch<256>("1KiB least-priority stream", lp, out, groups);
  // the null stream
  dispatch<256>("1KiB null stream", nullptr, out, groups);
  CK(hipDeviceSynchronize());
  printf("{\"done\": true}\n");
  return 0;
}
