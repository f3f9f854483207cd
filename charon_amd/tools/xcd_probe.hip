// Does a one-workgroup kernel's duration depend on the XCD it lands on?  (the n = 1 latency path: the
// octet check's duration cycles 7.2 - 9.8 ms with a period of 8 calls in the round-4 kernel trace.)
//
// Dispatches three one-wave kernels many times on one stream: an integer multiply-add chain (clock-bound), a
// private-segment round trip loop (scratch through the XCD's L2 to HBM) and a mix.  Each wave reads its XCC id
// (HW_REG_XCC_ID), the shader clock (s_memtime) and the constant 100 MHz real-time counter (s_memrealtime) at start
// and end, and lane 0 writes them with a vector store.  Per XCD: real time and clock rate.
//
//   hipcc --offload-arch=gfx950 -O2 -o xcd_probe xcd_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <map>
#include <vector>

#define CK(x)                                                                                \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) {                                                                  \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));      \
      exit(1);                                                                               \
    }                                                                                        \
  } while (0)

struct Rec {
  uint64_t t0, t1, c0, c1;
  uint32_t xcc, hwid, sink, pad;
};

__device__ inline uint32_t xcc_id() {
  uint32_t x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  return x;
}
__device__ inline uint32_t hw_id() {
  uint32_t x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(x));
  return x;
}

// mode 0: multiply-add chain; mode 1: scratch round trips; mode 2: both
__global__ void k_probe(Rec* out, int mode, int iters, uint32_t salt) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  const uint64_t c0 = __builtin_amdgcn_s_memtime();
  uint64_t a = threadIdx.x + salt, b = 0x9e3779b97f4a7c15ull;
  volatile uint32_t buf[1024];
  if (mode) {
    for (int i = 0; i < 1024; ++i) buf[i] = i ^ salt;
  }
  uint32_t s = 0;
  for (int it = 0; it < iters; ++it) {
    if (mode != 1) {
#pragma unroll 16
      for (int k = 0; k < 64; ++k) a = a * b + (a >> 17);
    }
    if (mode != 0) {
#pragma unroll 4
      for (int k = 0; k < 16; ++k) {
        const uint32_t j = (uint32_t)(a + k * 97 + it * 31 + s) & 1023;
        s += buf[j];
        buf[(j * 7 + 3) & 1023] = s;
      }
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
  const uint64_t c1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) {
    Rec r;
    r.t0 = t0;
    r.t1 = t1;
    r.c0 = c0;
    r.c1 = c1;
    r.xcc = xcc_id();
    r.hwid = hw_id();
    r.sink = (uint32_t)a + s;
    r.pad = 0;
    out[blockIdx.x] = r;
  }
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 32;
  Rec* d = nullptr;
  CK(hipMalloc(&d, 64 * sizeof(Rec)));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const char* names[3] = {"mad_chain", "scratch", "mix"};
  const int iters[3] = {20000, 4000, 4000};
  for (int mode = 0; mode < 3; ++mode) {
    std::map<uint32_t, std::vector<double>> us, mhz;
    for (int r = 0; r < reps; ++r) {
      // grid 1 (where does a lone workgroup land?) on even reps, grid 8 (one per XCD, side by side) on odd ones
      const int g = (r & 1) ? 8 : 1;
      hipLaunchKernelGGL(k_probe, dim3(g), dim3(64), 0, s, d, mode, iters[mode], (uint32_t)r);
      CK(hipGetLastError());
      CK(hipStreamSynchronize(s));
      Rec hs[8];
      CK(hipMemcpy(hs, d, g * sizeof(Rec), hipMemcpyDeviceToHost));
      for (int b = 0; b < g; ++b) {
        const Rec& h = hs[b];
        const double t = (double)(h.t1 - h.t0) / 100.0;  // 100 MHz counter -> us
        us[h.xcc].push_back(t);
        mhz[h.xcc].push_back((double)(h.c1 - h.c0) / t);
        printf("{\"kernel\": \"%s\", \"rep\": %d, \"grid\": %d, \"block\": %d, \"xcc\": %u, \"hw_id\": \"0x%08x\", "
               "\"us\": %.1f, \"clock_MHz\": %.0f}\n",
               names[mode], r, g, b, h.xcc, h.hwid, t, (double)(h.c1 - h.c0) / t);
      }
    }
    for (auto& kv : us) {
      double m = 0, f = 0;
      for (double x : kv.second) m += x;
      for (double x : mhz[kv.first]) f += x;
      printf("{\"summary\": \"%s\", \"xcc\": %u, \"n\": %zu, \"mean_us\": %.1f, \"mean_clock_MHz\": %.0f}\n", names[mode],
             kv.first, kv.second.size(), m / kv.second.size(), f / kv.second.size());
    }
    fflush(stdout);
  }
  return 0;
}
