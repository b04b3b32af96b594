// Which stream layouts give 4 chains on 4 distinct hardware queues?  One case
// per process (the runtime's queue pool keeps its state for the process):
//   ./queue_map <extra> <mode> <touch>
// `extra` normal-priority streams are created (and each used once) before the
// 4 chain streams; mode: normal | high | alt (alternating) | cumask (every CU
// enabled: hipExtStreamCreateWithCUMask).  touch 1: every rep also launches a
// tiny kernel on each extra stream.  Prints the time per chain of 11 5-us
// kernels with the 4 chains in flight (one chain alone: ~80 us; 4 distinct
// queues: ~21 us).
//   hipcc -O3 --offload-arch=gfx950 queue_map.hip -o queue_map
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

__global__ void k_spin(float* p, int ticks) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)ticks) __builtin_amdgcn_s_sleep(1);
  if (threadIdx.x == 0 && p) p[blockIdx.x] += 1.0f;
}

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      std::printf("%s failed: %s\n", #x, hipGetErrorString(e));            \
      return 1;                                                            \
    }                                                                      \
  } while (0)

int main(int argc, char** argv) {
  const int extra = argc > 1 ? std::atoi(argv[1]) : 0;
  const char* mode = argc > 2 ? argv[2] : "normal";
  const int touch = argc > 3 ? std::atoi(argv[3]) : 0;
  float* d = nullptr;
  CK(hipMalloc(&d, 1 << 20));
  CK(hipMemset(d, 0, 1 << 20));  // the null stream
  int lo = 0, hi = 0;
  CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
  std::vector<hipStream_t> ex(extra), st(4);
  for (auto& s : ex) {
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s, d, 0);
  }
  CK(hipDeviceSynchronize());
  for (int k = 0; k < 4; ++k) {
    if (!std::strcmp(mode, "cumask")) {
      std::vector<uint32_t> mask(8, 0xFFFFFFFFu);  // 256 CUs
      CK(hipExtStreamCreateWithCUMask(&st[k], (uint32_t)mask.size(), mask.data()));
    } else {
      const int pr = !std::strcmp(mode, "high") ? hi : (!std::strcmp(mode, "alt") && (k & 1) ? hi : lo);
      CK(hipStreamCreateWithPriority(&st[k], hipStreamNonBlocking, pr));
    }
  }
  const int chain = 11, reps = 60;
  std::vector<hipGraphExec_t> ge(4);
  for (int k = 0; k < 4; ++k) {
    hipGraph_t g;
    CK(hipStreamBeginCapture(st[k], hipStreamCaptureModeRelaxed));
    for (int c = 0; c < chain; ++c) hipLaunchKernelGGL(k_spin, dim3(256), dim3(256), 0, st[k], d, 500);
    CK(hipStreamEndCapture(st[k], &g));
    CK(hipGraphInstantiate(&ge[k], g, nullptr, nullptr, 0));
    CK(hipGraphDestroy(g));
  }
  auto rep = [&](int S) -> hipError_t {
    for (int k = 0; k < S; ++k) {
      hipError_t e = hipGraphLaunch(ge[k], st[k]);
      if (e != hipSuccess) return e;
    }
    if (touch)
      for (auto& s : ex) hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s, d, 0);
    return hipGetLastError();
  };
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::printf("extra %d mode %-6s touch %d:", extra, mode, touch);
  for (int S : {1, 4}) {
    for (int w = 0; w < 5; ++w) CK(rep(S));
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    CK(hipDeviceSynchronize());
    for (int r = 0; r < reps; ++r) CK(rep(S));
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::printf("  %d in flight %.2f us/chain", S, 1e3 * ms / (reps * S));
  }
  std::printf("\n");
  return 0;
}
