// Aggregate launch throughput with several streams in flight: S streams each
// run a chain of `chain` dependent kernels whose workgroups busy-wait `us`
// microseconds (s_memrealtime, 100 MHz), as a hipGraph replay or as plain
// stream launches.  If the streams' chains overlapped freely, S chains would
// take as long as one.
//   hipcc -O3 --offload-arch=gfx950 multi_stream.hip -o multi_stream
//   ./multi_stream [graph|stream] [prio]   (prio: streams alternate priorities)
#include <hip/hip_runtime.h>

#include <cstdio>
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
  const bool graph = argc < 2 || std::strcmp(argv[1], "stream") != 0;
  const bool prio = argc >= 3 && std::strcmp(argv[2], "prio") == 0;
  float* d = nullptr;
  CK(hipMalloc(&d, 1 << 20));
  CK(hipMemset(d, 0, 1 << 20));
  const int chain = 11, reps = 100;
  std::vector<hipStream_t> st(8);
  int lo = 0, hi = 0;
  CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
  for (int k = 0; k < 8; ++k) {
    if (prio) CK(hipStreamCreateWithPriority(&st[k], hipStreamNonBlocking, (k & 1) ? hi : lo));
    else CK(hipStreamCreateWithFlags(&st[k], hipStreamNonBlocking));
  }
  std::printf("mode %s%s (priority range %d..%d)\n", graph ? "graph" : "stream", prio ? " prio" : "", lo, hi);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int wgs : {256}) {
    for (int us : {0, 5}) {
      std::vector<hipGraphExec_t> ge(8);
      if (graph)
        for (int k = 0; k < 8; ++k) {
          hipGraph_t g;
          CK(hipStreamBeginCapture(st[k], hipStreamCaptureModeRelaxed));
          for (int c = 0; c < chain; ++c) hipLaunchKernelGGL(k_spin, dim3(wgs), dim3(256), 0, st[k], d, us * 100);
          CK(hipStreamEndCapture(st[k], &g));
          CK(hipGraphInstantiate(&ge[k], g, nullptr, nullptr, 0));
          CK(hipGraphDestroy(g));
        }
      auto run = [&](int k) -> hipError_t {
        if (graph) return hipGraphLaunch(ge[k], st[k]);
        for (int c = 0; c < chain; ++c) hipLaunchKernelGGL(k_spin, dim3(wgs), dim3(256), 0, st[k], d, us * 100);
        return hipGetLastError();
      };
      for (int S : {1, 2, 3, 4, 6, 8}) {
        for (int w = 0; w < 10; ++w)
          for (int k = 0; k < S; ++k) CK(run(k));
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, 0));
        CK(hipDeviceSynchronize());
        for (int r = 0; r < reps; ++r)
          for (int k = 0; k < S; ++k) CK(run(k));
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double per_chain = 1e3 * ms / (reps * S);
        std::printf("wgs %4d spin %2d us  streams %d: %.2f us per chain of %d (%.2f us per kernel, aggregate)\n",
                    wgs, us, S, per_chain, chain, per_chain / chain);
      }
      if (graph)
        for (auto& x : ge) CK(hipGraphExecDestroy(x));
    }
  }
  return 0;
}
