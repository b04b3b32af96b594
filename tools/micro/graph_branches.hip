// Does a hipGraph replay run independent branches concurrently?  A graph
// captured from two streams (fork / join by events): branch A = `chain`
// dependent spin kernels, branch B = the same; against one stream carrying
// both chains back to back.  Spin kernels of 256 workgroups busy-wait `us`.
//   hipcc -O3 --offload-arch=gfx950 graph_branches.hip -o graph_branches && ./graph_branches
#include <hip/hip_runtime.h>

#include <cstdio>

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

int main() {
  float* d = nullptr;
  CK(hipMalloc(&d, 1 << 20));
  CK(hipMemset(d, 0, 1 << 20));
  hipStream_t s0, s1;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  hipEvent_t fork, join, e0, e1;
  CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int chain = 10, reps = 50;
  for (int us : {2, 5, 10}) {
    for (int wgs : {64, 256}) {
      hipGraphExec_t ex[2];
      for (int par = 0; par < 2; ++par) {
        hipGraph_t g;
        CK(hipStreamBeginCapture(s0, hipStreamCaptureModeRelaxed));
        if (par) {
          CK(hipEventRecord(fork, s0));
          CK(hipStreamWaitEvent(s1, fork, 0));
          for (int c = 0; c < chain; ++c) hipLaunchKernelGGL(k_spin, dim3(wgs), dim3(256), 0, s0, d, us * 100);
          for (int c = 0; c < chain; ++c) hipLaunchKernelGGL(k_spin, dim3(wgs), dim3(256), 0, s1, d, us * 100);
          CK(hipEventRecord(join, s1));
          CK(hipStreamWaitEvent(s0, join, 0));
        } else {
          for (int c = 0; c < 2 * chain; ++c) hipLaunchKernelGGL(k_spin, dim3(wgs), dim3(256), 0, s0, d, us * 100);
        }
        CK(hipStreamEndCapture(s0, &g));
        CK(hipGraphInstantiate(&ex[par], g, nullptr, nullptr, 0));
        CK(hipGraphDestroy(g));
      }
      for (int par = 0; par < 2; ++par) {
        for (int w = 0; w < 5; ++w) CK(hipGraphLaunch(ex[par], s0));
        CK(hipStreamSynchronize(s0));
        CK(hipEventRecord(e0, s0));
        for (int r = 0; r < reps; ++r) CK(hipGraphLaunch(ex[par], s0));
        CK(hipEventRecord(e1, s0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        std::printf("spin %2d us  wgs %3d  %s: %.1f us per graph of %d kernels\n", us, wgs,
                    par ? "two branches" : "one chain   ", 1e3 * ms / reps, 2 * chain);
      }
      CK(hipGraphExecDestroy(ex[0]));
      CK(hipGraphExecDestroy(ex[1]));
    }
  }
  return 0;
}
