// Per-kernel cost of a chain of dependent launches (stream vs hipGraph) on
// this device: the floor a layer-per-kernel design pays per layer.
//   hipcc -O3 --offload-arch=gfx950 launch_gap.hip -o launch_gap && ./launch_gap
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

__global__ void k_touch(float* p, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = p[i] * 0.5f + 1.0f;
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
  const int maxn = 1 << 22;
  CK(hipMalloc(&d, maxn * 4));
  CK(hipMemset(d, 0, maxn * 4));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int chain = 12, reps = 200;
  for (int wgs : {1, 256, 1024, 4096}) {
    const int n = wgs * 256;
    // stream launches
    for (int w = 0; w < 20; ++w) hipLaunchKernelGGL(k_touch, dim3(wgs), dim3(256), 0, s, d, n);
    CK(hipEventRecord(e0, s));
    for (int r = 0; r < reps; ++r)
      for (int k = 0; k < chain; ++k) hipLaunchKernelGGL(k_touch, dim3(wgs), dim3(256), 0, s, d, n);
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms_stream = 0;
    CK(hipEventElapsedTime(&ms_stream, e0, e1));
    // graph of `chain` launches
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
    for (int k = 0; k < chain; ++k) hipLaunchKernelGGL(k_touch, dim3(wgs), dim3(256), 0, s, d, n);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int w = 0; w < 20; ++w) CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(e0, s));
    for (int r = 0; r < reps; ++r) CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms_graph = 0;
    CK(hipEventElapsedTime(&ms_graph, e0, e1));
    std::printf("wgs %5d: stream %.2f us/kernel, graph %.2f us/kernel (graph of %d: %.2f us)\n", wgs,
                1e3 * ms_stream / (reps * chain), 1e3 * ms_graph / (reps * chain), chain, 1e3 * ms_graph / reps);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }
  CK(hipFree(d));
  return 0;
}
