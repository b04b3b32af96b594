// Do 3 workgroups per CU really co-reside near the LDS limit?  768 workgroups
// of 256 threads that each compute for a fixed time, at dynamic LDS sizes
// around 160 KiB / 3: one round (256 CUs x 3) vs two rounds shows in the time.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ __launch_bounds__(256) void k(float* out, int iters) {
  extern __shared__ float s[];
  s[threadIdx.x] = threadIdx.x;
  __syncthreads();
  float a = s[(threadIdx.x * 7) & 255];
  for (int i = 0; i < iters; ++i) a = a * 0.999f + 1.0f;
  out[blockIdx.x * 256 + threadIdx.x] = a;
}
int main() {
  float* out;
  (void)hipMalloc(&out, 768 * 256 * 4);
  (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int bytes : {40000, 49024, 51648, 52992, 53248, 53952, 54272, 54592, 54656, 60000}) {
    hipLaunchKernelGGL(k, dim3(768), dim3(256), bytes, 0, out, 20000);
    (void)hipEventRecord(a);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(768), dim3(256), bytes, 0, out, 20000);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    int n = 0;
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k, 256, bytes);
    printf("%6d B: %.3f ms per launch (API: %d per CU)\n", bytes, ms / 5, n);
  }
  return 0;
}
