// Workgroups per CU that dynamic LDS allows (hipOccupancyMaxActiveBlocksPerMultiprocessor),
// to find gfx950's LDS allocation granule.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ __launch_bounds__(256) void k(float* p) {
  extern __shared__ float s[];
  s[threadIdx.x] = 1.f;
  __syncthreads();
  if (p) p[threadIdx.x] = s[255 - threadIdx.x];
}
int main() {
  (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  int last = -1;
  for (int bytes = 40000; bytes <= 84000; bytes += 64) {
    int n = 0;
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k, 256, bytes);
    if (n != last) printf("%d bytes -> %d per CU\n", bytes, n);
    last = n;
  }
  return 0;
}
