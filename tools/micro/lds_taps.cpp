// The decoder's depthwise tap reads from LDS (k_block MODE_DEC, 6x16 tile, 48
// channels): lane (r, g) = pixel block_pix(r) of a 16-pixel block, channels
// c0 + 4g..+3; 9 taps per pixel per 16-channel chunk.  Times the read loop for
// a per-pixel stride XS (floats) with and without the lane permutation.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f4 __attribute__((ext_vector_type(4)));
template <int XS, int PERM>
__global__ __launch_bounds__(256) void k(float* out, int reps) {
  extern __shared__ __attribute__((aligned(16))) float xt[];
  constexpr int TW = 16, TH = 6, IW = TW + 2, IH = TH + 2, NCH = 3;
  for (int i = threadIdx.x; i < IH * IW * XS; i += 256) xt[i] = (float)(i & 7);
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, r = lane & 15, g = lane >> 4;
  const int br = PERM ? (r < 4 ? r : (r < 12 ? r + 4 : r - 8)) : r;
  f4 acc = {0, 0, 0, 0};
  for (int it = 0; it < reps; ++it)
    for (int ck = 0; ck < NCH; ++ck)
      for (int pb = wave; pb < TH; pb += 4) {
        const int pix = pb * 16 + br, ly = pix / TW, lx = pix % TW;
#pragma unroll
        for (int ky = 0; ky < 3; ++ky)
#pragma unroll
          for (int kx = 0; kx < 3; ++kx)
            acc += *reinterpret_cast<const f4*>(xt + ((ly + ky) * IW + lx + kx) * XS + ck * 16 + 4 * g);
      }
  out[blockIdx.x * 256 + threadIdx.x] = acc.x + acc.y + acc.z + acc.w;
}
template <int XS, int PERM>
void run(float* out) {
  const int lds = 8 * 18 * XS * 4;
  hipFuncSetAttribute((const void*)k<XS, PERM>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  for (int w = 0; w < 2; ++w) hipLaunchKernelGGL((k<XS, PERM>), dim3(768), dim3(256), lds, 0, out, 50);
  hipEventRecord(a);
  hipLaunchKernelGGL((k<XS, PERM>), dim3(768), dim3(256), lds, 0, out, 200);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  printf("XS %d perm %d: %.3f ms\n", XS, PERM, ms);
}
int main() {
  float* out;
  hipMalloc(&out, 768 * 256 * 4);
  run<52, 0>(out); run<52, 1>(out); run<56, 0>(out); run<56, 1>(out); run<60, 0>(out); run<64, 0>(out);
  run<52, 0>(out); run<56, 1>(out);
  return 0;
}
