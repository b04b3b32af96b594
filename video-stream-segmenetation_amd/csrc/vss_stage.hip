// vss_stage.hip — host -> HBM staging of only the frame rows the seam reads.
//
// The tfjs-legacy resize (frameProcessorTest.ts:80; prep_tap in
// vss_kernels.hip) of an fh-row frame to Hm model rows reads rows
// y0 = floor(y * ry) and y1 = min(fh - 1, ceil(y * ry)) for y < Hm — about
// 1.7 Hm rows once fh / Hm > 2 (240 of 480 rows at 640x480 -> 144x256, 216 of
// 1080 at 1080p), and the post chain's guide image reads the same rows.  The
// queued host path therefore moves just those rows across PCIe: k_fetch_rows
// reads them from the pinned staging buffer (device loads of host memory, 16 B
// per lane where the rows allow) and writes each to its own place in the
// slot's HBM frame buffer, so every kernel after it addresses the frames
// exactly as if the whole frame had been copied.
#include <hip/hip_runtime.h>

#include "vss_kernels.h"

namespace vss {

// grid (rows, frames): one workgroup per (row, frame)
__global__ __launch_bounds__(256) void k_fetch_rows(FetchRowsParams p) {
  const int row = p.rows[blockIdx.x];
  const long off = (long)blockIdx.y * p.frame_stride + (long)row * p.row_stride;
  const uint8_t* src = p.src + off;
  uint8_t* dst = p.dst + off;
  if (p.vec16) {
    const uint4* s = reinterpret_cast<const uint4*>(src);
    uint4* d = reinterpret_cast<uint4*>(dst);
    const int n16 = p.row_bytes >> 4;
    // every load of the row in flight before the first store
    uint4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = (int)threadIdx.x + 256 * u;
      if (i < n16) v[u] = s[i];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = (int)threadIdx.x + 256 * u;
      if (i < n16) d[i] = v[u];
    }
    for (int i = (int)threadIdx.x + 1024; i < n16; i += 256) d[i] = s[i];
  } else {
    for (int i = threadIdx.x; i < p.row_bytes; i += 256) dst[i] = src[i];
  }
}

void launch_fetch_rows(const FetchRowsParams& p, int nrows, int nframes, hipStream_t s) {
  hipLaunchKernelGGL(k_fetch_rows, dim3(nrows, nframes), dim3(256), 0, s, p);
}

}  // namespace vss
