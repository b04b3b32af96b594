// vso_device.h — device helpers shared by the ONNX-session kernels
// (vso_kernels.hip, vso_conv.hip): the fused activation and the convolution
// epilogue (bias, residual source, activation).
#pragma once
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include "vso_kernels.h"

namespace vso {

typedef float f4 __attribute__((ext_vector_type(4)));

// The same pointer, provably wave-uniform (in SGPRs) for a buffer descriptor
// (the caller guarantees it is uniform; hipcc would otherwise waterfall every
// buffer op whose descriptor it cannot prove uniform).
__device__ __forceinline__ const void* uniform_ptr(const void* p) {
  const unsigned long long v = reinterpret_cast<unsigned long long>(p);
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
  return reinterpret_cast<const void*>(((unsigned long long)hi << 32) | lo);
}

// XCD-contiguous work items.  The dispatcher deals linear workgroup b to
// XCD b % 8; xcd_item(b, G) gives XCD x the contiguous items
// [x q + min(x, r), ...) of q = G / 8, r = G % 8, so neighbouring tiles — the
// halo rows they share, the 128-B lines their rows straddle — sit on one L2
// instead of eight (MODNet's k_conv_tile 3x3 at 72x128: 4.8x -> 1.0x the
// input's bytes fetched past L2).  A bijection on [0, G): the same items and
// arithmetic, placed differently.  (Measured and not kept on k_ir_b16 and the
// fused depthwise -> 1x1 k_conv_pw: fetched bytes 1.3-3x lower, no faster —
// latency-bound there — and MODNet b8 0.5 % slower, profiles/r06/r06u.)
__device__ __forceinline__ int xcd_item(int b, int G) {
  const int q = G >> 3, r = G & 7, x = b & 7;
  return x * q + min(x, r) + (b >> 3);
}

__device__ __forceinline__ float act_apply(float v, int act, float a0, float a1, const float* slope, int ch,
                                           int slope_stride) {
  switch (act) {
    case ACT_RELU: return fmaxf(v, 0.f);
    case ACT_CLIP: return fminf(fmaxf(v, a0), a1);
    case ACT_PRELU: return v < 0.f ? v * slope[ch * slope_stride] : v;
    case ACT_LEAKY: return v < 0.f ? v * a0 : v;
    case ACT_SIGMOID: return 1.f / (1.f + expf(-v));
    case ACT_TANH: return tanhf(v);
    case ACT_F16: return __half2float(__float2half_rn(v));
    default: return v;
  }
}

// The fused residual source's value for output (ch, idx) — n / pix: the
// output's image and pixel (res_mode 1 / 2 are addressed by them).
__device__ __forceinline__ float residual(const Epilogue& e, int ch, long idx, int n, int pix) {
  if (e.res_mode == 0) return e.res[idx];
  if (ch >= e.res_c) return 0.f;
  const long plane = (long)n * e.res_c + ch;
  if (e.res_mode == 1) return e.res[plane * e.out_hw + pix];
  const int y = pix / e.out_w, x = pix - y * e.out_w;
  const float* b = e.res + (plane * e.res_h + 2 * y) * e.res_w + 2 * x;
  return fmaxf(fmaxf(b[0], b[1]), fmaxf(b[e.res_w], b[e.res_w + 1]));
}

// o[k] = f(k, o[k]) for every k, in a loop that is NOT unrolled (one copy of
// f's code), each element moved in and out of the loop by selects over the
// array (a dynamic register index would go through scratch): for the rare
// epilogue forms, whose code inlined per output set whole kernels' register
// allocation.
template <int N, class F>
__device__ __forceinline__ void each_rare(float (&o)[N], F f) {
#pragma unroll 1
  for (int k = 0; k < N; ++k) {
    float v = o[0];
#pragma unroll
    for (int t = 1; t < N; ++t) v = k == t ? o[t] : v;
    v = f(k, v);
#pragma unroll
    for (int t = 0; t < N; ++t) o[t] = k == t ? v : o[t];
  }
}

// The activation over all N outputs a lane holds (channel ch_of(k) of output
// k): ONE uniform switch, then a loop per case.  A per-output switch (as in
// epilogue() below) inlined into each of k_conv_tile's 32 outputs per lane
// made a 17k-instruction kernel whose tanhf / expf paths set its register
// allocation (300+ VGPRs: one wave per SIMD).
template <int N, class ChOf>
__device__ __forceinline__ void act_block(float (&o)[N], ChOf ch_of, const Epilogue& e) {
  auto on = [&](int k) { return !(e.act_c_end && ch_of(k) >= e.act_c_end); };
  switch (e.act) {
    case ACT_RELU:
#pragma unroll
      for (int k = 0; k < N; ++k) o[k] = on(k) ? fmaxf(o[k], 0.f) : o[k];
      break;
    case ACT_CLIP:
#pragma unroll
      for (int k = 0; k < N; ++k) o[k] = on(k) ? fminf(fmaxf(o[k], e.a0), e.a1) : o[k];
      break;
    case ACT_NONE:
      break;
    case ACT_SIGMOID:
      if constexpr (N <= 16) {  // (the matte's last 1x1: a whole 288x512 layer of them)
#pragma unroll
        for (int k = 0; k < N; ++k) o[k] = on(k) ? 1.f / (1.f + expf(-o[k])) : o[k];
        break;
      }
      [[fallthrough]];
    default:
      each_rare(o, [&](int k, float v) {
        return on(k) ? act_apply(v, e.act, e.a0, e.a1, e.slope, ch_of(k), e.slope_stride) : v;
      });
  }
}

// n / pix: the output's image and pixel (the conv kernels know them; the
// fused residual sources of res_mode 1 / 2 are addressed by them)
__device__ __forceinline__ float epilogue(const Epilogue& e, float v, int ch, long idx, int n, int pix) {
  if (e.bias) v += e.bias[ch];
  if (e.res) {
    if (e.res_mode == 0) {
      v += e.res[idx];
    } else if (ch < e.res_c) {
      const long plane = (long)n * e.res_c + ch;
      if (e.res_mode == 1) {
        v += e.res[plane * e.out_hw + pix];
      } else {
        const int y = pix / e.out_w, x = pix - y * e.out_w;
        const float* b = e.res + (plane * e.res_h + 2 * y) * e.res_w + 2 * x;
        v += fmaxf(fmaxf(b[0], b[1]), fmaxf(b[e.res_w], b[e.res_w + 1]));
      }
    }
  }
  if (e.act_c_end && ch >= e.act_c_end) return v;
  return act_apply(v, e.act, e.a0, e.a1, e.slope, ch, e.slope_stride);
}

}  // namespace vso
