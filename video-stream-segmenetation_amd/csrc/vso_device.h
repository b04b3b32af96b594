// vso_device.h — device helpers shared by the ONNX-session kernels
// (vso_kernels.hip, vso_conv.hip): the fused activation and the convolution
// epilogue (bias, residual source, activation).
#pragma once
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include "vso_kernels.h"

namespace vso {

typedef float f4 __attribute__((ext_vector_type(4)));

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
