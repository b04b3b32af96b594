// vss_post.hip — §8(f) row 1: the reference's mask post-processing on the GPU.
//
// The chain processFrame applies to the seam's mask
// (/root/reference/client/src/core/frameProcessorTest.ts:115-169):
//   temporalEMA :218-227 -> morphologicalOpening :644-685 -> jointBilateral3x3
//   :230-266 (guide :315-321) -> refineAlphaOnce :270-313 -> alphaToImageData
//   :204-216.
// The reference computes in JS doubles and stores every intermediate in a
// Float32Array; these kernels do exactly that (double arithmetic, f32 stores,
// no FMA contraction), so they agree with the reference's own code run under
// Node (tests/golden/post_chain.npz) bit for bit up to the last-ulp
// differences of pow() between math libraries.  The guide image (a browser
// canvas resample in the reference) is defined as the model input's
// tfjs-legacy bilinear rounded half up to u8.
//
//   k_post_ema    : per pixel, the EMA recurrence over the batch's consecutive
//                   frames (all loads in flight), state = prevAlpha (:47).
//   k_post_filter : per frame and 8x32 output tile: 3x3 erosion then dilation
//                   (halo 3, the 1-px image border left 0), the guide, the
//                   joint bilateral (weights from a host-built exp table),
//                   refine, u8 alpha.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>

#include "vss_kernels.h"

namespace vss {

__global__ __launch_bounds__(256) void k_post_ema(PostEmaParams p) {
#pragma clang fp contract(off)
  const bool valid = *p.valid != 0;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < p.P; i += (long)gridDim.x * 256) {
    float prev = p.state[i];
    for (int t0 = 0; t0 < p.n; t0 += 8) {
      float x[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) x[u] = p.masks[(long)min(t0 + u, p.n - 1) * p.P + i];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int t = t0 + u;
        if (t < p.n) {
          // temporalEMA: the first frame of a stream passes through and seeds prevAlpha
          const float e = (!valid && t == 0) ? x[u] : (float)(p.a * (double)prev + (1.0 - p.a) * (double)x[u]);
          p.ema[(long)t * p.P + i] = e;
          prev = e;
        }
      }
    }
    p.state[i] = prev;
  }
}

// ---- §8(f) row 4: the face stabiliser's part of the chain ------------------
// Math.round: the nearest integer, ties toward +infinity (exact for every double)
__device__ __forceinline__ double js_round(double x) {
  const double r = floor(x);
  return x - r >= 0.5 ? r + 1.0 : r;
}

// One frame: warpAffineNearest(prevAlpha) (:335-353, invertAffine :323-333)
// blended 0.3 / 0.7 into the raw mask (:102-113), then temporalEMA (:218-227).
__global__ __launch_bounds__(256) void k_post_face_ema(PostFaceEmaParams p) {
#pragma clang fp contract(off)
  const bool valid = !p.first || *p.valid != 0;  // prevAlpha exists
  const FaceFrame f = *p.face;
  const bool warp = f.has_affine && valid;
  double ia11 = 0, ia12 = 0, itx = 0, ia21 = 0, ia22 = 0, ity = 0;
  if (warp) {
    const double a11 = f.affine[0], a12 = f.affine[1], tx = f.affine[2];
    const double a21 = f.affine[3], a22 = f.affine[4], ty = f.affine[5];
    const double det = a11 * a22 - a12 * a21;
    const double d = det != 0.0 ? det : 1e-6;
    ia11 = a22 / d;
    ia12 = -a12 / d;
    ia21 = -a21 / d;
    ia22 = a11 / d;
    itx = -(ia11 * tx + ia12 * ty);
    ity = -(ia21 * tx + ia22 * ty);
  }
  const long P = (long)p.H * p.W;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < P; i += (long)gridDim.x * 256) {
    float base = p.mask[i];
    if (warp) {
      const int x = (int)(i % p.W), y = (int)(i / p.W);
      const double sx = ia11 * x + ia12 * y + itx, sy = ia21 * x + ia22 * y + ity;
      const double xi = js_round(sx), yi = js_round(sy);
      const float w = (xi >= 0 && xi < p.W && yi >= 0 && yi < p.H) ? p.prev[(long)yi * p.W + (long)xi] : 0.f;
      base = (float)((double)w * 0.3 + (double)base * (1.0 - 0.3));
    }
    const float e = valid ? (float)(p.a * (double)p.prev[i] + (1.0 - p.a) * (double)base) : base;
    p.ema[i] = e;
    p.next[i] = e;
  }
}

void launch_post_face_ema(const PostFaceEmaParams& p, hipStream_t s) {
  const int grid = (int)std::min<long>(((long)p.H * p.W + 255) / 256, 2048);
  hipLaunchKernelGGL(k_post_face_ema, dim3(grid), dim3(256), 0, s, p);
}

// facePriorMask (:697-741) of a frame's box, in the reference's doubles
struct Prior {
  double cx, cy, rxd, ryd, thr;
};

__device__ __forceinline__ Prior make_prior(const FaceFrame& f, int W, int H, int fw, int fh) {
#pragma clang fp contract(off)
  const double vw = f.video_w > 0 ? f.video_w : fw, vh = f.video_h > 0 ? f.video_h : fh;
  const double sx = (double)W / vw, sy = (double)H / vh;
  const double x0 = floor(f.box[0] * sx), y0 = floor(f.box[1] * sy);
  const double x1 = ceil(f.box[2] * sx), y1 = ceil(f.box[3] * sy);
  Prior q;
  q.cx = (x0 + x1) / 2;
  q.cy = (y0 + y1) / 2;
  const double rx = (x1 - x0) * 0.56, ry = (y1 - y0) * 0.70;
  const double pad = fmax(4.0, floor((double)min(W, H) * 0.02));
  q.rxd = fmax(1e-6, rx);
  q.ryd = fmax(1e-6, ry);
  q.thr = 1 - (pad / fmax(rx, ry));
  return q;
}

__device__ __forceinline__ float prior_at(const Prior& q, int x, int y) {
#pragma clang fp contract(off)
  const double dx = (x - q.cx) / q.rxd, dy = (y - q.cy) / q.ryd;
  const double d2 = dx * dx + dy * dy;
  double v = 0;
  if (d2 <= 1) {
    const double t = sqrt(fmax(0.0, fmin(1.0, d2)));
    v = 0.5 - 0.5 * cos(M_PI * (1 - t));
    if (d2 > q.thr) v = fmax(v, 0.25);
  }
  return (float)v;
}

// guide pixel: tfjs-legacy bilinear of the frame at (y, x), rounded half up to u8
__device__ __forceinline__ unsigned guide_rgb(const uint8_t* f, long rs, int fc, int fh, int fw, float ry, float rx,
                                              int y, int x) {
#pragma clang fp contract(off)
  const float fy = (float)y * ry, fx = (float)x * rx;
  const int y0 = (int)floorf(fmaxf(fy, 0.f)), x0 = (int)floorf(fmaxf(fx, 0.f));
  const int y1 = min(fh - 1, (int)ceilf(fy)), x1 = min(fw - 1, (int)ceilf(fx));
  const float dy = fy - (float)y0, dx = fx - (float)x0;
  const uint8_t* t0 = f + (long)y0 * rs;
  const uint8_t* t1 = f + (long)y1 * rs;
  unsigned rgb = 0;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float tl = t0[x0 * fc + c], tr = t0[x1 * fc + c], bl = t1[x0 * fc + c], br = t1[x1 * fc + c];
    const float top = __builtin_fmaf(tr - tl, dx, tl);
    const float bot = __builtin_fmaf(br - bl, dx, bl);
    const float v = __builtin_fmaf(bot - top, dy, top);
    rgb |= (unsigned)floorf(v + 0.5f) << (8 * c);
  }
  return rgb;
}

// FACE: the frame may carry a face box: its prior, the 3x3 closing inside it
// (morphologicalClosingInPrior :743-787) after the opening, and the prior's
// clamp in refine; the tile then needs a halo of 5 (erosion, dilation,
// dilation, erosion, bilateral).
template <int TH, int TW, bool FACE>
__global__ __launch_bounds__(256) void k_post_filter(PostFilterParams p) {
#pragma clang fp contract(off)
  constexpr int HE = FACE ? 5 : 3;                                       // halo of the EMA tile
  constexpr int EH = TH + 2 * HE, EW = TW + 2 * HE;                      // EMA        (halo HE)
  constexpr int RH = EH - 2, RW = EW - 2;                                // erosion    (halo HE-1)
  constexpr int OH = RH - 2, OW = RW - 2;                                // opening    (halo HE-2)
  constexpr int DH = FACE ? TH + 4 : 1, DW = FACE ? TW + 4 : 1;          // closing's dilation / prior (halo 2)
  constexpr int CH = FACE ? TH + 2 : 1, CW = FACE ? TW + 2 : 1;          // closing    (halo 1)
  __shared__ float E[EH][EW];
  __shared__ float R[RH][RW];
  __shared__ float O[OH][OW];
  __shared__ float D[DH][DW];
  __shared__ float PR[DH][DW];
  __shared__ float C[CH][CW];
  __shared__ unsigned G[TH + 2][TW + 2];
  const int tid = threadIdx.x, t = blockIdx.z;
  const int y0 = blockIdx.y * TH, x0 = blockIdx.x * TW;
  const int H = p.H, W = p.W;
  const float* e = p.ema + (long)t * H * W;
  bool has_prior = false;
  Prior q{};
  if constexpr (FACE) {
    has_prior = p.faces[t].has_box != 0;
    if (has_prior) q = make_prior(p.faces[t], W, H, p.fw, p.fh);
  }
  // EMA values on the halo region (outside the image: never read as data)
  for (int i = tid; i < EH * EW; i += 256) {
    const int ly = i / EW, lx = i % EW;
    const int yy = min(max(y0 - HE + ly, 0), H - 1), xx = min(max(x0 - HE + lx, 0), W - 1);
    E[ly][lx] = e[(long)yy * W + xx];
  }
  // guide on the halo-1 region
  if (p.use_bilateral) {
    const uint8_t* f = p.frames + (long)t * p.frame_stride;
    for (int i = tid; i < (TH + 2) * (TW + 2); i += 256) {
      const int ly = i / (TW + 2), lx = i % (TW + 2);
      const int yy = y0 - 1 + ly, xx = x0 - 1 + lx;
      G[ly][lx] = (yy >= 0 && yy < H && xx >= 0 && xx < W)
                      ? guide_rgb(f, p.row_stride, p.fc, p.fh, p.fw, p.ry, p.rx, yy, xx) : 0u;
    }
  }
  if (has_prior)
    for (int i = tid; i < DH * DW; i += 256) {
      const int ly = i / DW, lx = i % DW;
      PR[ly][lx] = prior_at(q, x0 - 2 + lx, y0 - 2 + ly);
    }
  __syncthreads();
  // erosion (3x3 min, start 1.0) on the interior, 0 on the image border
  for (int i = tid; i < RH * RW; i += 256) {
    const int ly = i / RW, lx = i % RW;
    const int yy = y0 - (HE - 1) + ly, xx = x0 - (HE - 1) + lx;
    float m = 0.f;
    if (yy >= 1 && yy < H - 1 && xx >= 1 && xx < W - 1) {
      m = 1.0f;
#pragma unroll
      for (int dy = 0; dy < 3; ++dy)
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) m = E[ly + dy][lx + dx] < m ? E[ly + dy][lx + dx] : m;
    }
    R[ly][lx] = m;
  }
  __syncthreads();
  // dilation (3x3 max, start 0.0) of the erosion
  for (int i = tid; i < OH * OW; i += 256) {
    const int ly = i / OW, lx = i % OW;
    const int yy = y0 - (HE - 2) + ly, xx = x0 - (HE - 2) + lx;
    float m = 0.f;
    if (yy >= 1 && yy < H - 1 && xx >= 1 && xx < W - 1) {
#pragma unroll
      for (int dy = 0; dy < 3; ++dy)
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) m = R[ly + dy][lx + dx] > m ? R[ly + dy][lx + dx] : m;
    }
    O[ly][lx] = m;
  }
  __syncthreads();
  if constexpr (FACE) {
    if (has_prior) {
      // closing inside the prior: 3x3 max where prior > 0 (else the opening),
      // then 3x3 min where prior > 0 (else the dilation); the border stays 0
      for (int i = tid; i < DH * DW; i += 256) {
        const int ly = i / DW, lx = i % DW;
        const int yy = y0 - 2 + ly, xx = x0 - 2 + lx;
        float m = 0.f;
        if (yy >= 1 && yy < H - 1 && xx >= 1 && xx < W - 1) {
          if (PR[ly][lx] <= 0.f) {
            m = O[ly + 1][lx + 1];
          } else {
#pragma unroll
            for (int dy = 0; dy < 3; ++dy)
#pragma unroll
              for (int dx = 0; dx < 3; ++dx) m = O[ly + dy][lx + dx] > m ? O[ly + dy][lx + dx] : m;
          }
        }
        D[ly][lx] = m;
      }
      __syncthreads();
      for (int i = tid; i < CH * CW; i += 256) {
        const int ly = i / CW, lx = i % CW;
        const int yy = y0 - 1 + ly, xx = x0 - 1 + lx;
        float m = 0.f;
        if (yy >= 1 && yy < H - 1 && xx >= 1 && xx < W - 1) {
          if (PR[ly + 1][lx + 1] <= 0.f) {
            m = D[ly + 1][lx + 1];
          } else {
            m = 1.0f;
#pragma unroll
            for (int dy = 0; dy < 3; ++dy)
#pragma unroll
              for (int dx = 0; dx < 3; ++dx) m = D[ly + dy][lx + dx] < m ? D[ly + dy][lx + dx] : m;
          }
        }
        C[ly][lx] = m;
      }
    } else {
      for (int i = tid; i < CH * CW; i += 256) {
        const int ly = i / CW, lx = i % CW;
        C[ly][lx] = O[ly + 2][lx + 2];
      }
    }
    __syncthreads();
  }
  // the chain's value at halo 1: the opening, or the closing inside the prior
  auto A = [&](int ly, int lx) -> float {
    if constexpr (FACE) return C[ly][lx];
    else return O[ly][lx];
  };
  for (int i = tid; i < TH * TW; i += 256) {
    const int ly = i / TW, lx = i % TW;
    const int y = y0 + ly, x = x0 + lx;
    if (y >= H || x >= W) continue;
    float v = A(ly + 1, lx + 1);
    if (p.use_bilateral) {
      const unsigned c0 = G[ly + 1][lx + 1];
      const int r0 = c0 & 255, g0 = (c0 >> 8) & 255, b0 = (c0 >> 16) & 255;
      double sw = 0.0, sa = 0.0;
#pragma unroll
      for (int dy = -1; dy <= 1; ++dy) {
        if (y + dy < 0 || y + dy >= H) continue;
#pragma unroll
        for (int dx = -1; dx <= 1; ++dx) {
          if (x + dx < 0 || x + dx >= W) continue;
          const unsigned c = G[ly + 1 + dy][lx + 1 + dx];
          const int dr = (int)(c & 255) - r0, dg = (int)((c >> 8) & 255) - g0, db = (int)((c >> 16) & 255) - b0;
          const double wgt = p.sw[dx * dx + dy * dy] * p.rtab[dr * dr + dg * dg + db * db];
          sw += wgt;
          sa += wgt * (double)A(ly + 1 + dy, lx + 1 + dx);
        }
      }
      if (sw > 0.0) v = (float)(sa / sw);
    }
    // refineAlphaOnce (:270-313), with the face prior's clamp when present
    double r = v;
    if (r <= p.lo) r = 0.0;
    else if (r >= p.hi) r = 1.0;
    else r = pow((r - p.lo) / p.denom, p.gamma);
    if (has_prior) {
      const double pv = PR[ly + 2][lx + 2];
      if (pv > 0.25) r = fmax(r, fmin(1.0, 0.55 * pv + 0.15));
      else if (pv > 0) r = fmin(r, 0.35 + 0.15 * pv);
    }
    const float rf = (float)r;
    const long o = ((long)t * H + y) * W + x;
    if (p.alpha) p.alpha[o] = rf;
    if (p.alpha_u8) {
      const double a = rf < 0.f ? 0.0 : (rf > 1.f ? 1.0 : (double)rf);
      p.alpha_u8[o] = (uint8_t)floor(a * 255.0 + 0.5);  // Math.round(a * 255)
    }
  }
}

// destination-in compositing (frameProcessorTest.ts:170-178, output canvas =
// the video's size, main.ts:43-44): the frame's colour, alpha = the half-pixel
// bilinear of the mask's u8 alpha at frame resolution, rounded half up; colour
// 0 where alpha is 0 (a canvas stores premultiplied colour).  Thread = 4
// consecutive pixels of a row: one 16-B RGBA store; the alpha taps come from
// the L2-resident mask.  A tile of 256 x 4 pixels per workgroup.
__device__ __forceinline__ void up_coord(int o, float scale, int in, int& i0, int& i1, float& l) {
#pragma clang fp contract(off)
  float s = ((float)o + 0.5f) * scale - 0.5f;
  s = fmaxf(s, 0.f);
  const int a = min((int)s, in - 1);
  i0 = a;
  i1 = a < in - 1 ? a + 1 : a;
  l = s - (float)a;
}

__global__ __launch_bounds__(256) void k_composite(CompositeParams p) {
#pragma clang fp contract(off)
  const int t = blockIdx.z;
  const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
  const int x0 = (blockIdx.x * 64 + (threadIdx.x & 63)) * 4;
  if (y >= p.fh || x0 >= p.fw) return;
  int ya, yb;
  float ly;
  up_coord(y, p.sy, p.H, ya, yb, ly);
  const uint8_t* a = p.alpha + (long)t * p.H * p.W;
  const uint8_t* ra = a + (long)ya * p.W;
  const uint8_t* rb = a + (long)yb * p.W;
  const uint8_t* f = p.frames + (long)t * p.frame_stride + (long)y * p.row_stride;
  uint32_t px[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int x = min(x0 + k, p.fw - 1);
    int xa, xb;
    float lx;
    up_coord(x, p.sx, p.W, xa, xb, lx);
    const float a00 = ra[xa], a01 = ra[xb], a10 = rb[xa], a11 = rb[xb];
    const float top = __builtin_fmaf(a01 - a00, lx, a00), bot = __builtin_fmaf(a11 - a10, lx, a10);
    const uint32_t A = (uint32_t)floorf(__builtin_fmaf(bot - top, ly, top) + 0.5f);
    const uint8_t* q = f + (long)x * p.fc;
    const uint32_t rgb = (uint32_t)q[0] | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16);
    px[k] = A ? (rgb | (A << 24)) : 0u;
  }
  uint8_t* o = p.out + (long)t * p.out_frame_stride + (long)y * p.out_row_stride + (long)x0 * 4;
  if (x0 + 4 <= p.fw && (reinterpret_cast<uintptr_t>(o) & 15) == 0) {
    *reinterpret_cast<uint4*>(o) = make_uint4(px[0], px[1], px[2], px[3]);
  } else {
    for (int k = 0; k < 4 && x0 + k < p.fw; ++k) reinterpret_cast<uint32_t*>(o)[k] = px[k];
  }
}

// 4 output pixels per thread, one 16-B store; the taps' rows are L2-resident.
__global__ __launch_bounds__(256) void k_upmask(UpmaskParams p) {
#pragma clang fp contract(off)
  const int t = blockIdx.z;
  const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
  const int x0 = (blockIdx.x * 64 + (threadIdx.x & 63)) * 4;
  if (y >= p.fh || x0 >= p.fw) return;
  int ya, yb;
  float ly;
  up_coord(y, p.sy, p.H, ya, yb, ly);
  const float* ra = p.masks + ((long)t * p.H + ya) * p.W;
  const float* rb = p.masks + ((long)t * p.H + yb) * p.W;
  float v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int x = min(x0 + k, p.fw - 1);
    int xa, xb;
    float lx;
    up_coord(x, p.sx, p.W, xa, xb, lx);
    const float top = __builtin_fmaf(ra[xb] - ra[xa], lx, ra[xa]), bot = __builtin_fmaf(rb[xb] - rb[xa], lx, rb[xa]);
    v[k] = __builtin_fmaf(bot - top, ly, top);
  }
  float* o = p.out + ((long)t * p.fh + y) * p.fw + x0;
  if (x0 + 4 <= p.fw && (reinterpret_cast<uintptr_t>(o) & 15) == 0) {
    *reinterpret_cast<float4*>(o) = make_float4(v[0], v[1], v[2], v[3]);
  } else {
    for (int k = 0; k < 4 && x0 + k < p.fw; ++k) o[k] = v[k];
  }
}

void launch_upmask(const UpmaskParams& p, int n, hipStream_t s) {
  hipLaunchKernelGGL(k_upmask, dim3((p.fw + 255) / 256, (p.fh + 3) / 4, n), dim3(256), 0, s, p);
}

void launch_composite(const CompositeParams& p, int n, hipStream_t s) {
  hipLaunchKernelGGL(k_composite, dim3((p.fw + 255) / 256, (p.fh + 3) / 4, n), dim3(256), 0, s, p);
}

constexpr int kPostTH = 8, kPostTW = 32;

void launch_post_ema(const PostEmaParams& p, hipStream_t s) {
  const int grid = (int)std::min<long>((p.P + 255) / 256, 2048);
  hipLaunchKernelGGL(k_post_ema, dim3(grid), dim3(256), 0, s, p);
}

void launch_post_filter(const PostFilterParams& p, int n, hipStream_t s) {
  const dim3 grid((p.W + kPostTW - 1) / kPostTW, (p.H + kPostTH - 1) / kPostTH, n);
  if (p.faces)
    hipLaunchKernelGGL((k_post_filter<kPostTH, kPostTW, true>), grid, dim3(256), 0, s, p);
  else
    hipLaunchKernelGGL((k_post_filter<kPostTH, kPostTW, false>), grid, dim3(256), 0, s, p);
}

}  // namespace vss
