// vss_kernels.hip — gfx950 (CDNA4) kernels for the per-frame segmentation path.
//
// Replaces steps 1-2 of processFrame (/root/reference/client/src/core/
// frameProcessorTest.ts:78-97): tfjs preprocessing (:79-85) + the ORT
// session.run of the segmentation network (:91) + squeezeMaskTo2D (:94-97).
// Network = the build's own layer table (model/spec.json; the reference's
// model_q4f16.onnx is absent).
//
// Layout in HBM: activations NHWC f32 (channel counts are multiples of 16, so
// a pixel's channel vector is whole 64-B segments); frames u8 HWC with a row
// stride; masks [N][Hm][Wm] f32.
//
// Kernels (one launch each, 12 per forward for spec.json):
//   k_stem   : tfjs-legacy bilinear resize + /255 computed on the fly into an
//              LDS tile, fused with the 3x3 s2 stem conv + ReLU6 (VALU).
//   k_block  : one inverted-residual or decoder block.  The hidden (expanded)
//              tensor never touches HBM: the workgroup stages its input tile
//              (+halo) in LDS once, then walks the hidden channels in chunks
//              of 16: expand 1x1 (MFMA) -> dw 3x3 (VALU, LDS) -> project 1x1
//              (MFMA) accumulated in registers across chunks.  Decoder blocks
//              build the (instance-norm+ReLU'd, 2x bilinear upsampled src ++
//              skip) concat tile in the prologue and emit per-tile instance-
//              norm partial sums (deterministic, no atomics).
//   k_head   : norm+ReLU of d3, 1x1 -> logits in LDS, bilinear 2x, sigmoid.
//   k_prep   : standalone preprocess to the NCHW f32 ORT input tensor
//              (frameProcessorTest.ts:85) — bit-exact with the oracle.
#include <hip/hip_runtime.h>

#include "vss_kernels.h"

namespace vss {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ float relu6f(float v) { return fminf(fmaxf(v, 0.f), 6.f); }
__device__ __forceinline__ f4 relu6v(f4 v) {
  return f4{relu6f(v.x), relu6f(v.y), relu6f(v.z), relu6f(v.w)};
}
__device__ __forceinline__ f4 reluv(f4 v) {
  return f4{fmaxf(v.x, 0.f), fmaxf(v.y, 0.f), fmaxf(v.z, 0.f), fmaxf(v.w, 0.f)};
}

// ---------------------------------------------------------------------------
// a2/a3: tfjs 4.22 ResizeBilinear (alignCorners=false, halfPixelCenters=false,
// WebGL program form: f32, ratio = float(inH/outH)) followed by /255.
// Same operation order as oracle/vss_oracle.c:resize_px -> bit-identical.
__device__ __forceinline__ void prep_sample(const uint8_t* __restrict__ f, long rs, int fc, int fh,
                                            int fw, float ry, float rx, int y, int x,
                                            float& r, float& g, float& b) {
  const float fy = (float)y * ry, fx = (float)x * rx;
  const int y0 = (int)floorf(fmaxf(fy, 0.f)), x0 = (int)floorf(fmaxf(fx, 0.f));
  const int y1 = min(fh - 1, (int)ceilf(fy)), x1 = min(fw - 1, (int)ceilf(fx));
  const float dy = fy - (float)y0, dx = fx - (float)x0;
  const uint8_t* t0 = f + (long)y0 * rs;
  const uint8_t* t1 = f + (long)y1 * rs;
  float out[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float tl = t0[x0 * fc + c], tr = t0[x1 * fc + c];
    const float bl = t1[x0 * fc + c], br = t1[x1 * fc + c];
    const float top = __builtin_fmaf(tr - tl, dx, tl);
    const float bot = __builtin_fmaf(br - bl, dx, bl);
    const float v = __builtin_fmaf(bot - top, dy, top);
    out[c] = v / 255.0f;
  }
  r = out[0]; g = out[1]; b = out[2];
}

__global__ __launch_bounds__(256) void k_prep(PrepParams p) {
  const long plane = (long)p.Hm * p.Wm;
  const long total = plane * p.N;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int n = (int)(i / plane);
    const int rem = (int)(i - (long)n * plane);
    const int y = rem / p.Wm, x = rem - y * p.Wm;
    float r, g, b;
    prep_sample(p.frames + (long)n * p.frame_stride, p.row_stride, p.fc, p.fh, p.fw, p.ry, p.rx, y, x,
                r, g, b);
    float* o = p.out + (long)n * 3 * plane + rem;
    o[0] = r;
    o[plane] = g;
    o[2 * plane] = b;
  }
}

// ---------------------------------------------------------------------------
// Stem: output tile 8 x 32 pixels x 16 channels, one pixel per thread.
template <int COUT>
__global__ __launch_bounds__(256) void k_stem(StemParams p) {
  constexpr int TH = 8, TW = 32, IH = 2 * TH + 1, IW = 2 * TW + 1, IWP = IW + 1;
  __shared__ float xs[3][IH][IWP];
  __shared__ float ws[COUT * 27];
  __shared__ float bs[COUT];
  const int tid = threadIdx.x;
  const int n = blockIdx.z, oy0 = blockIdx.y * TH, ox0 = blockIdx.x * TW;
  const uint8_t* f = p.frames + (long)n * p.frame_stride;
  const int iy0 = 2 * oy0 - 1, ix0 = 2 * ox0 - 1;
  for (int i = tid; i < IH * IW; i += 256) {
    const int ly = i / IW, lx = i - ly * IW;
    const int yy = iy0 + ly, xx = ix0 + lx;
    float r = 0.f, g = 0.f, b = 0.f;
    if (yy >= 0 && yy < p.Hm && xx >= 0 && xx < p.Wm)
      prep_sample(f, p.row_stride, p.fc, p.fh, p.fw, p.ry, p.rx, yy, xx, r, g, b);
    xs[0][ly][lx] = r;
    xs[1][ly][lx] = g;
    xs[2][ly][lx] = b;
  }
  for (int i = tid; i < COUT * 27; i += 256) ws[i] = p.w[i];
  if (tid < COUT) bs[tid] = p.b[tid];
  __syncthreads();
  const int ly = tid / TW, lx = tid - ly * TW;
  float acc[COUT];
#pragma unroll
  for (int c = 0; c < COUT; ++c) acc[c] = bs[c];
#pragma unroll
  for (int ci = 0; ci < 3; ++ci)
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const float xv = xs[ci][2 * ly + ky][2 * lx + kx];
#pragma unroll
        for (int c = 0; c < COUT; ++c) acc[c] = __builtin_fmaf(ws[c * 27 + ci * 9 + ky * 3 + kx], xv, acc[c]);
      }
  const int oy = oy0 + ly, ox = ox0 + lx;
  if (oy < p.Ho && ox < p.Wo) {
    f4* o = reinterpret_cast<f4*>(p.y + (((long)n * p.Ho + oy) * p.Wo + ox) * COUT);
#pragma unroll
    for (int q = 0; q < COUT / 4; ++q)
      o[q] = f4{relu6f(acc[4 * q]), relu6f(acc[4 * q + 1]), relu6f(acc[4 * q + 2]), relu6f(acc[4 * q + 3])};
  }
}

// ---------------------------------------------------------------------------
// 16x16 output tile, K = 16 per call:  acc[row][col] += sum_k A[row][k] * B[k][col]
// lane l: r = l & 15, g = l >> 4.  The caller hands lane l
//   a = A[r][4g .. 4g+3]   (weights, row = output channel)
//   b = B[4g .. 4g+3][r]   (activations of pixel r, 4 consecutive channels)
// and gets back acc[i] = D[4g + i][r]  (4 consecutive output channels of pixel r).
template <int PREC> struct AFrag;
template <> struct AFrag<PREC_F32> { using T = f4; };
template <> struct AFrag<PREC_BF16X2> { using T = bf8; };

template <int PREC>
__device__ __forceinline__ typename AFrag<PREC>::T load_a(const void* w, int ldk, int row, int k);

template <>
__device__ __forceinline__ f4 load_a<PREC_F32>(const void* w, int ldk, int row, int k) {
  return *reinterpret_cast<const f4*>(static_cast<const float*>(w) + (long)row * ldk + k);
}
template <>
__device__ __forceinline__ bf8 load_a<PREC_BF16X2>(const void* w, int ldk, int row, int k) {
  // bf16-exact weights: elements 0-3 pair with the activation hi parts,
  // 4-7 (the same 4 weights) with the lo parts.
  const bf4 v = *reinterpret_cast<const bf4*>(static_cast<const __bf16*>(w) + (long)row * ldk + k);
  return bf8{v.x, v.y, v.z, v.w, v.x, v.y, v.z, v.w};
}

template <int PREC>
__device__ __forceinline__ f4 mma16(f4 acc, typename AFrag<PREC>::T a, f4 b);

template <>
__device__ __forceinline__ f4 mma16<PREC_F32>(f4 acc, f4 a, f4 b) {
  // 4 x v_mfma_f32_16x16x4_f32: MFMA j covers channel 4g + j of lane group g.
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b.x, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b.y, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b.z, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b.w, acc, 0, 0, 0);
  return acc;
}
template <>
__device__ __forceinline__ f4 mma16<PREC_BF16X2>(f4 acc, bf8 a, f4 b) {
  // f32 activation x = hi + lo (+ O(2^-17 |x|)); one v_mfma_f32_16x16x32_bf16
  // sums w*hi + w*lo over the 16 real channels (lane group g: k = 8g..8g+7 =
  // channels 4g..4g+3 as hi, then as lo).
  const __bf16 h0 = (__bf16)b.x, h1 = (__bf16)b.y, h2 = (__bf16)b.z, h3 = (__bf16)b.w;
  const __bf16 l0 = (__bf16)(b.x - (float)h0), l1 = (__bf16)(b.y - (float)h1);
  const __bf16 l2 = (__bf16)(b.z - (float)h2), l3 = (__bf16)(b.w - (float)h3);
  const bf8 bb{h0, h1, h2, h3, l0, l1, l2, l3};
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bb, acc, 0, 0, 0);
}

// Fused inverted-residual / decoder block (see header comment).
// LDS (floats): xt [P_in_pad][XS] | hid [P_in_pad][16] (EXPAND) | dwo [2][P_out][16]
//               | nrm [2][cin] (DEC) | st [4][2][cout] (DEC)
template <int MODE, int STRIDE, int PREC>
__global__ __launch_bounds__(256) void k_block(BlockParams p) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int n = blockIdx.z;
  const int TH = p.TH, TW = p.TW;
  const int oy0 = blockIdx.y * TH, ox0 = blockIdx.x * TW;
  const int IH = STRIDE == 2 ? 2 * TH + 1 : TH + 2;
  const int IW = STRIDE == 2 ? 2 * TW + 1 : TW + 2;
  const int iy0 = STRIDE * oy0 - 1, ix0 = STRIDE * ox0 - 1;
  const int P_in = IH * IW, P_in_pad = (P_in + 15) & ~15;
  const int P_out = TH * TW;
  const int CX = MODE == MODE_DEC ? p.cin + p.cskip : p.cin;
  const int XS = CX + 4;
  const int Ho = p.Ho, Wo = p.Wo;

  float* xt = smem;
  float* hid = xt + P_in_pad * XS;
  float* dwo = hid + (MODE == MODE_IR_EXPAND ? P_in_pad * 16 : 0);
  float* nrm = dwo + 2 * P_out * 16;
  float* st = nrm + (MODE == MODE_DEC ? 2 * p.cin : 0);

  // ---- prologue: stage the input tile (+halo), zero outside the image ----
  const int C4 = CX >> 2;
  if constexpr (MODE == MODE_DEC) {
    const int cl = p.cin;
    if (p.norm_in) {
      // instance-norm statistics of the producer, reduced in a fixed order
      for (int c = tid; c < cl; c += 256) {
        const float* pp = p.in_part + (long)n * p.in_tiles * 2 * cl;
        float s = 0.f, q = 0.f;
        for (int t = 0; t < p.in_tiles; ++t) {
          s += pp[(2 * t) * cl + c];
          q += pp[(2 * t + 1) * cl + c];
        }
        const float inv = 1.0f / (float)p.in_hw;
        const float mean = s * inv;
        const float var = fmaxf(q * inv - mean * mean, 0.f);
        const float rstd = 1.0f / sqrtf(var + p.eps);
        const float sc = rstd * p.in_gamma[c];
        nrm[c] = sc;
        nrm[cl + c] = p.in_beta[c] - mean * sc;
      }
      for (int c = tid; c < 4 * 2 * p.cout; c += 256) st[c] = 0.f;
      __syncthreads();
    } else {
      for (int c = tid; c < 4 * 2 * p.cout; c += 256) st[c] = 0.f;
    }
    const int h = p.H, w = p.W;  // low-res src dims (Ho = 2h, Wo = 2w)
    for (int i = tid; i < P_in_pad * C4; i += 256) {
      const int pix = i / C4, c4 = i - pix * C4;
      f4 v = {0.f, 0.f, 0.f, 0.f};
      const int ly = pix / IW, lx = pix - ly * IW;
      const int yy = iy0 + ly, xx = ix0 + lx;
      if (pix < P_in && yy >= 0 && yy < Ho && xx >= 0 && xx < Wo) {
        const int c = 4 * c4;
        if (c < cl) {
          // PyTorch upsample_bilinear2d(scale 2, align_corners=False)
          float sy = ((float)yy + 0.5f) * 0.5f - 0.5f;
          sy = fmaxf(sy, 0.f);
          const int y0 = (int)sy, y1 = y0 + (y0 < h - 1 ? 1 : 0);
          const float ly1 = sy - (float)y0, ly0 = 1.f - ly1;
          float sx = ((float)xx + 0.5f) * 0.5f - 0.5f;
          sx = fmaxf(sx, 0.f);
          const int x0 = (int)sx, x1 = x0 + (x0 < w - 1 ? 1 : 0);
          const float lx1 = sx - (float)x0, lx0 = 1.f - lx1;
          const float* base = p.x + (long)n * h * w * cl + c;
          f4 v00 = *reinterpret_cast<const f4*>(base + ((long)y0 * w + x0) * cl);
          f4 v01 = *reinterpret_cast<const f4*>(base + ((long)y0 * w + x1) * cl);
          f4 v10 = *reinterpret_cast<const f4*>(base + ((long)y1 * w + x0) * cl);
          f4 v11 = *reinterpret_cast<const f4*>(base + ((long)y1 * w + x1) * cl);
          if (p.norm_in) {
            const f4 sc = *reinterpret_cast<const f4*>(nrm + c);
            const f4 sh = *reinterpret_cast<const f4*>(nrm + cl + c);
            v00 = reluv(v00 * sc + sh);
            v01 = reluv(v01 * sc + sh);
            v10 = reluv(v10 * sc + sh);
            v11 = reluv(v11 * sc + sh);
          }
          v = ly0 * (lx0 * v00 + lx1 * v01) + ly1 * (lx0 * v10 + lx1 * v11);
        } else {
          v = *reinterpret_cast<const f4*>(p.skip + (((long)n * Ho + yy) * Wo + xx) * p.cskip + (c - cl));
        }
      }
      *reinterpret_cast<f4*>(xt + pix * XS + 4 * c4) = v;
    }
  } else {
    const int H = p.H, W = p.W;
    for (int i = tid; i < P_in_pad * C4; i += 256) {
      const int pix = i / C4, c4 = i - pix * C4;
      f4 v = {0.f, 0.f, 0.f, 0.f};
      const int ly = pix / IW, lx = pix - ly * IW;
      const int yy = iy0 + ly, xx = ix0 + lx;
      if (pix < P_in && yy >= 0 && yy < H && xx >= 0 && xx < W)
        v = *reinterpret_cast<const f4*>(p.x + (((long)n * H + yy) * W + xx) * p.cin + 4 * c4);
      *reinterpret_cast<f4*>(xt + pix * XS + 4 * c4) = v;
    }
  }
  __syncthreads();

  // ---- main loop over 16-channel chunks of the hidden / concat dim ----
  const int nchunks = p.chid >> 4;
  const int NPB = P_out >> 4, NT = (p.cout >> 4) * NPB;
  const int ldk2 = p.chid;  // project weight row length
  f4 acc[kMaxProjTiles];
#pragma unroll
  for (int j = 0; j < kMaxProjTiles; ++j) acc[j] = f4{0.f, 0.f, 0.f, 0.f};

  const int cg = tid & 3;  // dw: this thread's 4-channel group within the chunk

  for (int ck = 0; ck < nchunks; ++ck) {
    const int c0 = ck << 4;
    const float* src;
    int srcS;
    if constexpr (MODE == MODE_IR_EXPAND) {
      // expand: hid[pix][0..15] = relu6(W1[c0..c0+15][:] . x[pix][:] + b1), 0 outside image
      typename AFrag<PREC>::T aw[4];
      const int nk = p.cin >> 4;
#pragma unroll
      for (int s = 0; s < 4; ++s)
        if (s < nk) aw[s] = load_a<PREC>(p.w1, p.cin, c0 + r, 16 * s + 4 * g);
      const f4 bias = *reinterpret_cast<const f4*>(p.b1 + c0 + 4 * g);
      for (int cb = wave; cb < (P_in_pad >> 4); cb += 4) {
        const int pix = cb * 16 + r;
        f4 d = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 4; ++s)
          if (s < nk) d = mma16<PREC>(d, aw[s], *reinterpret_cast<const f4*>(xt + pix * XS + 16 * s + 4 * g));
        const int ly = pix / IW, lx = pix - ly * IW;
        const int yy = iy0 + ly, xx = ix0 + lx;
        const bool valid = pix < P_in && yy >= 0 && yy < p.H && xx >= 0 && xx < p.W;
        const f4 hv = valid ? relu6v(d + bias) : f4{0.f, 0.f, 0.f, 0.f};
        *reinterpret_cast<f4*>(hid + pix * 16 + 4 * g) = hv;
      }
      __syncthreads();
      src = hid;
      srcS = 16;
    } else {
      src = xt + c0;
      srcS = XS;
    }

    // depthwise 3x3 (VALU): dwo[ck&1][pix][0..15]
    {
      float* dout = dwo + (ck & 1) * P_out * 16;
      const int C = p.chid;
      f4 wk[9];
#pragma unroll
      for (int t = 0; t < 9; ++t) wk[t] = *reinterpret_cast<const f4*>(p.wdw + t * C + c0 + 4 * cg);
      const f4 bb = *reinterpret_cast<const f4*>(p.bdw + c0 + 4 * cg);
      for (int idx = tid; idx < P_out * 4; idx += 256) {
        const int pix = idx >> 2;
        const int ly = pix / TW, lx = pix - ly * TW;
        f4 a = bb;
#pragma unroll
        for (int ky = 0; ky < 3; ++ky)
#pragma unroll
          for (int kx = 0; kx < 3; ++kx) {
            const int sp = (STRIDE * ly + ky) * IW + (STRIDE * lx + kx);
            const f4 v = *reinterpret_cast<const f4*>(src + sp * srcS + 4 * cg);
            a = wk[ky * 3 + kx] * v + a;
          }
        if (p.relu6_dw) a = relu6v(a);
        *reinterpret_cast<f4*>(dout + pix * 16 + 4 * cg) = a;
      }
    }
    __syncthreads();

    // project: acc[tile] += W2[co][c0..c0+15] . dwo[pix][0..15]
    {
      const float* dout = dwo + (ck & 1) * P_out * 16;
#pragma unroll
      for (int j = 0; j < kMaxProjTiles; ++j) {
        const int t = wave + 4 * j;
        if (t < NT) {
          const int cb = t / NPB, pb = t - cb * NPB;
          const auto a = load_a<PREC>(p.w2, ldk2, cb * 16 + r, c0 + 4 * g);
          const f4 b = *reinterpret_cast<const f4*>(dout + (pb * 16 + r) * 16 + 4 * g);
          acc[j] = mma16<PREC>(acc[j], a, b);
        }
      }
    }
    // no barrier: the next chunk writes hid (last read by this chunk's dw,
    // fenced above) and the other dwo buffer (last read two chunks ago).
  }

  // ---- epilogue ----
#pragma unroll
  for (int j = 0; j < kMaxProjTiles; ++j) {
    const int t = wave + 4 * j;
    if (t < NT) {
      const int cb = t / NPB, pb = t - cb * NPB;
      const int pix = pb * 16 + r;
      const int ly = pix / TW, lx = pix - ly * TW;
      const int oy = oy0 + ly, ox = ox0 + lx;
      const bool valid = oy < Ho && ox < Wo;
      const int co = cb * 16 + 4 * g;
      f4 v = acc[j] + *reinterpret_cast<const f4*>(p.b2 + co);
      if (MODE != MODE_DEC && p.residual)
        v += *reinterpret_cast<const f4*>(xt + ((ly + 1) * IW + lx + 1) * XS + co);
      if (valid) *reinterpret_cast<f4*>(p.y + (((long)n * Ho + oy) * Wo + ox) * p.cout + co) = v;
      if constexpr (MODE == MODE_DEC) {
        f4 s = valid ? v : f4{0.f, 0.f, 0.f, 0.f};
        f4 q = s * s;
#pragma unroll
        for (int m = 1; m < 16; m <<= 1) {
          s.x += __shfl_xor(s.x, m); s.y += __shfl_xor(s.y, m);
          s.z += __shfl_xor(s.z, m); s.w += __shfl_xor(s.w, m);
          q.x += __shfl_xor(q.x, m); q.y += __shfl_xor(q.y, m);
          q.z += __shfl_xor(q.z, m); q.w += __shfl_xor(q.w, m);
        }
        if (r == 0) {
          float* sw = st + wave * 2 * p.cout;
          *reinterpret_cast<f4*>(sw + co) += s;
          *reinterpret_cast<f4*>(sw + p.cout + co) += q;
        }
      }
    }
  }
  if constexpr (MODE == MODE_DEC) {
    __syncthreads();
    const int tile = blockIdx.y * p.tiles_x + blockIdx.x;
    float* op = p.out_part + ((long)n * p.tiles_x * p.tiles_y + tile) * 2 * p.cout;
    for (int c = tid; c < 2 * p.cout; c += 256)
      op[c] = ((st[c] + st[2 * p.cout + c]) + st[4 * p.cout + c]) + st[6 * p.cout + c];
  }
}

// ---------------------------------------------------------------------------
// Head: mask tile 16 x 64; logits over the (10 x 34) low-res region in LDS.
__global__ __launch_bounds__(256) void k_head(HeadParams p) {
  constexpr int OTH = 16, OTW = 64, ZR = 10, ZC = 34, ZCP = 35;
  constexpr int CMAX = 64;
  __shared__ float z[ZR][ZCP];
  __shared__ float sc[CMAX], sh[CMAX], wv[CMAX];
  const int tid = threadIdx.x, n = blockIdx.z;
  const int oy0 = blockIdx.y * OTH, ox0 = blockIdx.x * OTW;
  const int h = p.h, w = p.w_, C = p.cin;
  for (int c = tid; c < C; c += 256) {
    const float* pp = p.in_part + (long)n * p.in_tiles * 2 * C;
    float s = 0.f, q = 0.f;
    for (int t = 0; t < p.in_tiles; ++t) {
      s += pp[(2 * t) * C + c];
      q += pp[(2 * t + 1) * C + c];
    }
    const float inv = 1.0f / (float)(h * w);
    const float mean = s * inv;
    const float var = fmaxf(q * inv - mean * mean, 0.f);
    const float rstd = 1.0f / sqrtf(var + p.eps);
    const float scale = rstd * p.gamma[c];
    sc[c] = scale;
    sh[c] = p.beta[c] - mean * scale;
    wv[c] = p.w[c];
  }
  __syncthreads();
  const int zr0 = oy0 / 2 - 1, zc0 = ox0 / 2 - 1;
  for (int i = tid; i < ZR * ZC; i += 256) {
    const int zr = i / ZC, zc = i - zr * ZC;
    const int yy = min(max(zr0 + zr, 0), h - 1), xx = min(max(zc0 + zc, 0), w - 1);
    const float* px = p.x + (((long)n * h + yy) * w + xx) * C;
    float acc = 0.f;
    for (int c = 0; c < C; c += 4) {
      const f4 v = *reinterpret_cast<const f4*>(px + c);
      const f4 a = reluv(v * *reinterpret_cast<const f4*>(sc + c) + *reinterpret_cast<const f4*>(sh + c));
      acc += a.x * wv[c] + a.y * wv[c + 1] + a.z * wv[c + 2] + a.w * wv[c + 3];
    }
    z[zr][zc] = acc + p.b;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < (OTH * OTW) / 256; ++k) {
    const int idx = tid + 256 * k;
    const int ly = idx / OTW, lx = idx - ly * OTW;
    const int oy = oy0 + ly, ox = ox0 + lx;
    if (oy < p.Hm && ox < p.Wm) {
      float sy = ((float)oy + 0.5f) * 0.5f - 0.5f;
      sy = fmaxf(sy, 0.f);
      const int y0 = (int)sy, y1 = y0 + (y0 < h - 1 ? 1 : 0);
      const float ly1 = sy - (float)y0, ly0 = 1.f - ly1;
      float sx = ((float)ox + 0.5f) * 0.5f - 0.5f;
      sx = fmaxf(sx, 0.f);
      const int x0 = (int)sx, x1 = x0 + (x0 < w - 1 ? 1 : 0);
      const float lx1 = sx - (float)x0, lx0 = 1.f - lx1;
      const float v = ly0 * (lx0 * z[y0 - zr0][x0 - zc0] + lx1 * z[y0 - zr0][x1 - zc0]) +
                      ly1 * (lx0 * z[y1 - zr0][x0 - zc0] + lx1 * z[y1 - zr0][x1 - zc0]);
      p.mask[((long)n * p.Hm + oy) * p.Wm + ox] = 1.0f / (1.0f + expf(-v));
    }
  }
}

// ---------------------------------------------------------------------------
// Host-visible launch table (used by vss_capi.hip).
using BlockFn = void (*)(BlockParams);

BlockFn block_kernel(int mode, int stride, int prec) {
#define VSS_SEL(M, S, P) \
  if (mode == M && stride == S && prec == P) return k_block<M, S, P>;
  VSS_SEL(MODE_IR_EXPAND, 1, PREC_F32)
  VSS_SEL(MODE_IR_EXPAND, 2, PREC_F32)
  VSS_SEL(MODE_IR_DIRECT, 1, PREC_F32)
  VSS_SEL(MODE_DEC, 1, PREC_F32)
  VSS_SEL(MODE_IR_EXPAND, 1, PREC_BF16X2)
  VSS_SEL(MODE_IR_EXPAND, 2, PREC_BF16X2)
  VSS_SEL(MODE_IR_DIRECT, 1, PREC_BF16X2)
  VSS_SEL(MODE_DEC, 1, PREC_BF16X2)
#undef VSS_SEL
  return nullptr;
}

void (*stem_kernel16())(StemParams) { return k_stem<16>; }
void (*head_kernel())(HeadParams) { return k_head; }
void (*prep_kernel())(PrepParams) { return k_prep; }

}  // namespace vss
