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
//              tensor never touches HBM: the workgroup stages the layer's
//              weights and its input tile (+halo) in LDS once; its 4 waves then
//              run independent units of 16 hidden channels: expand 1x1 (MFMA)
//              -> dw 3x3 (VALU, LDS) -> project 1x1 (MFMA) accumulated in
//              registers; the waves' partial sums meet in LDS in a fixed order.
//              Decoder blocks build the (instance-norm+ReLU'd, 2x bilinear
//              upsampled src ++ skip) concat tile in the prologue and emit
//              per-tile instance-norm partial sums (deterministic, no atomics).
//   k_head   : norm+ReLU of d3, 1x1 -> logits in LDS, bilinear 2x, sigmoid.
//   k_prep   : standalone preprocess to the NCHW f32 ORT input tensor
//              (frameProcessorTest.ts:85) — bit-exact with the oracle.
#include <hip/hip_runtime.h>

#include <vector>

#include "vss_kernels.h"

namespace vss {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef unsigned u4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));

// Activation tensors (and the instance-norm accumulators).  Layer launches use
// plain loads and stores.  The persistent forward (COH = true) hands them from
// workgroup to workgroup inside one launch, so there EVERY store and load of
// them is `sc1` — write-through stores, L1-bypassing loads — through a buffer
// descriptor built from a wave-uniform base (cdna_hip_programming.md
// Guideline 16, R1 with the sc1-load consumer form): no release or acquire
// fence per hand-off.  Indices are in floats; offsets stay below 2 GiB.
// The same pointer, provably wave-uniform (in SGPRs): the caller guarantees
// it is uniform; hipcc would otherwise waterfall every buffer op whose
// descriptor it cannot prove uniform (cdna_hip_programming.md T20).
__device__ __forceinline__ const void* uniform_ptr(const void* p) {
  const unsigned long long v = reinterpret_cast<unsigned long long>(p);
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
  return reinterpret_cast<const void*>(((unsigned long long)hi << 32) | lo);
}

template <bool COH>
struct Gm {
  const float* b;
  __amdgpu_buffer_rsrc_t r;
  __device__ __forceinline__ explicit Gm(const float* base) : b(base) {
    if constexpr (COH)
      r = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(uniform_ptr(base)), 0, 0x7FFFFFF0, 0x00020000);
  }
  __device__ __forceinline__ f4 ld(long i) const {
    if constexpr (COH)
      return __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)(i * 4), 0, 16));
    else
      return *reinterpret_cast<const f4*>(b + i);
  }
  // 32-bit element offset off a wave-uniform base: one global_load with an
  // SGPR base and a 32-bit VGPR byte offset, no 64-bit address arithmetic
  // (every activation tensor of a frame is far below 4 GiB)
  __device__ __forceinline__ f4 ldu(unsigned i) const {
    if constexpr (COH)
      return ld((long)i);
    else
      return *reinterpret_cast<const f4*>(reinterpret_cast<const char*>(b) + (i << 2));
  }
  __device__ __forceinline__ void st(long i, f4 v) const {
    if constexpr (COH)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, v), r, (int)(i * 4), 0, 16);
    else
      *reinterpret_cast<f4*>(const_cast<float*>(b) + i) = v;
  }
  __device__ __forceinline__ void st1(long i, float v) const {
    if constexpr (COH)
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, (int)(i * 4), 0, 16);
    else
      const_cast<float*>(b)[i] = v;
  }
};

// ReLU6 / ReLU as one v_med3_f32 per element (fminf(fmaxf()) compiles to a
// NaN-quieting v_max_f32 x, x, x plus the med3 in IEEE mode; the activations
// here are never NaN, and for every other input the value is the same)
__device__ __forceinline__ float relu6f(float v) { return __builtin_amdgcn_fmed3f(v, 0.f, 6.f); }
__device__ __forceinline__ f4 relu6v(f4 v) {
  return f4{relu6f(v.x), relu6f(v.y), relu6f(v.z), relu6f(v.w)};
}
// clamp to [0, lim]: ReLU6 where lim = 6, zero where lim = 0 (padding pixels)
__device__ __forceinline__ f4 clampv(f4 v, float lim) {
  return f4{__builtin_amdgcn_fmed3f(v.x, 0.f, lim), __builtin_amdgcn_fmed3f(v.y, 0.f, lim),
            __builtin_amdgcn_fmed3f(v.z, 0.f, lim), __builtin_amdgcn_fmed3f(v.w, 0.f, lim)};
}
__device__ __forceinline__ f4 reluv(f4 v) {
  constexpr float inf = __builtin_inff();
  return f4{__builtin_amdgcn_fmed3f(v.x, 0.f, inf), __builtin_amdgcn_fmed3f(v.y, 0.f, inf),
            __builtin_amdgcn_fmed3f(v.z, 0.f, inf), __builtin_amdgcn_fmed3f(v.w, 0.f, inf)};
}

// ---------------------------------------------------------------------------
// a2/a3: tfjs 4.22 ResizeBilinear (alignCorners=false, halfPixelCenters=false,
// WebGL program form: f32, ratio = float(inH/outH)) followed by /255.
// Same operation order as oracle/vss_oracle.c:resize_px -> bit-identical.
struct PrepTap {
  const uint8_t* t0;  // row y0
  const uint8_t* t1;  // row y1
  int o0, o1;         // byte offsets of columns x0, x1
  float dy, dx;
};

__device__ __forceinline__ PrepTap prep_tap(const uint8_t* __restrict__ f, long rs, int fc, int fh, int fw,
                                            float ry, float rx, int y, int x) {
  // hipcc contracts by default: keep `fy = y*ry` rounded before `fy - y0`
  // (an FMA there changes dy); the lerps below are explicit FMAs on both sides.
#pragma clang fp contract(off)
  const float fy = (float)y * ry, fx = (float)x * rx;
  const int y0 = (int)floorf(fmaxf(fy, 0.f)), x0 = (int)floorf(fmaxf(fx, 0.f));
  const int y1 = min(fh - 1, (int)ceilf(fy)), x1 = min(fw - 1, (int)ceilf(fx));
  PrepTap t;
  t.dy = fy - (float)y0;
  t.dx = fx - (float)x0;
  t.t0 = f + (long)y0 * rs;
  t.t1 = f + (long)y1 * rs;
  t.o0 = x0 * fc;
  t.o1 = x1 * fc;
  return t;
}

// v[0..2] = row y0 col x0 RGB, v[3..5] = (y0, x1), v[6..8] = (y1, x0), v[9..11] = (y1, x1)
__device__ __forceinline__ void prep_load(const PrepTap& t, uint32_t v[12]) {
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    v[c] = t.t0[t.o0 + c];
    v[3 + c] = t.t0[t.o1 + c];
    v[6 + c] = t.t1[t.o0 + c];
    v[9 + c] = t.t1[t.o1 + c];
  }
}

// v / 255.0f, correctly rounded, without the IEEE division sequence (div_scale,
// rcp, four FMAs, div_fmas, div_fixup): the reciprocal product corrected by one
// FMA residual.  Equal to the division for EVERY float in [0, 256] (and by
// symmetry [-256, 0]) — checked exhaustively, all 1,132,462,081 of them, by
// tools/div255_check.c (tests/test_div255.py); the resize's lerps of bytes
// never leave [0, 255].
__device__ __forceinline__ float div255(float v) {
#pragma clang fp contract(off)
  constexpr float kInv = 1.0f / 255.0f;
  const float q = v * kInv;
  return __builtin_fmaf(__builtin_fmaf(-q, 255.0f, v), kInv, q);
}

__device__ __forceinline__ void prep_finish(const uint32_t v[12], float dy, float dx, float out[3]) {
#pragma clang fp contract(off)
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float tl = (float)v[c], tr = (float)v[3 + c], bl = (float)v[6 + c], br = (float)v[9 + c];
    const float top = __builtin_fmaf(tr - tl, dx, tl);
    const float bot = __builtin_fmaf(br - bl, dx, bl);
    const float val = __builtin_fmaf(bot - top, dy, top);
    out[c] = div255(val);
  }
}

// prep_finish for two pixels at once: lane 0 / 1 of every float2 is pixel a /
// b, so each sub, mul and FMA is one packed-FP32 instruction (v_pk_add_f32,
// v_pk_mul_f32, v_pk_fma_f32: per lane the same IEEE operation as the scalar
// one) — the same floats as two prep_finish calls, in about half the VALU
// issue slots (b1's prologue is bound by VALU issue at 4.5 waves per SIMD).
typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f2 div255x2(f2 v) {
#pragma clang fp contract(off)
  constexpr float kInv = 1.0f / 255.0f;
  const f2 inv = {kInv, kInv}, c255 = {255.0f, 255.0f};
  const f2 q = v * inv;
  return __builtin_elementwise_fma(__builtin_elementwise_fma(-q, c255, v), inv, q);
}

__device__ __forceinline__ void prep_finish2(const uint32_t va[12], const uint32_t vb[12], float dya, float dxa,
                                             float dyb, float dxb, float outa[3], float outb[3]) {
#pragma clang fp contract(off)
  const f2 dy = {dya, dyb}, dx = {dxa, dxb};
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const f2 tl = {(float)va[c], (float)vb[c]}, tr = {(float)va[3 + c], (float)vb[3 + c]};
    const f2 bl = {(float)va[6 + c], (float)vb[6 + c]}, br = {(float)va[9 + c], (float)vb[9 + c]};
    const f2 top = __builtin_elementwise_fma(tr - tl, dx, tl);
    const f2 bot = __builtin_elementwise_fma(br - bl, dx, bl);
    const f2 o = div255x2(__builtin_elementwise_fma(bot - top, dy, top));
    outa[c] = o.x;
    outb[c] = o.y;
  }
}

__device__ __forceinline__ void prep_sample(const uint8_t* __restrict__ f, long rs, int fc, int fh, int fw,
                                            float ry, float rx, int y, int x, float& r, float& g, float& b) {
  const PrepTap t = prep_tap(f, rs, fc, fh, fw, ry, rx, y, x);
  uint32_t v[12];
  prep_load(t, v);
  float out[3];
  prep_finish(v, t.dy, t.dx, out);
  r = out[0]; g = out[1]; b = out[2];
}

#if !defined(VSS_SHARD) || VSS_SHARD == 0  // (one definition across the shard objects)
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
#endif

// ---------------------------------------------------------------------------
// The stem's 3x3 stride-2 conv (3 -> 16 channels) for a block of 16 output
// pixels on the MFMA (v_mfma_f32_16x16x4_f32): D[pixel][channel] = bias +
// sum over the 27 taps k = ci*9 + ky*3 + kx of x0[pixel][k] * w[channel][k],
// K padded to 28 with a zero weight, in 7 MFMAs of K = 4.  Lane (r, g) hands
// A[pixel r][tap 4s+g] (one LDS read) and B[tap 4s+g][channel r] (a register)
// and gets back D[pixel 4g+i][channel r].  Each output depends only on its own
// pixel's taps, so k_stem and the STEM_IN prologue (any tile) give bitwise the
// same activations.  (A per-lane FMA chain over the taps read 27 f4 weights
// and 27 x0 values from LDS per 4 outputs: LDS-bandwidth bound, 2.6 us.)
struct StemTaps {
  int off[7];  // LDS offset of tap 4s+g from the pixel's x0 corner (2py, 2px)
  float w[7];  // w[channel r][tap 4s+g]
};

// The four lane groups' offsets of tap 4s + g (g = 0..3) for one s, packed as
// 16-bit fields of a compile-time constant: a lane picks its field with one
// 64-bit shift by 16 g and a mask, instead of dividing 4s + g by 9 and 3 at
// run time (~12 VALU per tap: the taps' setup was a fifth of b1's VALU).
template <int PLANE, int ROW>
struct StemTapTable {
  static_assert(2 * PLANE + 2 * ROW + 2 < 65536, "tap offsets are 16-bit fields");
  static constexpr unsigned long long field(int s) {
    unsigned long long v = 0;
    for (int g = 0; g < 4; ++g) {
      const int k = 4 * s + g;
      const unsigned long long o = k < 27 ? (unsigned long long)((k / 9) * PLANE + ((k % 9) / 3) * ROW + k % 3) : 0ull;
      v |= o << (16 * g);
    }
    return v;
  }
  static constexpr unsigned long long c[7] = {field(0), field(1), field(2), field(3), field(4), field(5), field(6)};
};

template <int PLANE, int ROW>
__device__ __forceinline__ StemTaps stem_taps(const float* ws /* [tap][16], then the bias */, int r, int g) {
  StemTaps t;
  const unsigned sh = (unsigned)g << 4;
#pragma unroll
  for (int s = 0; s < 7; ++s) {
    t.off[s] = (int)((StemTapTable<PLANE, ROW>::c[s] >> sh) & 0xFFFFu);
    // tap 27 (s = 6, g = 3) is K's padding: weight 0 (its address reads the bias row, in bounds)
    const float wv = ws[(4 * s + g) * 16 + r];
    t.w[s] = (s == 6 && g == 3) ? 0.f : wv;
  }
  return t;
}

__device__ __forceinline__ f4 stem_mfma(const StemTaps& t, const float* x0, float bias) {
  f4 acc = {bias, bias, bias, bias};
#pragma unroll
  for (int s = 0; s < 7; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(x0[t.off[s]], t.w[s], acc, 0, 0, 0);
  return acc;
}

// The same products with the operands swapped (A = the weights, B = the taps):
// D[channel 4g+i][pixel r], i.e. lane (r, g) gets channels 4g..4g+3 of pixel
// r — one 16-B store per lane instead of four scalar ones.  Every output is the
// same sum of the same products over the same k (and the same C), so the
// activations are bitwise stem_mfma's transposed (test_stem_fusion_bitwise
// compares the fused stem with k_stem, which keeps stem_mfma).
__device__ __forceinline__ f4 stem_mfma_t(const StemTaps& t, const float* x0, f4 bias4) {
  f4 acc = bias4;
#pragma unroll
  for (int s = 0; s < 7; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(t.w[s], x0[t.off[s]], acc, 0, 0, 0);
  return acc;
}

// ---------------------------------------------------------------------------
// Stem: output tile 8 x 32 pixels x 16 channels, 16-pixel blocks on the MFMA.
template <int COUT, bool COH>
__device__ __forceinline__ void stem_body(const StemParams& p, int bx, int by, int n, float* smem) {
  constexpr int TH = kStemTH, TW = kStemTW, IH = kStemIH, IW = 2 * TW + 1, IWP = kStemIWP;
  static_assert(COUT == 16, "stem LDS carve (kStemLds) assumes 16 output channels");
  float (*xs)[IH][IWP] = reinterpret_cast<float (*)[IH][IWP]>(smem);  // [3][IH][IWP]
  float* ws = smem + r4(3 * IH * IWP);                                 // [tap][c]: 4 channels per LDS read
  float* bs = ws + 27 * COUT;
  const int tid = threadIdx.x;
  const int oy0 = by * TH, ox0 = bx * TW;
  const uint8_t* f = p.frames + (long)n * p.frame_stride;
  const int iy0 = 2 * oy0 - 1, ix0 = 2 * ox0 - 1;
  VSS_STAMP(0);
  // all frame gathers of this thread issued before any is consumed
  constexpr int NS = (IH * IW + 255) / 256, NW = (27 * COUT + 255) / 256;
  // the weights' loads go out first (they are consumed after the gathers)
  float wr[NW];
#pragma unroll
  for (int u = 0; u < NW; ++u) wr[u] = p.w[min(tid + 256 * u, 27 * COUT - 1)];
  const float br = p.b[min(tid, COUT - 1)];
  uint32_t raw[NS][12];
  float dys[NS], dxs[NS];
#pragma unroll
  for (int u = 0; u < NS; ++u) {
    const int i = min(tid + 256 * u, IH * IW - 1);
    const int ly = i / IW, lx = i - ly * IW;
    const int yy = min(max(iy0 + ly, 0), p.Hm - 1), xx = min(max(ix0 + lx, 0), p.Wm - 1);
    const PrepTap t = prep_tap(f, p.row_stride, p.fc, p.fh, p.fw, p.ry, p.rx, yy, xx);
    prep_load(t, raw[u]);
    dys[u] = t.dy;
    dxs[u] = t.dx;
  }
#pragma unroll
  for (int u = 0; u < NS; ++u) {
    const int i = tid + 256 * u;
    if (i < IH * IW) {
      const int ly = i / IW, lx = i - ly * IW;
      const int yy = iy0 + ly, xx = ix0 + lx;
      float o[3];
      prep_finish(raw[u], dys[u], dxs[u], o);
      const bool valid = yy >= 0 && yy < p.Hm && xx >= 0 && xx < p.Wm;
      xs[0][ly][lx] = valid ? o[0] : 0.f;
      xs[1][ly][lx] = valid ? o[1] : 0.f;
      xs[2][ly][lx] = valid ? o[2] : 0.f;
    }
  }
  // start of the forward: zero this frame's decoder norm accumulators
  // (write-through in the persistent forward: the decoders' atomics follow)
  if (bx == 0 && by == 0)
    for (int i = tid; i < p.acc_stride; i += 256) {
      if constexpr (COH)
        __hip_atomic_store(p.acc_zero + (long)n * p.acc_stride + i, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else
        p.acc_zero[(long)n * p.acc_stride + i] = 0ull;
    }
#pragma unroll
  for (int u = 0; u < NW; ++u) {
    const int i = tid + 256 * u;  // p.w is [c][27]
    if (i < 27 * COUT) ws[(i % 27) * COUT + i / 27] = wr[u];
  }
  if (tid < COUT) bs[tid] = br;
  __syncthreads();
  VSS_STAMP(1);
  VSS_STAMP(2);
  const int lane = tid & 63, wave = tid >> 6, r = lane & 15, g = lane >> 4;
  const StemTaps taps = stem_taps<IH * IWP, IWP>(ws, r, g);
  const float bias = bs[r];
  const Gm<COH> gy(p.y + (long)n * p.Ho * p.Wo * COUT);
#pragma unroll
  for (int blk = wave; blk < TH * TW / 16; blk += 4) {
    const int pa = blk * 16 + r, ly = pa / TW, lx = pa % TW;
    const f4 acc = stem_mfma(taps, &xs[0][2 * ly][2 * lx], bias);
#pragma unroll
    for (int i = 0; i < 4; ++i) {  // D[pixel 4g+i][channel r]
      const int pp = blk * 16 + 4 * g + i;
      const int oy = oy0 + pp / TW, ox = ox0 + pp % TW;
      if (oy < p.Ho && ox < p.Wo) gy.st1(((long)oy * p.Wo + ox) * COUT + r, relu6f(acc[i]));
    }
  }
  VSS_STAMP(3);
}

template <int COUT>
__global__ __launch_bounds__(256) void k_stem(StemParams p) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  stem_body<COUT, false>(p, blockIdx.x, blockIdx.y, blockIdx.z, smem);
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

// A fragment from the LDS weight image (bf16-exact pointwise weights, rows of
// `ld` bf16 elements): 4 consecutive weights of row `row` starting at k.
template <int PREC>
__device__ __forceinline__ typename AFrag<PREC>::T lds_a(const uint16_t* w, int ld, int row, int k);

template <>
__device__ __forceinline__ f4 lds_a<PREC_F32>(const uint16_t* w, int ld, int row, int k) {
  const uint2 v = *reinterpret_cast<const uint2*>(w + row * ld + k);
  return f4{__uint_as_float(v.x << 16), __uint_as_float(v.x & 0xFFFF0000u), __uint_as_float(v.y << 16),
            __uint_as_float(v.y & 0xFFFF0000u)};
}
template <>
__device__ __forceinline__ bf8 lds_a<PREC_BF16X2>(const uint16_t* w, int ld, int row, int k) {
  // elements 0-3 pair with the activation hi parts, 4-7 (the same weights) with the lo parts
  const bf4 b = __builtin_bit_cast(bf4, *reinterpret_cast<const uint2*>(w + row * ld + k));
  return bf8{b.x, b.y, b.z, b.w, b.x, b.y, b.z, b.w};
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

// B operands stored ready for the MFMA: f32 as is, or for the split mode the
// (hi, lo) bf16 pairs of mma16<PREC_BF16X2> packed in the same 16 bytes, so the
// conversion happens once when the tile is written, not once per use.
template <int PREC>
__device__ __forceinline__ f4 to_operand(f4 v) {
  if constexpr (PREC == PREC_F32) {
    return v;
  } else {
    const __bf16 h0 = (__bf16)v.x, h1 = (__bf16)v.y, h2 = (__bf16)v.z, h3 = (__bf16)v.w;
    const __bf16 l0 = (__bf16)(v.x - (float)h0), l1 = (__bf16)(v.y - (float)h1);
    const __bf16 l2 = (__bf16)(v.z - (float)h2), l3 = (__bf16)(v.w - (float)h3);
    return __builtin_bit_cast(f4, bf8{h0, h1, h2, h3, l0, l1, l2, l3});
  }
}

template <int PREC>
__device__ __forceinline__ f4 mma16_op(f4 acc, typename AFrag<PREC>::T a, f4 op) {
  if constexpr (PREC == PREC_F32)
    return mma16<PREC_F32>(acc, a, op);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, __builtin_bit_cast(bf8, op), acc, 0, 0, 0);
}

// Orders one wave's LDS writes before its other lanes' reads (and keeps the
// compiler from moving LDS accesses across it); no workgroup barrier.
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}


// Registers holding one thread's share of a TOTAL-item (16-B items) copy.
// issue(): every load of the copy in flight (unconditional at clamped indices:
// a conditional load makes hipcc branch and wait per element); commit():
// consume them (waits land at the first use).  Issuing several copies before
// committing any costs one memory round trip instead of one per copy.
template <int TOTAL>
struct Staged {
  static constexpr int PER = (TOTAL + 255) / 256;
  f4 v[PER > 0 ? PER : 1];
  template <class Load>
  __device__ __forceinline__ void issue(Load ld) {
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int i = (int)threadIdx.x + 256 * u;
      v[u] = ld(i < TOTAL ? i : TOTAL - 1);
    }
  }
  template <class Store>
  __device__ __forceinline__ void commit(Store st) const {
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int i = (int)threadIdx.x + 256 * u;
      if (i < TOTAL) st(i, v[u]);
    }
  }
};

// A staged copy of NI items of four consecutive float4s (16 channels of one
// pixel) from NP parts (the hidden-split partial sums) at the same offsets;
// commit_sum adds the parts in part order.  Two lane mappings:
//  WHOLE = true : a lane takes whole items — one index computation per 16
//    channels, its four loads at immediate offsets (16 B apart) off a 32-bit
//    offset from each part's wave-uniform base;
//  WHOLE = false: float4 j of the copy goes to lane j % 256 (a wave's load
//    instruction reads 1 KiB contiguous), one index computation per float4.
// Measured (4 batches in flight, A/B on one box): whole items for the
// inverted-residual input tile (fewer VALU, same time), float4s for the
// decoder's low-res / skip tiles (d2 7.18 -> 6.51 us, d3 8.83 -> 8.30 us).
#ifndef VSS_STAGE16
#define VSS_STAGE16 1      // the inverted-residual blocks' input tile
#endif
#ifndef VSS_STAGE16_DEC
#define VSS_STAGE16_DEC 0  // the decoder's low-res source and skip tiles
#endif
template <int NI, int NP, bool WHOLE>
struct Staged16 {
  static constexpr int PER = WHOLE ? (NI + 255) / 256 : (4 * NI + 255) / 256;
  static constexpr int V = WHOLE ? 4 : 1;
  f4 v[NP][PER > 0 ? PER : 1][V];
  template <class Off>
  __device__ __forceinline__ void issue(const float* const (&base)[NP], Off off) {
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int j = (int)threadIdx.x + 256 * u;
      unsigned o;
      if constexpr (WHOLE) {
        o = off(j < NI ? j : NI - 1);  // float offset of the item's first channel
      } else {
        const int jj = j < 4 * NI ? j : 4 * NI - 1;
        o = off(jj >> 2) + 4u * (unsigned)(jj & 3);
      }
#pragma unroll
      for (int q = 0; q < NP; ++q)
#pragma unroll
        for (int k = 0; k < V; ++k)
          v[q][u][k] = *reinterpret_cast<const f4*>(reinterpret_cast<const char*>(base[q]) + ((o + 4u * k) << 2));
    }
  }
  template <class Store>  // store(item, k, the parts' sum of float4 k of the item)
  __device__ __forceinline__ void commit_sum(Store st) const {
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int j = (int)threadIdx.x + 256 * u;
      constexpr int TOT = WHOLE ? NI : 4 * NI;  // items, or float4s
      if (TOT % 256 == 0 || j < TOT) {
#pragma unroll
        for (int k = 0; k < V; ++k) {
          f4 x = v[0][u][k];
#pragma unroll
          for (int q = 1; q < NP; ++q) x = x + v[q][u][k];
          if constexpr (WHOLE)
            st(j, k, x);
          else
            st(j >> 2, j & 3, x);
        }
      }
    }
  }
};

// The layer's weight image global -> LDS by LDS-DMA (VSS_WDMA, default on):
// 16 B per lane, 1 KiB per wave instruction, written straight into LDS — no
// register staging (Staged<WIMG_F4> held up to ~19 float4s per lane) and no
// commit stores; the prologue's closing barrier waits for it (dma_wait).
// Used by the decoders and the blocks whose image is >= 40 KiB (block_wdma):
// measured per layer against register staging (profiles/r05ac, isolated
// event pass, 3 interleaved runs): b7 6.70 -> 6.14 us, b6 6.43 -> 6.23,
// b5 5.88 -> 5.75, d1 5.06 -> 4.95, d2 6.48 -> 6.22, but b2 6.50 -> 6.85 and
// b4 5.40 -> 5.56 (small images: register staging kept there).
#ifndef VSS_WDMA
#define VSS_WDMA 1
#endif
#ifndef VSS_WDMA_ALL
#define VSS_WDMA_ALL 0  // (A/B knob: every layer)
#endif
#ifndef VSS_WDMA_FIRST
#define VSS_WDMA_FIRST 0  // (A/B knob: the DMA issued before the input tile's loads)
#endif
constexpr bool block_wdma(int mode, int wimg_f4) {
  return VSS_WDMA && (VSS_WDMA_ALL || mode == 2 || wimg_f4 >= 2560);
}
template <int N>
__device__ __forceinline__ void dma_f4(const f4* src, f4* dst) {
  const int lane = (int)threadIdx.x & 63;
  const int wb = __builtin_amdgcn_readfirstlane(((int)threadIdx.x >> 6) * 64);
  for (int o = wb; o < N; o += 256)
    if (N % 64 == 0 || o + lane < N)
      __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(src + o + lane),
                                       (__attribute__((address_space(3))) void*)(dst + o), 16, 0, 0);
}
struct NoStaged {  // Staged's interface for the DMA'd copy
  template <class Load>
  __device__ __forceinline__ void issue(Load) {}
  template <class Store>
  __device__ __forceinline__ void commit(Store) const {}
};
template <bool ON>
__device__ __forceinline__ void dma_wait() {
  if constexpr (ON) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <bool B>
struct ChunkTag {
  static constexpr bool value = B;
};

// Fused inverted-residual / decoder block, specialised on its whole shape
// (every tile and channel extent a compile-time constant: index math folds
// to shifts/multiplies, loops unroll, accumulators stay in registers).
//  prologue : every global load of the block issued first (the layer's weight
//             image, the input tile + halo, or for the decoder the low-res src
//             region, the skip tile and the src's norm scale/shift), then
//             committed to LDS; the decoder builds the 2x bilinear upsample
//             (norm + ReLU on the fly) ++ skip concat tile.
//  main     : independent per-wave work units, wave-level syncs only.
//             EXPAND: unit = 16 hidden channels: expand (MFMA) over the whole
//             input tile -> dw 3x3 (VALU) -> project (MFMA) into acc.
//             DIRECT/DEC: unit = (16 output pixels, 16 channels): dw -> project.
//  epilogue : per-wave accumulator slabs in LDS summed in a fixed order
//             (deterministic), + bias (+ residual), coalesced NHWC stores;
//             decoder: per-tile instance-norm partial sums, and the last
//             workgroup of each frame to arrive reduces them (fixed order) into
//             the frame's scale/shift for the consumer.
template <int MODE, int STRIDE, int TH, int TW, int CIN, int CSKIP, int CH, int COUT, int FLAGS, int PREC, bool COH>
__device__ __forceinline__ void block_body(const BlockParams& p, int bx, int by, int bz, float* smem) {
  constexpr bool STEM_IN = flags_stem_in(FLAGS);
  constexpr BlockLds L = block_lds(MODE, STRIDE, TH, TW, CIN, CSKIP, CH, COUT, STEM_IN);
  constexpr bool NORM_IN = (FLAGS & 1) != 0, RES = (FLAGS & 2) != 0;
  constexpr int XP = flags_xp(FLAGS), SP = flags_sp(FLAGS), KS = flags_ks(FLAGS);
  static_assert(KS == 1 || MODE == MODE_IR_EXPAND, "only expand layers split their hidden channels");
  static_assert(SP == 1 || MODE == MODE_DEC, "skip parts: decoder only");
  constexpr int IW = L.IW, P_IN = L.P_in, P_IN_PAD = L.P_in_pad, P_OUT = L.P_out, XS = L.XS;
  constexpr int NCB = L.NCB, NPB = L.NPB, NCHUNK = L.NCHUNK, PW = L.PW, CS = L.CS, NPBW = L.NPBW;
  constexpr int RS = L.RS, SS = L.slab_stride;
  static_assert(L.NACC <= kMaxAcc, "too many accumulators per wave");
  static_assert(CIN % 16 == 0 && CH % 16 == 0 && COUT % 16 == 0 && P_OUT % 16 == 0, "shape");
  static_assert(MODE != MODE_IR_EXPAND || CIN <= 64, "expand cin <= 64");
  static_assert(!RES || (STRIDE == 1 && CIN == COUT && MODE != MODE_DEC), "residual shape");
  static_assert(MODE != MODE_IR_EXPAND || CS == 4, "expand deals its chunks to the 4 waves");
  static_assert(NPB % PW == 0, "pixel blocks must split evenly over the wave groups");
  constexpr int XT_FLOATS = L.XQM ? P_IN_PAD * L.CX : r4(P_IN_PAD * XS);
  static_assert(MODE != MODE_DEC || (XT_FLOATS >= (NORM_IN ? kAccSlots * 2 * CIN * 2 : 0) &&
                                     (L.slab == L.xt ? L.stt == L.work : (L.stt == L.xt && XT_FLOATS >= 1024))),
                "decoder: xt holds the src's norm slots (prologue); the stats scratch (epilogue) sits in the "
                "work region when the slabs take xt, else in xt");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int n = KS == 1 ? bz : bz / KS;  // grid z = frame * KS + slice
  const int ks = KS == 1 ? 0 : bz % KS;
  const int oy0 = by * TH, ox0 = bx * TW;
  const int iy0 = STRIDE * oy0 - 1, ix0 = STRIDE * ox0 - 1;
  const int Ho = p.Ho, Wo = p.Wo;
  float* xt = smem + L.xt;
  const uint16_t* w1s = reinterpret_cast<const uint16_t*>(smem + L.w1);
  const uint16_t* w2s = reinterpret_cast<const uint16_t*>(smem + L.w2);
  const float* wdws = smem + L.wdw;
  const float* bdws = smem + L.bdw;
  const float* b1s = smem + L.b1;
  const float* b2s = smem + L.b2;
  float* work = smem + L.work;
  float* slabs = smem + L.slab;
  float* stt = smem + L.stt;
  // LDS layouts (vss_kernels.h, VSS_SWZ): float offsets of channel quad q of a
  // pixel in the input tile xt, an epilogue slab, the residual centre xr and
  // an expand wave's hidden chunk
  auto xq = [&](int pix, int q) {
    if constexpr (L.XQM) return q * L.XPL + 4 * pix;
    else return pix * XS + 4 * (q ^ gray_swz(pix, L.XSW));
  };
  auto sq = [&](int sl, int pix, int q) { return sl * SS + pix * RS + 4 * (q ^ gray_swz(pix, L.RSW)); };
  auto rq = [&](int pix, int q) { return pix * CIN + 4 * (q ^ (pix & (L.XRW - 1))); };
  VSS_STAMP(0);

  // ---- prologue: issue every load, then commit to LDS ----
  constexpr int WIMG_F4 = (L.wimg_end - L.w1) / 4;
  constexpr bool WDMA = block_wdma(MODE, WIMG_F4);
  const f4* wsrc = reinterpret_cast<const f4*>(p.wimg + ks * p.wimg_stride);
  f4* wdst = reinterpret_cast<f4*>(smem + L.w1);
  if constexpr (MODE == MODE_DEC) {
    constexpr int CL = CIN, C4L = CL / 4, SR = L.SR, SC = L.SC;
    const int h = p.H, w = p.W;
    float* lr = smem + L.lr;
    float* nrm = smem + L.nrm;
    const int sy0 = max(0, (oy0 - 1) / 2 - 1), sx0 = max(0, (ox0 - 1) / 2 - 1);
    const float* xn = p.x + (long)n * h * w * CL;
    const float* sn = p.skip + (long)n * Ho * Wo * CSKIP;
    // src instance norm: every slot of the frame's exact totals (issued first)
    constexpr int NSLOT16 = NORM_IN ? kAccSlots * 2 * CL / 2 : 0;  // 16-B items
    Staged<NSLOT16> st_slots;
    const Gm<COH> g_slots(reinterpret_cast<const float*>(p.in_acc + (long)n * p.acc_stride));
    if constexpr (NORM_IN) st_slots.issue([&](int i) { return g_slots.ld(4L * i); });
    static_assert(CL % 16 == 0 && CSKIP % 16 == 0, "16-channel staging items");
    constexpr int GL = CL / 16, GS = CSKIP / 16;  // 16-channel items per pixel
    Staged16<SR * SC * GL, XP, VSS_STAGE16_DEC> st_lr;
    Staged16<P_IN_PAD * GS, SP, VSS_STAGE16_DEC> st_sk;
    // The skip commit's 16-B stores go 8 lanes at a time (32 banks) over two
    // items; with one item per pixel and a pixel stride of 2 mod 4 quads (the
    // 16-wide decoder tiles' rows) two neighbouring pixels overlap by two bank
    // quads, pixels two apart do not: items take pixels 0, 2, 1, 3, 4, 6, ...
    // (a bijection within groups of four; P_IN_PAD is a multiple of 16)
    constexpr bool SKP = VSS_SWZ && GS == 1 && !L.XQM && VSS_STAGE16_DEC == 0 && (XS / 4) % 4 == 2;
    auto skip_pix = [&](int it) { return SKP ? (it & ~3) | ((it & 1) << 1) | ((it >> 1) & 1) : it; };
    std::conditional_t<WDMA, NoStaged, Staged<WIMG_F4>> st_w;
    {
      const float* xb[XP];
#pragma unroll
      for (int q = 0; q < XP; ++q) xb[q] = xn + q * p.x_part_stride;
      st_lr.issue(xb, [&](int i) {
        const int pr = i / GL, gq = i - pr * GL;
        const int yy = min(h - 1, sy0 + pr / SC), xx = min(w - 1, sx0 + pr % SC);
        return (unsigned)((yy * w + xx) * CL + 16 * gq);
      });
      const float* sb[SP];
#pragma unroll
      for (int q = 0; q < SP; ++q) sb[q] = sn + q * p.skip_part_stride;
      st_sk.issue(sb, [&](int i) {
        const int pix = skip_pix(i / GS), gq = i - (i / GS) * GS, py = pix / IW;
        const int yy = min(max(iy0 + py, 0), Ho - 1), xx = min(max(ix0 + pix - py * IW, 0), Wo - 1);
        return (unsigned)((yy * Wo + xx) * CSKIP + 16 * gq);
      });
    }
    if constexpr (WDMA) dma_f4<WIMG_F4>(wsrc, reinterpret_cast<f4*>(smem + L.w1));
    st_w.issue([&](int i) { return wsrc[i]; });
    VSS_STAMP(6);  // every load issued
    // the upsample's tap records, one per input-tile pixel, while the loads
    // are in flight: source coordinate max((o + 0.5) / 2 - 0.5, 0) in
    // integers — o = 0 -> (0, 0); odd o -> ((o - 1) / 2, 0.25); even o > 0 ->
    // (o / 2 - 1, 0.75), the same floats the float formula gives
    static_assert(SR * SC * CL < 65536, "tap offsets are u16");
    // even tiles start at an odd row and column of the output (iy0 = TH*by - 1),
    // so their input tile is whole 2x2 quads that share one 2x2 source window:
    // the upsample below runs per quad and needs no per-pixel tap records
    constexpr bool QUADS = VSS_QUADS && TH % 2 == 0 && TW % 2 == 0;
    unsigned* uc = reinterpret_cast<unsigned*>(smem + L.uc);
    if constexpr (!QUADS)
    for (int pix = tid; pix < P_IN_PAD; pix += 256) {
      const int yy = iy0 + pix / IW, xx = ix0 + pix % IW;
      uint4 rec = {0xFFFFFFFFu, 0u, 0u, 0u};  // outside the frame / padding: zeros
      if (pix < P_IN && yy >= 0 && yy < Ho && xx >= 0 && xx < Wo) {
        const int y0 = yy > 0 ? (yy - 1) >> 1 : 0, y1 = y0 + (y0 < h - 1 ? 1 : 0);
        const float ly1 = yy > 0 ? ((yy & 1) ? 0.25f : 0.75f) : 0.f;
        const int x0 = xx > 0 ? (xx - 1) >> 1 : 0, x1 = x0 + (x0 < w - 1 ? 1 : 0);
        const float lx1 = xx > 0 ? ((xx & 1) ? 0.25f : 0.75f) : 0.f;
        const int r0 = min(max(y0 - sy0, 0), SR - 1), r1 = min(max(y1 - sy0, 0), SR - 1);
        const int q0 = min(max(x0 - sx0, 0), SC - 1), q1 = min(max(x1 - sx0, 0), SC - 1);
        rec.x = (unsigned)((r0 * SC + q0) * CL) | ((unsigned)((r0 * SC + q1) * CL) << 16);
        rec.y = (unsigned)((r1 * SC + q0) * CL) | ((unsigned)((r1 * SC + q1) * CL) << 16);
        rec.z = __float_as_uint(ly1);
        rec.w = __float_as_uint(lx1);
      }
      reinterpret_cast<uint4*>(uc)[pix] = rec;
    }
    if constexpr (NORM_IN) {
      // sum the slots (exact, any order) -> the src's scale/shift; the slots
      // are staged in xt, whose contents are committed only after this
      const float gam = p.in_gamma[min(tid, CL - 1)], bet = p.in_beta[min(tid, CL - 1)];
      st_slots.commit([&](int i, f4 v) { reinterpret_cast<f4*>(xt)[i] = v; });
      __syncthreads();
      const unsigned long long* sl = reinterpret_cast<const unsigned long long*>(xt);
      if (tid < CL) {
        unsigned long long s_fx = 0, q_fx = 0;
#pragma unroll
        for (int k = 0; k < kAccSlots; ++k) {
          s_fx += sl[k * 2 * CL + tid];
          q_fx += sl[k * 2 * CL + CL + tid];
        }
        norm_affine(s_fx, q_fx, p.in_inv_hw, p.eps, gam, bet, nrm + tid, nrm + CL + tid);
      }
      __syncthreads();
      VSS_STAMP(5);
    }
    // the low-res src region; with norm_in, relu(src * scale + shift) applied
    // once per element as it is committed
    st_lr.commit_sum([&](int i, int k, f4 v) {
      // item i = (region pixel, 16-channel group): its floats are contiguous in lr
      if constexpr (NORM_IN) {
        const int c4 = (i % GL) * 4 + k;
        v = reluv(v * *reinterpret_cast<const f4*>(nrm + 4 * c4) + *reinterpret_cast<const f4*>(nrm + CL + 4 * c4));
      }
      reinterpret_cast<f4*>(lr)[4 * i + k] = v;
    });
    // the skip channels: zero outside the image (tiles at its edge only; the
    // loads were clamped to real pixels, and padding pixels are never read)
    const bool sk_interior = iy0 >= 0 && iy0 + L.IH <= Ho && ix0 >= 0 && ix0 + IW <= Wo;
    st_sk.commit_sum([&](int i, int k, f4 v) {
      const int pix = skip_pix(i / GS), gq = i - (i / GS) * GS;
      if (!sk_interior) {
        const int py = pix / IW, yy = iy0 + py, xx = ix0 + pix - py * IW;
        const bool valid = ((unsigned)yy < (unsigned)Ho) & ((unsigned)xx < (unsigned)Wo);
        v = valid ? v : f4{0.f, 0.f, 0.f, 0.f};
      }
      *reinterpret_cast<f4*>(xt + xq(pix, CL / 4 + 4 * gq + k)) = v;
    });
    st_w.commit([&](int i, f4 v) { wdst[i] = v; });
    VSS_STAMP(4);
    dma_wait<WDMA>();
    __syncthreads();
    // upsampled channels: PyTorch upsample_bilinear2d(scale 2, align_corners=False)
    // of relu(src * scale + shift) (the src's instance norm, applied per tap)
    if constexpr (QUADS) {
      // Output rows 2j+1, 2j+2 both lie between source rows j, j+1 (weights
      // 0.75 / 0.25 and 0.25 / 0.75), and so do columns: one 2x2 source window
      // per output quad.  Per source row the two horizontal interpolants
      // H1 = fma(0.25, R, 0.75 L) (column 2i+1) and H2 = fma(0.75, R, 0.25 L)
      // (column 2i+2), then each output = fma(ly1, H[j+1], ly0 H[j]) — exactly
      // the per-pixel form's operations (top / bot lerps, then the vertical
      // one), shared by the quad: the same floats with 4 tap reads per 4
      // pixels instead of 16.  At the image's edges the source index clamps
      // (row / column -1 -> 0, h -> h - 1), where both weights hit the same
      // value and the FMA returns it exactly — as the per-pixel form's
      // weight-0 taps do.  Outputs outside the image are zero (halo).
      constexpr int QH = L.IH / 2, QW = IW / 2, NQI = QH * QW * C4L, NQ = (NQI + 255) / 256;
      const int j0 = (iy0 - 1) / 2, i0 = (ix0 - 1) / 2;  // iy0, ix0 odd: exact (-1 -> -1)
      const int jr = j0 - sy0, ic = i0 - sx0;             // the quads' first source row / column in the region
      const bool interior = iy0 >= 0 && iy0 + L.IH <= Ho && ix0 >= 0 && ix0 + IW <= Wo;
      const f4 c25 = {0.25f, 0.25f, 0.25f, 0.25f}, c75 = {0.75f, 0.75f, 0.75f, 0.75f};
#pragma unroll
      for (int k = 0; k < NQ; ++k) {
        const int it = tid + 256 * k;
        if (NQI % 256 == 0 || it < NQI) {
          const int c4 = it % C4L, qq = it / C4L, qx = qq % QW, qy = qq / QW;
          // the source window's rows / columns, clamped to the region: the
          // region's rows (columns) past the source's last one were loaded
          // clamped, i.e. they hold that last row (column), and a row above
          // (left of) the source only occurs where the region starts at 0
          const int ra = min(max(qy + jr, 0), SR - 1), rb = min(max(qy + jr + 1, 0), SR - 1);
          const int ca = min(max(qx + ic, 0), SC - 1), cb = min(max(qx + ic + 1, 0), SC - 1);
          const float* la = lr + ra * (SC * CL) + 4 * c4;
          const float* lb = lr + rb * (SC * CL) + 4 * c4;
          const f4 taa = *reinterpret_cast<const f4*>(la + ca * CL);
          const f4 tab = *reinterpret_cast<const f4*>(la + cb * CL);
          const f4 tba = *reinterpret_cast<const f4*>(lb + ca * CL);
          const f4 tbb = *reinterpret_cast<const f4*>(lb + cb * CL);
          const f4 h1a = __builtin_elementwise_fma(c25, tab, c75 * taa), h2a = __builtin_elementwise_fma(c75, tab, c25 * taa);
          const f4 h1b = __builtin_elementwise_fma(c25, tbb, c75 * tba), h2b = __builtin_elementwise_fma(c75, tbb, c25 * tba);
          f4 o00 = __builtin_elementwise_fma(c25, h1b, c75 * h1a), o01 = __builtin_elementwise_fma(c25, h2b, c75 * h2a);
          f4 o10 = __builtin_elementwise_fma(c75, h1b, c25 * h1a), o11 = __builtin_elementwise_fma(c75, h2b, c25 * h2a);
          if (!interior) {
            const int yy = iy0 + 2 * qy, xx = ix0 + 2 * qx;  // the quad's top-left output pixel
            // (yy >= -1: the quad's second row is never above the image; a
            // partial tile's quads may lie past its bottom / right edge)
            const bool r0 = yy >= 0 && yy < Ho, r1 = yy + 1 < Ho, x0v = xx >= 0 && xx < Wo, x1v = xx + 1 < Wo;
            const f4 z = {0.f, 0.f, 0.f, 0.f};
            o00 = r0 && x0v ? o00 : z;
            o01 = r0 && x1v ? o01 : z;
            o10 = r1 && x0v ? o10 : z;
            o11 = r1 && x1v ? o11 : z;
          }
          const int p00 = (2 * qy) * IW + 2 * qx;
          *reinterpret_cast<f4*>(xt + xq(p00, c4)) = o00;
          *reinterpret_cast<f4*>(xt + xq(p00 + 1, c4)) = o01;
          *reinterpret_cast<f4*>(xt + xq(p00 + IW, c4)) = o10;
          *reinterpret_cast<f4*>(xt + xq(p00 + IW + 1, c4)) = o11;
        }
      }
    } else {
    // Every read of this thread's items is issued before any of its writes:
    // with a read -> write chain per item (the compiler cannot move an item's
    // LDS reads above the previous item's write into the same array) the
    // items ran one LDS round trip after another.  Reads are branch-free
    // (outside-the-frame records read a valid dummy address; their value is
    // dropped below).
    constexpr int NU = (P_IN_PAD * C4L + 255) / 256;
    uint4 rec[NU];
#pragma unroll
    for (int k = 0; k < NU; ++k)
      rec[k] = reinterpret_cast<const uint4*>(uc)[min(tid + 256 * k, P_IN_PAD * C4L - 1) / C4L];
    f4 t00[NU], t01[NU], t10[NU], t11[NU];
#pragma unroll
    for (int k = 0; k < NU; ++k) {
      const int c4 = min(tid + 256 * k, P_IN_PAD * C4L - 1) % C4L;
      const bool in = rec[k].x != 0xFFFFFFFFu;
      const unsigned a = in ? rec[k].x : 0u, b = in ? rec[k].y : 0u;
      t00[k] = *reinterpret_cast<const f4*>(lr + (a & 0xFFFFu) + 4 * c4);
      t01[k] = *reinterpret_cast<const f4*>(lr + (a >> 16) + 4 * c4);
      t10[k] = *reinterpret_cast<const f4*>(lr + (b & 0xFFFFu) + 4 * c4);
      t11[k] = *reinterpret_cast<const f4*>(lr + (b >> 16) + 4 * c4);
    }
#pragma unroll
    for (int k = 0; k < NU; ++k) {
      const int i = tid + 256 * k;
      if (i < P_IN_PAD * C4L) {
        const int pix = i / C4L, c4 = i % C4L;
        f4 v = {0.f, 0.f, 0.f, 0.f};
        if (rec[k].x != 0xFFFFFFFFu) {
          // the lerps as explicit FMAs: every tile variant compiles the same
          // operations (left to contraction, variants fused differently)
          const float ly1 = __uint_as_float(rec[k].z), ly0 = 1.f - ly1;
          const float lx1 = __uint_as_float(rec[k].w), lx0 = 1.f - lx1;
          const f4 lx0v = {lx0, lx0, lx0, lx0}, lx1v = {lx1, lx1, lx1, lx1};
          const f4 ly0v = {ly0, ly0, ly0, ly0}, ly1v = {ly1, ly1, ly1, ly1};
          const f4 top = __builtin_elementwise_fma(lx1v, t01[k], lx0v * t00[k]);
          const f4 bot = __builtin_elementwise_fma(lx1v, t11[k], lx0v * t10[k]);
          v = __builtin_elementwise_fma(ly1v, bot, ly0v * top);
        }
        *reinterpret_cast<f4*>(xt + xq(pix, c4)) = v;
      }
    }
    }
  } else if constexpr (STEM_IN) {
    // The input tile is the stem's output region (IH x IW at half model
    // resolution, halo included), computed here from the frame: resize taps of
    // its x0 region -> LDS, then the stem's 3x3 s2 conv + ReLU6 -> xt, in the
    // same operation order as k_stem (bitwise the same activations).
    static_assert(MODE == MODE_IR_DIRECT && STRIDE == 1 && CIN == 16 && XP == 1, "stem fusion shape");
    constexpr int IH = L.IH, XH = 2 * IH + 1, XW = 2 * IW + 1, XWP = stem_xwp(IW);
    static_assert(XWP >= XW, "x0 row pitch");
    const StemParams& sp = p.stem;
    const int H = p.H, W = p.W;  // the stem's output = this block's input
    const uint8_t* fr = sp.frames + (long)n * sp.frame_stride;
    const int r0 = 2 * iy0 - 1, c0 = 2 * ix0 - 1;  // x0 region origin (model resolution)
    float* x0s = work;                            // [3][XH][XWP]
    float* sws = work + r4(3 * XH * XWP);          // [tap][16]
    float* sbs = sws + 27 * 16;
    std::conditional_t<WDMA, NoStaged, Staged<WIMG_F4>> st_w;
    if constexpr (WDMA) dma_f4<WIMG_F4>(wsrc, reinterpret_cast<f4*>(smem + L.w1));
    st_w.issue([&](int i) { return wsrc[i]; });
    // the stem weights as [tap][16]: thread i loads w[channel i % 16][tap i / 16]
    // (sp.w is [c][27]) and stores word i (consecutive banks, no transposing store)
    float wr[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i = min(tid + 256 * u, 27 * 16 - 1);
      wr[u] = sp.w[(i % 16) * 27 + i / 16];
    }
    const float sb = sp.b[min(tid, 15)];
    // Each thread resizes two pixels of one row of the region, columns lx and
    // lx + HW2: the row's source rows, its weight and their byte offsets are
    // worked out once for both (the resize is separable), and every tap is a
    // 32-bit byte offset off the frame's base (one saddr load, no 64-bit
    // address arithmetic).  The per-pixel arithmetic is prep_tap / prep_finish's,
    // operation for operation (bitwise the same floats).
    constexpr int HW2 = (XW + 1) / 2, NPAIR = XH * HW2, NR = (NPAIR + 255) / 256;
    // the frame as a raw buffer (wave-uniform base, range = the frame's bytes)
    const __amdgpu_buffer_rsrc_t frsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<void*>(uniform_ptr(fr)), 0, (int)min(sp.frame_stride, (long)0x7FFFFFF0), 0x00020000);
    uint32_t raw[NR][2][12];
    float dys[NR], dxs[NR][2];
    int lys[NR], lxs[NR];
#pragma unroll
    for (int u = 0; u < NR; ++u) {
#pragma clang fp contract(off)
      const int i = min(tid + 256 * u, NPAIR - 1);
      const int ly = i / HW2, lx = i - ly * HW2;
      lys[u] = ly;
      lxs[u] = lx;
      const int yy = min(max(r0 + ly, 0), sp.Hm - 1);
      const float fy = (float)yy * sp.ry;
      const float y0f = floorf(fmaxf(fy, 0.f));
      const unsigned y1 = (unsigned)min(sp.fh - 1, (int)ceilf(fy));
      dys[u] = fy - y0f;
      const unsigned rs = (unsigned)sp.row_stride;
      const unsigned t0 = (unsigned)y0f * rs, t1 = y1 * rs;  // frame bytes < 4 GiB
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int xx = min(max(c0 + min(lx + e * HW2, XW - 1), 0), sp.Wm - 1);
        const float fx = (float)xx * sp.rx;
        const float x0f = floorf(fmaxf(fx, 0.f));
        const unsigned x1 = (unsigned)min(sp.fw - 1, (int)ceilf(fx));
        dxs[u][e] = fx - x0f;
        const unsigned o0 = (unsigned)x0f * (unsigned)sp.fc, o1 = x1 * (unsigned)sp.fc;
        // byte loads through the frame's buffer descriptor: the channel is the
        // instruction's immediate offset, so a tap is one address add, not three
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          raw[u][e][c] = __builtin_amdgcn_raw_buffer_load_b8(frsrc, (int)(t0 + o0) + c, 0, 0);
          raw[u][e][3 + c] = __builtin_amdgcn_raw_buffer_load_b8(frsrc, (int)(t0 + o1) + c, 0, 0);
          raw[u][e][6 + c] = __builtin_amdgcn_raw_buffer_load_b8(frsrc, (int)(t1 + o0) + c, 0, 0);
          raw[u][e][9 + c] = __builtin_amdgcn_raw_buffer_load_b8(frsrc, (int)(t1 + o1) + c, 0, 0);
        }
      }
    }
    VSS_STAMP(6);  // every load issued
    // the two pixels at once on packed FP32 (prep_finish2)
#pragma unroll
    for (int u = 0; u < NR; ++u) {
      float o[2][3];
      prep_finish2(raw[u][0], raw[u][1], dys[u], dxs[u][0], dys[u], dxs[u][1], o[0], o[1]);
      const int ly = lys[u], yy = r0 + ly;
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int lx = lxs[u] + e * HW2, xx = c0 + lx;
        const bool in = tid + 256 * u < NPAIR && lx < XW;
        const bool valid = ((unsigned)yy < (unsigned)sp.Hm) & ((unsigned)xx < (unsigned)sp.Wm);
        if (in) {
#pragma unroll
          for (int c = 0; c < 3; ++c) x0s[(c * XH + ly) * XWP + lx] = valid ? o[e][c] : 0.f;
        }
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i = tid + 256 * u;
      if (i < 27 * 16) sws[i] = wr[u];
    }
    if (tid < 16) sbs[tid] = sb;
    // start of the forward: zero this frame's decoder norm accumulators (the stem's job)
    if (bx == 0 && by == 0)
      for (int i = tid; i < sp.acc_stride; i += 256) {
        if constexpr (COH)
          __hip_atomic_store(sp.acc_zero + (long)n * sp.acc_stride + i, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else
          sp.acc_zero[(long)n * sp.acc_stride + i] = 0ull;
      }
    st_w.commit([&](int i, f4 v) { wdst[i] = v; });
    VSS_STAMP(4);
    dma_wait<WDMA>();
    __syncthreads();
    VSS_STAMP(5);  // resized region in LDS: the stem conv starts
    // stem outputs of the region, 16-pixel blocks on the MFMA (stem_mfma,
    // bitwise k_stem's), zero outside the image
    {
      const StemTaps taps = stem_taps<XH * XWP, XWP>(sws, r, g);
      // every pixel of the region first (the pixels past P_IN land in xt's
      // padding, which nothing reads); the stem pixels outside the image are
      // zeroed after, border only, in the tiles that have any (below)
      if constexpr (VSS_SWZ) {
        // transposed: lane (r, g) holds channels 4g..4g+3 of pixel r, one
        // 16-B store into quad g of xt's quad-major planes
        const f4 bias4 = *reinterpret_cast<const f4*>(sbs + 4 * g);
        for (int blk = wave; blk < P_IN_PAD / 16; blk += 4) {
          const int pa = min(blk * 16 + r, P_IN - 1), py = pa / IW, px = pa - py * IW;
          const f4 acc = stem_mfma_t(taps, x0s + 2 * py * XWP + 2 * px, bias4);
          *reinterpret_cast<f4*>(xt + xq(blk * 16 + r, g)) = relu6v(acc);
        }
      } else {
        const float bias = sbs[r];
        for (int blk = wave; blk < P_IN_PAD / 16; blk += 4) {
          const int pa = min(blk * 16 + r, P_IN - 1), py = pa / IW, px = pa - py * IW;
          const f4 acc = stem_mfma(taps, x0s + 2 * py * XWP + 2 * px, bias);
          const int p0 = blk * 16 + 4 * g;
#pragma unroll
          for (int i = 0; i < 4; ++i) xt[xq(p0 + i, r >> 2) + (r & 3)] = relu6f(acc[i]);  // D[pixel 4g+i][channel r]
        }
      }
      // a tile at the image's edge: its pixels outside the image (the halo
      // row / column, and a partial tile's columns / rows past the image) are
      // the dw's zero padding — one pass over the region, each pixel as 4
      // float4s, in those tiles only
      const bool interior = iy0 >= 0 && iy0 + L.IH <= H && ix0 >= 0 && ix0 + IW <= W;
      if (!interior) {
        __syncthreads();
        for (int i = tid; i < P_IN * 4; i += 256) {
          // (quad-major: consecutive threads take consecutive pixels of one plane)
          const int q = L.XQM ? i / P_IN : i & 3, e = L.XQM ? i - q * P_IN : i >> 2, qy = e / IW, qx = e - qy * IW;
          const int yy = iy0 + qy, xx = ix0 + qx;
          if (yy < 0 || yy >= H || xx < 0 || xx >= W)
            *reinterpret_cast<f4*>(xt + xq(qy * IW + qx, q)) = f4{0.f, 0.f, 0.f, 0.f};
        }
      }
    }

  } else {
    const int H = p.H, W = p.W;
    const float* xn = p.x + (long)n * H * W * CIN;
    static_assert(CIN % 16 == 0, "16-channel staging items");
    constexpr int GI = CIN / 16;  // 16-channel items per pixel
    Staged16<P_IN_PAD * GI, XP, VSS_STAGE16> st_x;
    std::conditional_t<WDMA, NoStaged, Staged<WIMG_F4>> st_w;
    if constexpr (WDMA && VSS_WDMA_FIRST) dma_f4<WIMG_F4>(wsrc, reinterpret_cast<f4*>(smem + L.w1));
    {
      const float* xb[XP];
#pragma unroll
      for (int q = 0; q < XP; ++q) xb[q] = xn + q * p.x_part_stride;
      st_x.issue(xb, [&](int i) {
        const int pix = i / GI, gq = i - pix * GI, py = pix / IW;
        const int yy = min(max(iy0 + py, 0), H - 1), xx = min(max(ix0 + pix - py * IW, 0), W - 1);
        return (unsigned)((yy * W + xx) * CIN + 16 * gq);
      });
    }
    if constexpr (WDMA && !VSS_WDMA_FIRST) dma_f4<WIMG_F4>(wsrc, reinterpret_cast<f4*>(smem + L.w1));
    st_w.issue([&](int i) { return wsrc[i]; });
    VSS_STAMP(6);  // every load issued
    st_x.commit_sum([&](int i, int k, f4 v) {
      const int pix = i / GI, c4 = (i - pix * GI) * 4 + k;
      if constexpr (MODE == MODE_IR_EXPAND) {
        // no validity test: an expand layer's input pixels outside the image
        // only feed hidden pixels that the expand loop zeroes (its clamp
        // limit is 0 there), and the loads were clamped to real pixels
        *reinterpret_cast<f4*>(xt + xq(pix, c4)) = to_operand<PREC>(v);
        if constexpr (RES) {
          const int py = pix / IW, px = pix - py * IW;
          if (py >= 1 && py <= TH && px >= 1 && px <= TW)
            *reinterpret_cast<f4*>(smem + L.xr + rq((py - 1) * TW + px - 1, c4)) = v;
        }
      } else {
        const int py = pix / IW, px = pix % IW;
        const int yy = iy0 + py, xx = ix0 + px;
        const bool valid = pix < P_IN && yy >= 0 && yy < H && xx >= 0 && xx < W;
        *reinterpret_cast<f4*>(xt + xq(pix, c4)) = valid ? v : f4{0.f, 0.f, 0.f, 0.f};
      }
    });
    st_w.commit([&](int i, f4 v) { wdst[i] = v; });
    VSS_STAMP(4);
  }
  dma_wait<WDMA>();
  __syncthreads();
  VSS_STAMP(1);

  // ---- main: per-wave work units ----
  // The accumulators start at a wave's first chunk, whose MFMAs take the
  // inline constant 0 as their C operand (the first chunk is peeled off the
  // chunk loop below): no zeroing moves (NACC x 4 VALU per wave).
  f4 acc[L.NACC];
  const int pw = wave % PW, cw = wave / PW;
  // dw pixel runs (dw_run): element j of super-block sb for this lane
  constexpr int XR = dw_run(TW, NPB, MODE == MODE_IR_EXPAND ? 1 : PW);
  static_assert(NPB % XR == 0 && NPBW % XR == 0, "dw runs");
  auto run_pix = [&](int sb, int j) {
    if constexpr (XR == 1) return sb * 16 + block_pix(r);
    else return (sb * (16 * XR / TW) + r / (TW / XR)) * TW + (r % (TW / XR)) * XR + j;
  };

  if constexpr (MODE == MODE_IR_EXPAND) {
    constexpr int HSD = hid_stride(STRIDE);
    // the wave's hidden chunk: quad-major planes of L.HPL floats (VSS_SWZ), or
    // pixel-major with HSD floats per pixel
    float* hid = work + wave * (L.HPL ? 4 * L.HPL : P_IN_PAD * HSD);
    auto hq = [&](int pix, int q) {
      if constexpr (L.HPL != 0) return q * L.HPL + 4 * pix;
      else return pix * HSD + 4 * q;
    };
    constexpr int NK = CIN / 16;
    constexpr int NCBI = P_IN_PAD / 16;
    static_assert(NCBI <= 32, "one validity bit per input pixel block");
    // bit cb: this lane's pixel cb * 16 + r of the input tile lies in the
    // image (else its hidden values are the dw's zero padding).  Once per
    // wave, and only in tiles at the image's edge; the chunk loop turns the
    // bit into the clamp limit of its ReLU6 (6, or 0 for a padding pixel),
    // one v_med3_f32 per element either way.  Pixels past P_IN are never read.
    unsigned vmask = ~0u;
    if (!(iy0 >= 0 && iy0 + L.IH <= p.H && ix0 >= 0 && ix0 + IW <= p.W)) {
      vmask = 0u;
#pragma unroll
      for (int cb = 0; cb < NCBI; ++cb) {
        const int pix = cb * 16 + r, py = pix / IW, yy = iy0 + py, xx = ix0 + pix - py * IW;
        vmask |= (yy >= 0 && yy < p.H && xx >= 0 && xx < p.W) ? 1u << cb : 0u;
      }
    }
    auto expand_chunk = [&](int ck, auto first) {
      constexpr bool FIRST = decltype(first)::value;
      const int c0 = ck << 4;
      typename AFrag<PREC>::T aw[NK];
#pragma unroll
      for (int s = 0; s < NK; ++s) aw[s] = lds_a<PREC>(w1s, L.LD1, c0 + r, 16 * s + 4 * g);
      const f4 bias = *reinterpret_cast<const f4*>(b1s + c0 + 4 * g);
      // (the unroll count from template parameters only: a lambda's pragma
      // cannot name the enclosing function's constexpr locals)
      constexpr int UNRL = block_lds(MODE, STRIDE, TH, TW, CIN, CSKIP, CH, COUT, STEM_IN).P_in_pad / 16 <= 6
                               ? block_lds(MODE, STRIDE, TH, TW, CIN, CSKIP, CH, COUT, STEM_IN).P_in_pad / 16
                               : 2;
#pragma unroll UNRL
      for (int cb = 0; cb < NCBI; ++cb) {
        const int pix = cb * 16 + r;
        f4 d = bias;  // the expand's bias enters as the MFMA accumulator
#pragma unroll
        for (int s = 0; s < NK; ++s) d = mma16_op<PREC>(d, aw[s], *reinterpret_cast<const f4*>(xt + xq(pix, 4 * s + g)));
        *reinterpret_cast<f4*>(hid + hq(pix, g)) = clampv(d, (vmask >> cb) & 1u ? 6.f : 0.f);
      }
      wave_sync();
      // dw 3x3 computed straight into the project MFMA's B layout: lane (r, g)
      // evaluates pixel r of the block for hidden channels c0+4g..c0+4g+3
      {
        f4 wk[9];
#pragma unroll
        for (int t = 0; t < 9; ++t) wk[t] = *reinterpret_cast<const f4*>(wdws + t * CH + c0 + 4 * g);
        const f4 bb = *reinterpret_cast<const f4*>(bdws + c0 + 4 * g);
        typename AFrag<PREC>::T a2[NCB];
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb) a2[cb] = lds_a<PREC>(w2s, L.LD2, cb * 16 + r, c0 + 4 * g);
#pragma unroll
        for (int q = 0; q < NPB / XR; ++q) {
          const int pix0 = run_pix(q, 0), ly = pix0 / TW, lx0 = pix0 % TW;
          f4 a[XR];
#pragma unroll
          for (int j = 0; j < XR; ++j) a[j] = bb;
#pragma unroll
          for (int ky = 0; ky < 3; ++ky) {
            constexpr int NT = STRIDE * (XR - 1) + 3;
            f4 t[NT];
#pragma unroll
            for (int u = 0; u < NT; ++u)
              t[u] = *reinterpret_cast<const f4*>(hid + hq((STRIDE * ly + ky) * IW + STRIDE * lx0 + u, g));
#pragma unroll
            for (int j = 0; j < XR; ++j)
#pragma unroll
              for (int kx = 0; kx < 3; ++kx) a[j] = __builtin_elementwise_fma(wk[ky * 3 + kx], t[STRIDE * j + kx], a[j]);
          }
#pragma unroll
          for (int j = 0; j < XR; ++j) {
            const f4 b = to_operand<PREC>(relu6v(a[j]));
#pragma unroll
            for (int cb = 0; cb < NCB; ++cb) {
              f4& ac = acc[(q * XR + j) * NCB + cb];
              if constexpr (FIRST)
                ac = mma16_op<PREC>(f4{0.f, 0.f, 0.f, 0.f}, a2[cb], b);
              else
                ac = mma16_op<PREC>(ac, a2[cb], b);
            }
          }
        }
      }
      wave_sync();  // this chunk's hid reads before the next chunk's expand writes
    };
    static_assert(NCHUNK >= 4, "every wave has a first chunk");
    expand_chunk(wave, ChunkTag<true>{});
    for (int ck = wave + 4; ck < NCHUNK; ck += 4) expand_chunk(ck, ChunkTag<false>{});
  } else {
    // dw 3x3 straight into the project MFMA's B layout (lane (r, g): pixel r
    // of the block, channels c0+4g..c0+4g+3); no LDS round trip, no syncs.
    // Chunk-outer: the chunk's dw taps and project fragments are read from
    // LDS once and reused for every pixel block of the wave (each
    // accumulator still sums its chunks in the same order).
    auto dw_chunk = [&](int ck, auto first) {
      constexpr bool FIRST = decltype(first)::value;
      const int c0 = ck << 4;
      f4 wk[9];
#pragma unroll
      for (int t = 0; t < 9; ++t) wk[t] = *reinterpret_cast<const f4*>(wdws + t * CH + c0 + 4 * g);
      const f4 bb = *reinterpret_cast<const f4*>(bdws + c0 + 4 * g);
      typename AFrag<PREC>::T a2[NCB];
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) a2[cb] = lds_a<PREC>(w2s, L.LD2, cb * 16 + r, c0 + 4 * g);
#pragma unroll
      for (int q = 0; q < NPBW / XR; ++q) {
        const int pix0 = run_pix(pw + q * PW, 0), ly = pix0 / TW, lx0 = pix0 % TW;
        f4 a[XR];
#pragma unroll
        for (int j = 0; j < XR; ++j) a[j] = bb;
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) {
          f4 t[XR + 2];
#pragma unroll
          for (int u = 0; u < XR + 2; ++u)
            t[u] = *reinterpret_cast<const f4*>(xt + xq((ly + ky) * IW + lx0 + u, (c0 >> 2) + g));
#pragma unroll
          for (int j = 0; j < XR; ++j)
#pragma unroll
            for (int kx = 0; kx < 3; ++kx) a[j] = __builtin_elementwise_fma(wk[ky * 3 + kx], t[j + kx], a[j]);
        }
#pragma unroll
        for (int j = 0; j < XR; ++j) {
          if constexpr (MODE == MODE_IR_DIRECT) a[j] = relu6v(a[j]);
          const f4 b = to_operand<PREC>(a[j]);
#pragma unroll
          for (int cb = 0; cb < NCB; ++cb) {
            f4& ac = acc[(q * XR + j) * NCB + cb];
            if constexpr (FIRST)
              ac = mma16_op<PREC>(f4{0.f, 0.f, 0.f, 0.f}, a2[cb], b);
            else
              ac = mma16_op<PREC>(ac, a2[cb], b);
          }
        }
      }
    };
    static_assert(CS <= NCHUNK, "every wave has a first chunk");
    dw_chunk(cw, ChunkTag<true>{});
    for (int ck = cw + CS; ck < NCHUNK; ck += CS) dw_chunk(ck, ChunkTag<false>{});
  }

  // ---- epilogue: slabs -> fixed-order sum, bias, residual, store ----
  if constexpr (MODE == MODE_IR_DIRECT && CS == 1) {
    // one wave computes every channel of its pixels (a single 16-channel
    // chunk): bias and residual added in registers and stored straight from
    // the accumulators — the same additions in the same order as the slab
    // path, without its LDS round trip and two barriers (b1)
    VSS_STAMP(2);
    const Gm<COH> gy(p.y + (long)n * Ho * Wo * COUT);
#pragma unroll
    for (int q = 0; q < NPBW / XR; ++q)
#pragma unroll
      for (int j = 0; j < XR; ++j) {
        const int pix = run_pix(pw + q * PW, j), ly = pix / TW, lx = pix % TW;
        const int oy = oy0 + ly, ox = ox0 + lx;
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb) {
          f4 v = acc[(q * XR + j) * NCB + cb] + *reinterpret_cast<const f4*>(b2s + cb * 16 + 4 * g);
          if constexpr (RES) v = v + *reinterpret_cast<const f4*>(xt + xq((ly + 1) * IW + lx + 1, cb * 4 + g));
          if (oy < Ho && ox < Wo) gy.st(((long)oy * Wo + ox) * COUT + cb * 16 + 4 * g, v);
        }
      }
  } else {
  __syncthreads();  // every wave is done with its scratch (reused as slabs)
  VSS_STAMP(2);
  {
#pragma unroll
    for (int q = 0; q < NPBW / XR; ++q)
#pragma unroll
      for (int j = 0; j < XR; ++j)
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb)
          *reinterpret_cast<f4*>(slabs + sq(cw, run_pix(pw + q * PW, j), cb * 4 + g)) = acc[(q * XR + j) * NCB + cb];
  }
  __syncthreads();
  constexpr int C4O = COUT / 4, NOUT = (P_OUT * C4O + 255) / 256;
  const Gm<COH> gy(p.y + ks * p.y_part_stride + (long)n * Ho * Wo * COUT);
  // the decoder keeps its outputs in registers until its stats are done: a
  // workgroup barrier waits for every store issued before it (vmcnt(0))
  f4 outv[MODE == MODE_DEC ? NOUT : 1];
#pragma unroll
  for (int k = 0; k < NOUT; ++k) {
    const int i = tid + 256 * k;
    if (i < P_OUT * C4O) {
      const int pix = i / C4O, c4 = i % C4O;
      const int ly = pix / TW, lx = pix % TW;
      const int oy = oy0 + ly, ox = ox0 + lx;
      const bool valid = oy < Ho && ox < Wo;
      // slabs of the CS waves that own this pixel block, summed in wave order
      f4 v = *reinterpret_cast<const f4*>(slabs + sq(0, pix, c4));
#pragma unroll
      for (int s = 1; s < CS; ++s) v = v + *reinterpret_cast<const f4*>(slabs + sq(s, pix, c4));
      if (KS == 1 || ks == 0) {  // bias and residual belong to part 0
        v = v + *reinterpret_cast<const f4*>(b2s + 4 * c4);
        if constexpr (RES) {
          if constexpr (MODE == MODE_IR_EXPAND)
            v = v + *reinterpret_cast<const f4*>(smem + L.xr + rq(pix, c4));
          else
            v = v + *reinterpret_cast<const f4*>(xt + xq((ly + 1) * IW + lx + 1, c4));
        }
      }
      if constexpr (MODE == MODE_DEC) {
        outv[k] = v;
        *reinterpret_cast<f4*>(slabs + sq(0, pix, c4)) = valid ? v : f4{0.f, 0.f, 0.f, 0.f};
      } else if (valid) {
        gy.st(((long)oy * Wo + ox) * COUT + 4 * c4, v);
      }
    }
  }
  if constexpr (MODE == MODE_DEC) {
    // this tile's exact fixed-point sums, added to the frame's accumulator
    // (integer adds are associative: the totals do not depend on the tiling
    // or on the order the workgroups arrive in)
    __syncthreads();
    constexpr int G = 256 / COUT;
    static_assert((P_OUT + G - 1) / G <= 16, "f64 lane sums: at most 16 terms (bound above)");
    long long* st64 = reinterpret_cast<long long*>(stt);
    const int c = tid % COUT, gg = tid / COUT;
    if (gg < G) {
      // the lane's terms are integers (rint of v*2^32, v*v*2^24); their f64 sums
      // are exact while no partial sum reaches 2^53.  The q terms are >= 0, so
      // q < 2^51 at the end means every partial q was exact, and then
      // sum |s terms| <= sqrt(T * sum v^2 2^64) = sqrt(T q 2^40) < 2^48 for
      // T = ceil(P_OUT/G) <= 16 — s was exact too.  Both sums are then
      // integers below 2^51 in magnitude, read out as int64 by the 1.5 * 2^52
      // bias (one f64 add and one 64-bit subtract, instead of an f64 -> i64
      // conversion sequence), the same integers as summing the terms as int64.
      // A lane whose q reaches 2^51 (|v| ~ 2.9k) adds its terms again as int64
      // (exact up to where the int64 frame totals overflow), so large pre-norm
      // activations cannot round silently or make the totals depend on the
      // tiling.  The asm statement keeps that rare path a branch: if-converted,
      // its int64 conversions ran on every lane (~60 VALU per wave).
      double s = 0.0, q = 0.0;
#pragma unroll
      for (int pix = 0; pix < P_OUT; pix += G) {
        if (pix + gg < P_OUT) {
          const float v = slabs[sq(0, pix + gg, c >> 2) + (c & 3)];
          s += (double)__builtin_rintf(v * 0x1p32f);
          q += (double)__builtin_rintf(v * v * 0x1p24f);
        }
      }
      constexpr double kBias = 0x1.8p52;
      long long si = __double_as_longlong(s + kBias) - __double_as_longlong(kBias);
      long long qi = __double_as_longlong(q + kBias) - __double_as_longlong(kBias);
      if (q >= 0x1p51) {
        asm volatile("" ::: "memory");
        si = 0;
        qi = 0;
        for (int pix = 0; pix < P_OUT; pix += G) {
          if (pix + gg < P_OUT) {
            const float v = slabs[sq(0, pix + gg, c >> 2) + (c & 3)];
            si += (long long)__builtin_rintf(v * 0x1p32f);
            qi += (long long)__builtin_rintf(v * v * 0x1p24f);
          }
        }
      }
      st64[gg * COUT + c] = si;
      st64[256 + gg * COUT + c] = qi;
    }
    __syncthreads();
    if (tid < 2 * COUT) {
      const int base = tid < COUT ? tid : 256 + (tid - COUT);
      long long t = 0;
#pragma unroll
      for (int k = 0; k < G; ++k) t += st64[base + k * COUT];
      const int slot = (by * p.tiles_x + bx) % kAccSlots;
      __hip_atomic_fetch_add(p.out_acc + (long)n * p.acc_stride + slot * 2 * COUT + tid, (unsigned long long)t,
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
#pragma unroll
    for (int k = 0; k < NOUT; ++k) {
      const int i = tid + 256 * k;
      if (i < P_OUT * C4O) {
        const int pix = i / C4O, c4 = i % C4O;
        const int oy = oy0 + pix / TW, ox = ox0 + pix % TW;
        if (oy < Ho && ox < Wo) gy.st(((long)oy * Wo + ox) * COUT + 4 * c4, outv[k]);
      }
    }
  }
  }  // slab epilogue
  if constexpr (STEM_IN) {
    // the stem activation itself (the tile centre of xt, intact through the
    // epilogue), only under VSS_OPT_KEEP_STEM (null otherwise: no layer reads
    // it): what vss_read_layer reports for the stem; last, so that no barrier
    // waits for these stores
    const Gm<COH> gst(p.stem.y + (long)n * p.H * p.W * 16);
    for (int i = tid; p.stem.y != nullptr && i < TH * TW * 4; i += 256) {
      const int pix = i >> 2, q = i & 3;
      const int yy = oy0 + pix / TW, xx = ox0 + pix % TW;
      if (yy < p.H && xx < p.W)
        gst.st(((long)yy * p.W + xx) * 16 + 4 * q,
               *reinterpret_cast<const f4*>(xt + xq((pix / TW + 1) * IW + pix % TW + 1, q)));
    }
  }
  VSS_STAMP(3);
}

template <int MODE, int STRIDE, int TH, int TW, int CIN, int CSKIP, int CH, int COUT, int FLAGS, int PREC>
__global__ __launch_bounds__(256) void k_block(BlockParams p) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const TileIdx t = xcd_tile();
  block_body<MODE, STRIDE, TH, TW, CIN, CSKIP, CH, COUT, FLAGS, PREC, false>(p, t.x, t.y, t.z, smem);
}

// ---------------------------------------------------------------------------
// b1 with the stem fused, on a wide workgroup (kWideThreads = 1024 threads, 16
// waves) and a tile four to eight times block_body's.  The arithmetic is
// block_body<MODE_IR_DIRECT, 1, .., 16, 0, 16, 16, STEM_IN | residual>'s,
// operation for operation (prep_tap / prep_load / prep_finish of the resize,
// stem_mfma, the dw taps in ky-major order, relu6, to_operand, one project
// MFMA, + bias, + residual), so the activations are bitwise the same
// (test_stem_fusion_bitwise, test_results_independent_of_tiling).  What
// changes is the overlap: a 4 x 16 tile recomputes its resized region 1.9x
// and its stem region 1.7x per output (the halo), an 8 x 32 tile 1.4x / 1.3x,
// and each of the 1024 threads has fewer resized pixels to gather and lerp
// (1.4 vs 1.9) — b1 is bound by the resize's VALU issue and byte gathers.
// Only for this layer shape (16 -> 16 direct, stride 1), so it lives outside
// the block registry's generator: block_registry() appends its entries.
template <int TH, int TW, int PREC>
__global__ __launch_bounds__(kWideThreads) void k_stem_b1(BlockParams p) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int WT = kWideThreads, NWAVE = WT / 64;
  constexpr StemB1Lds S = stem_b1_lds(TH, TW);
  constexpr int IH = S.IH, IW = S.IW, P_IN = S.P_IN, P_IN_PAD = S.P_IN_PAD, XS = S.XS;
  constexpr int XH = S.XH, XW = S.XW, XWP = S.XWP, NX = (XH * XW + WT - 1) / WT;
  constexpr BlockLds B = block_lds(MODE_IR_DIRECT, 1, TH, TW, 16, 0, 16, 16, 1);
  constexpr int WIMG4 = (B.wimg_end - B.w1) / 4;
  static_assert(WIMG4 <= WT && 27 * 16 <= WT, "one weight element per thread");
  float* x0s = smem + S.x0;
  float* sws = smem + S.sw;
  float* sbs = smem + S.sb;
  float* xt = smem + S.xt;
  float* wim = smem + S.wim;
  const TileIdx tl = xcd_tile();
  const int bx = tl.x, by = tl.y, n = tl.z;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 15, g = lane >> 4;
  const int oy0 = by * TH, ox0 = bx * TW, iy0 = oy0 - 1, ix0 = ox0 - 1;
  const StemParams& sp = p.stem;
  const int H = p.H, W = p.W;  // the stem's output = b1's input
  const uint8_t* fr = sp.frames + (long)n * sp.frame_stride;
  const int r0 = 2 * iy0 - 1, c0 = 2 * ix0 - 1;  // x0 region origin (model resolution)
  // every load issued first: the weight image, the stem's weights, the frame taps
  const f4 wv = reinterpret_cast<const f4*>(p.wimg)[min(tid, WIMG4 - 1)];
  const float swr = sp.w[min(tid, 27 * 16 - 1)];
  const float sb = sp.b[min(tid, 15)];
  uint32_t raw[NX][12];
  float dys[NX], dxs[NX];
#pragma unroll
  for (int u = 0; u < NX; ++u) {
    const int i = min(tid + WT * u, XH * XW - 1);
    const int ly = i / XW, lx = i - ly * XW;
    const int yy = min(max(r0 + ly, 0), sp.Hm - 1), xx = min(max(c0 + lx, 0), sp.Wm - 1);
    const PrepTap t = prep_tap(fr, sp.row_stride, sp.fc, sp.fh, sp.fw, sp.ry, sp.rx, yy, xx);
    prep_load(t, raw[u]);
    dys[u] = t.dy;
    dxs[u] = t.dx;
  }
  float o[NX][3];
#pragma unroll
  for (int u = 0; u < NX; u += 2) {
    if (u + 1 < NX)
      prep_finish2(raw[u], raw[u + 1], dys[u], dxs[u], dys[u + 1], dxs[u + 1], o[u], o[u + 1]);
    else
      prep_finish(raw[u], dys[u], dxs[u], o[u]);
  }
#pragma unroll
  for (int u = 0; u < NX; ++u) {
    const int i = tid + WT * u;
    if (i < XH * XW) {
      const int ly = i / XW, lx = i - ly * XW;
      const int yy = r0 + ly, xx = c0 + lx;
      const bool valid = yy >= 0 && yy < sp.Hm && xx >= 0 && xx < sp.Wm;
#pragma unroll
      for (int c = 0; c < 3; ++c) x0s[(c * XH + ly) * XWP + lx] = valid ? o[u][c] : 0.f;
    }
  }
  if (tid < WIMG4) reinterpret_cast<f4*>(wim)[tid] = wv;
  if (tid < 27 * 16) sws[(tid % 27) * 16 + tid / 27] = swr;  // sp.w is [c][27]
  if (tid < 16) sbs[tid] = sb;
  // start of the forward: zero this frame's decoder norm accumulators (the stem's job)
  if (bx == 0 && by == 0)
    for (int i = tid; i < sp.acc_stride; i += WT) sp.acc_zero[(long)n * sp.acc_stride + i] = 0ull;
  __syncthreads();
  // the stem over the region, 16-pixel blocks on the MFMA (stem_mfma), zero outside the image
  {
    const StemTaps taps = stem_taps<XH * XWP, XWP>(sws, r, g);
    const float bias = sbs[r];
    const bool interior = iy0 >= 0 && iy0 + IH <= H && ix0 >= 0 && ix0 + IW <= W;
    for (int blk = wave; blk < P_IN_PAD / 16; blk += NWAVE) {
      const int pa = min(blk * 16 + r, P_IN - 1), py = pa / IW, px = pa - py * IW;
      const f4 acc = stem_mfma(taps, x0s + 2 * py * XWP + 2 * px, bias);
      const int p0 = blk * 16 + 4 * g;
      if (interior) {
#pragma unroll
        for (int i = 0; i < 4; ++i) xt[(p0 + i) * XS + r] = p0 + i < P_IN ? relu6f(acc[i]) : 0.f;
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {  // D[pixel 4g+i][channel r]
          const int pp = p0 + i, qy = pp / IW, qx = pp - qy * IW;
          const int yy = iy0 + qy, xx = ix0 + qx;
          const bool valid = pp < P_IN && yy >= 0 && yy < H && xx >= 0 && xx < W;
          xt[pp * XS + r] = valid ? relu6f(acc[i]) : 0.f;
        }
      }
    }
  }
  __syncthreads();
  // b1: dw 3x3 -> relu6 -> project 16 -> 16 (one MFMA) -> + bias -> + residual;
  // lane (r, g) = pixel r of the wave's block, channels 4g..4g+3, in registers
  // from the dw taps to the store
  const uint16_t* w2s = reinterpret_cast<const uint16_t*>(wim + (B.w2 - B.w1));
  const float* wdws = wim + (B.wdw - B.w1);
  const float* bdws = wim + (B.bdw - B.w1);
  const float* b2s = wim + (B.b2 - B.w1);
  f4 wk[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) wk[t] = *reinterpret_cast<const f4*>(wdws + t * 16 + 4 * g);
  const f4 bb = *reinterpret_cast<const f4*>(bdws + 4 * g);
  const typename AFrag<PREC>::T a2 = lds_a<PREC>(w2s, B.LD2, r, 4 * g);
  const f4 bias2 = *reinterpret_cast<const f4*>(b2s + 4 * g);
  const int Ho = p.Ho, Wo = p.Wo;
  float* yn = p.y + (long)n * Ho * Wo * 16;
  float* st = p.stem.y ? p.stem.y + (long)n * H * W * 16 : nullptr;  // VSS_OPT_KEEP_STEM
  for (int pb = wave; pb < TH * TW / 16; pb += NWAVE) {
    const int pix = pb * 16 + block_pix(r), ly = pix / TW, lx = pix % TW;
    f4 a = bb;
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx)
        a = __builtin_elementwise_fma(wk[ky * 3 + kx], *reinterpret_cast<const f4*>(xt + ((ly + ky) * IW + lx + kx) * XS + 4 * g), a);
    a = relu6v(a);
    const f4 b = to_operand<PREC>(a);
    f4 v = mma16_op<PREC>(f4{0.f, 0.f, 0.f, 0.f}, a2, b);
    const f4 centre = *reinterpret_cast<const f4*>(xt + ((ly + 1) * IW + lx + 1) * XS + 4 * g);
    v = v + bias2;
    v = v + centre;
    const int oy = oy0 + ly, ox = ox0 + lx;
    if (oy < Ho && ox < Wo) {
      *reinterpret_cast<f4*>(yn + ((long)oy * Wo + ox) * 16 + 4 * g) = v;
      if (st) *reinterpret_cast<f4*>(st + ((long)oy * W + ox) * 16 + 4 * g) = centre;
    }
  }
}

// ---------------------------------------------------------------------------
// Head: mask tile 16 x 64; logits over the (10 x 34) low-res region in LDS.
template <int C, bool COH>
__device__ __forceinline__ void head_body(const HeadParams& p, int bx, int by, int n, float* smem) {
  constexpr int OTH = kHeadTH, OTW = kHeadTW, ZR = kHeadZR, ZC = kHeadZC, ZCP = kHeadZCP, NZ = (ZR * ZC + 255) / 256;
  static_assert(C == 16, "head LDS carve (kHeadLds) assumes 16 channels");
  unsigned long long* slots = reinterpret_cast<unsigned long long*>(smem);  // [kAccSlots][2][C]
  float (*z)[ZCP] = reinterpret_cast<float (*)[ZCP]>(smem + kAccSlots * 2 * C * 2);
  float* sc = smem + kAccSlots * 2 * C * 2 + r4(ZR * ZCP);
  float* sh = sc + C;
  float* wv = sh + C;
  const int tid = threadIdx.x;
  const int oy0 = by * OTH, ox0 = bx * OTW;
  const int h = p.h, w = p.w_;
  const int zr0 = oy0 / 2 - 1, zc0 = ox0 / 2 - 1;
  VSS_STAMP(0);
  // issue this thread's d3 loads before the statistics reduction
  const Gm<COH> gx(p.x + (long)n * h * w * C);
  f4 xv[NZ][C / 4];
#pragma unroll
  for (int u = 0; u < NZ; ++u) {
    const int i = min(tid + 256 * u, ZR * ZC - 1);
    const int zr = i / ZC, zc = i - zr * ZC;
    const int yy = min(max(zr0 + zr, 0), h - 1), xx = min(max(zc0 + zc, 0), w - 1);
#pragma unroll
    for (int q = 0; q < C / 4; ++q) xv[u][q] = gx.ldu((unsigned)((yy * w + xx) * C + 4 * q));
  }
  // the d3 norm: all slots of the frame's exact totals (2 x C int64 per slot)
  {
    const Gm<COH> ga(reinterpret_cast<const float*>(p.in_acc + (long)n * p.acc_stride));
    for (int i = tid; i < kAccSlots * C; i += 256) reinterpret_cast<f4*>(slots)[i] = ga.ld(4L * i);
  }
  if (tid < C) wv[tid] = p.w[tid];
  __syncthreads();
  if (tid < C) {
    unsigned long long s_fx = 0, q_fx = 0;
#pragma unroll
    for (int k = 0; k < kAccSlots; ++k) {
      s_fx += slots[k * 2 * C + tid];
      q_fx += slots[k * 2 * C + C + tid];
    }
    norm_affine(s_fx, q_fx, p.inv_hw, p.eps, p.gamma[tid], p.beta[tid], sc + tid, sh + tid);
  }
  __syncthreads();
  VSS_STAMP(1);
#pragma unroll
  for (int u = 0; u < NZ; ++u) {
    const int i = tid + 256 * u;
    if (i < ZR * ZC) {
      float acc = 0.f;
#pragma unroll
      for (int q = 0; q < C / 4; ++q) {
        const f4 a = reluv(xv[u][q] * *reinterpret_cast<const f4*>(sc + 4 * q) + *reinterpret_cast<const f4*>(sh + 4 * q));
        acc += a.x * wv[4 * q] + a.y * wv[4 * q + 1] + a.z * wv[4 * q + 2] + a.w * wv[4 * q + 3];
      }
      z[i / ZC][i % ZC] = acc + p.b;
    }
  }
  __syncthreads();
  VSS_STAMP(2);
  // bilinear x2 (align_corners=False) by 2 x 2 output blocks: output rows 2m
  // and 2m + 1 lie between logit rows (m - 1, m) at weights (0.25, 0.75) and
  // (m, m + 1) at (0.75, 0.25), columns alike, so one block reads a 3 x 3
  // logit window at constant weights: per logit row the two horizontal
  // interpolants, then the four vertical ones.  The region's rows / columns
  // outside the image hold the edge logits (clamped loads), which is the
  // clamp of the source index.  One block per thread (16 x 64 = 256 blocks).
  static_assert(OTH * OTW == 4 * 256 && OTW == 64 && ZR == OTH / 2 + 2 && ZC == OTW / 2 + 2, "head blocks");
  {
    const int by2 = tid >> 5, bx2 = tid & 31;
    float hz[3][2];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const float a = z[by2 + r][bx2], b = z[by2 + r][bx2 + 1], c = z[by2 + r][bx2 + 2];
      hz[r][0] = __builtin_fmaf(0.75f, b, 0.25f * a);  // column 2n
      hz[r][1] = __builtin_fmaf(0.25f, c, 0.75f * b);  // column 2n + 1
    }
    const int oy = oy0 + 2 * by2, ox = ox0 + 2 * bx2;
    float* mrow = p.mask + ((long)n * p.Hm + oy) * p.Wm + ox;
#pragma unroll
    for (int dy = 0; dy < 2; ++dy) {
      float o[2];
#pragma unroll
      for (int dx = 0; dx < 2; ++dx) {
        const float v = dy == 0 ? __builtin_fmaf(0.75f, hz[1][dx], 0.25f * hz[0][dx])
                                : __builtin_fmaf(0.25f, hz[2][dx], 0.75f * hz[1][dx]);
        // sigmoid from the hardware exp2 and reciprocal (v_exp_f32, v_rcp_f32:
        // ~1e-7 off the libm form, against the 1e-3 mask tolerance)
        o[dx] = __builtin_amdgcn_rcpf(1.0f + __expf(-v));
      }
      if (oy + dy < p.Hm) {
        if (ox + 1 < p.Wm)
          *reinterpret_cast<float2*>(mrow + dy * p.Wm) = float2{o[0], o[1]};
        else if (ox < p.Wm)
          mrow[dy * p.Wm] = o[0];
      }
    }
  }
  VSS_STAMP(3);
}

template <int C>
__global__ __launch_bounds__(256) void k_head(HeadParams p) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const TileIdx t = xcd_tile();
  head_body<C, false>(p, t.x, t.y, t.z, smem);
}

// ---------------------------------------------------------------------------
// Host-visible launch table (used by vss_capi.hip): one entry per compiled
// block shape, generated from the layer table by tools/gen_registry.py and
// dealt to kRegistryShards files (vss_registry_<k>.inc) so that the shapes
// compile in parallel: this file is compiled once per shard with
// -DVSS_SHARD=<k>; shard 0 also holds the stem, head and preprocessing
// kernels and the concatenated table.
#ifndef VSS_SHARD
#define VSS_SHARD 0
#endif
#define VSS_BLOCK(M, S, TH, TW, CI, CK, CH, CO, FL)                                    \
  {M, S, TH, TW, CI, CK, CH, CO, FL,                                                  \
   {k_block<M, S, TH, TW, CI, CK, CH, CO, FL, PREC_F32>,                              \
    k_block<M, S, TH, TW, CI, CK, CH, CO, FL, PREC_BF16X2>}},
#define VSS_STR2(x) #x
#define VSS_STR(x) VSS_STR2(x)
#define VSS_CAT2(a, b) a##b
#define VSS_CAT(a, b) VSS_CAT2(a, b)
static const BlockEntry kShardBlocks[] = {
#include VSS_STR(VSS_CAT(vss_registry_, VSS_SHARD).inc)
};
#undef VSS_BLOCK

const BlockEntry* VSS_CAT(registry_shard_, VSS_SHARD)(int* count) {
  *count = (int)(sizeof(kShardBlocks) / sizeof(kShardBlocks[0]));
  return kShardBlocks;
}

#if VSS_SHARD == 0
#define VSS_SHARD_FN(k) const BlockEntry* registry_shard_##k(int* count);
#include "vss_registry_shards.inc"
#undef VSS_SHARD_FN

// The wide stem + b1 kernel's tiles (k_stem_b1): 16 -> 16 direct, stride 1,
// residual, STEM_IN (block_flags(0, 1, 1, 1, 1, 1) = 258).
#define VSS_STEM_B1(TH, TW)                                                                              \
  {1, 1, TH, TW, 16, 0, 16, 16, 258, {k_stem_b1<TH, TW, PREC_F32>, k_stem_b1<TH, TW, PREC_BF16X2>}, kWideThreads, \
   VAR_STEM_B1_WIDE},
static const BlockEntry kStemB1Blocks[] = {VSS_STEM_B1(8, 32) VSS_STEM_B1(4, 64) VSS_STEM_B1(8, 64)};
#undef VSS_STEM_B1

const BlockEntry* block_registry(int* count) {
  static const std::vector<BlockEntry> all = [] {
    std::vector<BlockEntry> v;
    int n = 0;
    const BlockEntry* part = nullptr;
#define VSS_SHARD_FN(k)                              \
    part = registry_shard_##k(&n);                   \
    v.insert(v.end(), part, part + n);
#include "vss_registry_shards.inc"
#undef VSS_SHARD_FN
    v.insert(v.end(), std::begin(kStemB1Blocks), std::end(kStemB1Blocks));
    return v;
  }();
  *count = (int)all.size();
  return all.data();
}

void (*stem_kernel16())(StemParams) { return k_stem<16>; }
void (*head_kernel16())(HeadParams) { return k_head<16>; }
void (*prep_kernel())(PrepParams) { return k_prep; }
#endif

}  // namespace vss
