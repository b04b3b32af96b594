// vso_ir.hip — a MobileNetV2 inverted residual block of an ONNX session in ONE
// launch: 1x1 expand + Clip(ReLU6) -> 3x3 depthwise (stride 1 / 2) + Clip ->
// 1x1 project (+ the block's input as residual).  MODNet's backbone is eleven
// of them at /4../32 (tests/onnx_models.py modnet(); the reference runs that
// topology as model_q4f16.onnx, frameProcessorTest.ts:91, model.ts:12-29).
// As three launches (k_conv_pw, k_conv_dw_plane, k_conv_small) each block
// wrote its expanded tensor (6x the channels) to HBM and read it back twice,
// and the deep /16 - /32 blocks ran as a few dozen latency-bound workgroups:
// 38-57 us per block at batch 8, 288x512 (profiles/r04q).
//
// The seam's fused block (csrc/vss_kernels.hip k_block) on the session's NCHW
// f32 tensors: a workgroup owns a 4 x 16 output tile, all output channels and
// a slice of the hidden channels (KS slices per tile when the image has few
// tiles: each slice stores its plain partial sums and k_ir_reduce adds them in
// slice order — deterministic).  Prologue: the input region (tile + halo) for
// every input channel, staged in LDS as [c][pixel] (rows 4 mod 8 floats apart:
// the MFMA B reads of lanes (r, g), rows 4g apart, fall on complementary
// banks).  Two forms, the same chunk structure:
//  * k_ir (f32 sessions), per 16 hidden channels ("chunk"):
//   expand  — the region's 16-pixel blocks dealt to the 4 waves,
//             v_mfma_f32_16x16x4_f32 (exact f32 products, as k_conv_pw): D =
//             W1[chunk][c] x X[c][pixel], bias as the C operand, clip, zero
//             outside the image (the depthwise's padding), stored as four
//             quad-major planes (vss_kernels.h: conflict-free 16-B reads of
//             16-pixel runs; stride 2: planes one quad apart) — double
//             buffered, one workgroup barrier per chunk;
//   dw      — wave w computes output row w of the tile: lane (r, g) = pixel r,
//             channels 4g..4g+3, 9 taps in (ky, kx) order + bias + clip, in
//             registers in the project MFMA's B layout;
//   project — 4 MFMAs per 16 output channels (A = W2[out][chunk]), acc in
//             registers across the chunks.
//   Its weights are read from L2 per chunk, the depthwise / project ones in
//   flight during the expand, the next chunk's expand ones during the dw /
//   project; every operand stays f32.
//  * k_ir_b16 (bf16 / f16 sessions): every 1x1 product on
//   v_mfma_f32_16x16x32_bf16 over hi + lo bf16 splits of both operands (w x =
//   wh xh + wh xl + wl xh, ~2^-16 relative: about f32 precision — the
//   convolutions here are 1x1 / grouped, which onnx_ref.tiled_conv() rounds in
//   no session precision); the slice's weights pre-split and pre-ordered on
//   the host into one slab that the prologue copies to LDS by 16-byte LDS-DMA
//   (not read from L2 per chunk), the input region split once into registers,
//   projects per pair of chunks (32 hidden channels = one MFMA's K).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "vso_device.h"
#include "vso_kernels.h"

namespace vso {

// The input region of a tile: IH x IW pixels, one channel per PSTR floats.
// PSTR (>= P_IN) is 4 mod 8: the expand's B reads of lanes (r, g) (channels
// 4g apart) then fall on complementary banks.  The copy into LDS is one
// contiguous LDS-DMA stream over CIN x PSTR (the PSTR - P_IN gap floats of
// each channel take any image pixel; nothing reads them as data).
template <int S, int TH>
struct IrGeom {
  static constexpr int TW = 16;
  static constexpr int IH = S == 2 ? 2 * TH + 1 : TH + 2, IW = S == 2 ? 2 * TW + 1 : TW + 2;
  static constexpr int P_IN = IH * IW, NBI = (P_IN + 15) / 16, P_PAD = NBI * 16;
  static constexpr int pstr() {
    int v = P_IN;
    while (v % 8 != 4) ++v;
    return v;
  }
  static constexpr int PSTR = pstr();
  static constexpr int HQ = P_PAD + (S == 2 ? 1 : 0);  // quads per hidden plane
};

// floats of the staged region: CIN rows of PSTR, covering the last channel's
// reads up to P_PAD, rounded up to whole 256-element DMA blocks (the last
// block's lanes past the end write into the overhang)
__host__ __device__ constexpr int ir_xs_floats(int cin, int pstr, int p_pad) {
  const int f = (cin - 1) * pstr + (p_pad > pstr ? p_pad : pstr);
  return (f + 255) / 256 * 256;
}

// The epilogue of both forms: wave w owns output row w, lane (r, g) pixel r
// and channels cb * 16 + 4g + v.  ks == 1: + b2 (+ the residual res(ch) of
// this lane's output pixel, stride 1) and the store.  ks > 1: the slice's
// partial sums, plain stores into part [ks][N][COUT][Ho * Wo]; k_ir_reduce
// (the next launch) adds the slices in order, then b2 and the residual — the
// same operations in the same order as one workgroup summing them, spread
// over the whole chip.  (An in-kernel exchange — partials written through to
// L2, an arrival counter, the last workgroup of a tile reading every slice —
// cost 25-80 us per deep block at batch 8: one CU reading 0.4-2.4 MB.)
template <int NCB, typename Res>
__device__ __forceinline__ void ir_finish(const IrParams& p, f4 (&acc)[NCB], bool outw, int t, int ks, int n, int oy0,
                                          int ox0, Res res) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, r = lane & 15, g = lane >> 4;
  (void)t;
  if (!outw) return;
  const int oy = oy0 + wave, ox = ox0 + r;
  if (oy >= p.Ho || ox >= p.Wo) return;
  const long plane = (long)p.Ho * p.Wo;
  if (p.ks > 1 && !(p.probe & 16)) {
    float* pn = p.part + (((long)ks * p.N + n) * p.COUT) * plane + (long)oy * p.Wo + ox;
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int ch = cb * 16 + 4 * g + v;
        if (ch < p.COUT) pn[ch * plane] = acc[cb][v];
      }
    return;
  }
  float* yn = p.y + (long)n * ((long)p.COUT * plane + p.y_nx) + (long)oy * p.Wo + ox;
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int ch = cb * 16 + 4 * g + v;
      if (ch < p.COUT) {
        float o = acc[cb][v] + p.b2[ch];
        if (p.res) o += res(ch);
        yn[ch * plane] = o;
      }
    }
}

// y = sum over the ks slices of part (in slice order) + b2 (+ x): one output
// element per thread, the ks loads in flight together
__global__ __launch_bounds__(256) void k_ir_reduce(IrParams p) {
  const long plane = (long)p.Ho * p.Wo, per = (long)p.COUT * plane, total = (long)p.N * per;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int n = (int)(i / per);
  const long rem = i - (long)n * per;
  const int ch = (int)(rem / plane);
  const long px = rem - (long)ch * plane;
  float s = 0.f;
  for (int k0 = 0; k0 < p.ks; k0 += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = k0 + u < p.ks ? p.part[(long)(k0 + u) * total + i] : 0.f;
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (k0 + u < p.ks) s += v[u];
  }
  s += p.b2[ch];
  if (p.res) s += p.x[((long)n * p.CIN + ch) * plane + px];  // stride 1: the same plane
  p.y[(long)n * (per + p.y_nx) + rem] = s;
}

template <int NT, int NCB, int S, int TH>
__global__ __launch_bounds__(256) void k_ir(IrParams p) {
  using G = IrGeom<S, TH>;
  constexpr int TW = G::TW, IW = G::IW, P_IN = G::P_IN, NBI = G::NBI, HQ = G::HQ, PSTR = G::PSTR;
  static_assert(TH <= 4, "one output row per wave");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 15, g = lane >> 4;
  const int CIN = p.CIN, HID = p.HID, COUT = p.COUT, H = p.H, W = p.W;
  float* xs = smem;                                        // [CIN][PSTR] (+ overhang)
  float* hbuf = smem + ir_xs_floats(CIN, PSTR, G::P_PAD);  // 2 x [4 planes][HQ][4]
  const int t = blockIdx.x, ks = blockIdx.y, n = blockIdx.z;
  const int ty = t / p.tiles_x, tx = t - ty * p.tiles_x;
  const int oy0 = ty * TH, ox0 = tx * TW, iy0 = S * oy0 - 1, ix0 = S * ox0 - 1;

  // ---- prologue: the input region, global -> LDS by LDS-DMA (no register
  // stage, every load in flight at once).  Pixels outside the image load the
  // nearest image pixel: their expand outputs are zeroed below (the
  // depthwise's padding), so their inputs only need to be finite.
  {
    const float* xn = p.x + (long)n * CIN * H * W;
    const int total = CIN * PSTR;
    const int wbase = __builtin_amdgcn_readfirstlane((tid >> 6) << 6);
    for (int b0 = 0; b0 < total; b0 += 256) {
      const int i = min(b0 + tid, total - 1);
      const int c = i / PSTR, q = min(i - c * PSTR, P_IN - 1), ly = q / IW, lx = q - ly * IW;
      const int gy = min(max(iy0 + ly, 0), H - 1), gx = min(max(ix0 + lx, 0), W - 1);
      __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(xn + c * H * W + gy * W + gx),
                                       (__attribute__((address_space(3))) void*)(xs + b0 + wbase), 4, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();

  const int nch = HID / 16, c0 = ks * p.cps, c1 = min(c0 + p.cps, nch);
  const bool outw = wave < TH;
  // expand A fragments of chunk c: lane (r, g), MFMA 4u + e takes
  // W1[16c + r][16u + 4g + e] (one float4 per u; zero past CIN)
  f4 a1[NT];
  auto load_a1 = [&](int c) {
    const float* wr = p.w1 + (long)(c * 16 + r) * CIN;
#pragma unroll
    for (int u = 0; u < NT; ++u) {
      const int k = 16 * u + 4 * g;
      const f4 w = *reinterpret_cast<const f4*>(wr + min(k, CIN - 4));
      a1[u] = k < CIN ? w : f4{0.f, 0.f, 0.f, 0.f};
    }
  };
  f4 acc[NCB];
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb) acc[cb] = f4{0.f, 0.f, 0.f, 0.f};
  if (c0 < c1) load_a1(c0);
  for (int c = c0; c < c1; ++c) {
    float* hid = hbuf + ((c - c0) & 1) * (16 * HQ);
    const int h0 = c * 16;
    // this chunk's depthwise and project weights: in flight during the expand
    const f4 b1v = *reinterpret_cast<const f4*>(p.b1 + h0 + 4 * g);
    f4 wd[9], bd = f4{0.f, 0.f, 0.f, 0.f}, a2[NCB];
    if (outw) {
#pragma unroll
      for (int k = 0; k < 9; ++k) wd[k] = *reinterpret_cast<const f4*>(p.wdw + k * HID + h0 + 4 * g);
      bd = *reinterpret_cast<const f4*>(p.bdw + h0 + 4 * g);
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) {
        const int m = cb * 16 + r;
        const f4 w = *reinterpret_cast<const f4*>(p.w2 + (long)min(m, COUT - 1) * HID + h0 + 4 * g);
        a2[cb] = m < COUT ? w : f4{0.f, 0.f, 0.f, 0.f};
      }
    }
    // expand: D[hidden 4g + i][pixel r] of the region's 16-pixel blocks
    for (int pb = wave; pb < NBI; pb += 4) {
      f4 d = b1v;
      const float* xb = xs + pb * 16 + r;
#pragma unroll
      for (int u = 0; u < NT; ++u)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int k = min(16 * u + 4 * g + e, CIN - 1);  // (past CIN: weight 0, a finite value)
          d = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[u][e], xb[k * PSTR], d, 0, 0, 0);
        }
      const int pix = pb * 16 + r, ly = pix / IW, lx = pix - ly * IW;
      const bool in = pix < P_IN && (unsigned)(iy0 + ly) < (unsigned)H && (unsigned)(ix0 + lx) < (unsigned)W;
      f4 v;
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = in ? fminf(fmaxf(d[i], p.lo1), p.hi1) : 0.f;
      *reinterpret_cast<f4*>(hid + (g * HQ + pix) * 4) = v;
    }
    __syncthreads();
    if (c + 1 < c1) load_a1(c + 1);  // the next chunk's expand fragments, in flight during the dw / project
    if (outw) {
      // depthwise at output (oy0 + wave, ox0 + r), channels h0 + 4g .. + 3
      f4 a = bd;
#pragma unroll
      for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          const int rp = (S * wave + ky) * IW + S * r + kx;
          a = __builtin_elementwise_fma(wd[ky * 3 + kx], *reinterpret_cast<const f4*>(hid + (g * HQ + rp) * 4), a);
        }
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = fminf(fmaxf(a[i], p.lo2), p.hi2);
      // project: D[out cb*16 + 4g + v][pixel r] += W2[out][h0 + 4g' + j] x dw[h0 + 4g' + j][pixel r]
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[cb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a2[cb][j], a[j], acc[cb], 0, 0, 0);
    }
  }

  // ---- epilogue ----
  ir_finish<NCB>(p, acc, outw, t, ks, n, oy0, ox0, [&](int ch) { return xs[ch * PSTR + (wave + 1) * IW + r + 1]; });
}

// ---- the bf16x3 form (session precision bf16 / f16) ----
// The same block with every 1x1 product on v_mfma_f32_16x16x32_bf16 over a
// hi + lo bf16 split of both operands: w x = wh xh + wh xl + wl xh (+ wl xl,
// dropped: 2^-16 of the product, as are the splits' own residues) — about f32
// precision (these convolutions stay unrounded in onnx_ref's bf16 / f16
// oracle, tiled_conv()) at 3 bf16 MFMAs (48 cycles) per 32 channels where
// the f32 form takes 8 v_mfma_f32_16x16x4_f32 (256 cycles).
//   prologue — the slice's whole weight block (ir_slab_build: every operand
//             pre-split and pre-ordered) copied global -> LDS by 16-byte
//             LDS-DMA, and each wave's region blocks loaded straight into
//             registers and split once (lane (r, g) of block j: channels
//             32t + 8g .. + 7 of pixel r, 8 bf16 hi + 8 lo: the B operands of
//             every chunk) — one memory round trip per workgroup; the chunk
//             loop then reads LDS only (a first form read the weights from
//             L2 per chunk: the compiler's conservative vmcnt(0) waits exposed
//             three round trips per chunk, 60-80 us for the deep blocks);
//   expand  — A = the chunk's W1 rows from LDS (rows 2 mod 4 slots apart:
//             conflict-free ds_read_b128);
//   project — per PAIR of chunks (32 hidden channels = one MFMA's K): B = the
//             two chunks' depthwise outputs (lane (r, g): channels 4g..4g+3 of
//             each, split), A = W2 rows from LDS.  Slices hold whole pairs.
//   residual — read from x in HBM at the store (exact f32).
typedef __bf16 bf8v __attribute__((ext_vector_type(8)));
typedef __bf16 bf4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f4 mfma_bf(f4 a, f4 b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf8v, a), __builtin_bit_cast(bf8v, b), c, 0, 0, 0);
}

template <int NT2, int NCB, int S, int TH>
__global__ __launch_bounds__(256) void k_ir_b16(IrParams p) {
  using G = IrGeom<S, TH>;
  constexpr int IW = G::IW, P_IN = G::P_IN, NBI = G::NBI, HQ = G::HQ, NBW = (NBI + 3) / 4;
  static_assert(TH == 4, "one output row per wave, every wave");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  unsigned char* lds = reinterpret_cast<unsigned char*>(smem);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 15, g = lane >> 4;
  const int CIN = p.CIN, H = p.H, W = p.W, HW = H * W;
  float* hbuf = reinterpret_cast<float*>(lds + p.o_hid);  // 2 x [4 planes][HQ][4]
  const int t = blockIdx.x, ks = blockIdx.y, n = blockIdx.z;
  const int ty = t / p.tiles_x, tx = t - ty * p.tiles_x;
  const int oy0 = ty * TH, ox0 = G::TW * tx, iy0 = S * oy0 - 1, ix0 = S * ox0 - 1;

  // ---- prologue: the slice's weights -> LDS (DMA), the region -> registers.
  // Pixels outside the image (and past the region) load the nearest image
  // pixel: their expand outputs are zeroed below, so they only need to be finite.
  {
    const unsigned char* gsl = p.slab + (long)ks * p.sl_bytes;
    const int wb = __builtin_amdgcn_readfirstlane(wave * 1024);
    for (int o = wb; o < ((p.probe & 1) ? 0 : p.sl_bytes); o += 4096)
      __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(gsl + o + lane * 16),
                                       (__attribute__((address_space(3))) void*)(lds + o), 16, 0, 0);
  }
  f4 xh[NBW][NT2], xl[NBW][NT2];
  {
    const float* xn = p.x + (long)n * CIN * HW;
#pragma unroll
    for (int j = 0; j < NBW; ++j) {
      const int pix = min((wave + 4 * j) * 16 + r, P_IN - 1), ly = pix / IW, lx = pix - ly * IW;
      const int off = min(max(iy0 + ly, 0), H - 1) * W + min(max(ix0 + lx, 0), W - 1);
      float v[NT2][8];
#pragma unroll
      for (int u = 0; u < NT2; ++u)
#pragma unroll
        for (int e = 0; e < 8; ++e) v[u][e] = (p.probe & 2) ? 0.f : xn[min(32 * u + 8 * g + e, CIN - 1) * HW + off];
#pragma unroll
      for (int u = 0; u < NT2; ++u) {
        bf8v h, l;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float x = 32 * u + 8 * g + e < CIN ? v[u][e] : 0.f;
          const __bf16 b = (__bf16)x;
          h[e] = b;
          l[e] = (__bf16)(x - (float)b);
        }
        xh[j][u] = __builtin_bit_cast(f4, h);
        xl[j][u] = __builtin_bit_cast(f4, l);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const int nch = p.HID / 16, c0 = ks * p.cps, c1 = min(c0 + p.cps, nch), c16 = p.cps * 16;
  const unsigned char* w1h = lds;
  const unsigned char* w1l = lds + p.o_w1l;
  const unsigned char* w2h = lds + p.o_w2h;
  const unsigned char* w2l = lds + p.o_w2l;
  const float* wds = reinterpret_cast<const float*>(lds + p.o_wd);
  const float* bds = reinterpret_cast<const float*>(lds + p.o_bd);
  const float* b1s = reinterpret_cast<const float*>(lds + p.o_b1);
  f4 acc[NCB];
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb) acc[cb] = f4{0.f, 0.f, 0.f, 0.f};
  bf4v dh0 = bf4v{}, dl0 = bf4v{};  // the first chunk of a pair: its depthwise output, split
  for (int c = c0; c < c1; ++c) {
    const int cl = c - c0;
    const bool first = (cl & 1) == 0;
    float* hid = hbuf + (cl & 1) * (16 * HQ);
    // expand: D[hidden 4g + i][pixel r] of this wave's region blocks
    f4 a1h[NT2], a1l[NT2];
#pragma unroll
    for (int u = 0; u < NT2; ++u) {
      const int o = ((cl * 16 + r) * p.s1 + 4 * u + g) * 16;
      a1h[u] = *reinterpret_cast<const f4*>(w1h + o);
      a1l[u] = *reinterpret_cast<const f4*>(w1l + o);
    }
    const f4 b1v = *reinterpret_cast<const f4*>(b1s + cl * 16 + 4 * g);
#pragma unroll
    for (int j = 0; j < NBW; ++j) {
      const int pb = wave + 4 * j;
      if (pb < NBI) {
        f4 d = b1v;
        if (!(p.probe & 4)) {
#pragma unroll
          for (int u = 0; u < NT2; ++u) {
            d = mfma_bf(a1l[u], xh[j][u], d);
            d = mfma_bf(a1h[u], xl[j][u], d);
            d = mfma_bf(a1h[u], xh[j][u], d);
          }
        }
        const int pix = pb * 16 + r, ly = pix / IW, lx = pix - ly * IW;
        const bool in = pix < P_IN && (unsigned)(iy0 + ly) < (unsigned)H && (unsigned)(ix0 + lx) < (unsigned)W;
        f4 v;
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = in ? fminf(fmaxf(d[i], p.lo1), p.hi1) : 0.f;
        *reinterpret_cast<f4*>(hid + (g * HQ + pix) * 4) = v;
      }
    }
    __syncthreads();
    // depthwise at output (oy0 + wave, ox0 + r), channels 16c + 4g .. + 3
    f4 a = *reinterpret_cast<const f4*>(bds + cl * 16 + 4 * g);
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const f4 wk = *reinterpret_cast<const f4*>(wds + (ky * 3 + kx) * c16 + cl * 16 + 4 * g);
        const int rp = (S * wave + ky) * IW + S * r + kx;
        a = __builtin_elementwise_fma(wk, *reinterpret_cast<const f4*>(hid + (g * HQ + rp) * 4), a);
      }
    bf4v dh, dl;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float v = fminf(fmaxf(a[i], p.lo2), p.hi2);
      const __bf16 b = (__bf16)v;
      dh[i] = b;
      dl[i] = (__bf16)(v - (float)b);
    }
    if (first && c + 1 < c1) {
      dh0 = dh;
      dl0 = dl;
    } else {
      // project the pair: B lane (r, g) = (first chunk's 4g..4g+3, second's)
      const bf4v z = bf4v{};
      const bf8v bh = first ? __builtin_shufflevector(dh, z, 0, 1, 2, 3, 4, 5, 6, 7)
                            : __builtin_shufflevector(dh0, dh, 0, 1, 2, 3, 4, 5, 6, 7);
      const bf8v bl = first ? __builtin_shufflevector(dl, z, 0, 1, 2, 3, 4, 5, 6, 7)
                            : __builtin_shufflevector(dl0, dl, 0, 1, 2, 3, 4, 5, 6, 7);
      const f4 fh = __builtin_bit_cast(f4, bh), fl = __builtin_bit_cast(f4, bl);
      const int qo = (cl >> 1) * 4 + g;
#pragma unroll
      for (int cb = 0; cb < ((p.probe & 8) ? 0 : NCB); ++cb) {
        const int o = ((cb * 16 + r) * p.s2 + qo) * 16;
        const f4 ah = *reinterpret_cast<const f4*>(w2h + o), al = *reinterpret_cast<const f4*>(w2l + o);
        acc[cb] = mfma_bf(al, fh, acc[cb]);
        acc[cb] = mfma_bf(ah, fl, acc[cb]);
        acc[cb] = mfma_bf(ah, fh, acc[cb]);
      }
    }
  }

  // ---- epilogue ----
  const float* xres = p.x + (long)n * CIN * HW + (long)(oy0 + wave) * W + ox0 + r;
  ir_finish<NCB>(p, acc, true, t, ks, n, oy0, ox0, [&](int ch) { return xres[(long)ch * HW]; });
}

// ---- the bf16x3 form, wave-private (small input channel counts) ----
// k_ir_b16 with no workgroup barrier in the chunk loop: wave w expands the
// three region rows its own output row reads (S w .. S w + 2; the rows
// between two waves' outputs are expanded by both — 2x the expand MFMAs at
// stride 1, 1.33x at stride 2) into its own hidden planes, so the waves only
// meet once, after the prologue's DMA.  For the wide, shallow blocks (MODNet
// at /2 - /8: 16-64 input channels, 6-9 chunks, ~1000 workgroups) whose
// chunks carry little MFMA work: there the per-chunk barrier and its LDS
// round trips set the pace.  Same slab, operands, rounding and sums as
// k_ir_b16 (bitwise the same outputs).
template <int S>
struct IrWaveGeom {
  static constexpr int IW = IrGeom<S, 4>::IW, PW = 3 * IW, NB = (PW + 15) / 16;
  static constexpr int HQ = NB * 16 + (S == 2 ? 1 : 0);  // quads per hidden plane
};

__device__ __forceinline__ void wave_fence() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int NT2, int NCB, int S>
__global__ __launch_bounds__(256) void k_ir_b16w(IrParams p) {
  using WG = IrWaveGeom<S>;
  constexpr int IW = WG::IW, PW = WG::PW, NB = WG::NB, HQ = WG::HQ, TW = 16, TH = 4;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  unsigned char* lds = reinterpret_cast<unsigned char*>(smem);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 15, g = lane >> 4;
  const int CIN = p.CIN, H = p.H, W = p.W, HW = H * W;
  float* hid = reinterpret_cast<float*>(lds + p.o_hid) + wave * (16 * HQ);  // this wave's [4 planes][HQ][4]
  const int t = blockIdx.x, ks = blockIdx.y, n = blockIdx.z;
  const int ty = t / p.tiles_x, tx = t - ty * p.tiles_x;
  const int oy0 = ty * TH, ox0 = TW * tx;
  const int ry0 = S * (oy0 + wave) - 1, ix0 = S * ox0 - 1;  // this wave's region: rows ry0 .. ry0 + 2
  {
    const unsigned char* gsl = p.slab + (long)ks * p.sl_bytes;
    const int wb = __builtin_amdgcn_readfirstlane(wave * 1024);
    for (int o = wb; o < ((p.probe & 1) ? 0 : p.sl_bytes); o += 4096)
      __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(gsl + o + lane * 16),
                                       (__attribute__((address_space(3))) void*)(lds + o), 16, 0, 0);
  }
  f4 xh[NB][NT2], xl[NB][NT2];
  {
    const float* xn = p.x + (long)n * CIN * HW;
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int pix = min(j * 16 + r, PW - 1), ly = pix / IW, lx = pix - ly * IW;
      const int off = min(max(ry0 + ly, 0), H - 1) * W + min(max(ix0 + lx, 0), W - 1);
      float v[NT2][8];
#pragma unroll
      for (int u = 0; u < NT2; ++u)
#pragma unroll
        for (int e = 0; e < 8; ++e) v[u][e] = (p.probe & 2) ? 0.f : xn[min(32 * u + 8 * g + e, CIN - 1) * HW + off];
#pragma unroll
      for (int u = 0; u < NT2; ++u) {
        bf8v h, l;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float x = 32 * u + 8 * g + e < CIN ? v[u][e] : 0.f;
          const __bf16 b = (__bf16)x;
          h[e] = b;
          l[e] = (__bf16)(x - (float)b);
        }
        xh[j][u] = __builtin_bit_cast(f4, h);
        xl[j][u] = __builtin_bit_cast(f4, l);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const int nch = p.HID / 16, c0 = ks * p.cps, c1 = min(c0 + p.cps, nch), c16 = p.cps * 16;
  const unsigned char* w1h = lds;
  const unsigned char* w1l = lds + p.o_w1l;
  const unsigned char* w2h = lds + p.o_w2h;
  const unsigned char* w2l = lds + p.o_w2l;
  const float* wds = reinterpret_cast<const float*>(lds + p.o_wd);
  const float* bds = reinterpret_cast<const float*>(lds + p.o_bd);
  const float* b1s = reinterpret_cast<const float*>(lds + p.o_b1);
  f4 acc[NCB];
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb) acc[cb] = f4{0.f, 0.f, 0.f, 0.f};
  bf4v dh0 = bf4v{}, dl0 = bf4v{};
  for (int c = c0; c < c1; ++c) {
    const int cl = c - c0;
    const bool first = (cl & 1) == 0;
    f4 a1h[NT2], a1l[NT2];
#pragma unroll
    for (int u = 0; u < NT2; ++u) {
      const int o = ((cl * 16 + r) * p.s1 + 4 * u + g) * 16;
      a1h[u] = *reinterpret_cast<const f4*>(w1h + o);
      a1l[u] = *reinterpret_cast<const f4*>(w1l + o);
    }
    const f4 b1v = *reinterpret_cast<const f4*>(b1s + cl * 16 + 4 * g);
    wave_fence();  // the previous chunk's depthwise reads of hid are done
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      f4 d = b1v;
      if (!(p.probe & 4)) {
#pragma unroll
        for (int u = 0; u < NT2; ++u) {
          d = mfma_bf(a1l[u], xh[j][u], d);
          d = mfma_bf(a1h[u], xl[j][u], d);
          d = mfma_bf(a1h[u], xh[j][u], d);
        }
      }
      const int pix = j * 16 + r, ly = pix / IW, lx = pix - ly * IW;
      const bool in = pix < PW && (unsigned)(ry0 + ly) < (unsigned)H && (unsigned)(ix0 + lx) < (unsigned)W;
      f4 v;
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = in ? fminf(fmaxf(d[i], p.lo1), p.hi1) : 0.f;
      *reinterpret_cast<f4*>(hid + (g * HQ + pix) * 4) = v;
    }
    wave_fence();
    f4 a = *reinterpret_cast<const f4*>(bds + cl * 16 + 4 * g);
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const f4 wk = *reinterpret_cast<const f4*>(wds + (ky * 3 + kx) * c16 + cl * 16 + 4 * g);
        const int rp = ky * IW + S * r + kx;
        a = __builtin_elementwise_fma(wk, *reinterpret_cast<const f4*>(hid + (g * HQ + rp) * 4), a);
      }
    bf4v dh, dl;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float v = fminf(fmaxf(a[i], p.lo2), p.hi2);
      const __bf16 b = (__bf16)v;
      dh[i] = b;
      dl[i] = (__bf16)(v - (float)b);
    }
    if (first && c + 1 < c1) {
      dh0 = dh;
      dl0 = dl;
    } else {
      const bf4v z = bf4v{};
      const bf8v bh = first ? __builtin_shufflevector(dh, z, 0, 1, 2, 3, 4, 5, 6, 7)
                            : __builtin_shufflevector(dh0, dh, 0, 1, 2, 3, 4, 5, 6, 7);
      const bf8v bl = first ? __builtin_shufflevector(dl, z, 0, 1, 2, 3, 4, 5, 6, 7)
                            : __builtin_shufflevector(dl0, dl, 0, 1, 2, 3, 4, 5, 6, 7);
      const f4 fh = __builtin_bit_cast(f4, bh), fl = __builtin_bit_cast(f4, bl);
      const int qo = (cl >> 1) * 4 + g;
#pragma unroll
      for (int cb = 0; cb < ((p.probe & 8) ? 0 : NCB); ++cb) {
        const int o = ((cb * 16 + r) * p.s2 + qo) * 16;
        const f4 ah = *reinterpret_cast<const f4*>(w2h + o), al = *reinterpret_cast<const f4*>(w2l + o);
        acc[cb] = mfma_bf(al, fh, acc[cb]);
        acc[cb] = mfma_bf(ah, fl, acc[cb]);
        acc[cb] = mfma_bf(ah, fh, acc[cb]);
      }
    }
  }
  const float* xres = p.x + (long)n * CIN * HW + (long)(oy0 + wave) * W + ox0 + r;
  ir_finish<NCB>(p, acc, true, t, ks, n, oy0, ox0, [&](int ch) { return xres[(long)ch * HW]; });
}

// ---- host side ----
namespace {
struct IrEntry {
  int nt, ncb, s, th;
  void (*fn)(IrParams);
  const char* name;
};
// (names as the other launches': the kernel's demangled signature)
#define VSO_IR(NT, NCB, S, TH) \
  {NT, NCB, S, TH, k_ir<NT, NCB, S, TH>, "void vso::k_ir<" #NT ", " #NCB ", " #S ", " #TH ">(vso::IrParams)"},
#define VSO_IR16(NT2, NCB, S, TH) \
  {NT2, NCB, S, TH, k_ir_b16<NT2, NCB, S, TH>, "void vso::k_ir_b16<" #NT2 ", " #NCB ", " #S ", " #TH ">(vso::IrParams)"},
// MobileNetV2 1.0's blocks (t = 6): input channels / 16 (rounded up), output
// channels / 16 (rounded up), stride — 16->24 s2, 24->24, 24->32 s2, 32->32,
// 32->64 s2, 64->64, 64->96, 96->96, 96->160 s2, 160->160, 160->320
const IrEntry kIr[] = {
    VSO_IR(1, 2, 2, 4) VSO_IR(2, 2, 1, 4) VSO_IR(2, 2, 2, 4) VSO_IR(2, 4, 2, 4) VSO_IR(4, 4, 1, 4)
    VSO_IR(4, 6, 1, 4) VSO_IR(6, 6, 1, 4) VSO_IR(6, 10, 2, 4) VSO_IR(10, 10, 1, 4) VSO_IR(10, 20, 1, 4)
    VSO_IR(4, 4, 2, 4) VSO_IR(6, 6, 2, 4)};
// the same blocks by input channels / 32 (the bf16x3 form's K step)
const IrEntry kIr16[] = {
    VSO_IR16(1, 2, 2, 4) VSO_IR16(1, 2, 1, 4) VSO_IR16(1, 4, 2, 4) VSO_IR16(2, 4, 1, 4) VSO_IR16(2, 6, 1, 4)
    VSO_IR16(3, 6, 1, 4) VSO_IR16(3, 10, 2, 4) VSO_IR16(5, 10, 1, 4) VSO_IR16(5, 20, 1, 4) VSO_IR16(2, 4, 2, 4)
    VSO_IR16(3, 6, 2, 4)};
// the wave-private form (k_ir_b16w) for <= 64 input channels
#define VSO_IR16W(NT2, NCB, S) \
  {NT2, NCB, S, 4, k_ir_b16w<NT2, NCB, S>, "void vso::k_ir_b16w<" #NT2 ", " #NCB ", " #S ">(vso::IrParams)"},
const IrEntry kIr16w[] = {VSO_IR16W(1, 2, 2) VSO_IR16W(1, 2, 1) VSO_IR16W(1, 4, 2) VSO_IR16W(2, 4, 1)
                              VSO_IR16W(2, 6, 1) VSO_IR16W(2, 4, 2)};
#undef VSO_IR
#undef VSO_IR16
#undef VSO_IR16W

const IrEntry* ir_entry(const IrParams& p) {
  const int nt = p.b16 ? (p.CIN + 31) / 32 : (p.CIN + 15) / 16, ncb = (p.COUT + 15) / 16;
  const IrEntry* t = p.wv ? kIr16w : p.b16 ? kIr16 : kIr;
  const size_t n = p.wv ? sizeof(kIr16w) / sizeof(kIr16w[0])
                        : p.b16 ? sizeof(kIr16) / sizeof(kIr16[0]) : sizeof(kIr) / sizeof(kIr[0]);
  for (size_t i = 0; i < n; ++i)
    if (t[i].nt == nt && t[i].ncb == ncb && t[i].s == p.stride && t[i].th == kIrTH) return &t[i];
  return nullptr;
}
}  // namespace

int ir_pstr(int stride) { return stride == 2 ? IrGeom<2, kIrTH>::PSTR : IrGeom<1, kIrTH>::PSTR; }

static size_t ir_hid_bytes(int stride) {
  return 2 * 16 * (size_t)(stride == 2 ? IrGeom<2, kIrTH>::HQ : IrGeom<1, kIrTH>::HQ) * 4;
}

size_t ir_lds_bytes(const IrParams& p) {
  if (p.wv)
    return (size_t)p.o_hid + 4 * 16 * (size_t)(p.stride == 2 ? IrWaveGeom<2>::HQ : IrWaveGeom<1>::HQ) * 4;
  if (p.b16) return (size_t)p.o_hid + ir_hid_bytes(p.stride);
  const int pad = p.stride == 2 ? IrGeom<2, kIrTH>::P_PAD : IrGeom<1, kIrTH>::P_PAD;
  return (size_t)ir_xs_floats(p.CIN, ir_pstr(p.stride), pad) * 4 + ir_hid_bytes(p.stride);
}

// The b16 slab: per slice, W1 hi / lo planes [cps * 16 rows][s1 slots of 16 B]
// (slot t of row j: W1[16 c + j][8 t .. 8 t + 7], the expand A operand of lane
// group t % 4 in K step t / 4), W2 hi / lo planes [16 NCB rows][s2 slots]
// (slot 4 q + g of row m: W2[m][32 q' + 4g + i] (i < 4) then W2[m][32 q' + 16 +
// 4g + i], q' the slice's q-th chunk pair: the project A operand of lane group
// g), the depthwise taps [9][cps * 16], its bias, the expand bias (f32).  Row
// strides of 2 mod 4 slots: the ds_read_b128 lane groups of an A read (rows
// r, slots g) hit 16 distinct 16-byte bank groups.  sl_bytes is a whole
// number of KiB (the prologue's DMA moves 1 KiB per wave instruction).
static void ir_slab_layout(IrParams* p) {
  const int nt2 = (p->CIN + 31) / 32, ncb = (p->COUT + 15) / 16, c16 = p->cps * 16;
  p->s1 = 4 * nt2 + 2;
  p->s2 = 4 * ((p->cps + 1) / 2) + 2;
  const int w1 = c16 * p->s1 * 16, w2 = ncb * 16 * p->s2 * 16;
  p->o_w1l = w1;
  p->o_w2h = 2 * w1;
  p->o_w2l = p->o_w2h + w2;
  p->o_wd = p->o_w2l + w2;
  p->o_bd = p->o_wd + 9 * c16 * 4;
  p->o_b1 = p->o_bd + c16 * 4;
  p->sl_bytes = (p->o_b1 + c16 * 4 + 1023) / 1024 * 1024;
  p->o_hid = p->sl_bytes;
}

bool ir_slab_plan(IrParams* p, long wgs, int cps_target) {
  const int nch = p->HID / 16;
  const long wg0 = (long)p->N * p->tiles;
  int ks = (int)std::min<long>(nch, std::max<long>(1, (wgs + wg0 / 2) / wg0));
  if (cps_target > 0) {  // about cps_target chunks per slice, at least one chip's worth of workgroups
    ks = (nch + cps_target - 1) / cps_target;
    if (wg0 * ks < 256) ks = (int)std::min<long>(nch, (256 + wg0 - 1) / wg0);
    static const long one_slice = [] {  // tiles x images from which a block is not split (VSO_IR_KS1)
      const char* e = std::getenv("VSO_IR_KS1");
      return e ? std::atol(e) : 1024L;
    }();
    if (wg0 >= one_slice) ks = 1;
  }
  int cps = (nch + ks - 1) / ks;
  if (cps < nch) cps += cps & 1;  // slices of whole chunk pairs
  for (;;) {
    p->cps = cps;
    ir_slab_layout(p);
    if (ir_lds_bytes(*p) <= 160 * 1024) break;
    if (cps <= 2) return false;
    cps = cps >= nch ? (nch - 1) & ~1 : cps - 2;
    if (cps < 2) return false;
  }
  p->ks = (nch + p->cps - 1) / p->cps;
  return true;
}

void ir_slab_build(const IrParams& p, const float* w1, const float* b1, const float* wdt, const float* bd,
                   const float* w2, std::vector<unsigned char>* out) {
  const int nch = p.HID / 16, c16 = p.cps * 16, ncb = (p.COUT + 15) / 16;
  out->assign((size_t)p.ks * p.sl_bytes, 0);
  auto bf = [](float f) {  // nearest even (f finite)
    uint32_t u;
    std::memcpy(&u, &f, 4);
    u += 0x7fffu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
  };
  auto split = [&](float w, uint16_t* h, uint16_t* l) {
    *h = bf(w);
    const uint32_t hb = (uint32_t)*h << 16;
    float hf;
    std::memcpy(&hf, &hb, 4);
    *l = bf(w - hf);
  };
  for (int k = 0; k < p.ks; ++k) {
    unsigned char* b = out->data() + (size_t)k * p.sl_bytes;
    const int c0 = k * p.cps, cn = std::min(p.cps, nch - c0);
    for (int cl = 0; cl < cn; ++cl)
      for (int j = 0; j < 16; ++j) {
        const int h = 16 * (c0 + cl) + j;
        for (int c = 0; c < p.CIN; ++c) {
          const size_t o = ((size_t)(cl * 16 + j) * p.s1 + c / 8) * 16 + (c % 8) * 2;
          split(w1[(size_t)h * p.CIN + c], reinterpret_cast<uint16_t*>(b + o),
                reinterpret_cast<uint16_t*>(b + p.o_w1l + o));
        }
        for (int t = 0; t < 9; ++t)
          std::memcpy(b + p.o_wd + ((size_t)t * c16 + cl * 16 + j) * 4, &wdt[(size_t)t * p.HID + h], 4);
        std::memcpy(b + p.o_bd + (size_t)(cl * 16 + j) * 4, &bd[h], 4);
        std::memcpy(b + p.o_b1 + (size_t)(cl * 16 + j) * 4, &b1[h], 4);
      }
    for (int m = 0; m < p.COUT; ++m)
      for (int q = 0; q < (cn + 1) / 2; ++q)
        for (int gg = 0; gg < 4; ++gg)
          for (int i = 0; i < 8; ++i) {
            const int h = 16 * c0 + 32 * q + (i < 4 ? 4 * gg + i : 16 + 4 * gg + i - 4);
            if (h >= std::min(16 * (c0 + cn), p.HID)) continue;
            const size_t o = ((size_t)m * p.s2 + 4 * q + gg) * 16 + i * 2;
            split(w2[(size_t)m * p.HID + h], reinterpret_cast<uint16_t*>(b + p.o_w2h + o),
                  reinterpret_cast<uint16_t*>(b + p.o_w2l + o));
          }
    (void)ncb;
  }
}

void ir_tiles(int Ho, int Wo, int* tiles_x, int* tiles) {
  *tiles_x = (Wo + 15) / 16;
  *tiles = *tiles_x * ((Ho + kIrTH - 1) / kIrTH);
}

bool ir_supported(const IrParams& p) {
  // the kernels index an image's input planes with 32-bit offsets
  if ((long)p.CIN * p.H * p.W >= (1L << 31)) return false;
  return p.CIN % 4 == 0 && p.HID % 16 == 0 && (p.stride == 1 || p.stride == 2) && ir_entry(p) != nullptr &&
         ir_lds_bytes(p) <= 160 * 1024 && (!p.res || (p.stride == 1 && p.CIN == p.COUT));
}

const char* ir_kernel_name(const IrParams& p) {
  const IrEntry* e = ir_entry(p);
  return e ? e->name : (p.wv ? "vso::k_ir_b16w<?>" : p.b16 ? "vso::k_ir_b16<?>" : "vso::k_ir<?>");
}

void launch_ir_reduce(const IrParams& p, hipStream_t s) {
  const long total = (long)p.N * p.COUT * p.Ho * p.Wo;
  hipLaunchKernelGGL(k_ir_reduce, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, p);
}

void launch_ir(const IrParams& p, hipStream_t s) {
  const IrEntry* e = ir_entry(p);
  if (!e) return;
  const size_t lds = ir_lds_bytes(p);
  (void)hipFuncSetAttribute((const void*)e->fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(e->fn, dim3(p.tiles, p.ks, p.N), dim3(256), lds, s, p);
}

}  // namespace vso
