// vso_conv.hip — the dense k x k convolutions of the ONNX sessions
// (include/vso.h) as LDS-tiled implicit GEMMs on gfx950 MFMA.
//
// MODNet (the reference's model_q4f16.onnx, model.ts:12-29, run at 288x512 by
// frameProcessorTest.ts:91) spends ~90 % of its 8.7 GMAC per frame in dense
// 3x3 / 5x5 convolutions with 16-99 input and 16-96 output channels at
// 72x128 .. 288x512 pixels.  k_conv_tile computes one
// TH x TW output tile x BM output channels per workgroup:
//
//   * the input tile of 32 channels at a time (its halo included) is staged
//     from the f32 NCHW tensor into LDS as [pixel][32 channels] in the MFMA
//     operand type T, every element once per chunk (the im2col gather of all
//     KS*KS taps then reads LDS), the next chunk's global loads in flight
//     during the current chunk's MFMAs;
//   * each wave owns TH*TW/64 blocks of 16 consecutive output pixels of one
//     row and all BM output channels; per tap it reads one 16-byte B fragment
//     per block from LDS (8 channels of one pixel) and the A fragments (8
//     channels of one output channel's tap weights, packed at create as
//     [tap][Mp][Cp] in T) from global memory / L2;
//   * T = float: v_mfma_f32_16x16x4_f32, exact f32 products (8 MFMAs per 32
//     channels); T = bf16 / f16: v_mfma_f32_16x16x32_{bf16,f16} (one MFMA per
//     32 channels, 16x the rate), operands rounded to nearest-even, f32
//     accumulation;
//   * bias, residual and activation fused into the epilogue (vso_device.h);
//   * the tile (8x32 .. 2x32 / 16x16 .. 4x16 pixels) is the largest that
//     still gives ~4 workgroups per CU: at batch 1 MODNet's layers are small
//     (36864 pixels x 64 channels), and a workgroup's global-load latency is
//     only hidden by other workgroups on the same CU;
//   * when even the smallest tile leaves the chip half empty the 32-channel
//     chunks are split over ksplit workgroups: each writes its partial sums,
//     and the last of them to arrive (a per-output-block arrival counter)
//     adds all ksplit partials in split order — deterministic — and applies
//     the epilogue, so no reduction launch is needed.
//
// Compiled once per operand precision (-DVSO_CONV_PREC=0/1/2: the template
// instances) and once with -DVSO_CONV_DISPATCH (planning and dispatch).
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "vso_device.h"
#include "vso_kernels.h"

namespace vso {

typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
// 16 bytes as a clang vector (HIP's uint4 is a struct with a union: arrays of
// it in registers were not promoted by SROA and went to scratch)
typedef unsigned u4 __attribute__((ext_vector_type(4)));

constexpr int CK = 32;  // input channels per staged chunk

template <int PREC> struct Elem;
template <> struct Elem<PREC_F32> { using T = float; };
template <> struct Elem<PREC_BF16> { using T = __bf16; };
template <> struct Elem<PREC_F16> { using T = _Float16; };

// 16 bytes of the LDS pixel row: 4 f32 or 8 16-bit channels
template <int PREC> __device__ __forceinline__ u4 pack_quad(const float* v);
template <> __device__ __forceinline__ u4 pack_quad<PREC_F32>(const float* v) {
  return u4{__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3])};
}
template <> __device__ __forceinline__ u4 pack_quad<PREC_BF16>(const float* v) {
  bf8 b;
#pragma unroll
  for (int e = 0; e < 8; ++e) b[e] = (__bf16)v[e];
  return __builtin_bit_cast(u4, b);
}
template <> __device__ __forceinline__ u4 pack_quad<PREC_F16>(const float* v) {
  h8 b;
#pragma unroll
  for (int e = 0; e < 8; ++e) b[e] = (_Float16)v[e];
  return __builtin_bit_cast(u4, b);
}

// acc += A (16 out channels x 32 in channels) * B (32 in channels x 16 pixels).
// a / b: this lane's fragments — 16-bit: one quad (channels 8g .. 8g+7);
// f32: two quads (channels 4g .. 4g+3 and 16+4g .. 16+4g+3), MFMA s taking
// element s (the same channel on both sides: the sum over all 32 channels).
template <int PREC> __device__ __forceinline__ f4 mma32(const u4* a, const u4* b, f4 acc);
template <> __device__ __forceinline__ f4 mma32<PREC_F32>(const u4* a, const u4* b, f4 acc) {
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a[h].x), __uint_as_float(b[h].x), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a[h].y), __uint_as_float(b[h].y), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a[h].z), __uint_as_float(b[h].z), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a[h].w), __uint_as_float(b[h].w), acc, 0, 0, 0);
  }
  return acc;
}
template <> __device__ __forceinline__ f4 mma32<PREC_BF16>(const u4* a, const u4* b, f4 acc) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf8, a[0]), __builtin_bit_cast(bf8, b[0]), acc,
                                                  0, 0, 0);
}
template <> __device__ __forceinline__ f4 mma32<PREC_F16>(const u4* a, const u4* b, f4 acc) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, a[0]), __builtin_bit_cast(h8, b[0]), acc, 0,
                                                 0, 0);
}

#ifdef VSO_CONV_PREC
// Workgroups per CU the kernel's LDS allows (160 KiB per CU), as a register
// budget (amdgpu_waves_per_eu; one wave per SIMD per workgroup) — an A/B knob,
// off: held to the LDS occupancy the compiler spills (8x32 tiles, 72-184 B of
// scratch) and MODNet batch 8 bf16 measured 2.38 ms per run against 2.31
// without the cap (r04c).
#ifndef VSO_CONV_WPE
#define VSO_CONV_WPE 0
#endif
// LDS layouts free of bank conflicts for the MFMA fragment reads
// (MI355X_MICROARCH.md §LDS: ds_read_b128 serves lane groups {0-3, 12-15,
// 20-27}, ... of 16 lanes on 16 four-bank 16-B slots).  A B read is 16
// consecutive pixels (lane r = l & 15) x quad g = l >> 4: with a pixel stride
// of QS quads the group's slots mod 16 are distinct iff QS = 2 mod 4 at
// stride 1 (pixels r) and QS odd at stride 2 (pixels 2r, i.e. 2 QS = 2 mod 4);
// the odd stride of round 4 gave 2-way conflicts at stride 1.  An A read is
// row r of 16 weight rows x quad g at a row stride of NQ = 4 quads (16-bit):
// 2-way on every group, 4 extra cycles per read; the quads of row m are
// XOR-swizzled by (-(m >> 2)) & 3 instead (no padding: the slab stays the
// largest LDS user), which puts the group's 16 lanes on 16 slots.
// VSO_CONV_SWZ (a build-time A/B knob, bits): 1 the f32 B stride, 2 the
// 16-bit B stride, 4 the A swizzle; 0 = round 4's layouts.  Default 5: the
// 16-bit B stride's 20 % larger pixel tile cost occupancy — MODNet batch 8
// bf16 1.360-1.363 ms with it, 1.345-1.347 without, 1.366-1.370 without the
// A swizzle, 1.356-1.357 with neither; f32 3.51 against 3.72 with neither
// (profiles/r05x).
#ifndef VSO_CONV_SWZ
#define VSO_CONV_SWZ 5
#endif
// Persistent, software-pipelined workgroups (conv_tile_body_persist) for f32 operands
constexpr bool conv_tile_persist(int prec) { return prec == PREC_F32; }
__device__ __forceinline__ int wsw(int m) { return (VSO_CONV_SWZ & 4) ? (-(m >> 2)) & 3 : 0; }
template <int PREC, int S>
constexpr int conv_qs() {
  constexpr int nq = CK * (PREC == PREC_F32 ? 4 : 2) / 16;
  return nq + (S == 1 && (VSO_CONV_SWZ & (PREC == PREC_F32 ? 1 : 2)) ? 2 : 1);
}
template <int PREC, int KS, int S, int TH, int TW, int BM>
constexpr int conv_tile_wpe() {
  if (!VSO_CONV_WPE) return 1;
  constexpr int sz = PREC == PREC_F32 ? 4 : 2, NQ = CK * sz / 16, IH = (TH - 1) * S + KS, IW = (TW - 1) * S + KS;
  constexpr bool WL = PREC != PREC_F32 && (KS <= 3 || BM <= 32);
  constexpr int lds = IH * IW * conv_qs<PREC, S>() * 16 + (WL ? KS * KS * BM * NQ * 16 : 16);
  return std::max(1, std::min(VSO_CONV_WPE == 2 ? 2 : 4, 163840 / lds));
}

// UP: the 32-channel chunks in [p.up_c0, p.up_c1) of the input are not read
// from c.x but computed while staging — the 2x linear upsample (ONNX Resize,
// half_pixel / pytorch_half_pixel, scale 2) of p.up, k_resize's arithmetic: a
// Resize whose output only feeds this convolution (directly or through a
// Concat) runs inside it instead of writing and re-reading a 4x larger
// tensor.  As in the seam's decoders, the chunk's low-resolution source region
// (SR x SC pixels) is loaded once (coalesced along its rows) into LDS and the
// tile's items interpolate from there.
template <int PREC, int KS, int S, int TH, int TW, int BM, bool UP>
__device__ __forceinline__ void conv_tile_body(const ConvTileParams& p) {
  using T = typename Elem<PREC>::T;
  constexpr int NQ = CK * (int)sizeof(T) / 16;     // quads of one pixel's chunk: 8 (f32) / 4
  constexpr int QS = conv_qs<PREC, S>();           // LDS pixel stride in quads (above)
  constexpr int CG = 16 / (int)sizeof(T);          // channels per quad
  constexpr int NF = PREC == PREC_F32 ? 2 : 1;     // fragment quads per lane
  constexpr int IH = (TH - 1) * S + KS, IW = (TW - 1) * S + KS, NPIX = IH * IW;
  constexpr int ITEMS = NPIX * NQ;                 // quads staged per chunk
  constexpr int PER = (ITEMS + 255) / 256;
  constexpr int NB = TH * TW / 16, PBW = NB / 4;   // 16-pixel blocks per tile / per wave
  constexpr int MI = BM / 16;
  static_assert(NB % 4 == 0 && TW % 16 == 0, "tile: a multiple of 64 pixels, rows of 16");
  // 16-bit operands, k <= 3 (and 5x5 on 16 / 32-channel tiles: <= 51 KB): the chunk's weights of all taps staged in LDS too
  // ([tap][BM rows][NQ quads]), loaded once per workgroup instead of once
  // per wave and tap from L2 (whose latency the per-tap MFMAs cannot cover)
  constexpr bool WL = PREC != PREC_F32 && (KS <= 3 || BM <= 32);
  constexpr int QW = NQ;
  constexpr int WITEMS = KS * KS * BM * NQ;
  constexpr int PERW = WL ? (WITEMS + 255) / 256 : 1;
  __shared__ u4 xs[NPIX * QS];
  __shared__ u4 wsm[WL ? KS * KS * BM * QW : 1];

  const ConvParams& c = p.c;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 15, g = lane >> 4;
  // 1-D grid, split index fastest: workgroups b and b + 8 share an XCD
  // (round-robin dispatch), so with ksplit a multiple of 8 each XCD's L2 holds
  // the weights of its own splits only (MODNet's 5x5 1280 -> 96 layer: 6 MB
  // of bf16 weights, re-read per pixel tile, no longer from HBM).
  // Without a split (p.xcd) the items are dealt to the XCDs in contiguous
  // runs instead: XCD x = b % 8 runs items [x q + min(x, r), ...) of the
  // grid's q = G / 8, r = G % 8 split, in raster order, so the halo rows a
  // tile shares with the tiles above and below it and the 128-B lines its
  // 34-pixel rows straddle are read once into that XCD's L2 rather than
  // once per XCD (3x3 64 -> 64 at 72x128, batch 8: ~2.4x the input's bytes
  // fetched past L2 in round-robin order).  A bijection on [0, G).
  int L = blockIdx.x;
  if (p.xcd && p.ksplit == 1) L = xcd_item(L, gridDim.x);
  const int kz = L % p.ksplit;
  const int rest = L / p.ksplit;
  const int t = rest % p.tiles, mt = (rest / p.tiles) % p.mtiles, n = rest / (p.tiles * p.mtiles);
  const int oy0 = (t / p.tiles_x) * TH, ox0 = (t % p.tiles_x) * TW;
  const int m0 = mt * BM;
  const int nch = p.Cp / CK;
  const int cbeg = kz * p.cps, cend = min(nch, cbeg + p.cps);
  const int iy0 = oy0 * S - c.pt, ix0 = ox0 * S - c.pl;
  const float* xn = c.x + (long)n * c.C * c.H * c.W;
  const long plane = (long)c.H * c.W;

  // The image as a raw buffer (wave-uniform base, range = its C planes): every
  // staging load is unconditional, at a 32-bit byte offset, and the hardware's
  // range check returns 0 for the halo outside the image (its offset is moved
  // past the range) and for channels past C (their offsets lie past the last
  // plane).  The per-element conditional loads this replaced compiled to a
  // branch and an exec-mask swap per element (~5k instructions per chunk).
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(uniform_ptr(xn)), 0, (int)((long)c.C * plane * 4), 0x00020000);
  // (the chunks from p.x2_c0 on: the Concat's last input, its own tensor)
  const __amdgpu_buffer_rsrc_t xr2 = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(uniform_ptr(p.x2 ? p.x2 + (long)n * p.x2_C * plane : xn)), 0,
      (int)((long)(p.x2 ? p.x2_C : c.C) * plane * 4), 0x00020000);
  const unsigned plane4 = (unsigned)plane * 4u;
  unsigned soff[PER];  // per item: the byte offset of (channel q * CG, pixel) in the chunk, or out of range
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int idx = tid + 256 * u;
    const int q = idx / NPIX, pix = idx - q * NPIX;
    const int iy = pix / IW, ix = pix - iy * IW;
    const int gy = iy0 + iy, gx = ix0 + ix;
    const bool in = idx < ITEMS && (unsigned)gy < (unsigned)c.H && (unsigned)gx < (unsigned)c.W;
    soff[u] = in ? (unsigned)(q * CG) * plane4 + (unsigned)(gy * c.W + gx) * 4u : 0x80000000u;
  }
  // UP: the chunk's source region [CK][SR][SC] from the low-resolution image
  // (rows / columns clamped to it; the halo's zeros come from the items'
  // validity), copied global -> LDS with no register stage (LDS-DMA: the
  // destination is linear in the region's order) while the previous chunk's
  // MFMAs run; the barrier that opens the next chunk waits for it
  constexpr int SR = UP ? IH / 2 + 2 : 1, SC = UP ? IW / 2 + 2 : 1, SRC = SR * SC;
  constexpr int RITEMS = SRC * CK, PR = UP ? (RITEMS + 255) / 256 : 1;
  __shared__ float lrs[UP ? PR * 256 : 1];
  const int up_plane = UP ? p.up_H * p.up_W : 0;
  const int ry0 = max(0, (iy0 - 1) >> 1), rx0 = max(0, (ix0 - 1) >> 1);  // the region's origin
  const float* upn = UP ? p.up + (long)n * (p.up_c1 - p.up_c0) * up_plane : xn;
  // is chunk ch an upsampled one (uniform: the range is whole chunks)
  auto up_chunk = [&](int ch) { return UP && ch * CK >= p.up_c0 && ch * CK < p.up_c1; };
  // (the chunk's CK planes as a buffer: 32-bit byte offsets, no 64-bit
  // address arithmetic per element — it was ~25 VALU per element, as many
  // as the interpolation's)
  auto load_region = [&](int ch) {
    const int c0 = ch * CK - p.up_c0;
    const int wbase = __builtin_amdgcn_readfirstlane((tid >> 6) << 6);
    const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<void*>(uniform_ptr(upn + (long)c0 * up_plane)), 0, CK * up_plane * 4, 0x00020000);
#pragma unroll
    for (int u = 0; u < PR; ++u) {
      const int idx = min(tid + 256 * u, RITEMS - 1);
      const int cc = idx / SRC, rem = idx - cc * SRC, a = rem / SC, b = rem - a * SC;
      const int yy = min(ry0 + a, p.up_H - 1), xx = min(rx0 + b, p.up_W - 1);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rr, (__attribute__((address_space(3))) void*)(lrs + 256 * u + wbase), 4,
                                               (cc * up_plane + yy * p.up_W + xx) * 4, 0, 0, 0);
    }
  };
  float st[PER][CG];
  auto load = [&](int ch) {
    if (up_chunk(ch)) {
      load_region(ch);
      return;
    }
    const bool sec = p.x2 && ch * CK >= p.x2_c0;  // (uniform) from the Concat's last input
    const __amdgpu_buffer_rsrc_t r = sec ? xr2 : xr;
    const unsigned cofs = (unsigned)(sec ? ch * CK - p.x2_c0 : ch * CK) * plane4;  // the chunk's first plane
    // quads with no channel below C (a partial last chunk: MODNet's 35 -> 16
    // fusion layer stages 3 real channels of 32) skip their loads — one
    // branch per item; the zeros are those the range check would return
    const int cend_ch = sec ? p.x2_c0 + p.x2_C : (p.x2 ? p.x2_c0 : c.C);
    const int qv = p.qskip ? min(NQ, (cend_ch - ch * CK + CG - 1) / CG) : NQ;
    const int uend = (qv * NPIX + 255) / 256;  // items u >= uend hold only such quads (uniform)
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const unsigned o = soff[u] + cofs;  // out-of-range items stay out of range (no wrap: < 2 GiB added)
      if (u < uend) {
#pragma unroll
        for (int e = 0; e < CG; ++e)
          st[u][e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)(o + e * plane4), 0, 0));
      } else {
#pragma unroll
        for (int e = 0; e < CG; ++e) st[u][e] = 0.f;
      }
    }
  };
  const u4* wq = static_cast<const u4*>(p.wp);  // [tap][Mp][Cp] in quads of T
  const int cq = p.Cp / CG;                            // quads per weight row
  // weight staging: item u of a chunk is quad idx of [tap][BM rows][NQ], its
  // LDS slot; its global quad index at chunk 0 worked out once (the index is
  // clamped: items past WITEMS load a valid quad and store nothing).  A lambda
  // with a fully unrolled loop: the macro form left stw[] in scratch.
  unsigned woff[PERW];
  u4 stw[PERW];
#pragma unroll
  for (int u = 0; u < PERW; ++u) {
    const int idx = min(tid + 256 * u, WITEMS - 1);
    const int tap = idx / (BM * NQ), rem = idx - tap * (BM * NQ);
    const int m = rem / NQ, q = rem - m * NQ;
    woff[u] = (unsigned)((tap * p.Mp + m0 + m) * cq + q);
  }
  auto load_w = [&](int chw) {
    if constexpr (WL) {
#pragma unroll
      for (int u = 0; u < PERW; ++u) stw[u] = wq[woff[u] + (unsigned)(chw * NQ)];
    }
  };
  f4 acc[MI][PBW];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < PBW; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

  // this wave's blocks: LDS pixel of lane r at tap (0, 0)
  int bpix[PBW];
#pragma unroll
  for (int j = 0; j < PBW; ++j) {
    const int b = wave * PBW + j;
    const int ty = b / (TW / 16), tx = (b % (TW / 16)) * 16 + r;
    bpix[j] = ty * S * IW + tx * S;
  }
  // UP: a plain chunk right after the upsampled one (staged by DMA, no
  // registers) loads into its registers from the start, in flight with the
  // source region instead of after the interpolation (MODNet's 35 -> 16
  // fusion layer: the image's 3 channels behind the 32 upsampled ones)
  bool ahead = false;
  if (cbeg < cend) {
    load(cbeg);
    load_w(cbeg);
    if (UP && up_chunk(cbeg) && cbeg + 1 < cend && !up_chunk(cbeg + 1)) {
      load(cbeg + 1);
      ahead = true;
    }
  }
  for (int ch = cbeg; ch < cend; ++ch) {
    __syncthreads();  // the previous chunk's fragment reads are done
    if (up_chunk(ch)) {
      if constexpr (UP) {
        // items of one pixel and QI quads (QI x CG channels): the pixel's
        // source coordinates and taps worked out once per item rather than
        // once per quad (the coordinate and address arithmetic was most of
        // this loop's VALU: ~150 per 8-channel item, 36 of them the lerps)
        constexpr int QI = NQ % 2 == 0 ? 2 : 1, NIT = NPIX * (NQ / QI), PERI = (NIT + 255) / 256;
#pragma unroll 1
        for (int u = 0; u < PERI; ++u) {
          const int idx = tid + 256 * u;
          if (idx < NIT) {
            const int qh = idx / NPIX, pix = idx - qh * NPIX;
            const int iy = pix / IW, ix = pix - iy * IW;
            const int gy = iy0 + iy, gx = ix0 + ix;
            const bool in = (unsigned)gy < (unsigned)c.H && (unsigned)gx < (unsigned)c.W;
            const float sy = fminf(fmaxf(((float)gy + 0.5f) * 0.5f - 0.5f, 0.f), (float)(p.up_H - 1));
            const float sx = fminf(fmaxf(((float)gx + 0.5f) * 0.5f - 0.5f, 0.f), (float)(p.up_W - 1));
            const int y0 = (int)sy, x0 = (int)sx;
            const float ly = sy - (float)y0, lx = sx - (float)x0;
            // region pixels (clamped into the region: only out-of-image items, whose value is dropped, clamp)
            const int a0 = min(max(y0 - ry0, 0), SR - 1), a1 = min(max(min(y0 + 1, p.up_H - 1) - ry0, 0), SR - 1);
            const int b0 = min(max(x0 - rx0, 0), SC - 1), b1 = min(max(min(x0 + 1, p.up_W - 1) - rx0, 0), SC - 1);
            const int t00 = a0 * SC + b0, t01 = a0 * SC + b1, t10 = a1 * SC + b0, t11 = a1 * SC + b1;
            const float keep = in ? 1.f : 0.f;
#pragma unroll 1
            for (int qq = 0; qq < QI; ++qq) {
              const int q = qh * QI + qq;
              const float* l = lrs + q * CG * SRC;
              // every tap read unconditionally (the clamped taps lie in the
              // region), all 4 x CG in flight at once, the halo's zero applied
              // after as a product with 0 / 1 (finite values: the same as the
              // select): with `in ? interp : 0` the compiler sank the reads
              // into a branch per channel, an exposed LDS round trip each
              float t0[CG], t1[CG], t2[CG], t3[CG];
#pragma unroll
              for (int e = 0; e < CG; ++e) {
                t0[e] = l[e * SRC + t00];
                t1[e] = l[e * SRC + t01];
                t2[e] = l[e * SRC + t10];
                t3[e] = l[e * SRC + t11];
              }
              float v[CG];
#pragma unroll
              for (int e = 0; e < CG; ++e)
                v[e] = keep * ((1.f - ly) * ((1.f - lx) * t0[e] + lx * t1[e]) + ly * ((1.f - lx) * t2[e] + lx * t3[e]));
              xs[pix * QS + q] = pack_quad<PREC>(v);
            }
          }
        }
      }
    } else {
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        const int idx = tid + 256 * u;
        if (idx < ITEMS) {
          const int q = idx / NPIX, pix = idx - q * NPIX;
          xs[pix * QS + q] = pack_quad<PREC>(st[u]);
        }
      }
    }
    if constexpr (WL) {
      static_assert(QW == 4 && NQ == 4, "item idx = row idx / 4, quad idx % 4");
#pragma unroll
      for (int u = 0; u < PERW; ++u) {
        const int idx = tid + 256 * u;
        if (WITEMS % 256 == 0 || idx < WITEMS) wsm[idx ^ wsw(idx >> 2)] = stw[u];
      }
    }
    __syncthreads();
    if (ch + 1 < cend) {  // in flight during this chunk's MFMAs
      if (!(ahead && ch == cbeg)) load(ch + 1);
      load_w(ch + 1);
    }
    const int wc = ch * (CK / CG);    // this chunk's first quad in a weight row
#pragma unroll
    for (int ky = 0; ky < KS; ++ky) {
#pragma unroll
      for (int kx = 0; kx < KS; ++kx) {
        const int tap = ky * KS + kx;
        u4 a[MI][NF];
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          if (WL) {
            a[i][0] = wsm[(tap * BM + 16 * i + r) * QW + (g ^ wsw(r))];  // (tap * BM + 16 i) = 0 mod 16
          } else {
            const u4* row = wq + ((long)tap * p.Mp + m0 + 16 * i + r) * cq + wc;
#pragma unroll
            for (int f = 0; f < NF; ++f) a[i][f] = row[g + 4 * f];
          }
        }
#pragma unroll
        for (int j = 0; j < PBW; ++j) {
          u4 b[NF];
          const u4* px = xs + (bpix[j] + ky * IW + kx) * QS;
#pragma unroll
          for (int f = 0; f < NF; ++f) b[f] = px[g + 4 * f];
#pragma unroll
          for (int i = 0; i < MI; ++i) acc[i][j] = mma32<PREC>(a[i], b, acc[i][j]);
        }
      }
    }
  }

  // acc[i][j][v] = out channel m0 + 16 i + 4 g + v, pixel r of block j
  const int P = c.Ho * c.Wo;
  if (p.ksplit > 1) {
    // the partial tile in accumulator order: [output block][split][i, j][thread] as
    // f4, stored write-through (8-byte agent-scope stores: sc1) so the last
    // workgroup to arrive — on any XCD — reads them from memory with sc1 loads
    // (MI355X_MICROARCH.md, hand-off table row 1: no fences)
    const long blk = ((long)n * p.mtiles + mt) * p.tiles + t;
    uint64_t* part = reinterpret_cast<uint64_t*>(p.part) + (blk * p.ksplit + kz) * (MI * PBW * 256 * 2);
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < PBW; ++j) {
        const uint64_t lo = (uint64_t)__float_as_uint(acc[i][j][0]) | ((uint64_t)__float_as_uint(acc[i][j][1]) << 32);
        const uint64_t hi = (uint64_t)__float_as_uint(acc[i][j][2]) | ((uint64_t)__float_as_uint(acc[i][j][3]) << 32);
        uint64_t* q = part + ((i * PBW + j) * 256 + tid) * 2;
        __hip_atomic_store(q, lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(q + 1, hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    // Ordering: the hardware side is the vmcnt(0) drain below (every sc1 store
    // has left the CU before the arrival is counted) and sc1 loads on the
    // consumer side (L1 bypassed) — the measured protocol of
    // MI355X_MICROARCH.md's hand-off table, row 1.  The compiler side is the
    // asm's memory clobber plus the signal fences (no load or store moves
    // across them).  An acq_rel agent-scope fetch_add instead would add a
    // buffer_wbl2 + buffer_inv per workgroup (~3.5 us each, measured 2x slower
    // for the whole layer in round 1).
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __shared__ int last;
    __syncthreads();
    if (tid == 0) {
      int* cnt = p.counters + blk;
      const int prev = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last = prev == p.ksplit - 1;
      if (last) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // ready for the next run
    }
    __syncthreads();
    if (!last) return;
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    const uint64_t* base = reinterpret_cast<const uint64_t*>(p.part) + blk * p.ksplit * (MI * PBW * 256 * 2);
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < PBW; ++j) {
        f4 sum = f4{0.f, 0.f, 0.f, 0.f};
        for (int k0 = 0; k0 < p.ksplit; k0 += 8) {  // 8 splits' loads in flight, summed in split order
          uint64_t lo[8], hi[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            if (k0 + u < p.ksplit) {
              const uint64_t* q = base + (((k0 + u) * MI * PBW + i * PBW + j) * 256 + tid) * 2;
              lo[u] = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              hi[u] = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
          }
#pragma unroll
          for (int u = 0; u < 8; ++u)
            if (k0 + u < p.ksplit)
              sum += f4{__uint_as_float((uint32_t)lo[u]), __uint_as_float((uint32_t)(lo[u] >> 32)),
                        __uint_as_float((uint32_t)hi[u]), __uint_as_float((uint32_t)(hi[u] >> 32))};
        }
        acc[i][j] = sum;
      }
  }
  // epilogue: bias, residual, then the activation over all the lane's outputs
  // under one uniform switch (act_block), then the stores.  Output k = (i, j,
  // v): channel m0 + 16 i + 4 g + v, pixel r of block j.
  const Epilogue& ep = c.ep;
  constexpr int NO = MI * PBW * 4;
  float o[NO];
  auto ch_of = [&](int k) { return m0 + 16 * (k / (PBW * 4)) + 4 * g + (k & 3); };
  int pixj[PBW];
  bool okj[PBW];
#pragma unroll
  for (int j = 0; j < PBW; ++j) {
    const int b = wave * PBW + j;
    const int oy = oy0 + b / (TW / 16), ox = ox0 + (b % (TW / 16)) * 16 + r;
    okj[j] = oy < c.Ho && ox < c.Wo;
    pixj[j] = okj[j] ? oy * c.Wo + ox : 0;
  }
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int ch = m0 + 16 * i + 4 * g + v;
      const float bv = ep.bias ? ep.bias[min(ch, c.M - 1)] : 0.f;
#pragma unroll
      for (int j = 0; j < PBW; ++j) o[(i * PBW + j) * 4 + v] = acc[i][j][v] + bv;
    }
  // 32-bit offsets off the image's planes (uniform bases)
  if (ep.res) {
    if (ep.res_mode == 0) {
      const float* rn = ep.res + (long)n * c.M * P;
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < PBW; ++j)
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            const int ch = m0 + 16 * i + 4 * g + v;
            if (okj[j] && ch < c.M) o[(i * PBW + j) * 4 + v] += rn[ch * P + pixj[j]];
          }
    } else {  // the fused Pad / MaxPool residuals (face models): rare, one copy of the code
      each_rare(o, [&](int k, float v) {
        const int j = (k >> 2) % PBW, ch = ch_of(k);
        int pj = pixj[0];
        bool ok = okj[0];
#pragma unroll
        for (int t = 1; t < PBW; ++t) {
          pj = j == t ? pixj[t] : pj;
          ok = j == t ? okj[t] : ok;
        }
        ok = ok && ch < c.M;
        return ok ? v + residual(ep, ch, ((long)n * c.M + ch) * P + pj, n, pj) : v;
      });
    }
  }
  act_block(o, ch_of, ep);
  float* yn = c.y + (long)n * ((long)c.M * P + c.y_nx);
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < PBW; ++j)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int ch = m0 + 16 * i + 4 * g + v;
        if (okj[j] && ch < c.M) yn[ch * P + pixj[j]] = o[(i * PBW + j) * 4 + v];
      }
}

template <int PREC, int KS, int S, int TH, int TW, int BM, bool UP>
__device__ __forceinline__ void conv_tile_body_persist(const ConvTileParams& p) {
  using T = typename Elem<PREC>::T;
  constexpr int NQ = CK * (int)sizeof(T) / 16;     // quads of one pixel's chunk: 8 (f32) / 4
  constexpr int QS = conv_qs<PREC, S>();           // LDS pixel stride in quads (above)
  constexpr int CG = 16 / (int)sizeof(T);          // channels per quad
  constexpr int NF = PREC == PREC_F32 ? 2 : 1;     // fragment quads per lane
  constexpr int IH = (TH - 1) * S + KS, IW = (TW - 1) * S + KS, NPIX = IH * IW;
  constexpr int ITEMS = NPIX * NQ;                 // quads staged per chunk
  constexpr int PER = (ITEMS + 255) / 256;
  constexpr int NB = TH * TW / 16, PBW = NB / 4;   // 16-pixel blocks per tile / per wave
  constexpr int MI = BM / 16;
  static_assert(NB % 4 == 0 && TW % 16 == 0, "tile: a multiple of 64 pixels, rows of 16");
  // 16-bit operands, k <= 3 (and 5x5 on 16 / 32-channel tiles: <= 51 KB): the chunk's weights of all taps staged in LDS too
  // ([tap][BM rows][NQ quads]), loaded once per workgroup instead of once
  // per wave and tap from L2 (whose latency the per-tap MFMAs cannot cover)
  constexpr bool WL = PREC != PREC_F32 && (KS <= 3 || BM <= 32);
  constexpr int QW = NQ;
  constexpr int WITEMS = KS * KS * BM * NQ;
  constexpr int PERW = WL ? (WITEMS + 255) / 256 : 1;
  __shared__ u4 xs[NPIX * QS];
  __shared__ u4 wsm[WL ? KS * KS * BM * QW : 1];

  const ConvParams& c = p.c;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 15, g = lane >> 4;
  // Work items L = (n, M tile, pixel tile, split), split index fastest: items
  // L and L + 8 share an XCD (round-robin dispatch, a grid of a multiple of 8
  // workgroups), so with ksplit a multiple of 8 each XCD's L2 holds the
  // weights of its own splits only (MODNet's 5x5 1280 -> 96 layer: 6 MB of
  // bf16 weights, re-read per pixel tile, no longer from HBM).  A workgroup
  // runs items blockIdx.x, + gridDim.x, ... < p.items, software-pipelined: the
  // next item's first chunk loads while this item's last chunk runs its MFMAs
  // and epilogue, so a workgroup's staging latency is exposed once per launch
  // rather than once per tile (gridDim.x = p.items: one item per workgroup).
  // Instantiated for f32 operands only (conv_tile_persist): in the 16-bit
  // forms this loop's registers crossed the occupancy steps (114 -> 172,
  // 218 -> 262 VGPRs) and MODNet b8 bf16 went 1.35 -> 1.51 ms, while f32
  // gained 3.52 -> 3.39 (profiles/r05z); they keep conv_tile_body.
  constexpr bool PERSIST = true;
  struct Item {
    int L, kz, t, mt, n, oy0, ox0, m0, cbeg, cend, iy0, ix0, ry0, rx0;
  };
  const int nch = p.Cp / CK;
  auto item_of = [&](int L) {
    Item it;
    it.L = L;
    it.kz = L % p.ksplit;
    const int rest = L / p.ksplit;
    it.t = rest % p.tiles;
    it.mt = (rest / p.tiles) % p.mtiles;
    it.n = rest / (p.tiles * p.mtiles);
    it.oy0 = (it.t / p.tiles_x) * TH;
    it.ox0 = (it.t % p.tiles_x) * TW;
    it.m0 = it.mt * BM;
    it.cbeg = it.kz * p.cps;
    it.cend = min(nch, it.cbeg + p.cps);
    it.iy0 = it.oy0 * S - c.pt;
    it.ix0 = it.ox0 * S - c.pl;
    it.ry0 = max(0, (it.iy0 - 1) >> 1);  // UP: the source region's origin
    it.rx0 = max(0, (it.ix0 - 1) >> 1);
    return it;
  };
  if ((int)blockIdx.x >= p.items) return;
  Item cur = item_of(blockIdx.x);
  const long plane = (long)c.H * c.W;

  // The image as a raw buffer (wave-uniform base, range = its C planes): every
  // staging load is unconditional, at a 32-bit byte offset, and the hardware's
  // range check returns 0 for the halo outside the image (its offset is moved
  // past the range) and for channels past C (their offsets lie past the last
  // plane).  The per-element conditional loads this replaced compiled to a
  // branch and an exec-mask swap per element (~5k instructions per chunk).
  // (the state below is the loading item's: set by set_load_item)
  __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(uniform_ptr(c.x)), 0, (int)((long)c.C * plane * 4), 0x00020000);
  __amdgpu_buffer_rsrc_t xr2 = xr;  // (the Concat's last input: conv_tile_body)
  const unsigned plane4 = (unsigned)plane * 4u;
  unsigned soff[PER];  // per item: the byte offset of (channel q * CG, pixel) in the chunk, or out of range
  auto set_soff = [&](const Item& it) {
    const float* xn = c.x + (long)it.n * c.C * c.H * c.W;
    xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(uniform_ptr(xn)), 0, (int)((long)c.C * plane * 4),
                                           0x00020000);
    xr2 = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<void*>(uniform_ptr(p.x2 ? p.x2 + (long)it.n * p.x2_C * plane : xn)), 0,
        (int)((long)(p.x2 ? p.x2_C : c.C) * plane * 4), 0x00020000);
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int idx = tid + 256 * u;
      const int q = idx / NPIX, pix = idx - q * NPIX;
      const int iy = pix / IW, ix = pix - iy * IW;
      const int gy = it.iy0 + iy, gx = it.ix0 + ix;
      const bool in = idx < ITEMS && (unsigned)gy < (unsigned)c.H && (unsigned)gx < (unsigned)c.W;
      soff[u] = in ? (unsigned)(q * CG) * plane4 + (unsigned)(gy * c.W + gx) * 4u : 0x80000000u;
    }
  };
  // UP: the chunk's source region [CK][SR][SC] from the low-resolution image
  // (rows / columns clamped to it; the halo's zeros come from the items'
  // validity), copied global -> LDS with no register stage (LDS-DMA: the
  // destination is linear in the region's order) while the previous chunk's
  // MFMAs run; the barrier that opens the next chunk waits for it
  constexpr int SR = UP ? IH / 2 + 2 : 1, SC = UP ? IW / 2 + 2 : 1, SRC = SR * SC;
  constexpr int RITEMS = SRC * CK, PR = UP ? (RITEMS + 255) / 256 : 1;
  __shared__ float lrs[UP ? PR * 256 : 1];
  const int up_plane = UP ? p.up_H * p.up_W : 0;
  int lry0 = 0, lrx0 = 0;  // the loading item's region origin and image
  const float* upn = p.up;
  // is chunk ch an upsampled one (uniform: the range is whole chunks)
  auto up_chunk = [&](int ch) { return UP && ch * CK >= p.up_c0 && ch * CK < p.up_c1; };
  auto load_region = [&](int ch) {
    const int c0 = ch * CK - p.up_c0;
    const int wbase = __builtin_amdgcn_readfirstlane((tid >> 6) << 6);
#pragma unroll
    for (int u = 0; u < PR; ++u) {
      const int idx = min(tid + 256 * u, RITEMS - 1);
      const int cc = idx / SRC, rem = idx - cc * SRC, a = rem / SC, b = rem - a * SC;
      const int yy = min(lry0 + a, p.up_H - 1), xx = min(lrx0 + b, p.up_W - 1);
      __builtin_amdgcn_global_load_lds(
          (__attribute__((address_space(1))) void*)(upn + (c0 + cc) * up_plane + yy * p.up_W + xx),
          (__attribute__((address_space(3))) void*)(lrs + 256 * u + wbase), 4, 0, 0);
    }
  };
  float st[PER][CG];
  auto load = [&](int ch) {
    if (up_chunk(ch)) {
      load_region(ch);
      return;
    }
    const bool sec = p.x2 && ch * CK >= p.x2_c0;  // (uniform) from the Concat's last input
    const __amdgpu_buffer_rsrc_t r = sec ? xr2 : xr;
    const unsigned cofs = (unsigned)(sec ? ch * CK - p.x2_c0 : ch * CK) * plane4;  // the chunk's first plane
    // quads with no channel below C (a partial last chunk: MODNet's 35 -> 16
    // fusion layer stages 3 real channels of 32) skip their loads — one
    // branch per item; the zeros are those the range check would return
    const int cend_ch = sec ? p.x2_c0 + p.x2_C : (p.x2 ? p.x2_c0 : c.C);
    const int qv = p.qskip ? min(NQ, (cend_ch - ch * CK + CG - 1) / CG) : NQ;
    const int uend = (qv * NPIX + 255) / 256;  // items u >= uend hold only such quads (uniform)
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const unsigned o = soff[u] + cofs;  // out-of-range items stay out of range (no wrap: < 2 GiB added)
      if (u < uend) {
#pragma unroll
        for (int e = 0; e < CG; ++e)
          st[u][e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)(o + e * plane4), 0, 0));
      } else {
#pragma unroll
        for (int e = 0; e < CG; ++e) st[u][e] = 0.f;
      }
    }
  };
  const u4* wq = static_cast<const u4*>(p.wp);  // [tap][Mp][Cp] in quads of T
  const int cq = p.Cp / CG;                            // quads per weight row
  // weight staging: item u of a chunk is quad idx of [tap][BM rows][NQ], its
  // LDS slot; its global quad index at chunk 0 worked out once (the index is
  // clamped: items past WITEMS load a valid quad and store nothing).  A lambda
  // with a fully unrolled loop: the macro form left stw[] in scratch.
  unsigned woff[PERW];
  u4 stw[PERW];
  auto set_load_item = [&](const Item& it) {
    set_soff(it);
    lry0 = it.ry0;
    lrx0 = it.rx0;
    if constexpr (UP) upn = p.up + (long)it.n * (p.up_c1 - p.up_c0) * up_plane;
#pragma unroll
    for (int u = 0; u < PERW; ++u) {
      const int idx = min(tid + 256 * u, WITEMS - 1);
      const int tap = idx / (BM * NQ), rem = idx - tap * (BM * NQ);
      const int m = rem / NQ, q = rem - m * NQ;
      woff[u] = (unsigned)((tap * p.Mp + it.m0 + m) * cq + q);
    }
  };
  auto load_w = [&](int chw) {
    if constexpr (WL) {
#pragma unroll
      for (int u = 0; u < PERW; ++u) stw[u] = wq[woff[u] + (unsigned)(chw * NQ)];
    }
  };
  f4 acc[MI][PBW];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < PBW; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

  // this wave's blocks: LDS pixel of lane r at tap (0, 0)
  int bpix[PBW];
#pragma unroll
  for (int j = 0; j < PBW; ++j) {
    const int b = wave * PBW + j;
    const int ty = b / (TW / 16), tx = (b % (TW / 16)) * 16 + r;
    bpix[j] = ty * S * IW + tx * S;
  }
  auto epilogue = [&](const Item& it) {
    const int n = it.n, mt = it.mt, t = it.t, kz = it.kz, m0 = it.m0, oy0 = it.oy0, ox0 = it.ox0;
    // acc[i][j][v] = out channel m0 + 16 i + 4 g + v, pixel r of block j
    const int P = c.Ho * c.Wo;
    if (p.ksplit > 1) {
      // the partial tile in accumulator order: [output block][split][i, j][thread] as
      // f4, stored write-through (8-byte agent-scope stores: sc1) so the last
      // workgroup to arrive — on any XCD — reads them from memory with sc1 loads
      // (MI355X_MICROARCH.md, hand-off table row 1: no fences)
      const long blk = ((long)n * p.mtiles + mt) * p.tiles + t;
      uint64_t* part = reinterpret_cast<uint64_t*>(p.part) + (blk * p.ksplit + kz) * (MI * PBW * 256 * 2);
  #pragma unroll
      for (int i = 0; i < MI; ++i)
  #pragma unroll
        for (int j = 0; j < PBW; ++j) {
          const uint64_t lo = (uint64_t)__float_as_uint(acc[i][j][0]) | ((uint64_t)__float_as_uint(acc[i][j][1]) << 32);
          const uint64_t hi = (uint64_t)__float_as_uint(acc[i][j][2]) | ((uint64_t)__float_as_uint(acc[i][j][3]) << 32);
          uint64_t* q = part + ((i * PBW + j) * 256 + tid) * 2;
          __hip_atomic_store(q, lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(q + 1, hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      // Ordering: the hardware side is the vmcnt(0) drain below (every sc1 store
      // has left the CU before the arrival is counted) and sc1 loads on the
      // consumer side (L1 bypassed) — the measured protocol of
      // MI355X_MICROARCH.md's hand-off table, row 1.  The compiler side is the
      // asm's memory clobber plus the signal fences (no load or store moves
      // across them).  An acq_rel agent-scope fetch_add instead would add a
      // buffer_wbl2 + buffer_inv per workgroup (~3.5 us each, measured 2x slower
      // for the whole layer in round 1).
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __atomic_signal_fence(__ATOMIC_SEQ_CST);
      __shared__ int last;
      __syncthreads();
      if (tid == 0) {
        int* cnt = p.counters + blk;
        const int prev = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = prev == p.ksplit - 1;
        if (last) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // ready for the next run
      }
      __syncthreads();
      if (!last) return;
      __atomic_signal_fence(__ATOMIC_SEQ_CST);
      const uint64_t* base = reinterpret_cast<const uint64_t*>(p.part) + blk * p.ksplit * (MI * PBW * 256 * 2);
  #pragma unroll
      for (int i = 0; i < MI; ++i)
  #pragma unroll
        for (int j = 0; j < PBW; ++j) {
          f4 sum = f4{0.f, 0.f, 0.f, 0.f};
          for (int k0 = 0; k0 < p.ksplit; k0 += 8) {  // 8 splits' loads in flight, summed in split order
            uint64_t lo[8], hi[8];
  #pragma unroll
            for (int u = 0; u < 8; ++u) {
              if (k0 + u < p.ksplit) {
                const uint64_t* q = base + (((k0 + u) * MI * PBW + i * PBW + j) * 256 + tid) * 2;
                lo[u] = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                hi[u] = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              }
            }
  #pragma unroll
            for (int u = 0; u < 8; ++u)
              if (k0 + u < p.ksplit)
                sum += f4{__uint_as_float((uint32_t)lo[u]), __uint_as_float((uint32_t)(lo[u] >> 32)),
                          __uint_as_float((uint32_t)hi[u]), __uint_as_float((uint32_t)(hi[u] >> 32))};
          }
          acc[i][j] = sum;
        }
    }
    // epilogue: bias, residual, then the activation over all the lane's outputs
    // under one uniform switch (act_block), then the stores.  Output k = (i, j,
    // v): channel m0 + 16 i + 4 g + v, pixel r of block j.
    const Epilogue& ep = c.ep;
    constexpr int NO = MI * PBW * 4;
    float o[NO];
    auto ch_of = [&](int k) { return m0 + 16 * (k / (PBW * 4)) + 4 * g + (k & 3); };
    int pixj[PBW];
    bool okj[PBW];
  #pragma unroll
    for (int j = 0; j < PBW; ++j) {
      const int b = wave * PBW + j;
      const int oy = oy0 + b / (TW / 16), ox = ox0 + (b % (TW / 16)) * 16 + r;
      okj[j] = oy < c.Ho && ox < c.Wo;
      pixj[j] = okj[j] ? oy * c.Wo + ox : 0;
    }
  #pragma unroll
    for (int i = 0; i < MI; ++i)
  #pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int ch = m0 + 16 * i + 4 * g + v;
        const float bv = ep.bias ? ep.bias[min(ch, c.M - 1)] : 0.f;
  #pragma unroll
        for (int j = 0; j < PBW; ++j) o[(i * PBW + j) * 4 + v] = acc[i][j][v] + bv;
      }
    // 32-bit offsets off the image's planes (uniform bases)
    if (ep.res) {
      if (ep.res_mode == 0) {
        const float* rn = ep.res + (long)n * c.M * P;
  #pragma unroll
        for (int i = 0; i < MI; ++i)
  #pragma unroll
          for (int j = 0; j < PBW; ++j)
  #pragma unroll
            for (int v = 0; v < 4; ++v) {
              const int ch = m0 + 16 * i + 4 * g + v;
              if (okj[j] && ch < c.M) o[(i * PBW + j) * 4 + v] += rn[ch * P + pixj[j]];
            }
      } else {  // the fused Pad / MaxPool residuals (face models): rare, one copy of the code
        each_rare(o, [&](int k, float v) {
          const int j = (k >> 2) % PBW, ch = ch_of(k);
          int pj = pixj[0];
          bool ok = okj[0];
  #pragma unroll
          for (int t = 1; t < PBW; ++t) {
            pj = j == t ? pixj[t] : pj;
            ok = j == t ? okj[t] : ok;
          }
          ok = ok && ch < c.M;
          return ok ? v + residual(ep, ch, ((long)n * c.M + ch) * P + pj, n, pj) : v;
        });
      }
    }
    act_block(o, ch_of, ep);
    float* yn = c.y + (long)n * ((long)c.M * P + c.y_nx);
  #pragma unroll
    for (int i = 0; i < MI; ++i)
  #pragma unroll
      for (int j = 0; j < PBW; ++j)
  #pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int ch = m0 + 16 * i + 4 * g + v;
          if (okj[j] && ch < c.M) yn[ch * P + pixj[j]] = o[(i * PBW + j) * 4 + v];
        }
  };

  set_load_item(cur);
  int ch = cur.cbeg;
  load(ch);
  load_w(ch);
  for (;;) {
    __syncthreads();  // the previous chunk's fragment reads are done
    const int iy0 = cur.iy0, ix0 = cur.ix0, ry0 = cur.ry0, rx0 = cur.rx0, m0 = cur.m0;
    if (up_chunk(ch)) {
      if constexpr (UP) {
#pragma unroll 1
        for (int u = 0; u < PER; ++u) {
          const int idx = tid + 256 * u;
          if (idx < ITEMS) {
            const int q = idx / NPIX, pix = idx - q * NPIX;
            const int iy = pix / IW, ix = pix - iy * IW;
            const int gy = iy0 + iy, gx = ix0 + ix;
            const bool in = (unsigned)gy < (unsigned)c.H && (unsigned)gx < (unsigned)c.W;
            const float sy = fminf(fmaxf(((float)gy + 0.5f) * 0.5f - 0.5f, 0.f), (float)(p.up_H - 1));
            const float sx = fminf(fmaxf(((float)gx + 0.5f) * 0.5f - 0.5f, 0.f), (float)(p.up_W - 1));
            const int y0 = (int)sy, x0 = (int)sx;
            const float ly = sy - (float)y0, lx = sx - (float)x0;
            // region pixels (clamped into the region: only out-of-image items, whose value is dropped, clamp)
            const int a0 = min(max(y0 - ry0, 0), SR - 1), a1 = min(max(min(y0 + 1, p.up_H - 1) - ry0, 0), SR - 1);
            const int b0 = min(max(x0 - rx0, 0), SC - 1), b1 = min(max(min(x0 + 1, p.up_W - 1) - rx0, 0), SC - 1);
            const int t00 = a0 * SC + b0, t01 = a0 * SC + b1, t10 = a1 * SC + b0, t11 = a1 * SC + b1;
            const float* l = lrs + q * CG * SRC;
            // (a form reading every tap unconditionally, all 4 x CG in flight
            // at once, measured slower: the 8 x 32 x 32 tile's 258 VGPRs left
            // one wave per SIMD — MODNet b8 bf16 1.358 against 1.347 ms, r05y / r05z)
            float v[CG];
#pragma unroll
            for (int e = 0; e < CG; ++e)
              v[e] = in ? (1.f - ly) * ((1.f - lx) * l[e * SRC + t00] + lx * l[e * SRC + t01]) +
                              ly * ((1.f - lx) * l[e * SRC + t10] + lx * l[e * SRC + t11])
                        : 0.f;
            xs[pix * QS + q] = pack_quad<PREC>(v);
          }
        }
      }
    } else {
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        const int idx = tid + 256 * u;
        if (idx < ITEMS) {
          const int q = idx / NPIX, pix = idx - q * NPIX;
          xs[pix * QS + q] = pack_quad<PREC>(st[u]);
        }
      }
    }
    if constexpr (WL) {
      static_assert(QW == 4 && NQ == 4, "item idx = row idx / 4, quad idx % 4");
#pragma unroll
      for (int u = 0; u < PERW; ++u) {
        const int idx = tid + 256 * u;
        if (WITEMS % 256 == 0 || idx < WITEMS) wsm[idx ^ wsw(idx >> 2)] = stw[u];
      }
    }
    __syncthreads();
    // the next chunk — this item's, or the next item's first — in flight
    // during this chunk's MFMAs (and, at an item's last chunk, its epilogue)
    const bool more = ch + 1 < cur.cend;
    Item nxt = cur;
    int chn = ch + 1;
    bool have = more;
    if constexpr (PERSIST) {
      if (!more) {
        const int Ln = cur.L + (int)gridDim.x;
        have = Ln < p.items;
        if (have) {
          nxt = item_of(Ln);
          chn = nxt.cbeg;
          set_load_item(nxt);
        }
      }
    }
    if (have) {
      load(chn);
      load_w(chn);
    }
    const int wc = ch * (CK / CG);    // this chunk's first quad in a weight row
#pragma unroll
    for (int ky = 0; ky < KS; ++ky) {
#pragma unroll
      for (int kx = 0; kx < KS; ++kx) {
        const int tap = ky * KS + kx;
        u4 a[MI][NF];
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          if (WL) {
            a[i][0] = wsm[(tap * BM + 16 * i + r) * QW + (g ^ wsw(r))];  // (tap * BM + 16 i) = 0 mod 16
          } else {
            const u4* row = wq + ((long)tap * p.Mp + m0 + 16 * i + r) * cq + wc;
#pragma unroll
            for (int f = 0; f < NF; ++f) a[i][f] = row[g + 4 * f];
          }
        }
#pragma unroll
        for (int j = 0; j < PBW; ++j) {
          u4 b[NF];
          const u4* px = xs + (bpix[j] + ky * IW + kx) * QS;
#pragma unroll
          for (int f = 0; f < NF; ++f) b[f] = px[g + 4 * f];
#pragma unroll
          for (int i = 0; i < MI; ++i) acc[i][j] = mma32<PREC>(a[i], b, acc[i][j]);
        }
      }
    }
    if (!more) {
      epilogue(cur);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < PBW; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
    }
    if (!have) break;
    cur = nxt;
    ch = chn;
  }
}

template <int PREC, int KS, int S, int TH, int TW, int BM>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(conv_tile_wpe<PREC, KS, S, TH, TW, BM>(), 8)))
void k_conv_tile(ConvTileParams p) {
  if constexpr (conv_tile_persist(PREC))
    conv_tile_body_persist<PREC, KS, S, TH, TW, BM, false>(p);
  else
    conv_tile_body<PREC, KS, S, TH, TW, BM, false>(p);
}

// The upsample tiles whose LDS (pixel tile, weights, source region) leaves two
// workgroups per CU are held to 256 VGPRs (two waves per SIMD): the 8 x 32 x
// 32 tile sits at 253-258 by the compiler's choice, and one VGPR past 256
// halves its occupancy (49 -> 69 us, profiles/r05x r05y).
template <int PREC, int KS, int S, int TH, int TW, int BM>
constexpr int conv_tile_up_wpe() {
  constexpr int NQ = CK * (PREC == PREC_F32 ? 4 : 2) / 16, IH = (TH - 1) * S + KS, IW = (TW - 1) * S + KS;
  constexpr bool WL = PREC != PREC_F32 && (KS <= 3 || BM <= 32);
  constexpr int SRC = (IH / 2 + 2) * (IW / 2 + 2), PR = (SRC * CK + 255) / 256;
  constexpr int lds = IH * IW * conv_qs<PREC, S>() * 16 + (WL ? KS * KS * BM * NQ * 16 : 16) + PR * 256 * 4;
  // (3x3, <= 32 output channels: the planner's upsample tiles; the larger
  // ones spill under the cap)
  return KS == 3 && BM <= 32 && 163840 / lds >= 2 ? 2 : 1;
}
template <int PREC, int KS, int S, int TH, int TW, int BM>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(conv_tile_up_wpe<PREC, KS, S, TH, TW, BM>(), 8)))
void k_conv_tile_up(ConvTileParams p) {
  conv_tile_body<PREC, KS, S, TH, TW, BM, true>(p);
}
#endif

// ---- instantiations (one precision per compile unit) and dispatch ---------------
// (KS, S, TH, TW): stride 1 (3x3, 5x5) on 8x32, 4x32, 2x32, 16x16, 4x16 tiles;
// stride 2 (3x3) on 2x32, 4x16
#define VSO_TILE_SHAPES_S1(X, PR, K, BMV) \
  X(PR, K, 1, 8, 32, BMV) X(PR, K, 1, 4, 32, BMV) X(PR, K, 1, 2, 32, BMV) X(PR, K, 1, 16, 16, BMV) X(PR, K, 1, 4, 16, BMV)
#define VSO_TILE_SHAPES(X, PR, BMV) \
  VSO_TILE_SHAPES_S1(X, PR, 3, BMV) VSO_TILE_SHAPES_S1(X, PR, 5, BMV) \
  X(PR, 3, 2, 2, 32, BMV) X(PR, 3, 2, 4, 16, BMV)

template <int PREC>
void launch_conv_tile_prec(const ConvTileParams& p, const ConvTileShape& t, hipStream_t s);

#ifdef VSO_CONV_PREC
// Workgroups for `items` work items: one per item, or for the persistent
// forms (conv_tile_persist; VSO_CONV_PERSIST=0: off) as many as are resident
// at once — the kernel's occupancy per CU x the CUs, rounded down to a
// multiple of 8 (XCDs) — each running its items software-pipelined
template <class K>
static void launch_items(K kern, const ConvTileParams& p, long items, hipStream_t s) {
  static const bool persist = conv_tile_persist(VSO_CONV_PREC) && [] {
    const char* e = std::getenv("VSO_CONV_PERSIST");
    return !e || std::atoi(e) != 0;
  }();
  ConvTileParams q = p;
  q.items = (int)items;
  long grid = items;
  if (persist) {
    int dev = 0, cus = 0, per_cu = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 256, 0) == hipSuccess) {
      const long resident = (long)per_cu * cus / 8 * 8;
      if (resident > 0) grid = std::min(grid, resident);
    }
  }
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(256), 0, s, q);
}

template <>
void launch_conv_tile_prec<VSO_CONV_PREC>(const ConvTileParams& p, const ConvTileShape& t, hipStream_t s) {
  const long items = (long)t.tiles * (t.Mp / t.bm) * p.c.N * t.ksplit;
#define VSO_TILE_CASE(PR, KSV, SV, THV, TWV, BMV)                                              \
  if (!t.up && t.ks == KSV && t.s == SV && t.th == THV && t.tw == TWV && t.bm == BMV) {         \
    launch_items(k_conv_tile<PR, KSV, SV, THV, TWV, BMV>, p, items, s);                         \
  } else
#define VSO_TILE_CASE_UP(PR, KSV, SV, THV, TWV, BMV)                                           \
  if (t.up && t.ks == KSV && t.s == SV && t.th == THV && t.tw == TWV && t.bm == BMV) {          \
    launch_items(k_conv_tile_up<PR, KSV, SV, THV, TWV, BMV>, p, items, s);                      \
  } else
  VSO_TILE_SHAPES(VSO_TILE_CASE, VSO_CONV_PREC, 16) VSO_TILE_SHAPES(VSO_TILE_CASE, VSO_CONV_PREC, 32)
  VSO_TILE_SHAPES(VSO_TILE_CASE, VSO_CONV_PREC, 64)
#if VSO_CONV_PREC != 0  // the fused upsample: 16-bit operands, stride 1
  VSO_TILE_SHAPES_S1(VSO_TILE_CASE_UP, VSO_CONV_PREC, 3, 16) VSO_TILE_SHAPES_S1(VSO_TILE_CASE_UP, VSO_CONV_PREC, 3, 32)
  VSO_TILE_SHAPES_S1(VSO_TILE_CASE_UP, VSO_CONV_PREC, 3, 64) VSO_TILE_SHAPES_S1(VSO_TILE_CASE_UP, VSO_CONV_PREC, 5, 16)
  VSO_TILE_SHAPES_S1(VSO_TILE_CASE_UP, VSO_CONV_PREC, 5, 32) VSO_TILE_SHAPES_S1(VSO_TILE_CASE_UP, VSO_CONV_PREC, 5, 64)
#endif
  {
    std::fprintf(stderr, "vso: no k_conv_tile instance for %s\n", conv_tile_name(t));
  }
#undef VSO_TILE_CASE
#undef VSO_TILE_CASE_UP
}
#endif

#ifdef VSO_CONV_DISPATCH
bool conv_tile_shape(const ConvParams& c, int prec, ConvTileShape* sh) {
  if (prec < PREC_F32 || prec > PREC_F16) return false;
  if (c.G != 1 || c.kh != c.kw || c.dh != 1 || c.dw != 1 || c.sh != c.sw || c.pre.w) return false;
  const int ks = c.kh, s = c.sh;
  if (!((s == 1 && (ks == 1 || ks == 3 || ks == 5)) || (s == 2 && ks == 3))) return false;
  // 1x1: a plain GEMM with K = C, faster on k_conv_small's LDS-free 16x16
  // wave tiles in f32 than here in any precision (measured: MODNet's 1x1
  // layers 240 us per frame there, 630 here in f32 and 16-bit alike)
  if (ks == 1) return false;
  // k_conv_tile stages through a buffer descriptor (num_records = C*H*W*4
  // bytes, 32-bit offsets, out-of-range marker 0x80000000) and its epilogue
  // offsets are int: an image of 2 GiB or more keeps the 64-bit kernels
  // (k_conv_gemm / k_conv_small), as pw_kernel and thin_conv_fits do
  if ((long)c.C * c.H * c.W * 4 >= (1L << 31) || (long)c.M * c.Ho * c.Wo >= (1L << 31)) return false;
  ConvTileShape t{};
  t.up = sh->up;  // (input: the k_conv_tile_up shape is wanted)
  t.prec = prec;
  t.ks = ks;
  t.s = s;
  // 32-channel tiles for 16-bit 5x5: their 25 taps' weights then fit LDS
  // (k_conv_tile's WL) instead of 25 exposed L2 round trips per chunk
  // (16-channel tiles for M <= 16: MODNet's 35 -> 16 fusion layer at 288x512
  // ran half its MFMAs and weight traffic on padding in a 32-channel tile)
  // (VSO_CONV_BM_MAX=32: an A/B knob — 64-channel tiles take up to 300 VGPRs)
  static const int bm_max = [] {
    const char* e = std::getenv("VSO_CONV_BM_MAX");
    return e ? std::atoi(e) : 64;
  }();
  t.bm = c.M <= 16 ? 16 : (c.M <= 32 || bm_max <= 32 || (ks == 5 && prec != PREC_F32)) ? 32 : 64;
  t.Mp = (c.M + t.bm - 1) / t.bm * t.bm;
  t.Cp = (c.C + CK - 1) / CK * CK;
  // candidate tiles, largest first: the first giving >= kWant workgroups wins,
  // else the smallest
  static const int s1w[][2] = {{8, 32}, {4, 32}, {2, 32}}, s1n[][2] = {{16, 16}, {4, 16}};
  static const int s2w[][2] = {{2, 32}}, s2n[][2] = {{4, 16}};
  const int(*cand)[2];
  int nc;
  if (s == 1) { cand = c.Wo >= 32 ? s1w : s1n; nc = c.Wo >= 32 ? 3 : 2; }
  else { cand = c.Wo >= 32 ? s2w : s2n; nc = 1; }
  // ~4 workgroups per CU (VSO_CONV_WANT: an A/B knob)
  static const long kWant = [] {
    const char* e = std::getenv("VSO_CONV_WANT");
    return e ? std::atol(e) : 1024L;
  }();
  // With 16-bit operands the tile height is capped at 2 rows
  // (VSO_CONV_MAX_TH; 0 = no cap): the 8x32 / 4x32 tiles' 180-300 VGPRs leave
  // one or two workgroups per CU, and the 2x32 tiles measured faster overall
  // despite twice the halo rows — MODNet batch 8 bf16 2.054-2.057 against
  // 2.070-2.072 ms, two interleaved rounds (profiles/r04l/); a cap of 4
  // measured 2.08, 32-channel tiles for the 64-channel layers
  // (VSO_CONV_BM_MAX=32) 2.10-2.11.  f32 operands keep the uncapped choice
  // (their 2x32 tiles measured 4.45 against 4.08 ms, profiles/r04m/).
  static const int max_th_env = [] {
    const char* e = std::getenv("VSO_CONV_MAX_TH");
    return e ? std::atoi(e) : -1;
  }();
  // k_conv_tile_up keeps the uncapped choice: a taller tile interpolates each
  // staged source region for more pixels (MODNet's 35 -> 16 layer at 288x512:
  // 146 us at 2 x 32, 113 at 8 x 32; the 64 -> 32 at 144x256: 59.7 -> 49.1)
  // (64-channel upsample tiles, VSO_UP_BM64: capped like the plain 16-bit
  // ones — 8 x 32 x 64 ran at 319 VGPRs, one wave per SIMD: 99 us against the
  // 2 x 32 x 64 tile's 50, profiles/r05x r05ao)
  static const int up_max_th = [] {  // (A/B knob: a height cap for the upsample tiles too)
    const char* e = std::getenv("VSO_UP_MAX_TH");
    return e ? std::atoi(e) : 0;
  }();
  const int max_th = (t.up && t.bm <= 32) ? up_max_th : max_th_env >= 0 ? max_th_env : (prec == PREC_F32 ? 0 : 2);
  long wgs = 0;
  for (int k = 0; k < nc; ++k) {
    if (max_th > 0 && cand[k][0] > max_th && k + 1 < nc) continue;
    t.th = cand[k][0];
    t.tw = cand[k][1];
    t.tiles_x = (c.Wo + t.tw - 1) / t.tw;
    t.tiles = t.tiles_x * ((c.Ho + t.th - 1) / t.th);
    wgs = (long)t.tiles * (t.Mp / t.bm) * c.N;
    if (wgs >= kWant) break;
  }
  const int nch = t.Cp / CK;
  // a deep 16-bit 5x5 on few pixels (MODNet's LR 1280 -> 96 at /16) is split
  // over K anyway: there a 4 x 32 tile (two 16-pixel blocks per wave: 4 LDS
  // fragment reads per 4 MFMAs instead of 3 per 2) with more splits keeps the
  // workgroup count and feeds the MFMAs better: batch 8, 102.4 -> 78.6 us,
  // MFMA busy 14.8 % (VSO_CONV_DEEP_TILE=0: off; 2: 8 x 32 tiles)
  static const int deep_tile = [] {
    const char* e = std::getenv("VSO_CONV_DEEP_TILE");
    return e ? std::atoi(e) : 1;
  }();
  if (deep_tile > 0 && ks == 5 && s == 1 && prec != PREC_F32 && c.Wo >= 32 && wgs < kWant / 2 && nch >= 16 &&
      t.th == 2) {
    t.th = deep_tile == 2 ? 8 : 4;
    t.tw = 32;
    t.tiles_x = (c.Wo + t.tw - 1) / t.tw;
    t.tiles = t.tiles_x * ((c.Ho + t.th - 1) / t.th);
    wgs = (long)t.tiles * (t.Mp / t.bm) * c.N;
  }
  t.ksplit = 1;
  t.cps = nch;
  if (wgs < kWant / 2 && nch > 1) {
    int k = (int)std::min<long>(nch, (kWant + wgs - 1) / wgs);
    if (k > 8) k = k / 8 * 8;  // a multiple of 8: one XCD per split residue (the grid order above)
    t.cps = (nch + k - 1) / k;
    t.ksplit = (nch + t.cps - 1) / t.cps;
  }
  *sh = t;
  return true;
}

void launch_conv_tile(const ConvTileParams& p, const ConvTileShape& t, hipStream_t s) {
  if (t.prec == PREC_F32) launch_conv_tile_prec<PREC_F32>(p, t, s);
  else if (t.prec == PREC_BF16) launch_conv_tile_prec<PREC_BF16>(p, t, s);
  else launch_conv_tile_prec<PREC_F16>(p, t, s);
}
#endif

#ifdef VSO_CONV_DISPATCH
const char* conv_tile_name(const ConvTileShape& t) {
  static thread_local char buf[128];
  std::snprintf(buf, sizeof buf, "void vso::k_conv_tile%s<%d, %d, %d, %d, %d, %d>(vso::ConvTileParams)",
                t.up ? "_up" : "", t.prec, t.ks, t.s, t.th, t.tw, t.bm);
  return buf;
}
#endif

}  // namespace vso
