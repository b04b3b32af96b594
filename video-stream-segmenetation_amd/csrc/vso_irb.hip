// vso_irb.hip — a MobileNetV2 inverted-residual block of an ONNX session in
// one launch (the backbone of MODNet, model.ts:12-29: 16 such blocks):
//
//   x [N][Cin][H][W] -> Conv 1x1 Cin -> Ch (+ bias, Relu / Clip)
//                    -> depthwise 3x3, stride S, pad 1 (+ bias, Relu / Clip)
//                    -> Conv 1x1 Ch -> Cout (+ bias) [+ x]  -> y
//
// Unfused, the expanded tensor (Ch = 6 Cin channels) makes an HBM round trip
// between two or three launches.  Here a workgroup owns TH x 16 output pixels
// of one image:
//   * its input tile with the depthwise halo ((TH-1)S+3) x (15S+3) pixels x
//     Cin channels is staged once into LDS, channel-major ([Cin][NP], NP = 16 mod
//     32 so the expand MFMA's B reads of 16 pixels x 4 channels hit 32 banks);
//   * per 16 hidden channels (a chunk): the four waves compute the expand for
//     the tile's pixel blocks on v_mfma_f32_16x16x4_f32 (A = weights from
//     global / L1, B = the LDS tile) into an LDS chunk [16][NP] (zero outside
//     the image: the depthwise padding), then the depthwise 3x3 of the chunk
//     for the output pixels into LDS [16][TH*16], then each wave accumulates
//     the project 1x1 for its output-channel blocks in registers;
//   * the hidden chunks may be split over ksplit workgroups when the grid is
//     small (the low-resolution blocks: 10 tiles at 18x32): each writes its
//     partial project tile write-through, and the last to arrive sums them in
//     split order and runs the epilogue (bias, residual) — vso_conv.hip's
//     hand-off, no fences.
// Exact f32 products, f32 accumulation (the session's f32 semantics).
//
// Opt-in (env VSO_IRB=1 at vso_create): measured slower than the unfused
// launches on MODNet 288x512 (bf16 session, batch 1: 1.22 vs 0.95 ms per
// frame; batch 8: 0.49 vs 0.40 ms).  A workgroup's latency chain — staging,
// two barriers per 16-channel chunk, the split hand-off's write-through
// round trips — outweighs the expanded tensor's HBM round trip, which at
// these sizes is only a few MB; per-wave independent chunks (vss's k_block
// layout) would be the next design to try.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>

#include "vso_device.h"
#include "vso_kernels.h"

namespace vso {

__device__ __forceinline__ float irb_act(float v, int act, float lo, float hi) {
  if (act == ACT_RELU) return fmaxf(v, 0.f);
  if (act == ACT_CLIP) return fminf(fmaxf(v, lo), hi);
  return v;
}

template <int S, int TH, int CBW>
__global__ __launch_bounds__(256) void k_irb(IrbParams p) {
  constexpr int TW = 16, P_OUT = TH * TW, NPB = TH;
  constexpr int IH = (TH - 1) * S + 3, IW = (TW - 1) * S + 3, NPIX = IH * IW;
  constexpr int NP = irb_np(S, TH);
  extern __shared__ float lds[];
  float* xt = lds;                       // [Cin][NP]
  float* hid = xt + (size_t)p.Cin * NP;  // [16][NP]
  float* dwo = hid + 16 * NP;            // [16][P_OUT]
  float* wts = dwo + 16 * P_OUT;         // per chunk of the split: irb_chunk_floats(Cin, Cout)
  const int W1S = p.Cin + 1;             // w1 row stride (odd: the A reads of 16 rows spread over banks)
  const int CF = irb_chunk_floats(p.Cin, p.Cout);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int L = blockIdx.x;
  const int kz = L % p.ksplit, rest = L / p.ksplit;
  const int t = rest % p.tiles, n = rest / p.tiles;
  const int oy0 = (t / p.tiles_x) * TH, ox0 = (t % p.tiles_x) * TW;
  const int iy0 = oy0 * S - 1, ix0 = ox0 * S - 1;
  const float* xn = p.x + (long)n * p.Cin * p.H * p.W;

  // the input tile (zeros outside the image and in the pixel padding), 8
  // loads per thread in flight at a time (a load-then-store loop would wait
  // out each global load's latency in turn: 70 of them for 160 channels)
  {
    const int total = p.Cin * NP;
    for (int base = 0; base < total; base += 256 * 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int idx = base + tid + 256 * u;
        const int c = idx / NP, pix = idx - c * NP;
        const int iy = pix / IW, ix = pix - (pix / IW) * IW;
        const int gy = iy0 + iy, gx = ix0 + ix;
        const bool in = idx < total && pix < NPIX && gy >= 0 && gy < p.H && gx >= 0 && gx < p.W;
        v[u] = in ? xn[((long)c * p.H + gy) * p.W + gx] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int idx = base + tid + 256 * u;
        if (idx < total) xt[idx] = v[u];
      }
    }
  }
  __syncthreads();

  const int nchunk = p.Ch / 16;
  const int cbeg = kz * p.cps, cend = min(nchunk, cbeg + p.cps);
  // every weight this workgroup's chunks use, staged once (8 loads in flight
  // per thread): per chunk w1 [16][Cin+1], wd [16][9], b1 [16], bd [16],
  // w2 [Cout][17] (its 16 columns of the project) — the chunk loop below then
  // reads only LDS
  {
    const int nck = cend - cbeg, total = nck * CF;
    for (int base = 0; base < total; base += 256 * 8) {
      float v[8];
      int dst[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int idx = base + tid + 256 * u;
        dst[u] = -1;
        v[u] = 0.f;
        if (idx < total) {
          const int ck = idx / CF, o = idx - ck * CF;
          const int h0 = (cbeg + ck) * 16;
          dst[u] = ck * CF + o;
          if (o < 16 * p.Cin) {
            const int rr = o / p.Cin, k = o - rr * p.Cin;
            v[u] = p.w1[(long)(h0 + rr) * p.Cin + k];
            dst[u] = ck * CF + rr * W1S + k;
          } else if (o < 16 * W1S) {
            dst[u] = -1;  // the pad column
          } else if (o < 16 * W1S + 144) {
            const int q = o - 16 * W1S;
            v[u] = p.wd[(long)h0 * 9 + q];
          } else if (o < 16 * W1S + 160) {
            v[u] = p.b1[h0 + o - 16 * W1S - 144];
          } else if (o < 16 * W1S + 176) {
            v[u] = p.bd[h0 + o - 16 * W1S - 160];
          } else {
            const int q = o - 16 * W1S - 176, co = q / 17, kk = q - co * 17;
            v[u] = kk < 16 ? p.w2[(long)co * p.Ch + h0 + kk] : 0.f;
          }
        }
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (dst[u] >= 0) wts[dst[u]] = v[u];
    }
  }
  __syncthreads();
  const int cob = (p.Cout + 15) / 16;  // output-channel blocks; wave w takes w, w + 4, ...
  f4 acc[CBW][NPB];
#pragma unroll
  for (int i = 0; i < CBW; ++i)
#pragma unroll
    for (int j = 0; j < NPB; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

  for (int hc = cbeg; hc < cend; ++hc) {
    const float* wc = wts + (hc - cbeg) * CF;
    const float* wdc = wc + 16 * W1S;
    const float* b1c = wdc + 144;
    const float* bdc = b1c + 16;
    const float* w2c = bdc + 16;
    // ---- expand: 16 hidden channels x the tile's NP / 16 pixel blocks ----
    const float* w1 = wc + r * W1S;
    for (int pb = wave; pb < NP / 16; pb += 4) {
      f4 e = f4{0.f, 0.f, 0.f, 0.f};
      for (int k0 = 0; k0 < p.Cin; k0 += 32) {
        float a[8], b[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int k = k0 + 4 * u + g;
          const bool in = k < p.Cin;
          a[u] = in ? w1[k] : 0.f;
          b[u] = in ? xt[k * NP + pb * 16 + r] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (k0 + 4 * u < p.Cin) e = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u], b[u], e, 0, 0, 0);
      }
      // e[v] = hidden channel h0 + 4g + v at pixel pb*16 + r
      const int pix = pb * 16 + r;
      const int iy = pix / IW, ix = pix - (pix / IW) * IW;
      const int gy = iy0 + iy, gx = ix0 + ix;
      const bool inside = pix < NPIX && gy >= 0 && gy < p.H && gx >= 0 && gx < p.W;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        hid[(4 * g + v) * NP + pix] = inside ? irb_act(e[v] + b1c[4 * g + v], p.act1, p.lo1, p.hi1) : 0.f;
      }
    }
    __syncthreads();
    // ---- depthwise 3x3 of the chunk for the output pixels ----
    for (int o = tid; o < 16 * P_OUT; o += 256) {
      const int ch = o / P_OUT, px = o - ch * P_OUT;
      const int oy = px / TW, ox = px - oy * TW;
      const float* hb = hid + ch * NP + (oy * S) * IW + ox * S;
      const float* wd = wdc + ch * 9;
      float s = bdc[ch];
#pragma unroll
      for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) s = __builtin_fmaf(wd[ky * 3 + kx], hb[ky * IW + kx], s);
      dwo[ch * P_OUT + px] = irb_act(s, p.act2, p.lo2, p.hi2);
    }
    __syncthreads();
    // ---- project: this wave's output-channel blocks += W2[:, chunk] x dwo ----
#pragma unroll
    for (int i = 0; i < CBW; ++i) {
      const int cb = wave + 4 * i;
      if (cb >= cob) break;
      const int co = cb * 16 + r;
      const float* w2 = w2c + (co < p.Cout ? co : 0) * 17;
      float a[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) a[s] = co < p.Cout ? w2[4 * s + g] : 0.f;
#pragma unroll
      for (int j = 0; j < NPB; ++j)
#pragma unroll
        for (int s = 0; s < 4; ++s)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], dwo[(4 * s + g) * P_OUT + j * 16 + r], acc[i][j], 0,
                                                           0, 0);
    }
    // the next chunk's expand overwrites hid only: dw of this chunk is done
    // (barrier above); its dw overwrites dwo after the next barrier, which every
    // wave reaches only after this project
  }

  if (p.ksplit > 1) {  // vso_conv.hip's hand-off: write-through partials, last arrival sums in split order
    const long blk = (long)n * p.tiles + t;
    constexpr int PER = CBW * NPB * 256 * 2;  // 8-byte words per partial tile
    uint64_t* part = reinterpret_cast<uint64_t*>(p.part) + (blk * p.ksplit + kz) * PER;
#pragma unroll
    for (int i = 0; i < CBW; ++i)
#pragma unroll
      for (int j = 0; j < NPB; ++j) {
        const uint64_t lo = (uint64_t)__float_as_uint(acc[i][j][0]) | ((uint64_t)__float_as_uint(acc[i][j][1]) << 32);
        const uint64_t hi = (uint64_t)__float_as_uint(acc[i][j][2]) | ((uint64_t)__float_as_uint(acc[i][j][3]) << 32);
        uint64_t* q = part + ((i * NPB + j) * 256 + tid) * 2;
        __hip_atomic_store(q, lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(q + 1, hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __shared__ int last;
    __syncthreads();
    if (tid == 0) {
      int* cnt = p.counters + blk;
      const int prev = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last = prev == p.ksplit - 1;
      if (last) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (!last) return;
    const uint64_t* base = reinterpret_cast<const uint64_t*>(p.part) + blk * p.ksplit * PER;
#pragma unroll
    for (int i = 0; i < CBW; ++i)
#pragma unroll
      for (int j = 0; j < NPB; ++j) {
        f4 sum = f4{0.f, 0.f, 0.f, 0.f};
        for (int k0 = 0; k0 < p.ksplit; k0 += 8) {
          uint64_t lo[8], hi[8];
#pragma unroll
          for (int u = 0; u < 8; ++u)
            if (k0 + u < p.ksplit) {
              const uint64_t* q = base + (long)(k0 + u) * PER + ((i * NPB + j) * 256 + tid) * 2;
              lo[u] = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              hi[u] = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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

  // epilogue: acc[i][j][v] = output channel (wave + 4i)*16 + 4g + v, pixel (oy0 + j, ox0 + r)
#pragma unroll
  for (int i = 0; i < CBW; ++i) {
    const int cb = wave + 4 * i;
    if (cb >= cob) break;
#pragma unroll
    for (int j = 0; j < NPB; ++j) {
      const int oy = oy0 + j, ox = ox0 + r;
      if (oy >= p.Ho || ox >= p.Wo) continue;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int co = cb * 16 + 4 * g + v;
        if (co >= p.Cout) continue;
        float y = acc[i][j][v] + p.b2[co];
        if (p.res) y += xn[((long)co * p.H + oy) * p.W + ox];
        p.y[(((long)n * p.Cout + co) * p.Ho + oy) * p.Wo + ox] = y;
      }
    }
  }
}

// ---- planning and dispatch ------------------------------------------------
bool irb_shape(int N, int Cin, int Ch, int Cout, int Ho, int Wo, int S, IrbShape* sh) {
  if (S != 1 && S != 2) return false;
  if (Cin % 4 || Ch % 16 || Cout > 16 * 4 * 3) return false;
  IrbShape t{};
  t.s = S;
  t.th = S == 1 ? 4 : 2;
  t.cbw = (((Cout + 15) / 16) + 3) / 4;
  if (t.cbw < 1) t.cbw = 1;
  const size_t fixed = ((size_t)Cin * irb_np(S, t.th) + 16 * irb_np(S, t.th) + 16 * t.th * 16) * 4;
  const size_t per_chunk = (size_t)irb_chunk_floats(Cin, Cout) * 4;
  constexpr size_t kLdsMax = 128 * 1024;
  if (fixed + per_chunk > kLdsMax) return false;
  t.tiles_x = (Wo + 15) / 16;
  t.tiles = t.tiles_x * ((Ho + t.th - 1) / t.th);
  const long base = (long)t.tiles * N;
  const int nch = Ch / 16;
  // chunks per workgroup: enough workgroups to fill the chip, and the chunks'
  // weights within the LDS budget
  const int fit = (int)((kLdsMax - fixed) / per_chunk);
  int k = 1;
  if (base < 512 && nch > 1) {
    k = (int)std::min<long>(nch, (1024 + base - 1) / base);
    if (k > 8) k = k / 8 * 8;
  }
  t.cps = (nch + k - 1) / k;
  if (t.cps > fit) t.cps = fit;
  t.ksplit = (nch + t.cps - 1) / t.cps;
  t.lds = fixed + (size_t)t.cps * per_chunk;
  *sh = t;
  return true;
}

const char* irb_name(const IrbShape& t) {
  static thread_local char buf[96];
  std::snprintf(buf, sizeof buf, "void vso::k_irb<%d, %d, %d>(vso::IrbParams)", t.s, t.th, t.cbw);
  return buf;
}

void launch_irb(const IrbParams& p, const IrbShape& t, hipStream_t s) {
  const dim3 grid((unsigned)((long)t.tiles * p.N * t.ksplit));
#define VSO_IRB(SV, THV, CBWV)                                                                     \
  if (t.s == SV && t.th == THV && t.cbw == CBWV) {                                                 \
    hipLaunchKernelGGL((k_irb<SV, THV, CBWV>), grid, dim3(256), t.lds, s, p);                      \
    return;                                                                                        \
  }
  VSO_IRB(1, 4, 1) VSO_IRB(1, 4, 2) VSO_IRB(1, 4, 3) VSO_IRB(2, 2, 1) VSO_IRB(2, 2, 2) VSO_IRB(2, 2, 3)
#undef VSO_IRB
  std::fprintf(stderr, "vso: no k_irb instance for %s\n", irb_name(t));
}

bool irb_set_lds_limit() {
  // dynamic LDS beyond 64 KiB must be allowed per kernel
  const void* fns[] = {(const void*)k_irb<1, 4, 1>, (const void*)k_irb<1, 4, 2>, (const void*)k_irb<1, 4, 3>,
                       (const void*)k_irb<2, 2, 1>, (const void*)k_irb<2, 2, 2>, (const void*)k_irb<2, 2, 3>};
  for (const void* f : fns)
    if (hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024) != hipSuccess) return false;
  return true;
}

}  // namespace vso
