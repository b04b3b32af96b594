// vso_kernels.hip — gfx950 kernels of the ONNX sessions (include/vso.h):
// the operators of the reference's ORT models (MODNet, MediaPipe face
// detector and landmarks; client/src/core/model.ts) on float32 NCHW tensors.
//
//   k_conv_gemm : dense / grouped convolution as an implicit GEMM per (image,
//                 group): D[m][p] = sum_k W[m][k] * X^[k][p], k = (c, ky, kx),
//                 p = output pixel; 64x64 output tile per workgroup, K in
//                 steps of 16 staged through LDS (the im2col gather happens in
//                 the staging loads, never in HBM; the next step's loads are in
//                 flight while the current one computes), four wave64s each
//                 running 16 rows x 64 columns on v_mfma_f32_16x16x4_f32;
//                 bias, residual and activation fused into the epilogue.
//   k_conv_dw   : depthwise convolution (groups == channels), direct.
//   the rest    : broadcast binary ops, unary activations, one strided
//                 gather-copy for Transpose / Slice / Split / Concat / Pad,
//                 pooling, per-row reductions (GlobalAveragePool,
//                 InstanceNormalization, Softmax), channel affine
//                 (BatchNormalization), Resize and a small batched GEMM.
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include "vso_device.h"
#include "vso_kernels.h"

namespace vso {

// ---------------------------------------------------------------------------
constexpr int BM = 64, BP = 64, BK = 16;

__global__ __launch_bounds__(256) void k_conv_gemm(ConvParams p) {
  __shared__ float As[BM][BK + 1];
  __shared__ float Bs[BK][BP + 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 15, g4 = lane >> 4;
  const int P = p.Ho * p.Wo;
  const int p0 = blockIdx.x * BP, m0 = blockIdx.y * BM;
  const int n = blockIdx.z / p.G, grp = blockIdx.z % p.G;
  const int khw = p.kh * p.kw;
  const int K = p.Cg * khw;
  const float* xg = p.x + ((long)n * p.C + (long)grp * p.Cg) * p.H * p.W;
  const float* wg = p.w + (long)grp * p.Mg * K;
  float ra[4], rb[4];
  auto load = [&](int k0) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int idx = tid + 256 * u;
      {  // A: weights, row m (output channel), 16 consecutive k
        const int m = idx >> 4, kk = idx & 15;
        const int gm = m0 + m, k = k0 + kk;
        ra[u] = (gm < p.Mg && k < K) ? wg[(long)gm * K + k] : 0.f;
      }
      {  // B: the im2col element (k, pixel), gathered from the input
        const int kk = idx >> 6, pp = idx & 63;
        const int k = k0 + kk, pix = p0 + pp;
        float v = 0.f;
        if (k < K && pix < P) {
          const int c = k / khw, rem = k - c * khw;
          const int ky = rem / p.kw, kx = rem - ky * p.kw;
          const int oy = pix / p.Wo, ox = pix - oy * p.Wo;
          const int iy = oy * p.sh - p.pt + ky * p.dh, ix = ox * p.sw - p.pl + kx * p.dw;
          if (iy >= 0 && iy < p.H && ix >= 0 && ix < p.W) v = xg[((long)c * p.H + iy) * p.W + ix];
        }
        rb[u] = v;
      }
    }
  };
  f4 acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = f4{0.f, 0.f, 0.f, 0.f};
  load(0);
  for (int k0 = 0; k0 < K; k0 += BK) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int idx = tid + 256 * u;
      As[idx >> 4][idx & 15] = ra[u];
      Bs[idx >> 6][idx & 63] = rb[u];
    }
    __syncthreads();
    if (k0 + BK < K) load(k0 + BK);  // next step's loads in flight during this step's MFMAs
#pragma unroll
    for (int s = 0; s < BK / 4; ++s) {
      const float a = As[16 * wave + r][4 * s + g4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, Bs[4 * s + g4][16 * j + r], acc[j], 0, 0, 0);
    }
    __syncthreads();
  }
  // acc[j][v] = D[row 16*wave + 4*g4 + v][column 16*j + r]
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    const int gm = m0 + 16 * wave + 4 * g4 + v;
    if (gm >= p.Mg) continue;
    const int ch = grp * p.Mg + gm;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int pix = p0 + 16 * j + r;
      if (pix < P) {
        const long o = ((long)n * p.M + ch) * P + pix;
        p.y[o + n * p.y_nx] = epilogue(p.ep, acc[j][v], ch, o, n, pix);
      }
    }
  }
}

// Depthwise -> 1x1 pair in one launch (the face models' 32 / 20 dw layers each
// paid a whole launch, ~4.6 us, for a few MFLOP).  A workgroup owns 16 output
// pixels and 64 output channels: its 256 threads first compute the depthwise
// outputs of those pixels for all C channels into LDS (k_conv_dw's arithmetic:
// the same floats), then each wave runs one 16x16 MFMA tile of the 1x1 over
// them (A = weights from global / L1, B = the LDS tile), in k order as
// k_conv_small does.  Only the final output reaches HBM.
__global__ __launch_bounds__(256) void k_conv_dwpw(ConvParams p) {
  __shared__ float bs[kDwPwMaxC][17];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int P = p.Ho * p.Wo, K = p.C;
  const int tp = blockIdx.x, n = blockIdx.z;
  const DwPre& q = p.pre;
  // phase 1: depthwise outputs of pixels 16 tp .. 16 tp + 15, channels 0 .. K-1.
  // 3x3: four outputs per thread per pass, all 36 taps' loads issued together
  // (an absent tap loads nothing and adds 0: the value of k_conv_dw's skip,
  // up to the sign of a zero)
  if (q.kh == 3 && q.kw == 3) {
    for (int e0 = tid; e0 < K * 16; e0 += 1024) {
      float t[4][9], wv[4][9];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int e = e0 + 256 * u, c = min(e >> 4, K - 1), pix = tp * 16 + (e & 15);
        const int oy = pix / p.Wo, ox = pix - oy * p.Wo;
        const float* xc = p.x + ((long)n * K + c) * q.H * q.W;
#pragma unroll
        for (int k = 0; k < 9; ++k) {
          const int iy = oy * q.sh - q.pt + (k / 3) * q.dh, ix = ox * q.sw - q.pl + (k % 3) * q.dw;
          const bool in = e < K * 16 && pix < P && iy >= 0 && iy < q.H && ix >= 0 && ix < q.W;
          t[u][k] = in ? xc[(long)iy * q.W + ix] : 0.f;
          wv[u][k] = q.w[(long)c * 9 + k];
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int e = e0 + 256 * u;
        if (e >= K * 16) break;
        const int c = e >> 4, pl = e & 15, pix = tp * 16 + pl;
        float acc = 0.f;
#pragma unroll
        for (int k = 0; k < 9; ++k) acc = __builtin_fmaf(wv[u][k], t[u][k], acc);
        bs[c][pl] = pix < P ? epilogue(q.ep, acc, c, 0, n, pix) : 0.f;
      }
    }
  } else {
    for (int e = tid; e < K * 16; e += 256) {
      const int c = e >> 4, pl = e & 15, pix = tp * 16 + pl;
      float v = 0.f;
      if (pix < P) {
        const int oy = pix / p.Wo, ox = pix - oy * p.Wo;
        const float* xc = p.x + ((long)n * K + c) * q.H * q.W;
        const float* wc = q.w + (long)c * q.kh * q.kw;
        float acc = 0.f;
        for (int ky = 0; ky < q.kh; ++ky) {
          const int iy = oy * q.sh - q.pt + ky * q.dh;
          if (iy < 0 || iy >= q.H) continue;
          for (int kx = 0; kx < q.kw; ++kx) {
            const int ix = ox * q.sw - q.pl + kx * q.dw;
            if (ix >= 0 && ix < q.W) acc = __builtin_fmaf(wc[ky * q.kw + kx], xc[(long)iy * q.W + ix], acc);
          }
        }
        v = epilogue(q.ep, acc, c, 0, n, pix);
      }
      bs[c][pl] = v;
    }
  }
  __syncthreads();
  // phase 2: this wave's 16 output channels x the 16 pixels
  const int m0 = blockIdx.y * 64 + wave * 16;
  if (m0 >= p.M) return;
  const int m = m0 + r;
  const bool m_ok = m < p.M;
  const float* wrow = p.w + (long)(m_ok ? m : 0) * K;
  f4 acc = f4{0.f, 0.f, 0.f, 0.f};
  constexpr int CH = 8;
  if ((K & 15) == 0 && (reinterpret_cast<uintptr_t>(p.w) & 15) == 0) {
    // as k_conv_small: MFMA 4t + e takes k = k0 + 16 t + 4 g + e, a lane's
    // four weights of MFMAs 4t .. 4t+3 one float4 (K % 16 == 0: every MFMA full)
    for (int k0 = 0; k0 < K; k0 += 4 * CH) {
      f4 a4[CH / 4];
#pragma unroll
      for (int t = 0; t < CH / 4; ++t) {
        const int kb = k0 + 16 * t + 4 * g;
        a4[t] = (m_ok && kb < K) ? *reinterpret_cast<const f4*>(wrow + kb) : f4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int t = 0; t < CH / 4; ++t)
        if (k0 + 16 * t < K)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[t][e], bs[k0 + 16 * t + 4 * g + e][r], acc, 0, 0, 0);
    }
  } else {
    for (int k0 = 0; k0 < K; k0 += 4 * CH) {
      float a[CH];
#pragma unroll
      for (int s = 0; s < CH; ++s) {
        const int k = k0 + 4 * s + g;
        a[s] = (m_ok && k < K) ? wrow[k] : 0.f;
      }
#pragma unroll
      for (int s = 0; s < CH; ++s) {
        const int k = k0 + 4 * s + g;
        if (k0 + 4 * s < K) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], k < K ? bs[k][r] : 0.f, acc, 0, 0, 0);
      }
    }
  }
  const int pix = tp * 16 + r;
  if (pix >= P) return;
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    const int ch = m0 + 4 * g + v;
    if (ch >= p.M) continue;
    const long o = ((long)n * p.M + ch) * P + pix;
    p.y[o + n * p.y_nx] = epilogue(p.ep, acc[v], ch, o, n, pix);
  }
}

// Small convolutions (few 64x64 tiles: the deep layers of the face models ran
// 8-22 workgroups of k_conv_gemm, each walking its K serially through LDS —
// latency bound at 13-36 us).  Here a 16 (output channels) x 16 (output
// pixels) tile reads its A / B operands straight from global memory into
// registers (lane (r, g) supplies W[m r][k 4s+g] and the im2col element
// X^[k 4s+g][pixel r]; 16 consecutive pixels per k are one coalesced 64-B
// read) and runs v_mfma_f32_16x16x4f32 on them: CH MFMAs per chunk, all of a
// chunk's loads in flight together and the next chunk's issued before this
// one's MFMAs.  No LDS, no barriers, 4-16x the workgroups of k_conv_gemm.
//   SPLIT = false: one wave per tile, the wave walks all of K;
//   SPLIT = true : one workgroup per tile, its four waves take a quarter of K
//                  each and reduce through LDS (K > 128: a quarter of the
//                  serial load latency).
// PW: 1x1 stride-1 unpadded (the im2col element is X[k][pixel]).
template <bool PW, int CH, bool SPLIT>
__global__ __launch_bounds__(256) void k_conv_small(ConvParams p, int tiles_m, int tiles_p) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long tile = SPLIT ? (long)blockIdx.x : (long)blockIdx.x * 4 + wave;
  const long per_img = (long)tiles_m * tiles_p;
  if (tile >= per_img * p.N * p.G) return;  // SPLIT: uniform per workgroup
  const int ng = (int)(tile / per_img);
  const int rem = (int)(tile - (long)ng * per_img);
  const int tm = rem / tiles_p, tp = rem - tm * tiles_p;  // neighbouring tiles: same weights
  const int n = ng / p.G, grp = ng - n * p.G;
  const int r = lane & 15, g = lane >> 4;
  const int P = p.Ho * p.Wo;
  const int khw = p.kh * p.kw;
  const int K = p.Cg * khw;
  // this wave's K range
  const int kq = SPLIT ? ((K + 15) / 16) * 4 : K;
  const int kbeg = SPLIT ? wave * kq : 0;
  const int kend = SPLIT ? min(K, kbeg + kq) : K;
  const float* xg = p.x + ((long)n * p.C + (long)grp * p.Cg) * p.H * p.W;
  const int m = tm * 16 + r, pix = tp * 16 + r;
  const bool m_ok = m < p.Mg, pix_ok = pix < P;
  const float* wrow = p.w + ((long)grp * p.Mg + (m_ok ? m : 0)) * K;
  const int oy = pix / p.Wo, ox = pix - oy * p.Wo;
  const int iy0 = oy * p.sh - p.pt, ix0 = ox * p.sw - p.pl;
  // Branch-free: every element is loaded from a valid (clamped) address and
  // selected afterwards — a conditional load compiled to a branch and an exec
  // swap per element.
  const int pixc = pix_ok ? pix : 0;
  auto bval = [&](int k) -> float {
    const bool ok = pix_ok && k < kend;
    const int kc = min(k, K - 1);
    if (PW) {
      const float v = xg[(long)kc * P + pixc];
      return ok ? v : 0.f;
    }
    const int c = kc / khw, rr = kc - c * khw;
    const int ky = rr / p.kw, kx = rr - ky * p.kw;
    const int iy = iy0 + ky * p.dh, ix = ix0 + kx * p.dw;
    const bool in = ok && iy >= 0 && iy < p.H && ix >= 0 && ix < p.W;
    const float v = xg[((long)c * p.H + min(max(iy, 0), p.H - 1)) * p.W + min(max(ix, 0), p.W - 1)];
    return in ? v : 0.f;
  };
  // A operands: with K % 4 == 0 and 16-B aligned weights, MFMA 4t + e of a
  // chunk takes k = k0 + 16 t + 4 g + e, so a lane's four A elements of MFMAs
  // 4t .. 4t+3 are one float4 of its weight row (a quarter of the load
  // instructions); otherwise MFMA s takes k = k0 + 4 s + g, one float each.
  const bool av = (K & 3) == 0 && (reinterpret_cast<uintptr_t>(p.w) & 15) == 0;
  auto kof = [&](int k0, int s) { return av ? k0 + 16 * (s >> 2) + 4 * g + (s & 3) : k0 + 4 * s + g; };
  auto load_chunk = [&](int k0, float* a, float* b) {
    if (av) {
#pragma unroll
      for (int t = 0; t < CH / 4; ++t) {
        const int kb = k0 + 16 * t + 4 * g;  // kend % 4 == 0: all four or none
        const f4 w4l = *reinterpret_cast<const f4*>(wrow + min(kb, K - 4));  // clamped, selected (no branch)
        const f4 w4 = (m_ok && kb < kend) ? w4l : f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int e = 0; e < 4; ++e) a[4 * t + e] = w4[e];
      }
    } else {
#pragma unroll
      for (int s = 0; s < CH; ++s) {
        const int k = kof(k0, s);
        const float wl = wrow[min(k, K - 1)];
        a[s] = (m_ok && k < kend) ? wl : 0.f;
      }
    }
#pragma unroll
    for (int s = 0; s < CH; ++s) b[s] = bval(kof(k0, s));
  };
  float a[CH], b[CH];
  load_chunk(kbeg, a, b);
  f4 acc = f4{0.f, 0.f, 0.f, 0.f};
  for (int k0 = kbeg; k0 < kend; k0 += 4 * CH) {
    const bool more = k0 + 4 * CH < kend;
    float an[CH], bn[CH];
    if (more) load_chunk(k0 + 4 * CH, an, bn);  // the next chunk's loads, in flight during this chunk's MFMAs
#pragma unroll
    for (int s = 0; s < CH; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], b[s], acc, 0, 0, 0);
    if (more) {
#pragma unroll
      for (int s = 0; s < CH; ++s) {
        a[s] = an[s];
        b[s] = bn[s];
      }
    }
  }
  if (SPLIT) {  // sum the four waves' partial tiles (fixed order: deterministic)
    __shared__ f4 part[4][64];
    part[wave][lane] = acc;
    __syncthreads();
    if (wave != 0) return;
    acc = part[0][lane];
#pragma unroll
    for (int w2 = 1; w2 < 4; ++w2) acc += part[w2][lane];
  }
  // acc[v] = D[channel 16 tm + 4g + v][pixel 16 tp + r]
  if (!pix_ok) return;
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    const int gm = tm * 16 + 4 * g + v;
    if (gm >= p.Mg) continue;
    const int ch = grp * p.Mg + gm;
    const long o = ((long)n * p.M + ch) * P + pix;
    p.y[o + n * p.y_nx] = epilogue(p.ep, acc[v], ch, o, n, pix);
  }
}

// 1x1 convolutions (stride 1, unpadded, ungrouped) as one GEMM per image,
// Y[m][p] = sum_k W[m][k] X[k][p], on NCHW f32 with v_mfma_f32_16x16x4_f32
// (exact f32 products, like k_conv_small).  DWK = 3 / 5: X is a depthwise
// DWK x DWK convolution computed on the fly (a fused dw -> 1x1 pair: k_conv_dw's
// arithmetic, taps in ky, kx order, then its bias / activation — an absent tap
// adds w * 0, as k_conv_dwpw did).  A workgroup owns PT = 64 WP pixels x
// BM = 16 WM output channels (WM x WP = 4 waves, WM from the channel count:
// the 16-channel project layers keep every wave busy on pixels); wave (wm, wp)
// computes 16 channels x 64 pixels (4 MFMA blocks).  K runs in chunks of 32
// channels staged through LDS as [k][pixel]: a thread stages one pixel of the
// tile for 32 / (256 / PT) channels — lanes on consecutive pixels, so every
// load is coalesced along the row and its pixel / tap geometry is worked out
// once — and the next chunk's loads are in flight during this chunk's MFMAs.
// Replaces k_conv_dwpw (16 pixels per workgroup: its 18k workgroups at
// 144x256 were launch- and latency-bound, 104 us for a 7 us layer), and
// k_conv_gemm / k_conv_small for the 1x1 convolutions.
template <int WM, int DWK>
__global__ __launch_bounds__(256) void k_conv_pw(ConvParams p) {
  constexpr int WP = 4 / WM, PT = 64 * WP, BM = 16 * WM, KC = 32;
  constexpr int KPT = 256 / PT;       // channels staged per pass (threads per pixel column)
  constexpr int NS = KC / KPT;        // staged elements per thread and chunk
  constexpr int XSTR = PT + 4;        // LDS row stride: rows 4 apart land 16 banks apart
  constexpr int KT = DWK * DWK;       // depthwise taps (0: none)
  __shared__ float xs[KC * XSTR];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 15, g = lane >> 4;
  const int wm = wave % WM, wp = wave / WM;
  const int P = p.Ho * p.Wo, K = p.C;
  const int p0 = blockIdx.x * PT, n = blockIdx.z;
  const int px = tid % PT, kq = tid / PT;  // this thread's staged pixel and its first channel in a chunk
  const int pix = p0 + px;
  const bool pix_ok = pix < P;
  const int pixc = pix_ok ? pix : P - 1;
  const int nch = (K + KC - 1) / KC;
  // the depthwise taps of this pixel: offsets in the input plane, and validity
  int toff[KT > 0 ? KT : 1];
  bool tok[KT > 0 ? KT : 1];
  const DwPre& q = p.pre;
  if constexpr (KT > 0) {
    const int oy = pixc / p.Wo, ox = pixc - oy * p.Wo;
#pragma unroll
    for (int t = 0; t < KT; ++t) {
      const int iy = oy * q.sh - q.pt + (t / DWK) * q.dh, ix = ox * q.sw - q.pl + (t % DWK) * q.dw;
      tok[t] = pix_ok && iy >= 0 && iy < q.H && ix >= 0 && ix < q.W;
      toff[t] = min(max(iy, 0), q.H - 1) * q.W + min(max(ix, 0), q.W - 1);
    }
  }
  const int plane_in = KT > 0 ? q.H * q.W : P;
  const float* xn = p.x + (long)n * K * plane_in;  // image n's input (32-bit offsets below)
  float st[NS];
  auto stage = [&](int ch) {
#pragma unroll
    for (int u = 0; u < NS; ++u) {
      const int k = ch * KC + kq + KPT * u;  // wave-uniform (PT >= 64)
      const int kc = min(k, K - 1);
      if constexpr (KT == 0) {
        const float v = xn[kc * P + pixc];
        st[u] = (k < K && pix_ok) ? v : 0.f;
      } else {
        const int cu = __builtin_amdgcn_readfirstlane(kc);
        const float* xc = xn + cu * plane_in;
        const float* wc = q.w + cu * KT;
        float acc = 0.f;
#pragma unroll
        for (int t = 0; t < KT; ++t) {
          const float v = xc[toff[t]];
          acc = __builtin_fmaf(wc[t], tok[t] ? v : 0.f, acc);
        }
        st[u] = acc;
      }
    }
  };
  // the depthwise epilogue (bias, activation) at commit, then zero for k >= K
  auto commit = [&](int ch) {
    if constexpr (KT > 0) {
#pragma unroll
      for (int u = 0; u < NS; ++u) {
        const int k = min(ch * KC + kq + KPT * u, K - 1);
        if (q.ep.bias) st[u] += q.ep.bias[__builtin_amdgcn_readfirstlane(k)];
      }
      act_block(st, [&](int u) { return ch * KC + kq + KPT * u; }, q.ep);
    }
#pragma unroll
    for (int u = 0; u < NS; ++u) {
      const int k = ch * KC + kq + KPT * u;
      xs[(kq + KPT * u) * XSTR + px] = (k < K && pix_ok) ? st[u] : 0.f;
    }
  };
  // A operands: lane (r, g) of MFMA 4t + e takes W[m][k0 + 16 t + 4 g + e]
  // (as k_conv_small: four consecutive k per lane and t, one float4 when the
  // rows are 16-B aligned), B the same k of pixel r of its block
  const int m = blockIdx.y * BM + wm * 16 + r;
  const bool m_ok = m < p.M;
  const float* wrow = p.w + (long)(m_ok ? m : 0) * K;
  const bool av = (K & 3) == 0 && (reinterpret_cast<uintptr_t>(p.w) & 15) == 0;
  float a[8];
  auto load_a = [&](int ch) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int kb = ch * KC + 16 * t + 4 * g;
      if (av) {
        const f4 w4 = *reinterpret_cast<const f4*>(wrow + min(kb, K - 4));
        const bool ok = m_ok && kb < K;  // K % 4 == 0: all four or none
#pragma unroll
        for (int e = 0; e < 4; ++e) a[4 * t + e] = ok ? w4[e] : 0.f;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float w1 = wrow[min(kb + e, K - 1)];
          a[4 * t + e] = (m_ok && kb + e < K) ? w1 : 0.f;
        }
      }
    }
  };
  f4 acc[4];
#pragma unroll
  for (int b = 0; b < 4; ++b) acc[b] = f4{0.f, 0.f, 0.f, 0.f};
  stage(0);
  for (int ch = 0; ch < nch; ++ch) {
    if (ch > 0) __syncthreads();  // the previous chunk's B reads are done
    commit(ch);
    load_a(ch);
    __syncthreads();
    if (ch + 1 < nch) stage(ch + 1);  // in flight during this chunk's MFMAs
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float* row = xs + (16 * t + 4 * g + e) * XSTR + wp * 64 + r;
#pragma unroll
        for (int b = 0; b < 4; ++b)
          acc[b] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[4 * t + e], row[16 * b], acc[b], 0, 0, 0);
      }
  }
  // acc[b][v] = D[channel m0 + 4 g + v][pixel p0 + wp * 64 + 16 b + r]
  const Epilogue& ep = p.ep;
  const int m0 = blockIdx.y * BM + wm * 16;
  float o[16];
  auto ch_of = [&](int k) { return m0 + 4 * g + (k & 3); };
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    const int chn = m0 + 4 * g + v;
    const float bv = ep.bias ? ep.bias[min(chn, p.M - 1)] : 0.f;
#pragma unroll
    for (int b = 0; b < 4; ++b) o[4 * b + v] = acc[b][v] + bv;
  }
  const int pb0 = p0 + wp * 64 + r;
  if (ep.res) {
    if (ep.res_mode == 0) {
      const float* rn = ep.res + (long)n * p.M * P;
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int chn = m0 + 4 * g + v, px2 = pb0 + 16 * b;
          if (chn < p.M && px2 < P) o[4 * b + v] += rn[chn * P + px2];
        }
    } else {
      each_rare(o, [&](int k, float v) {
        const int chn = ch_of(k), px2 = pb0 + 16 * (k >> 2);
        return chn < p.M && px2 < P ? v + residual(ep, chn, ((long)n * p.M + chn) * P + px2, n, px2) : v;
      });
    }
  }
  act_block(o, ch_of, ep);
  float* yn = p.y + (long)n * ((long)p.M * P + p.y_nx);
#pragma unroll
  for (int b = 0; b < 4; ++b)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int chn = m0 + 4 * g + v, px2 = pb0 + 16 * b;
      if (chn < p.M && px2 < P) yn[chn * P + px2] = o[4 * b + v];
    }
}

// k_conv_pw's workgroups for a 1x1 convolution of M channels over N images of
// P pixels (WM waves along the channels, PT = 64 (4 / WM) pixels per workgroup)
static long pw_workgroups(int N, long P, int M, int* wm) {
  *wm = M <= 16 ? 1 : (M <= 32 ? 2 : 4);
  const long pt = 64L * (4 / *wm), bm = 16L * *wm;
  return ((P + pt - 1) / pt) * ((M + bm - 1) / bm) * N;
}

// Where k_conv_pw pays (MODNet batch 8, per layer against the kernels it
// replaces, profiles/r04e): a plain 1x1 always when it has >= 256 workgroups
// or a shallow K (expand layers 16 -> 96 at 144x256 61 -> 44 us, 96 -> 576 at
// 18x32 28 -> 18 us); a fused depthwise -> 1x1 pair only with >= 512
// workgroups — a workgroup walks all of K serially with its depthwise
// recomputed per chunk, which won at 144x256 and 72x128 (104 -> 35, 86 -> 56
// us) and lost below (a 960-channel pair at 9x16: 72 workgroups, 26 -> 157 us),
// where k_conv_dwpw's 16-pixel workgroups or k_conv_dw + k_conv_small's
// split K keep the chip busy.
bool pw_fused_pays(int N, long P, int M) {
  int wm;
  return pw_workgroups(N, P, M, &wm) >= 512;
}

bool pw_pair_fits(int N, long C, long pre_hw, long P, int M) {
  if (C * pre_hw >= (1L << 31) || (long)M * P >= (1L << 31)) return false;  // pw_kernel's limits
  return pw_fused_pays(N, P, M);
}

// k_conv_pw serves this 1x1 convolution (or dw -> 1x1 pair); WM: waves along
// the output channels (the rest along pixels)
static bool pw_kernel(const ConvParams& p, int* wm, int* dwk) {
  const bool one = p.kh == 1 && p.kw == 1 && p.sh == 1 && p.sw == 1 && p.pt == 0 && p.pl == 0 && p.Ho == p.H &&
                   p.Wo == p.W && p.G == 1;
  if (!one) return false;
  const long P = (long)p.Ho * p.Wo, wgs = pw_workgroups(p.N, P, p.M, wm);  // (sets *wm for the launch)
  *dwk = 0;
  if (p.pre.w) {
    if (p.pre.kh != p.pre.kw || (p.pre.kh != 3 && p.pre.kh != 5)) return false;
    *dwk = p.pre.kh;
    return pw_pair_fits(p.N, p.C, (long)p.pre.H * p.pre.W, P, p.M);
  }
  if ((long)p.C * P >= (1L << 31) || (long)p.M * P >= (1L << 31)) return false;  // 32-bit offsets within an image
  static const bool plain_on = [] {  // (VSO_PW=0: plain 1x1s on k_conv_small / k_conv_gemm, an A/B knob)
    const char* e = std::getenv("VSO_PW");
    return !(e && e[0] == '0');
  }();
  return plain_on && (wgs >= 256 || p.C <= 192);
}

// Index arithmetic in 32 bits whenever the tensor allows (I = int): a 64-bit
// division is a ~40-instruction software sequence on CDNA, a 32-bit one a few
// VALU ops; the elementwise kernels below choose per launch (uniform branch).
template <typename I>
__device__ __forceinline__ void unravel(I i, int nd, const int* dims, int* idx) {
  for (int d = nd - 1; d >= 0; --d) {
    idx[d] = (int)(i % (I)dims[d]);
    i /= (I)dims[d];
  }
}

constexpr long kIdx32 = 1L << 30;  // totals below this index in int (grid-stride steps cannot overflow)

// k_conv_dw's four-outputs-per-thread form: 3x3, dilation 1, stride 1 or 2,
// rows of a multiple of 4 outputs, a 16-B aligned output, and at least 1024
// workgroups of quads (4 per CU; MODNet's 648-workgroup layer measured 12.3 us
// as quads against 10.1 us one output per thread)
// VSO_DW_PLANE=0: the flat k_conv_dw for every quad-shaped depthwise (A/B)
static bool dw_plane_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("VSO_DW_PLANE");
    return !(e && e[0] == '0');
  }();
  return on;
}

__host__ __device__ inline bool dw_quad(const ConvParams& p) {
  const long total = (long)p.N * p.M * p.Ho * p.Wo;
  return p.kh == 3 && p.kw == 3 && p.dh == 1 && p.dw == 1 && (p.sw == 1 || p.sw == 2) && (p.Wo & 3) == 0 &&
         (reinterpret_cast<uintptr_t>(p.y) & 15) == 0 && total / 4 >= 1024L * 256 && total < kIdx32;
}

template <typename I>
__device__ __forceinline__ void conv_dw_body(const ConvParams& p, I total) {
  for (I o = (I)blockIdx.x * 256 + (I)threadIdx.x; o < total; o += (I)gridDim.x * 256) {
    const int ox = (int)(o % (I)p.Wo);
    const I t = o / (I)p.Wo;
    const int oy = (int)(t % (I)p.Ho);
    const I nc = t / (I)p.Ho;
    const int ch = (int)(nc % (I)p.M);
    const float* xc = p.x + (long)nc * p.H * p.W;  // depthwise: input channel = output channel
    const float* wc = p.w + (long)ch * p.kh * p.kw;
    float acc = 0.f;
    for (int ky = 0; ky < p.kh; ++ky) {
      const int iy = oy * p.sh - p.pt + ky * p.dh;
      if (iy < 0 || iy >= p.H) continue;
      for (int kx = 0; kx < p.kw; ++kx) {
        const int ix = ox * p.sw - p.pl + kx * p.dw;
        if (ix >= 0 && ix < p.W) acc = __builtin_fmaf(wc[ky * p.kw + kx], xc[(long)iy * p.W + ix], acc);
      }
    }
    const int n = (int)(nc / (I)p.M);
    p.y[(long)o + n * p.y_nx] = epilogue(p.ep, acc, ch, (long)o, n, oy * p.Wo + ox);
  }
}

// 3x3 depthwise, dilation 1, stride SW, four consecutive outputs of a row per
// thread: each input row's 3 SW + 3 columns are loaded once for the four
// (18 loads per 4 outputs at stride 1 instead of 36), one float4 store.  Per
// output the same operations as conv_dw_body: the taps in ky, kx order, an
// absent tap skipped.
template <int SW>
__device__ __forceinline__ void conv_dw3_quad(const ConvParams& p, int total4) {
  constexpr int NC = 3 * SW + 3;  // input columns of the four outputs
  for (int q = blockIdx.x * 256 + threadIdx.x; q < total4; q += gridDim.x * 256) {
    const int o = 4 * q;
    const int ox = o % p.Wo, t = o / p.Wo, oy = t % p.Ho, nc = t / p.Ho;
    const int ch = nc % p.M;
    const float* xc = p.x + (long)nc * p.H * p.W;
    const float* wc = p.w + (long)ch * 9;
    float wv[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) wv[k] = wc[k];
    const int ix0 = ox * SW - p.pl;
    f4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const int iy = oy * p.sh - p.pt + ky;
      if (iy < 0 || iy >= p.H) continue;
      float r[NC];
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int ix = ix0 + c;
        r[c] = (ix >= 0 && ix < p.W) ? xc[(long)iy * p.W + ix] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          const int ix = ix0 + j * SW + kx;
          if (ix >= 0 && ix < p.W) acc[j] = __builtin_fmaf(wv[ky * 3 + kx], r[j * SW + kx], acc[j]);
        }
    }
    f4 out;
    const int n = nc / p.M;
#pragma unroll
    for (int j = 0; j < 4; ++j) out[j] = epilogue(p.ep, acc[j], ch, (long)o + j, n, oy * p.Wo + ox + j);
    *reinterpret_cast<f4*>(p.y + o + n * p.y_nx) = out;
  }
}

// conv_dw3_quad with one (image, channel) plane per blockIdx.y and a wave
// per workgroup: the channel, its 9 weights, bias and activation are uniform
// (scalar loads, a uniform branch) and the only runtime division is by the
// plane's quads per row — the flat form divides five times per quad and
// loads the weights per lane.  Same taps, FMA order and epilogue: bit for
// bit k_conv_dw's values.
template <int SW>
__global__ __launch_bounds__(64) void k_conv_dw_plane(ConvParams p) {
  constexpr int NC = 3 * SW + 3;
  const int nc = blockIdx.y;
  const int qrow = p.Wo >> 2;
  const int q = blockIdx.x * 64 + threadIdx.x;
  if (q >= qrow * p.Ho) return;
  const int oy = q / qrow, ox = (q - oy * qrow) * 4;
  const int n = nc / p.M, ch = nc - n * p.M;
  const float* xc = p.x + (long)nc * p.H * p.W;
  const float* wc = p.w + (long)ch * 9;
  float wv[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) wv[k] = wc[k];
  const int ix0 = ox * SW - p.pl;
  f4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ky = 0; ky < 3; ++ky) {
    const int iy = oy * p.sh - p.pt + ky;
    if (iy < 0 || iy >= p.H) continue;
    float r[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int ix = ix0 + c;
      r[c] = (ix >= 0 && ix < p.W) ? xc[(long)iy * p.W + ix] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const int ix = ix0 + j * SW + kx;
        if (ix >= 0 && ix < p.W) acc[j] = __builtin_fmaf(wv[ky * 3 + kx], r[j * SW + kx], acc[j]);
      }
  }
  const int pix = oy * p.Wo + ox;
  const long o = (long)nc * p.Ho * p.Wo + pix;
  f4 out;
#pragma unroll
  for (int j = 0; j < 4; ++j) out[j] = epilogue(p.ep, acc[j], ch, o + j, n, pix + j);
  *reinterpret_cast<f4*>(p.y + o + n * p.y_nx) = out;
}

__host__ inline bool dw_plane(const ConvParams& p) {
  return dw_quad(p) && (long)p.N * p.M <= 65535 && dw_plane_enabled();
}

__global__ __launch_bounds__(256) void k_conv_dw(ConvParams p) {
  const long total = (long)p.N * p.M * p.Ho * p.Wo;
  if (dw_quad(p)) {
    if (p.sw == 1) conv_dw3_quad<1>(p, (int)(total / 4));
    else conv_dw3_quad<2>(p, (int)(total / 4));
    return;
  }
  if (total < kIdx32) conv_dw_body<int>(p, (int)total);
  else conv_dw_body<long>(p, total);
}

static int grid_for(long n) { return (int)((n + 255) / 256 < 65536 ? (n + 255) / 256 : 65536); }

enum ConvKind { CONV_DW, CONV_SMALL_PW, CONV_SMALL, CONV_GEMM };

static ConvKind conv_kind(const ConvParams& p) {
  if (p.G == p.C && p.G == p.M) return CONV_DW;
  const long P = (long)p.Ho * p.Wo;
  const long tiles64 = ((P + BP - 1) / BP) * ((p.Mg + BM - 1) / BM) * p.N * p.G;
  if (tiles64 >= 1024) return CONV_GEMM;  // enough 64x64 tiles to fill 256 CUs
  const bool pw = p.kh == 1 && p.kw == 1 && p.sh == 1 && p.sw == 1 && p.pt == 0 && p.pl == 0 && p.Ho == p.H &&
                  p.Wo == p.W;
  return pw ? CONV_SMALL_PW : CONV_SMALL;
}

const char* conv_kernel_name(const ConvParams& p) {
  int wm, dwk;
  if (pw_kernel(p, &wm, &dwk)) {
    static const char* names[3][3] = {
        {"void vso::k_conv_pw<1, 0>(vso::ConvParams)", "void vso::k_conv_pw<2, 0>(vso::ConvParams)",
         "void vso::k_conv_pw<4, 0>(vso::ConvParams)"},
        {"void vso::k_conv_pw<1, 3>(vso::ConvParams)", "void vso::k_conv_pw<2, 3>(vso::ConvParams)",
         "void vso::k_conv_pw<4, 3>(vso::ConvParams)"},
        {"void vso::k_conv_pw<1, 5>(vso::ConvParams)", "void vso::k_conv_pw<2, 5>(vso::ConvParams)",
         "void vso::k_conv_pw<4, 5>(vso::ConvParams)"}};
    return names[dwk / 2][wm / 2];
  }
  if (p.pre.w) return "vso::k_conv_dwpw(vso::ConvParams)";
  switch (conv_kind(p)) {
    case CONV_DW:
      if (dw_plane(p))
        return p.sw == 1 ? "void vso::k_conv_dw_plane<1>(vso::ConvParams)" : "void vso::k_conv_dw_plane<2>(vso::ConvParams)";
      return "vso::k_conv_dw(vso::ConvParams)";
    case CONV_SMALL_PW:
    case CONV_SMALL: {
      static const char* names[2][4] = {
          {"void vso::k_conv_small<false, 8, false>(vso::ConvParams, int, int)",
           "void vso::k_conv_small<false, 16, false>(vso::ConvParams, int, int)",
           "void vso::k_conv_small<false, 32, false>(vso::ConvParams, int, int)",
           "void vso::k_conv_small<false, 16, true>(vso::ConvParams, int, int)"},
          {"void vso::k_conv_small<true, 8, false>(vso::ConvParams, int, int)",
           "void vso::k_conv_small<true, 16, false>(vso::ConvParams, int, int)",
           "void vso::k_conv_small<true, 32, false>(vso::ConvParams, int, int)",
           "void vso::k_conv_small<true, 16, true>(vso::ConvParams, int, int)"}};
      const int K = p.Cg * p.kh * p.kw;
      return names[conv_kind(p) == CONV_SMALL_PW][K <= 32 ? 0 : K <= 64 ? 1 : K <= 128 ? 2 : 3];
    }
    default: return "vso::k_conv_gemm(vso::ConvParams)";
  }
}

void launch_conv(const ConvParams& p, hipStream_t s, const char** name) {
  if (name) *name = conv_kernel_name(p);
  int wm, dwk;
  if (pw_kernel(p, &wm, &dwk)) {
    const dim3 grid((unsigned)((p.Ho * p.Wo + 64 * (4 / wm) - 1) / (64 * (4 / wm))),
                    (unsigned)((p.M + 16 * wm - 1) / (16 * wm)), (unsigned)p.N);
#define VSO_PW(WMV, DWKV) \
  if (wm == WMV && dwk == DWKV) { hipLaunchKernelGGL((k_conv_pw<WMV, DWKV>), grid, dim3(256), 0, s, p); return; }
    VSO_PW(1, 0) VSO_PW(2, 0) VSO_PW(4, 0) VSO_PW(1, 3) VSO_PW(2, 3) VSO_PW(4, 3) VSO_PW(1, 5) VSO_PW(2, 5) VSO_PW(4, 5)
#undef VSO_PW
  }
  if (p.pre.w) {
    const dim3 grid((unsigned)((p.Ho * p.Wo + 15) / 16), (unsigned)((p.M + 63) / 64), (unsigned)p.N);
    hipLaunchKernelGGL(k_conv_dwpw, grid, dim3(256), 0, s, p);
    return;
  }
  const ConvKind kind = conv_kind(p);
  if (kind == CONV_DW) {
    const long total = (long)p.N * p.M * p.Ho * p.Wo;
    if (dw_plane(p)) {
      const dim3 grid((unsigned)(((p.Wo >> 2) * p.Ho + 63) / 64), (unsigned)(p.N * p.M));
      if (p.sw == 1) hipLaunchKernelGGL(k_conv_dw_plane<1>, grid, dim3(64), 0, s, p);
      else hipLaunchKernelGGL(k_conv_dw_plane<2>, grid, dim3(64), 0, s, p);
      return;
    }
    hipLaunchKernelGGL(k_conv_dw, dim3(grid_for(dw_quad(p) ? total / 4 : total)), dim3(256), 0, s, p);
  } else if (kind == CONV_GEMM) {
    const dim3 grid((p.Ho * p.Wo + BP - 1) / BP, (p.Mg + BM - 1) / BM, p.N * p.G);
    hipLaunchKernelGGL(k_conv_gemm, grid, dim3(256), 0, s, p);
  } else {  // 16x16 tiles: one wave each, or one workgroup each with K split four ways
    const int tm = (p.Mg + 15) / 16, tp = (p.Ho * p.Wo + 15) / 16;
    const long tiles = (long)tm * tp * p.N * p.G;
    const int K = p.Cg * p.kh * p.kw;
    const bool pw = kind == CONV_SMALL_PW;
    if (K > 128) {
      const dim3 grid((unsigned)tiles);
      if (pw)
        hipLaunchKernelGGL((k_conv_small<true, 16, true>), grid, dim3(256), 0, s, p, tm, tp);
      else
        hipLaunchKernelGGL((k_conv_small<false, 16, true>), grid, dim3(256), 0, s, p, tm, tp);
    } else {  // a chunk just covers K (no MFMAs on zero padding)
      const dim3 grid((unsigned)((tiles + 3) / 4));
#define VSO_SMALL(PWV, CHV) hipLaunchKernelGGL((k_conv_small<PWV, CHV, false>), grid, dim3(256), 0, s, p, tm, tp)
      if (K <= 32) {
        if (pw) VSO_SMALL(true, 8); else VSO_SMALL(false, 8);
      } else if (K <= 64) {
        if (pw) VSO_SMALL(true, 16); else VSO_SMALL(false, 16);
      } else {
        if (pw) VSO_SMALL(true, 32); else VSO_SMALL(false, 32);
      }
#undef VSO_SMALL
    }
  }
}

// ---------------------------------------------------------------------------

__device__ __forceinline__ float bin_op(int op, float a, float b) {
  switch (op) {
    case BIN_ADD: return a + b;
    case BIN_SUB: return a - b;
    case BIN_MUL: return a * b;
    case BIN_DIV: return a / b;
    default: return a < 0.f ? a * b : a;  // PRELU
  }
}

// a 4-D contiguous a (op) b of one value per (n, c) plane (the SE blocks'
// channel gate, MODNet 288x512: 8 x 1280 planes of 144): float4s of a, b's
// value per plane, y contiguous — the general form's per-element unravel ran
// this at 0.8 TB/s (15 us)
__global__ __launch_bounds__(256) void k_binary_planes(BinParams p) {
  const long inner = (long)p.dims[2] * p.dims[3];
  const long n4 = p.n / 4;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    const long plane = (4 * i) / inner;
    const long nn = plane / p.dims[1], cc = plane - nn * p.dims[1];
    const float bv = p.b[nn * p.sb[0] + cc * p.sb[1]];
    const f4 av = reinterpret_cast<const f4*>(p.a)[i];
    reinterpret_cast<f4*>(p.y)[i] = f4{bin_op(p.op, av.x, bv), bin_op(p.op, av.y, bv), bin_op(p.op, av.z, bv),
                                       bin_op(p.op, av.w, bv)};
  }
}
bool binary_planes(const BinParams& p) {
  static const bool on = [] {
    const char* e = std::getenv("VSO_BIN_PLANES");
    return !e || std::atoi(e) != 0;
  }();
  if (!on) return false;
  const auto al = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  if (p.nd != 4 || p.sb[2] != 0 || p.sb[3] != 0 || ((long)p.dims[2] * p.dims[3]) % 4 != 0) return false;
  if (p.sa[3] != 1 || p.sa[2] != p.dims[3] || p.sa[1] != (long)p.dims[2] * p.dims[3] ||
      (p.dims[0] > 1 && p.sa[0] != (long)p.dims[1] * p.sa[1]))
    return false;
  return al(p.a) && al(p.y);
}

template <typename I>
__device__ __forceinline__ void binary_body(const BinParams& p) {
  for (I i = (I)blockIdx.x * 256 + (I)threadIdx.x; i < (I)p.n; i += (I)gridDim.x * 256) {
    int idx[kMaxDims];
    unravel<I>(i, p.nd, p.dims, idx);
    long oa = 0, ob = 0;
    for (int d = 0; d < p.nd; ++d) {
      oa += idx[d] * p.sa[d];
      ob += idx[d] * p.sb[d];
    }
    const float a = p.a[oa], b = p.b[ob];
    float v;
    switch (p.op) {
      case BIN_ADD: v = a + b; break;
      case BIN_SUB: v = a - b; break;
      case BIN_MUL: v = a * b; break;
      case BIN_DIV: v = a / b; break;
      default: v = a < 0.f ? a * b : a; break;  // PRELU
    }
    p.y[i] = v;
  }
}

__global__ __launch_bounds__(256) void k_binary(BinParams p) {
  if (p.n < kIdx32) binary_body<int>(p);
  else binary_body<long>(p);
}

__global__ __launch_bounds__(256) void k_unary(UnaryParams p) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < p.n; i += (long)gridDim.x * 256)
    p.y[i] = act_apply(p.x[i], p.act, p.a0, p.a1, nullptr, 0, 0);
}

template <typename I>
__device__ __forceinline__ void copy_body(const CopyParams& p) {
  for (I i = (I)blockIdx.x * 256 + (I)threadIdx.x; i < (I)p.n; i += (I)gridDim.x * 256) {
    int idx[kMaxDims];
    unravel<I>(i, p.nd, p.size, idx);
    long od = p.dst_base, os = p.src_base;
    bool in = true;
    for (int d = 0; d < p.nd; ++d) {
      od += idx[d] * p.dst_stride[d];
      const int c = idx[d] * p.step[d] + p.start[d];
      in = in && c >= 0 && c < p.lim[d];
      os += (long)c * p.src_stride[d];
    }
    p.dst[od] = in ? p.src[os] : p.fill;
  }
}

__global__ __launch_bounds__(256) void k_copy(CopyParams p) {
  if (p.n < kIdx32) copy_body<int>(p);
  else copy_body<long>(p);
}

// grid (ceil(inner / (256 * 4 * U)), rows); VEC: 16-byte moves (every offset a multiple of 4)
template <bool VEC>
__global__ __launch_bounds__(256) void k_copy_rows(RowCopyParams p) {
  constexpr int U = 4;
  const float* src = p.src + p.src_base + (long)blockIdx.y * p.src_row;
  float* dst = p.dst + p.dst_base + (long)blockIdx.y * p.dst_row;
  if (VEC) {
    const long n4 = p.inner >> 2;
    const long i0 = (long)blockIdx.x * 256 * U + threadIdx.x;
    f4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i0 + 256 * u < n4) v[u] = reinterpret_cast<const f4*>(src)[i0 + 256 * u];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i0 + 256 * u < n4) reinterpret_cast<f4*>(dst)[i0 + 256 * u] = v[u];
  } else {
    const long i0 = (long)blockIdx.x * 256 * U * 4 + threadIdx.x;
    for (int u = 0; u < U * 4; ++u)
      if (i0 + 256 * u < p.inner) dst[i0 + 256 * u] = src[i0 + 256 * u];
  }
}

static bool rows_vec(const RowCopyParams& p) {
  const auto al = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  return p.inner % 4 == 0 && p.src_row % 4 == 0 && p.dst_row % 4 == 0 && p.src_base % 4 == 0 &&
         p.dst_base % 4 == 0 && al(p.src) && al(p.dst);
}

void launch_copy_rows(const RowCopyParams& p, hipStream_t s) {
  const dim3 grid((unsigned)((p.inner + 4096 - 1) / 4096), (unsigned)p.rows);
  if (rows_vec(p)) hipLaunchKernelGGL(k_copy_rows<true>, grid, dim3(256), 0, s, p);
  else hipLaunchKernelGGL(k_copy_rows<false>, grid, dim3(256), 0, s, p);
}

const char* row_copy_name(const RowCopyParams& p) {
  return rows_vec(p) ? "void vso::k_copy_rows<true>(vso::RowCopyParams)" : "void vso::k_copy_rows<false>(vso::RowCopyParams)";
}

template <typename I>
__device__ __forceinline__ void pool_body(const PoolParams& p, I total) {
  for (I o = (I)blockIdx.x * 256 + (I)threadIdx.x; o < total; o += (I)gridDim.x * 256) {
    const int ox = (int)(o % (I)p.Wo);
    const I t = o / (I)p.Wo;
    const int oy = (int)(t % (I)p.Ho);
    const I nc = t / (I)p.Ho;
    const float* xc = p.x + (long)nc * p.H * p.W;
    float m = -INFINITY, s = 0.f;
    int cnt = 0;
    for (int ky = 0; ky < p.kh; ++ky) {
      const int iy = oy * p.sh - p.pt + ky * p.dh;
      if (iy < 0 || iy >= p.H) continue;
      for (int kx = 0; kx < p.kw; ++kx) {
        const int ix = ox * p.sw - p.pl + kx * p.dw;
        if (ix < 0 || ix >= p.W) continue;
        const float v = xc[(long)iy * p.W + ix];
        m = fmaxf(m, v);
        s += v;
        ++cnt;
      }
    }
    p.y[o] = p.max_mode ? m : s / (float)(p.count_include_pad ? p.kh * p.kw : (cnt > 0 ? cnt : 1));
  }
}

__global__ __launch_bounds__(256) void k_pool(PoolParams p) {
  const long total = (long)p.N * p.C * p.Ho * p.Wo;
  if (total < kIdx32) pool_body<int>(p, (int)total);
  else pool_body<long>(p, total);
}

__device__ __forceinline__ float block_sum(float v, float* sh) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int wave = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[wave] = v;
  __syncthreads();
  return sh[0] + sh[1] + sh[2] + sh[3];
}

__device__ __forceinline__ float block_max(float v, float* sh) {
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  const int wave = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[wave] = v;
  __syncthreads();
  return fmaxf(fmaxf(sh[0], sh[1]), fmaxf(sh[2], sh[3]));
}

__global__ __launch_bounds__(256) void k_gap(RowParams p) {
  __shared__ float sh[4];
  const float* x = p.x + (long)blockIdx.x * p.inner;
  float s = 0.f;
  for (long i = threadIdx.x; i < p.inner; i += 256) s += x[i];
  s = block_sum(s, sh);
  if (threadIdx.x == 0) p.y[blockIdx.x] = s / (float)p.inner;
}

// Short planes (inner <= kGapWaveMax): a wave per plane, four per workgroup —
// MODNet's SE pool (8 x 1280 planes of 9 x 16 at 288x512): 14.1 -> 8.3 us
// against 10240 workgroups of 256 threads summing 144 elements each (r05ag).
// (A wave per output column for the SE's few-row GEMMs measured slower than
// k_gemm's 16 x 16 MFMA tiles: 20 against 13 us each.)
__global__ __launch_bounds__(256) void k_gap_wave(RowParams p) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= p.rows) return;  // (whole waves)
  const float* x = p.x + row * p.inner;
  float s = 0.f;
  for (long i = lane; i < p.inner; i += 64) s += x[i];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if (lane == 0) p.y[row] = s / (float)p.inner;
}

// Planes whose length is a multiple of 4 (and 16-B aligned tensors) move
// float4s: 4 elements per load / store instruction, a quarter of the
// instructions of the scalar form (MODNet 288x512: 2 x 24 launches per run).
__device__ __forceinline__ bool norm_vec(const NormParams& p) {
  return (p.inner & 3) == 0 && (reinterpret_cast<uintptr_t>(p.x) & 15) == 0 &&
         (reinterpret_cast<uintptr_t>(p.y) & 15) == 0;
}

// InstanceNorm of planes of at most 256 x PER elements: one workgroup per
// plane holds it in registers — statistics and apply in one launch, one read
// and one write (k_norm_stats + k_norm_apply read it twice, launch twice:
// ~5 us each at MODNet's /8 and /16 planes, where the launches, not the
// bytes, set the time).
template <int NT>
__device__ __forceinline__ float block_sum_n(float v, float* sh) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) t += sh[w];
  return t;
}

template <int PER, int NT>
__global__ __launch_bounds__(NT) void k_norm_plane(NormParams p) {
  static_assert(PER % 4 == 0, "float4 pieces");
  __shared__ float sh[NT / 64];
  const int row = blockIdx.x, n = row / p.C, c = row - n * p.C;
  const long off = ((long)n * p.ctot + p.c0 + c) * p.inner;
  const int cnt = (int)p.inner;
  const bool vec = norm_vec(p);
  auto elem = [&](int i) { return vec ? 4 * (int)threadIdx.x + 4 * NT * (i >> 2) + (i & 3) : (int)threadIdx.x + NT * i; };
  float v[PER];
  if (vec) {
#pragma unroll
    for (int i = 0; i < PER; i += 4) {
      const int e = elem(i);
      const f4 t = e < cnt ? *reinterpret_cast<const f4*>(p.x + off + e) : f4{0.f, 0.f, 0.f, 0.f};
      v[i] = t[0]; v[i + 1] = t[1]; v[i + 2] = t[2]; v[i + 3] = t[3];
    }
  } else {
#pragma unroll
    for (int i = 0; i < PER; ++i) v[i] = elem(i) < cnt ? p.x[off + elem(i)] : 0.f;
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) s += v[i];
  const float mean = block_sum_n<NT>(s, sh) / (float)cnt;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const float d = v[i] - mean;
    if (elem(i) < cnt) q += d * d;
  }
  q = block_sum_n<NT>(q, sh);
  const float sc = p.scale[c] / sqrtf(q / (float)cnt + p.eps), sf = p.shift[c];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    v[i] = (v[i] - mean) * sc + sf;
    if (p.act == ACT_RELU) v[i] = fmaxf(v[i], 0.f);
  }
  if (vec) {
#pragma unroll
    for (int i = 0; i < PER; i += 4) {
      const int e = elem(i);
      if (e < cnt) *reinterpret_cast<f4*>(p.y + off + e) = f4{v[i], v[i + 1], v[i + 2], v[i + 3]};
    }
  } else {
#pragma unroll
    for (int i = 0; i < PER; ++i)
      if (elem(i) < cnt) p.y[off + elem(i)] = v[i];
  }
}

bool norm_plane_fits(long inner) { return inner > 0 && inner <= kNormPlaneMax; }

// (256 threads x 16 / 48 elements up to 12288; 1024 x 36 up to 36864:
// MODNet's 144x256 planes, 128-256 of them, one per CU)
const char* norm_plane_name(long inner) {
  return inner <= 4096    ? "void vso::k_norm_plane<16, 256>(vso::NormParams)"
         : inner <= 12288 ? "void vso::k_norm_plane<48, 256>(vso::NormParams)"
                          : "void vso::k_norm_plane<36, 1024>(vso::NormParams)";
}

void launch_norm_plane(const NormParams& p, hipStream_t s) {
  const dim3 grid((unsigned)(p.N * p.C));
  if (p.inner <= 4096) hipLaunchKernelGGL((k_norm_plane<16, 256>), grid, dim3(256), 0, s, p);
  else if (p.inner <= 12288) hipLaunchKernelGGL((k_norm_plane<48, 256>), grid, dim3(256), 0, s, p);
  else hipLaunchKernelGGL((k_norm_plane<36, 1024>), grid, dim3(1024), 0, s, p);
}

// A plane's statistics from k_norm_stats' pieces ((mean, M2, count) each),
// merged by one wave: every lane folds pieces lane, lane + 64, ... in order,
// then the lanes' partials combine in a butterfly (Chan et al.'s pairwise
// update); every lane ends with the whole.  (k_conv_thin: its sequential fold
// over 36 pieces per channel measured 25.7 against 20.9 us for MODNet's
// matte head; k_norm_apply, one channel per workgroup, keeps the sequential
// fold — the butterfly measured slower there.)
__device__ __forceinline__ void merge_stats(const float* st, int chunks, float& mean, float& m2, float& cnt) {
  const int lane = threadIdx.x & 63;
  mean = 0.f; m2 = 0.f; cnt = 0.f;
  auto fold = [&](float mb, float m2b, float nb) {
    if (nb == 0.f) return;
    const float nab = cnt + nb, d = mb - mean;
    mean += d * (nb / nab);
    m2 += m2b + d * d * (cnt * nb / nab);
    cnt = nab;
  };
  for (int k = lane; k < chunks; k += 64) fold(st[3 * k], st[3 * k + 1], st[3 * k + 2]);
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float mb = __shfl_xor(mean, o), m2b = __shfl_xor(m2, o), nb = __shfl_xor(cnt, o);
    // (both partners compute the same merge: the lower lane's partial first)
    if (lane & o) {
      const float ma = mean, m2a = m2, na = cnt;
      mean = mb; m2 = m2b; cnt = nb;
      fold(ma, m2a, na);
    } else {
      fold(mb, m2b, nb);
    }
  }
}

__global__ __launch_bounds__(256) void k_norm_stats(NormParams p) {
  __shared__ float sh[4];
  constexpr int PER = kNormChunk / 256;
  static_assert(PER % 4 == 0, "float4 pieces");
  const int row = blockIdx.y, n = row / p.C, c = row - n * p.C;
  const float* x = p.x + ((long)n * p.ctot + p.c0 + c) * p.inner;
  const long beg = (long)blockIdx.x * p.chunk;
  const int cnt = (int)min((long)p.chunk, p.inner - beg);
  // element e of the chunk: v[i] = e = threadIdx.x + 256 * i (scalar form) or
  // e = 4 * threadIdx.x + 1024 * (i / 4) + i % 4 (float4 form)
  const bool vec = norm_vec(p);
  auto elem = [&](int i) { return vec ? 4 * (int)threadIdx.x + 1024 * (i >> 2) + (i & 3) : (int)threadIdx.x + 256 * i; };
  float v[PER];
  float s = 0.f;
  if (vec) {
#pragma unroll
    for (int i = 0; i < PER; i += 4) {
      const int e = elem(i);  // cnt is a multiple of 4 here
      const f4 t = e < cnt ? *reinterpret_cast<const f4*>(x + beg + e) : f4{0.f, 0.f, 0.f, 0.f};
      v[i] = t[0];
      v[i + 1] = t[1];
      v[i + 2] = t[2];
      v[i + 3] = t[3];
    }
  } else {
#pragma unroll
    for (int i = 0; i < PER; ++i) v[i] = elem(i) < cnt ? x[beg + elem(i)] : 0.f;
  }
#pragma unroll
  for (int i = 0; i < PER; ++i) s += v[i];
  const float mean = block_sum(s, sh) / (float)cnt;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const float d = v[i] - mean;
    if (elem(i) < cnt) q += d * d;
  }
  q = block_sum(q, sh);
  if (threadIdx.x == 0) {
    float* st = p.stats + ((long)row * p.chunks + blockIdx.x) * 3;
    st[0] = mean;
    st[1] = q;
    st[2] = (float)cnt;
  }
}

__global__ __launch_bounds__(256) void k_norm_apply(NormParams p) {
  const int row = blockIdx.y, n = row / p.C, c = row - n * p.C;
  const long off = ((long)n * p.ctot + p.c0 + c) * p.inner;
  // the plane's statistics: its pieces merged in piece order (every thread alike)
  const float* st = p.stats + (long)row * p.chunks * 3;
  float mean = st[0], m2 = st[1], cnt = st[2];
  for (int k = 1; k < p.chunks; ++k) {
    const float mb = st[3 * k], m2b = st[3 * k + 1], nb = st[3 * k + 2];
    const float nab = cnt + nb, d = mb - mean;
    mean += d * (nb / nab);
    m2 += m2b + d * d * (cnt * nb / nab);
    cnt = nab;
  }
  const float sc = p.scale[c] / sqrtf(m2 / cnt + p.eps), sf = p.shift[c];
  const long beg = (long)blockIdx.x * p.chunk;
  const long end = min(beg + p.chunk, p.inner);
  if (norm_vec(p)) {
    for (long i = beg + 4 * threadIdx.x; i < end; i += 1024) {
      f4 y = *reinterpret_cast<const f4*>(p.x + off + i);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        y[j] = (y[j] - mean) * sc + sf;
        if (p.act == ACT_RELU) y[j] = fmaxf(y[j], 0.f);
      }
      *reinterpret_cast<f4*>(p.y + off + i) = y;
    }
    return;
  }
  for (long i = beg + threadIdx.x; i < end; i += 256) {
    float y = (p.x[off + i] - mean) * sc + sf;
    if (p.act == ACT_RELU) y = fmaxf(y, 0.f);
    p.y[off + i] = y;
  }
}

// k_conv_thin (vso_kernels.h).  Workgroup: 1024 pixels of one image, 4 per
// thread (one float4 per input channel when the plane is 16-byte aligned);
// the normalised channels' (mean, scale, shift) merged from the statistics
// pieces as k_norm_apply does, once per workgroup, into LDS.  Memory bound:
// C x 4 bytes in and M x 4 out per pixel.
template <int M>
__global__ __launch_bounds__(256) void k_conv_thin(ConvParams p, NormParams q, int has_norm) {
  __shared__ float nrm[3][256];
  const int n = blockIdx.y;
  const long P = (long)p.Ho * p.Wo;
  const long pix0 = ((long)blockIdx.x * 256 + threadIdx.x) * 4;
  const bool vec = (P & 3) == 0 && pix0 + 3 < P;
  const float* xn = p.x + (long)n * p.C * P;
  auto load = [&](int c) {
    f4 v;
    if (vec) {
      v = *reinterpret_cast<const f4*>(xn + c * P + pix0);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = pix0 + j < P ? xn[c * P + pix0 + j] : 0.f;
    }
    return v;
  };
  if (has_norm) {
    for (int c = threadIdx.x >> 6; c < q.C; c += 4) {  // a wave per channel
      float mean, m2, cnt;
      merge_stats(q.stats + ((long)n * q.C + c) * q.chunks * 3, q.chunks, mean, m2, cnt);
      if ((threadIdx.x & 63) == 0) {
        nrm[0][c] = mean;
        nrm[1][c] = q.scale[c] / sqrtf(m2 / cnt + q.eps);
        nrm[2][c] = q.shift[c];
      }
    }
    __syncthreads();
  }
  if (pix0 >= P) return;
  float acc[M][4] = {};
  auto step = [&](int c, f4 v) {
    const int k = c - q.c0;
    if (has_norm && k >= 0 && k < q.C) {
      const float mean = nrm[0][k], sc = nrm[1][k], sf = nrm[2][k];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v[j] = (v[j] - mean) * sc + sf;
        if (q.act == ACT_RELU) v[j] = fmaxf(v[j], 0.f);
      }
    }
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const float w = p.w[m * p.C + c];
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[m][j] = fmaf(w, v[j], acc[m][j]);
    }
  };
#pragma unroll 8
  for (int c = 0; c < p.C; ++c) step(c, load(c));  // (unrolled: 8 loads in flight per thread)
  float* yn = p.y + (long)n * (M * P + p.y_nx);
#pragma unroll
  for (int m = 0; m < M; ++m) {
    if (m >= p.M) break;
    f4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const long pix = pix0 + j;
      o[j] = epilogue(p.ep, acc[m][j], m, ((long)n * p.M + m) * P + pix, n, (int)pix);
    }
    if (vec) {
      *reinterpret_cast<f4*>(yn + m * P + pix0) = o;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (pix0 + j < P) yn[m * P + pix0 + j] = o[j];
    }
  }
}

bool thin_conv_fits(const ConvParams& p) {
  return p.G == 1 && p.M >= 1 && p.M <= kThinMaxM && p.kh == 1 && p.kw == 1 && p.sh == 1 && p.sw == 1 &&
         p.pt == 0 && p.pl == 0 && p.Ho == p.H && p.Wo == p.W && !p.pre.w && (long)p.C * p.H * p.W < (1L << 31);
}

void launch_conv_thin(const ConvParams& p, const NormParams* norm, hipStream_t s) {
  const long P = (long)p.Ho * p.Wo;
  const dim3 grid((unsigned)((P + 1023) / 1024), (unsigned)p.N);
  NormParams q{};
  if (norm) q = *norm;
  const int has = norm ? 1 : 0;
  // (M a template parameter: the accumulators stay in registers)
  switch (p.M) {
    case 1: hipLaunchKernelGGL(k_conv_thin<1>, grid, dim3(256), 0, s, p, q, has); break;
    case 2: hipLaunchKernelGGL(k_conv_thin<2>, grid, dim3(256), 0, s, p, q, has); break;
    case 3: hipLaunchKernelGGL(k_conv_thin<3>, grid, dim3(256), 0, s, p, q, has); break;
    default: hipLaunchKernelGGL(k_conv_thin<4>, grid, dim3(256), 0, s, p, q, has); break;
  }
}

const char* conv_thin_name(int M) {
  static const char* names[] = {"void vso::k_conv_thin<1>(vso::ConvParams, vso::NormParams, int)",
                                "void vso::k_conv_thin<2>(vso::ConvParams, vso::NormParams, int)",
                                "void vso::k_conv_thin<3>(vso::ConvParams, vso::NormParams, int)",
                                "void vso::k_conv_thin<4>(vso::ConvParams, vso::NormParams, int)"};
  return names[std::min(std::max(M, 1), kThinMaxM) - 1];
}

__global__ __launch_bounds__(256) void k_softmax(RowParams p) {
  __shared__ float sh[4];
  const float* x = p.x + (long)blockIdx.x * p.inner;
  float* y = p.y + (long)blockIdx.x * p.inner;
  float m = -INFINITY;
  for (long i = threadIdx.x; i < p.inner; i += 256) m = fmaxf(m, x[i]);
  m = block_max(m, sh);
  float s = 0.f;
  for (long i = threadIdx.x; i < p.inner; i += 256) s += expf(x[i] - m);
  s = block_sum(s, sh);
  for (long i = threadIdx.x; i < p.inner; i += 256) y[i] = expf(x[i] - m) / s;
}

__global__ __launch_bounds__(256) void k_affine(AffineParams p) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < p.n; i += (long)gridDim.x * 256) {
    const int c = (int)((i / p.inner) % p.C);
    p.y[i] = p.x[i] * p.scale[c] + p.shift[c];
  }
}

__device__ __forceinline__ float resize_src(int o, float scale, int in, int out, int ctm) {
  switch (ctm) {
    case 0: return ((float)o + 0.5f) / scale - 0.5f;
    case 1: return out > 1 ? ((float)o + 0.5f) / scale - 0.5f : 0.f;
    case 2: return out > 1 ? (float)o * (float)(in - 1) / (float)(out - 1) : 0.f;
    default: return (float)o / scale;
  }
}

__device__ __forceinline__ int nearest_idx(float v, int mode, int in) {
  float r;
  if (mode == 0) r = (v == floorf(v) + 0.5f) ? floorf(v) : rintf(v);        // round_prefer_floor
  else if (mode == 1) r = floorf(v + 0.5f);                                   // round_prefer_ceil
  else if (mode == 2) r = floorf(v);
  else r = ceilf(v);
  const int i = (int)r;
  return i < 0 ? 0 : (i > in - 1 ? in - 1 : i);
}

// The source coordinate with the division by the scale as a multiplication
// when the scale is a power of two (2, 0.5, ...: the reciprocal is exact, so
// the value is the division's bit for bit); other scales divide.
__device__ __forceinline__ float resize_src_fast(int o, float scale, float inv, bool pow2, int in, int out, int ctm) {
  if ((ctm == 0 || (ctm == 1 && out > 1)) && pow2) return ((float)o + 0.5f) * inv - 0.5f;
  return resize_src(o, scale, in, out, ctm);
}

// One output row's source rows (linear) or row (nearest), worked out once
// for all the outputs of a thread (they share oy).
struct ResizeRow {
  const float* r0;
  const float* r1;
  float ly;
};

__device__ __forceinline__ ResizeRow resize_row(const ResizeParams& p, const float* __restrict__ xc, int oy, float inv,
                                                bool pow2) {
  const float fy = resize_src_fast(oy, p.sy, inv, pow2, p.H, p.Ho, p.ctm);
  if (!p.linear) {
    const float* r = xc + nearest_idx(fy, p.nearest, p.H) * p.W;
    return {r, r, 0.f};
  }
  const float sy = fminf(fmaxf(fy, 0.f), (float)(p.H - 1));
  const int y0 = (int)sy, y1 = min(y0 + 1, p.H - 1);
  return {xc + y0 * p.W, xc + y1 * p.W, sy - (float)y0};
}

__device__ __forceinline__ float resize_col(const ResizeParams& p, const ResizeRow& rw, int ox, float inv, bool pow2) {
  const float fx = resize_src_fast(ox, p.sx, inv, pow2, p.W, p.Wo, p.ctm);
  if (!p.linear) return rw.r0[nearest_idx(fx, p.nearest, p.W)];
  const float sx = fminf(fmaxf(fx, 0.f), (float)(p.W - 1));
  const int x0 = (int)sx, x1 = min(x0 + 1, p.W - 1);
  const float ly = rw.ly, lx = sx - (float)x0;
  const float v00 = rw.r0[x0], v01 = rw.r0[x1], v10 = rw.r1[x0], v11 = rw.r1[x1];
  return (1.f - ly) * ((1.f - lx) * v00 + lx * v01) + ly * ((1.f - lx) * v10 + lx * v11);
}

__device__ __forceinline__ bool pow2f(float v) { return v > 0.f && (__float_as_uint(v) & 0x7FFFFFu) == 0; }

// Four consecutive outputs of one row per thread (rows of a multiple of 4:
// one index split and one source row per 4 outputs, one float4 store; other
// widths one output per thread), 32-bit index math — the flat 64-bit index's
// three 64-bit divisions per output were most of the old kernel's
// instructions.  The row's coordinate once per thread; the same arithmetic
// per output as before (a power-of-two scale's division is its reciprocal's
// multiplication, exactly).
template <bool QUAD>
__global__ __launch_bounds__(256) void k_resize(ResizeParams p) {
  const int total = p.N * p.C * p.Ho * p.Wo, step = QUAD ? 4 : 1;
  const float iy = 1.f / p.sy, ix = 1.f / p.sx;
  const bool py = pow2f(p.sy), px = pow2f(p.sx);
  for (long ol = (blockIdx.x * 256L + threadIdx.x) * step; ol < total; ol += gridDim.x * 256L * step) {
    const int o = (int)ol, ox = o % p.Wo, t = o / p.Wo, oy = t % p.Ho, nc = t / p.Ho;
    const float* xc = p.x + (long)nc * p.H * p.W;
    const ResizeRow rw = resize_row(p, xc, oy, iy, py);
    if constexpr (QUAD) {
      f4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = resize_col(p, rw, ox + e, ix, px);
      *reinterpret_cast<f4*>(p.y + o + (nc / p.C) * p.y_nx) = v;
    } else {
      p.y[o + (nc / p.C) * p.y_nx] = resize_col(p, rw, ox, ix, px);
    }
  }
}

// y[b][m][n] = act(alpha * sum_k A[b][m][k] B[b][k][n] + beta * c[m][n]) on
// v_mfma_f32_16x16x4_f32: one workgroup per 16 x 16 output tile, its four
// waves each taking a quarter of K (partial tiles summed through LDS in wave
// order: deterministic).  VEC (A rows and B columns contiguous in k — Gemm
// transB, MatMul with a constant B stored transposed, MatMulNBits' [N][K]
// weights — K % 4 == 0, 16-byte aligned): lane (r, g) loads float4
// A[m0 + r][k + 4g ..] and B[k + 4g ..][n0 + r] and issues 4 MFMAs, element e
// of both in MFMA e (every k once per 16); 8 such loads in flight per lane.
// Otherwise one element per lane per MFMA.  The SE blocks' [1, 1280] x
// [1280, 320] layers ran 214 us on the old one-thread-per-output kernel.
template <bool VEC>
__global__ __launch_bounds__(256) void k_gemm(GemmParams p, int tiles_m, int tiles_n) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int tile = blockIdx.x;
  const int bt = tile / (tiles_m * tiles_n), rem = tile - bt * tiles_m * tiles_n;
  const int m0 = (rem / tiles_n) * 16, n0 = (rem % tiles_n) * 16;
  const int m = m0 + r, nn = n0 + r;
  const bool m_ok = m < p.M, n_ok = nn < p.N;
  const float* a = p.a + bt * p.sab + (long)(m_ok ? m : 0) * p.sam;
  const float* b = p.b + bt * p.sbb + (long)(n_ok ? nn : 0) * p.sbn;
  const int kq = VEC ? ((p.K + 63) / 64) * 16 : ((p.K + 15) / 16) * 4;  // this wave's quarter of K
  const int kbeg = wave * kq, kend = min(p.K, kbeg + kq);
  f4 acc = f4{0.f, 0.f, 0.f, 0.f};
  if (VEC) {
    constexpr int U = 8;
    for (int k0 = kbeg; k0 < kend; k0 += 16 * U) {
      f4 av[U], bv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int k = k0 + 16 * u + 4 * g;
        const bool in = k < kend;
        av[u] = (in && m_ok) ? *reinterpret_cast<const f4*>(a + k) : f4{0.f, 0.f, 0.f, 0.f};
        bv[u] = (in && n_ok) ? *reinterpret_cast<const f4*>(b + k) : f4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (k0 + 16 * u >= kend) break;
#pragma unroll
        for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u][e], bv[u][e], acc, 0, 0, 0);
      }
    }
  } else {
    constexpr int U = 8;
    for (int k0 = kbeg; k0 < kend; k0 += 4 * U) {
      float av[U], bv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int k = k0 + 4 * u + g;
        const bool in = k < kend;
        av[u] = (in && m_ok) ? a[(long)k * p.sak] : 0.f;
        bv[u] = (in && n_ok) ? b[(long)k * p.sbk] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (k0 + 4 * u >= kend) break;
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], bv[u], acc, 0, 0, 0);
      }
    }
  }
  __shared__ f4 part[4][64];
  part[wave][lane] = acc;
  __syncthreads();
  if (wave != 0) return;
  acc = part[0][lane];
#pragma unroll
  for (int w2 = 1; w2 < 4; ++w2) acc += part[w2][lane];
  // acc[v] = D[row m0 + 4g + v][column n0 + r]
  if (!n_ok) return;
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    const int mm = m0 + 4 * g + v;
    if (mm >= p.M) continue;
    float y = p.alpha * acc[v];
    if (p.c) y += p.beta * p.c[mm * p.scm + nn * p.scn];
    p.y[((long)bt * p.M + mm) * p.N + nn] = act_apply(y, p.ep.act, p.ep.a0, p.ep.a1, p.ep.slope, nn, p.ep.slope_stride);
  }
}

bool gemm_vec(const GemmParams& p) {
  const auto al = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  return p.sak == 1 && p.sbk == 1 && p.K % 4 == 0 && p.sam % 4 == 0 && p.sbn % 4 == 0 && p.sab % 4 == 0 &&
         p.sbb % 4 == 0 && al(p.a) && al(p.b);
}


const char* binary_kernel_name(const BinParams& p) {
  return binary_planes(p) ? "void vso::k_binary_planes(vso::BinParams)" : "vso::k_binary(vso::BinParams)";
}
void launch_binary(const BinParams& p, hipStream_t s) {
  if (binary_planes(p))
    hipLaunchKernelGGL(k_binary_planes, dim3(grid_for(p.n / 4)), dim3(256), 0, s, p);
  else
    hipLaunchKernelGGL(k_binary, dim3(grid_for(p.n)), dim3(256), 0, s, p);
}
void launch_unary(const UnaryParams& p, hipStream_t s) {
  hipLaunchKernelGGL(k_unary, dim3(grid_for(p.n)), dim3(256), 0, s, p);
}
void launch_copy(const CopyParams& p, hipStream_t s) {
  hipLaunchKernelGGL(k_copy, dim3(grid_for(p.n)), dim3(256), 0, s, p);
}
void launch_pool(const PoolParams& p, hipStream_t s) {
  hipLaunchKernelGGL(k_pool, dim3(grid_for((long)p.N * p.C * p.Ho * p.Wo)), dim3(256), 0, s, p);
}
static bool gap_wave(const RowParams& p) {
  static const bool on = [] {
    const char* e = std::getenv("VSO_GAP_WAVE");
    return !e || std::atoi(e) != 0;
  }();
  return on && p.inner <= kGapWaveMax;
}
const char* gap_kernel_name(const RowParams& p) {
  return gap_wave(p) ? "void vso::k_gap_wave(vso::RowParams)" : "void vso::k_gap(vso::RowParams)";
}
void launch_gap(const RowParams& p, hipStream_t s) {
  if (gap_wave(p))
    hipLaunchKernelGGL(k_gap_wave, dim3((unsigned)((p.rows + 3) / 4)), dim3(256), 0, s, p);
  else
    hipLaunchKernelGGL(k_gap, dim3((unsigned)p.rows), dim3(256), 0, s, p);
}
void launch_norm_stats(const NormParams& p, hipStream_t s) {
  hipLaunchKernelGGL(k_norm_stats, dim3((unsigned)p.chunks, (unsigned)(p.N * p.C)), dim3(256), 0, s, p);
}
void launch_norm_apply(const NormParams& p, hipStream_t s) {
  hipLaunchKernelGGL(k_norm_apply, dim3((unsigned)p.chunks, (unsigned)(p.N * p.C)), dim3(256), 0, s, p);
}
void launch_softmax(const RowParams& p, hipStream_t s) {
  hipLaunchKernelGGL(k_softmax, dim3((unsigned)p.rows), dim3(256), 0, s, p);
}
void launch_affine(const AffineParams& p, hipStream_t s) {
  hipLaunchKernelGGL(k_affine, dim3(grid_for(p.n)), dim3(256), 0, s, p);
}
static bool resize_quad(const ResizeParams& p) {
  return (p.Wo & 3) == 0 && (reinterpret_cast<uintptr_t>(p.y) & 15) == 0;
}
const char* resize_kernel_name(const ResizeParams& p) {
  return resize_quad(p) ? "void vso::k_resize<true>(vso::ResizeParams)" : "void vso::k_resize<false>(vso::ResizeParams)";
}
void launch_resize(const ResizeParams& p, hipStream_t s) {
  const long total = (long)p.N * p.C * p.Ho * p.Wo;  // < 2^31: checked by the planner
  if (resize_quad(p))
    hipLaunchKernelGGL(k_resize<true>, dim3(grid_for(total / 4)), dim3(256), 0, s, p);
  else
    hipLaunchKernelGGL(k_resize<false>, dim3(grid_for(total)), dim3(256), 0, s, p);
}
void launch_gemm(const GemmParams& p, hipStream_t s) {
  const int tm = (p.M + 15) / 16, tn = (p.N + 15) / 16;
  const dim3 grid((unsigned)(tm * tn * p.batch));
  if (gemm_vec(p)) hipLaunchKernelGGL(k_gemm<true>, grid, dim3(256), 0, s, p, tm, tn);
  else hipLaunchKernelGGL(k_gemm<false>, grid, dim3(256), 0, s, p, tm, tn);
}

const char* gemm_kernel_name(const GemmParams& p) {
  return gemm_vec(p) ? "void vso::k_gemm<true>(vso::GemmParams, int, int)"
                     : "void vso::k_gemm<false>(vso::GemmParams, int, int)";
}

}  // namespace vso
