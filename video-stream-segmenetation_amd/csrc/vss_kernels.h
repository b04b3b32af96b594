// vss_kernels.h — launch parameter blocks shared by the HIP kernels
// (vss_kernels.hip) and the host planner (vss_capi.hip).  Plain structs
// passed by value as kernel arguments; no torch types anywhere.
#pragma once
#include <cstddef>
#include <cstdint>

namespace vss {

// Arithmetic used for the pointwise (1x1) GEMMs.
//   PREC_F32    : v_mfma_f32_16x16x4_f32 (exact f32 fma chain)
//   PREC_BF16X2 : v_mfma_f32_16x16x32_bf16 on a hi+lo bf16 split of the f32
//                 activation against bf16-exact weights (K=16 per MFMA)
//   PREC_BF16   : same MFMA, activations rounded to bf16 (lo dropped) — the
//                 lossy "pure bf16" mode; parity only vs the bf16-emulating oracle
enum Prec : int { PREC_F32 = 0, PREC_BF16X2 = 1, PREC_BF16 = 2 };

enum BlockMode : int { MODE_IR_EXPAND = 0, MODE_IR_DIRECT = 1, MODE_DEC = 2 };

constexpr int kThreads = 256;       // 4 wave64 per workgroup
constexpr int kMaxProjTiles = 8;    // 16x16 project tiles per wave (cout/16 * pout/16 / 4)

// Fused block: [prologue: stage X tile (or upsample+concat)] ->
//   for each 16-channel chunk c0 of the hidden/concat dim:
//     (expand pw on MFMA) -> dw3x3 (VALU) -> project pw accumulate (MFMA)
//   -> epilogue (bias, residual, store, instance-norm partial stats)
struct BlockParams {
  const float* x;        // IR input [N][H][W][cin]   | DEC low-res src [N][h][w][cin]
  const float* skip;     // DEC skip [N][Ho][Wo][cskip]
  float* y;              // output [N][Ho][Wo][cout]
  // weights (row-major [rows][K]); f32 or bf16 bits depending on prec
  const void* w1;        // expand [chid][cin]
  const float* b1;       // [chid]
  const float* wdw;      // [chid or ccat][9]
  const float* bdw;
  const void* w2;        // project [cout][chid or ccat]
  const float* b2;       // [cout]
  // instance norm on the input (DEC whose src is DEC): src partial stats
  const float* in_part;  // [N][in_tiles][2][cin]
  const float* in_gamma;
  const float* in_beta;
  int in_tiles;          // tiles per frame of the producer
  int in_hw;             // pixels per frame of the producer
  float eps;
  // instance norm stats of this layer's output (DEC)
  float* out_part;       // [N][tiles_y*tiles_x][2][cout]
  int N, H, W;           // input spatial (IR: x dims; DEC: skip/output dims)
  int Ho, Wo;            // output spatial
  int cin, cskip, chid, cout;   // chid = hidden (IR expand) or channels fed to dw
  int stride;
  int relu6_dw;          // IR: relu6 after dw; DEC: none
  int residual;
  int TH, TW;            // output tile
  int tiles_x, tiles_y;
  int norm_in;           // DEC: src needs norm+relu
};

struct StemParams {
  const uint8_t* frames; // [N] frames, row_stride / frame_stride bytes
  long row_stride, frame_stride;
  int fh, fw, fc;        // frame geometry, fc = 3 or 4
  int Hm, Wm;            // model input resolution
  float ry, rx;          // (float)((double)fh/Hm), (float)((double)fw/Wm)
  const float* w;        // [cout][3][3][3]
  const float* b;
  float* y;              // [N][Ho][Wo][cout]
  int Ho, Wo, cout;
};

struct HeadParams {
  const float* x;        // pre-norm dec output [N][h][w][cin]
  const float* in_part;  // [N][in_tiles][2][cin]
  const float* gamma;
  const float* beta;
  int in_tiles;
  float eps;
  const float* w;        // [cin]
  float b;
  float* mask;           // [N][Hm][Wm] f32
  int N, h, w_, cin;
  int Hm, Wm;
};

struct PrepParams {      // standalone preprocess: frames -> [N][3][Hm][Wm] f32
  const uint8_t* frames;
  long row_stride, frame_stride;
  int fh, fw, fc;
  int Hm, Wm;
  float ry, rx;
  float* out;
  int N;
};

}  // namespace vss
