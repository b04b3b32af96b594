// vso_kernels.h — launch parameter blocks of the ONNX-session kernels
// (vso_kernels.hip), shared with the session planner (vso_model.hip).
// float32 NCHW tensors; plain structs passed by value.
#pragma once
#include <cstdint>
#include <vector>

#include <hip/hip_runtime.h>

namespace vso {

constexpr int kMaxDims = 6;

// Activations fused into the producing kernel's epilogue (and the unary kernel).
enum Act : int { ACT_NONE = 0, ACT_RELU = 1, ACT_CLIP = 2, ACT_PRELU = 3, ACT_LEAKY = 4, ACT_SIGMOID = 5, ACT_TANH = 6,
                 ACT_F16 = 7 /* Cast to float16: round to the nearest half (ties to even), kept as f32 */ };

struct Epilogue {
  const float* bias;   // [M] or null
  const float* res;    // residual added before the activation (same layout as y) or null
  int act;             // Act
  float a0, a1;        // CLIP lo/hi, LEAKY alpha
  const float* slope;  // PRELU: per output channel ([M]) or one value (slope_stride 0)
  int slope_stride;
  // res_mode 1: res is [N][res_c][Ho][Wo], channels >= res_c add 0 (an ONNX Pad
  // of the channel axis, fused); 2: res is [N][res_c][res_h][res_w] and the
  // value added is its 2x2 stride-2 max (a MaxPool, fused, then that Pad)
  int res_mode, res_c, res_h, res_w;
  int out_c, out_hw, out_w;  // the output's M, Ho*Wo, Wo (res_mode != 0)
  int act_c_end;             // > 0: the activation applies to channels < act_c_end only (an IBNorm's BN half)
};

// A depthwise convolution fused in front of a 1x1 one (k_conv_dwpw): `x` is
// the depthwise conv's input; its output — the 1x1's input — exists only in
// LDS.  Same FMA order and epilogue as k_conv_dw: the values k_conv_dw would
// have stored, bit for bit.
struct DwPre {
  const float* w;  // [C][kh][kw]; null: no fused producer
  int H, W;        // the depthwise input's size
  int kh, kw, sh, sw, dh, dw, pt, pl;
  Epilogue ep;     // bias / activation (no residual)
};

struct ConvParams {
  const float* x;  // [N][C][H][W]
  const float* w;  // [M][Cg][kh][kw]
  float* y;        // [N][M][Ho][Wo]
  int N, C, H, W, M, Ho, Wo;
  int G, Cg, Mg;   // groups, input / output channels per group
  int kh, kw, sh, sw, dh, dw, pt, pl;
  Epilogue ep;
  DwPre pre;       // k_conv_dwpw only (x is then the depthwise input)
  // extra output elements per image: y is a channel range of a wider
  // [N][ctot][Ho][Wo] tensor (a Concat input written in place), image n's
  // output at y + n * (M * Ho * Wo + y_nx); 0 = a tensor of its own
  long y_nx;
};

// Operand precision of the dense convolutions (vso_conv.hip; vso_options.conv_precision)
enum ConvPrec : int { PREC_F32 = 0, PREC_BF16 = 1, PREC_F16 = 2 };

// k_conv_tile's plan: tile shape, padding of the packed weights, K split
struct ConvTileShape {
  int prec, ks, s, th, tw, bm;
  int up;              // k_conv_tile_up: channels [up_c0, up_c1) upsampled from ConvTileParams::up
  int tiles_x, tiles;  // pixel tiles per tile row / per image
  int Mp, Cp;          // output channels padded to bm, input channels to 32
  int ksplit, cps;     // workgroups splitting the 32-channel chunks, chunks per split
};

struct ConvTileParams {
  ConvParams c;        // geometry, x, y, epilogue
  const void* wp;      // weights packed [kh*kw][Mp][Cp] in the operand type
  int Mp, Cp, tiles_x, tiles, mtiles, ksplit, cps;
  float* part;         // ksplit > 1: partial tiles [output block][ksplit][bm/16][th*tw/64][256 threads] as f4
  int* counters;       // ksplit > 1: arrivals per output block [N][M tiles][tiles], zero between runs
  // k_conv_tile_up: input channels [up_c0, up_c1) (whole 32-channel chunks)
  // are the 2x linear (half-pixel) upsample of up ([N][up_c1 - up_c0][up_H][up_W])
  const float* up;
  int up_c0, up_c1, up_H, up_W;
  // a Concat's last input read from its own tensor instead of copied into the
  // concatenation: channels [x2_c0, x2_c0 + x2_C) ([N][x2_C][H][W]; x2_c0 a
  // multiple of 32), or x2 = null
  const float* x2;
  int x2_c0, x2_C;
  int items;           // work items (pixel tile x M tile x image x split); set by launch_conv_tile
  int qskip;           // skip the loads of quads past C in a partial last chunk (VSO_CONV_QSKIP=0: off)
  int xcd;             // XCD-contiguous item order (k_conv_tile, ksplit 1; VSO_CONV_XCD=0: off)
};

constexpr int kDwPwMaxC = 256;  // channels a fused depthwise -> 1x1 pair may have

enum BinOp : int { BIN_ADD = 0, BIN_SUB = 1, BIN_MUL = 2, BIN_DIV = 3, BIN_PRELU = 4 };

struct BinParams {  // y = a (op) b with numpy broadcasting (strides 0 on broadcast dims)
  const float* a;
  const float* b;
  float* y;
  long n;
  int nd;
  int dims[kMaxDims];
  long sa[kMaxDims], sb[kMaxDims];
  int op;
};

struct UnaryParams {
  const float* x;
  float* y;
  long n;
  int act;
  float a0, a1;
};

// dst[dst_base + sum_d i_d * dst_stride_d] = src[src_base + sum_d c_d * src_stride_d]
// with c_d = i_d * step_d + start_d, or `fill` when some c_d is outside [0, lim_d):
// Transpose, Slice, Split, Concat (one launch per input), Pad.
struct CopyParams {
  const float* src;
  float* dst;
  long n;
  int nd;
  int size[kMaxDims];
  long dst_stride[kMaxDims], src_stride[kMaxDims];
  int start[kMaxDims], step[kMaxDims], lim[kMaxDims];
  long dst_base, src_base;
  float fill;
};

// dst[dst_base + r * dst_row + i] = src[src_base + r * src_row + i], i < inner,
// r < rows: a Concat / Split / Slice of whole trailing dimensions
struct RowCopyParams {
  const float* src;
  float* dst;
  long inner, rows, src_row, dst_row, src_base, dst_base;
};

struct PoolParams {
  const float* x;
  float* y;
  int N, C, H, W, Ho, Wo, kh, kw, sh, sw, dh, dw, pt, pl;
  int max_mode;           // 1 max, 0 average
  int count_include_pad;
};

struct RowParams {  // per-row reductions over `inner` contiguous elements (rows = N*C)
  const float* x;
  float* y;
  long rows, inner;
  const float* scale;  // InstanceNormalization gamma [C] (rows % C), beta
  const float* shift;
  int C;
  float eps;
};

// InstanceNormalization of N*C planes of `inner` elements, plane (n, c) at
// x + (n * ctot + c0 + c) * inner (c0 / ctot: an IBNorm's InstanceNorm half
// of a convolution's output, normalised in place), in two parallel passes:
// k_norm_stats writes each `chunk`-element piece's (mean, M2, count), then
// k_norm_apply merges a plane's pieces in order (Chan et al.) and normalises
// its piece, with an optional Relu.
struct NormParams {
  const float* x;
  float* y;  // addressed as x (may be x)
  int N, C, c0, ctot;
  long inner;
  const float* scale;  // [C]
  const float* shift;
  float eps;
  int act;             // ACT_NONE or ACT_RELU
  float* stats;        // [N*C][chunks][3]
  int chunks, chunk;
};

struct AffineParams {  // y = x * scale[c] + shift[c] over NC(HW)
  const float* x;
  float* y;
  long n, inner;
  int C;
  const float* scale;
  const float* shift;
};

// Resize of [N][C][H][W] -> [N][C][Ho][Wo]; ctm: 0 half_pixel, 1 pytorch_half_pixel,
// 2 align_corners, 3 asymmetric; nearest: 0 round_prefer_floor, 1 round_prefer_ceil, 2 floor, 3 ceil
struct ResizeParams {
  const float* x;
  float* y;
  int N, C, H, W, Ho, Wo;
  float sy, sx;  // scales (output / input)
  int linear, ctm, nearest;
  long y_nx;     // as ConvParams::y_nx (C * Ho * Wo + y_nx elements per image)
};

constexpr long kGapWaveMax = 1024;  // k_gap_wave: planes of at most this many elements
struct GemmParams {  // y[b][m][n] = alpha * sum_k A[b][m][k] B[b][k][n] + beta * c
  const float* a;
  const float* b;
  const float* c;     // broadcast over (m, n) with strides cm, cn (0 = broadcast) or null
  float* y;
  int batch, M, N, K;
  long sab, sam, sak;  // A strides (batch, m, k)
  long sbb, sbk, sbn;  // B strides
  long scm, scn;
  float alpha, beta;
  Epilogue ep;         // act only
};

// A MobileNetV2 inverted residual block — 1x1 expand + Clip -> 3x3 depthwise
// (stride 1 / 2) + Clip -> 1x1 project (+ the block input) — in one launch
// (vso_ir.hip, k_ir): output tiles of kIrTH x 16 pixels, all output channels,
// a slice of the hidden channels per workgroup (ks slices of cps 16-channel
// chunks, the partial tiles summed in slice order by the last to arrive).
constexpr int kIrTH = 4;
struct IrParams {
  const float* x;     // [N][CIN][H][W]
  const float* w1;    // [HID][CIN], b1 [HID]: expand, then clip to [lo1, hi1]
  const float* b1;
  const float* wdw;   // [9][HID] (tap-major), bdw [HID]: depthwise, then clip to [lo2, hi2]
  const float* bdw;
  const float* w2;    // [COUT][HID], b2 [COUT]: project
  const float* b2;
  // b16 (k_ir_b16, bf16 / f16 sessions): each hidden-channel slice's weights
  // as one contiguous block of sl_bytes (ir_slab_build: the 1x1 weights split
  // into bf16 hi / lo planes in the MFMA operand order, rows padded for
  // conflict-free LDS reads, then the depthwise taps and biases in f32),
  // copied into LDS by the workgroup's prologue; o_*: byte offsets of the
  // parts, s1 / s2: 16-byte slots per W1 / W2 row, o_hid: the hidden planes
  const unsigned char* slab;
  int b16, sl_bytes, o_w1l, o_w2h, o_w2l, o_wd, o_bd, o_b1, o_hid, s1, s2;
  int wv;     // b16 with CIN <= 64: the wave-private form (k_ir_b16w; opt-in, VSO_IR_WAVE=1)
  int probe;  // timing probes (VSO_IR_PROBE, results invalid): 1 no slab DMA, 2 no x loads,
              // 4 no expand MFMAs, 8 no project MFMAs, 16 no split-K exchange
  float* y;           // [N][COUT][Ho][Wo], image n at y + n * (COUT * Ho * Wo + y_nx)
  long y_nx;
  int N, CIN, H, W, HID, COUT, Ho, Wo, stride, res;  // res: + x (stride 1, CIN == COUT)
  float lo1, hi1, lo2, hi2;
  int pstr;           // floats between the staged input channels' rows in LDS (ir_pstr)
  int tiles_x, tiles; // output tiles per tile row / per image (ir_tiles)
  int ks, cps;        // hidden-channel slices per tile, 16-channel chunks per slice
  float* part;        // ks > 1: the slices' partial sums [ks][N][COUT][Ho][Wo] (k_ir_reduce adds them)
};
bool ir_supported(const IrParams& p);
int ir_pstr(int stride);
size_t ir_lds_bytes(const IrParams& p);
// b16: choose the slices (p->cps / ks, LDS budget and ~wgs workgroups) and the
// slab's layout (p->sl_bytes, offsets); then ir_slab_build writes every
// slice's block: w1 [HID][CIN], b1 [HID], wdt [9][HID] (tap-major), bd [HID],
// w2 [COUT][HID]
bool ir_slab_plan(IrParams* p, long wgs, int cps_target);
void ir_slab_build(const IrParams& p, const float* w1, const float* b1, const float* wdt, const float* bd,
                   const float* w2, std::vector<unsigned char>* out);
void ir_tiles(int Ho, int Wo, int* tiles_x, int* tiles);
const char* ir_kernel_name(const IrParams& p);
void launch_ir(const IrParams& p, hipStream_t s);
void launch_ir_reduce(const IrParams& p, hipStream_t s);  // ks > 1: the launch after launch_ir

const char* conv_kernel_name(const ConvParams& p);
// a depthwise -> 1x1 pair of N images of P pixels into M channels runs fused
// on k_conv_pw (vso_kernels.hip: where that measured faster)
bool pw_fused_pays(int N, long P, int M);
// the same decision with pw_kernel's 32-bit offset limits: a C-channel depthwise
// over pre_hw input pixels per image into P output pixels, then 1x1 to M
// channels — what the planner must ask before deferring a depthwise whose
// channels exceed k_conv_dwpw's LDS tile (kDwPwMaxC)
bool pw_pair_fits(int N, long C, long pre_hw, long P, int M);
// false: not a k_conv_tile convolution (grouped, dilated, other kernel sizes)
bool conv_tile_shape(const ConvParams& p, int prec, ConvTileShape* sh);
const char* conv_tile_name(const ConvTileShape& t);
void launch_conv_tile(const ConvTileParams& p, const ConvTileShape& t, hipStream_t s);

void launch_conv(const ConvParams& p, hipStream_t s, const char** name);

// k_conv_thin: a 1x1 convolution to at most kThinMaxM output channels (a
// matte / logit head) — a per-pixel dot product over the input channels on
// the VALU, 4 pixels per thread — optionally normalising input channels
// [norm.c0, norm.c0 + norm.C) on the way in: an InstanceNorm (+ Relu) whose
// statistics k_norm_stats computed (NormParams, its apply step not launched:
// the IBNorm in front of MODNet's matte head)
constexpr int kThinMaxM = 4;
bool thin_conv_fits(const ConvParams& p);
void launch_conv_thin(const ConvParams& p, const NormParams* norm, hipStream_t s);
const char* conv_thin_name(int M);
void launch_binary(const BinParams& p, hipStream_t s);
void launch_unary(const UnaryParams& p, hipStream_t s);
void launch_copy(const CopyParams& p, hipStream_t s);
void launch_copy_rows(const RowCopyParams& p, hipStream_t s);
const char* row_copy_name(const RowCopyParams& p);
void launch_pool(const PoolParams& p, hipStream_t s);
void launch_gap(const RowParams& p, hipStream_t s);
void launch_norm_stats(const NormParams& p, hipStream_t s);
void launch_norm_apply(const NormParams& p, hipStream_t s);
// k_norm_plane: statistics and apply of planes up to kNormPlaneMax elements in one launch
constexpr long kNormPlaneMax = 36864;
bool norm_plane_fits(long inner);
const char* norm_plane_name(long inner);
void launch_norm_plane(const NormParams& p, hipStream_t s);
constexpr int kNormChunk = 4096;  // elements per k_norm_stats / k_norm_apply workgroup
void launch_softmax(const RowParams& p, hipStream_t s);
void launch_affine(const AffineParams& p, hipStream_t s);
const char* resize_kernel_name(const ResizeParams& p);  // the kernel launch_resize picks (profiles)
void launch_resize(const ResizeParams& p, hipStream_t s);
void launch_gemm(const GemmParams& p, hipStream_t s);
bool gemm_vec(const GemmParams& p);
const char* binary_kernel_name(const BinParams& p);
const char* gap_kernel_name(const RowParams& p);
const char* gemm_kernel_name(const GemmParams& p);

}  // namespace vso
