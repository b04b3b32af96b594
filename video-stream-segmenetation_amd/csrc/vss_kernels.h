// vss_kernels.h — launch parameter blocks shared by the HIP kernels
// (vss_kernels.hip) and the host planner (vss_capi.hip).  Plain structs
// passed by value as kernel arguments; no torch types anywhere.
#pragma once
#include <cstddef>
#include <cstdint>

#include <hip/hip_runtime.h>

namespace vss {

// Arithmetic used for the pointwise (1x1) GEMMs.
//   PREC_F32    : v_mfma_f32_16x16x4_f32 (exact f32 fma chain)
//   PREC_BF16X2 : v_mfma_f32_16x16x32_bf16 on a hi+lo bf16 split of the f32
//                 activation against bf16-exact weights (K=16 per MFMA)
//   PREC_BF16   : same MFMA, activations rounded to bf16 (lo dropped) — the
//                 lossy "pure bf16" mode; parity only vs the bf16-emulating oracle
enum Prec : int { PREC_F32 = 0, PREC_BF16X2 = 1, PREC_BF16 = 2 };

enum BlockMode : int { MODE_IR_EXPAND = 0, MODE_IR_DIRECT = 1, MODE_DEC = 2 };

// k_block FLAGS: bit 0 the decoder's src needs instance norm + ReLU, bit 1
// residual add, bits 2-3 XP-1, bits 4-5 SP-1, bits 6-7 KS-1, bit 8 STEM_IN where
//   STEM_IN = the block's input is the stem's output, computed in the block's
//        prologue from the frame (stem fused into its only consumer: one launch
//        and one HBM round trip fewer); the block still writes the stem
//        activation's tile so every layer stays readable;
//   KS = hidden-channel split of this (expand) layer: KS workgroups per tile,
//        slice s owns hidden channels [s*chid/KS, (s+1)*chid/KS) and writes
//        its partial project sum to part s of the output (bias and residual
//        in part 0): deep low-res layers get KS x the workgroups and 1/KS of
//        the weights per workgroup;
//   XP / SP = parts of the x / skip input, summed in part order (fixed, so
//        results never depend on the tiling) as the prologue loads them.
__host__ __device__ constexpr int block_flags(int norm_in, int residual, int xp, int sp, int ks, int stem_in = 0) {
  return (norm_in ? 1 : 0) | (residual ? 2 : 0) | ((xp - 1) << 2) | ((sp - 1) << 4) | ((ks - 1) << 6) |
         (stem_in ? 256 : 0);
}
__host__ __device__ constexpr bool flags_stem_in(int f) { return (f & 256) != 0; }
__host__ __device__ constexpr int flags_xp(int f) { return ((f >> 2) & 3) + 1; }
__host__ __device__ constexpr int flags_sp(int f) { return ((f >> 4) & 3) + 1; }
__host__ __device__ constexpr int flags_ks(int f) { return ((f >> 6) & 3) + 1; }

constexpr int kThreads = 256;       // 4 wave64 per workgroup
// gfx950 allocates LDS to workgroups in 2 KiB granules, 80 per CU (measured:
// tools/micro/lds_resident.cpp; hipOccupancyMaxActiveBlocksPerMultiprocessor
// assumes a finer granule and reports 3 per CU up to 54,613 B where only
// 53,248 B fit three)
constexpr int kLdsGranule = 2048, kLdsGranulesPerCu = 80;
__host__ __device__ constexpr int lds_wg_per_cu(int bytes) {
  return kLdsGranulesPerCu / ((bytes + kLdsGranule - 1) / kLdsGranule);
}
constexpr int kMaxAcc = 16;         // 16x16 project accumulators per wave
// LDS layout of the input tile and the expand waves' hidden chunks.  Measured
// (round 2, tools/lds_model.py + tools/micro/lds_taps.cpp + tools/ab_pinned.sh):
// gfx950's ds_read_b128 serves lane groups {0-3,12-15,20-27}, {4-11,16-19,28-31}
// (and +32), so a 16-pixel block read with a pixel stride of 5 or 13 bank quads
// (the padding below) is 2-way conflicted.  A layout that is conflict-free for
// every depthwise tap (VSS_PERM=1: lanes {0-3,12-15} take pixels 0-7, lanes
// {4-11} pixels 8-15; VSS_XS_PAD=8 and VSS_HS1=24: 2 mod 4 quads per pixel)
// has 4.5x fewer conflict cycles (model; SQ_LDS_BANK_CONFLICT agreed within
// 5 %) and makes the tap reads alone 1.6x faster, but its extra LDS costs
// occupancy (LDS is allocated in 2 KiB granules, 80 per CU — d3's 6x16 tile
// went from 3 to 2 workgroups per CU at 53,952 B) and the whole layers
// measured equal or slower except d2 (-5 %): the default stays the tight one.
#ifndef VSS_PERM
#define VSS_PERM 0
#endif
#ifndef VSS_XS_PAD
#define VSS_XS_PAD 4
#endif
#ifndef VSS_HS1
#define VSS_HS1 20
#endif
// decoders with even tiles upsample by 2x2 quads (VSS_QUADS=0: per pixel,
// from tap records, as odd tiles always do — an A/B knob)
#ifndef VSS_QUADS
#define VSS_QUADS 1
#endif
__host__ __device__ constexpr int block_pix(int r) { return VSS_PERM ? (r < 4 ? r : (r < 12 ? r + 4 : r - 8)) : r; }
// floats per pixel of an expand wave's hidden chunk in LDS (16 channels + pad)
// (the padded layout, VSS_SWZ=0)
__host__ __device__ constexpr int hid_stride(int stride) { return stride == 2 ? 20 : VSS_HS1; }

// Bank-conflict-free LDS layouts (round 5, VSS_SWZ=1; tools/lds_sites.py models
// every access site lane by lane against gfx950's bank rules).  The access
// pattern that sets them: a ds_read_b128 of a 16-pixel block, lane (r, g) =
// pixel r, channel quad g, is served in lane groups {0-3,12-15,20-27},
// {4-11,16-19,28-31} (+32) over 64 banks (16 bank quads); a pixel stride of
// 5 or 13 quads — the +4 float pads — is 2-way conflicted, and a plain 16-B
// write (8 contiguous lanes, 32 banks) wants the opposite of what the reads
// want from a pad.  Three layouts, no padding:
//  * quad-major planes ("QM"): quad q of pixel p at q * PLANE + 4 p floats.  A
//    lane group's 16 pixels are consecutive quads of one or two planes; with
//    PLANE a multiple of 16 quads the two channel quads of a group fall on
//    complementary pixel sets, so a run of 16 consecutive pixels is
//    conflict-free, and so is a write of 8 consecutive pixels of one plane —
//    at any pixel offset, so the taps keep immediate offsets (no VALU).
//    Stride-2 taps read every other pixel: their planes are PLANE + 1 quads
//    apart.  For b1's input tile and every expand layer's hidden chunk;
//  * XOR-swizzled pixel-major ("SW"): quad q of pixel p at p * CX + 4 (q ^
//    gray(p) % M), M = the largest power of two dividing the pixel's quads
//    (<= 16).  For the expand layers' input tile (the MFMA B reads take
//    pixel cb * 16 + r, whose swizzle is the lane's own for M <= 8), the
//    epilogue slabs and the residual centre;
//  * the decoders with 16-wide tiles keep pixel-major rows padded to 8 mod 16
//    floats (2 mod 4 quads: conflict-free for runs of 16 pixels).
#ifndef VSS_SWZ
#define VSS_SWZ 1
#endif
__host__ __device__ constexpr int pow2div16(int q) {
  return q % 16 == 0 ? 16 : (q % 8 == 0 ? 8 : (q % 4 == 0 ? 4 : (q % 2 == 0 ? 2 : 1)));
}
__host__ __device__ constexpr int gray_swz(int pix, int m) { return (pix ^ (pix >> 1)) & (m - 1); }
constexpr int kAccSlots = 4;        // instance-norm accumulator slots per frame and layer
                                    // (spreads the producers' atomics over 16x the cache lines)

__host__ __device__ constexpr int r4(int v) { return (v + 3) & ~3; }
__host__ __device__ constexpr int cmax(int a, int b) { return a > b ? a : b; }

// dw pixel runs: the output pixels of XR consecutive pixel blocks are dealt
// to lanes in horizontal runs — lane r of a "super-block" evaluates the XR
// adjacent pixels (row, c0 .. c0 + XR - 1) — so the 3 x 3 taps those pixels
// share are read from LDS once: per tap row STRIDE * (XR - 1) + 3 reads for
// XR pixels instead of 3 * XR (stride 1, XR = 4: 18 reads per 4 pixels, not
// 36).  Element j of the run is pixel block sb * XR + j's column r, so the
// MFMAs still take one 16-pixel block per call, and every output pixel's
// arithmetic is unchanged (bitwise the same activations for any XR / tile).
// XR = the largest of 4, 2, 1 that tiles the TW-wide rows and deals evenly
// to the PW pixel-block groups of waves.
__host__ __device__ constexpr int dw_run(int TW, int NPB, int PW) {
  return (TW % 4 == 0 && 16 % (TW / 4) == 0 && NPB % 4 == 0 && (NPB / 4) % PW == 0)   ? 4
         : (TW % 2 == 0 && 16 % (TW / 2) == 0 && NPB % 2 == 0 && (NPB / 2) % PW == 0) ? 2
                                                                                      : 1;
}

// Geometry + LDS carve (floats) of one k_block instantiation.  Evaluated at
// compile time in the kernel and at run time by the host planner, so the two
// can never disagree.  Every region is a multiple of 4 floats (16-B aligned).
struct BlockLds {
  int IH, IW, P_in, P_in_pad, P_out, CX, XS, LD1, LD2, SR, SC;
  // layouts (VSS_SWZ): XQM = xt quad-major (plane XPL floats; XS = 4 then),
  // XSW / RSW / XRW = the xt / slab / residual-centre swizzle modulus (1 = none),
  // HPL = the hidden chunk's plane (floats; 0 = the padded pixel-major chunk)
  bool XQM;
  int XPL, XSW, HPL, RS, RSW, XRW;
  int NCB, NPB, NCHUNK, PW, CS, NPBW, NACC;  // CS = chunk groups, PW = pixel-block groups
  int xt, xr, w1, w2, wdw, bdw, b1, b2, wimg_end, lr, nrm, uc, work, stt, total;  // [w1, wimg_end): the weight image
  int slab_stride;  // floats per wave slab = P_out * (cout + 4)
  int slab;         // the epilogue's accumulator slabs: the work region, or (decoder) the input tile
};

// Row pitch (floats) of the fused stem's resized region x0 [3][2*IH+1][XWP]:
// its XW = 2*IW+1 columns are written two per thread, columns lx and lx + HW2
// (HW2 = (XW+1)/2) of row ly by thread ly*HW2 + lx, so a pitch = HW2 mod 32
// makes consecutive threads hit consecutive banks (ds_write_b32: 32 banks);
// being odd it also puts the stem MFMA's paired taps on opposite bank parities
// (tools/lds_sites.py: 125 -> 19 conflict cycles per b1 wave with the rest of
// the round-5 layouts).  VSS_SWZ=0: XW + 1.
__host__ __device__ constexpr int stem_xwp(int IW) {
  if (!VSS_SWZ) return 2 * IW + 2;
  const int xw = 2 * IW + 1, hw2 = IW + 1;
  int x = xw;
  while ((x - hw2) % 32 != 0) ++x;
  return x;
}
// LDS the fused stem needs (x0 region [3][2*IH+1][stem_xwp(IW)] + stem weights), in the work region
__host__ __device__ constexpr int stem_in_lds(int IH, int IW) {
  return r4(3 * (2 * IH + 1) * stem_xwp(IW)) + 27 * 16 + 16;
}

__host__ __device__ constexpr BlockLds block_lds(int mode, int stride, int TH, int TW, int cin, int cskip, int chid,
                                                 int cout, int stem_in = 0) {
  BlockLds L{};
  L.IH = stride == 2 ? 2 * TH + 1 : TH + 2;
  L.IW = stride == 2 ? 2 * TW + 1 : TW + 2;
  L.P_in = L.IH * L.IW;
  L.P_in_pad = (L.P_in + 15) & ~15;
  L.P_out = TH * TW;
  L.CX = mode == 2 /*MODE_DEC*/ ? cin + cskip : cin;
  L.XQM = VSS_SWZ && mode == 1;
  L.XS = !VSS_SWZ ? L.CX + VSS_XS_PAD : (L.XQM ? 4 : (mode == 2 ? L.CX + (TW == 16 ? 8 : VSS_XS_PAD) : L.CX));
  L.XPL = L.XQM ? 4 * L.P_in_pad : 0;
  L.XSW = VSS_SWZ && mode == 0 ? pow2div16(L.CX / 4) : 1;

  L.RS = VSS_SWZ ? cout : cout + 4;
  L.RSW = VSS_SWZ ? pow2div16(cout / 4) : 1;
  L.XRW = VSS_SWZ ? pow2div16(cin / 4) : 1;
  L.LD1 = cin + 8;   // bf16 elements per W1 row in LDS (16-B aligned rows)
  L.LD2 = chid + 8;  // bf16 elements per W2 row
  L.SR = (TH + 1) / 2 + 3;
  L.SC = (TW + 1) / 2 + 3;
  L.NCB = cout / 16;
  L.NPB = L.P_out / 16;
  L.NCHUNK = chid / 16;
  // work split: the 16-channel chunks are dealt to CS = GC groups of waves,
  // GC in {1, 2, 4} fixed by the channel count alone (so the order in which a
  // pixel's partial sums are added never depends on the tile: results are
  // bitwise identical for every tile the planner may pick); the remaining
  // PW = 4 / GC waves of a group split the pixel blocks.  EXPAND has GC = 4.
  L.CS = L.NCHUNK >= 4 ? 4 : (L.NCHUNK >= 2 ? 2 : 1);
  L.PW = 4 / L.CS;
  L.NPBW = L.NPB / L.PW;
  L.NACC = L.NPBW * L.NCB;
  // the hidden chunk quad-major where the dw reads runs of 16 pixels (XR = 1);
  // the 2- and 4-pixel runs of XR > 1 meet its planes 4-way: they keep HSD
  L.HPL = VSS_SWZ && mode == 0 && dw_run(TW, L.NPB, 1) == 1 ? 4 * (L.P_in_pad + (stride == 2 ? 1 : 0)) : 0;
  L.slab_stride = L.P_out * L.RS;
  const int xt_floats = L.XQM ? L.P_in_pad * L.CX : r4(L.P_in_pad * L.XS);
  int o = 0;
  L.xt = o;  o += xt_floats;
  // expand blocks keep xt as MFMA operands (bf16 hi/lo pairs in the split
  // mode); the residual-capable shape keeps the exact f32 centre here
  L.xr = o;  o += (mode == 0 && stride == 1 && cin == cout) ? r4(L.P_out * cin) : 0;
  L.w1 = o;  o += mode == 0 ? r4(chid * L.LD1 / 2) : 0;
  L.w2 = o;  o += r4(cout * L.LD2 / 2);
  L.wdw = o; o += r4(9 * chid);
  L.bdw = o; o += r4(chid);
  L.b1 = o;  o += mode == 0 ? r4(chid) : 0;
  L.b2 = o;  o += r4(cout);
  L.wimg_end = o;
  // per-wave scratch during the main loop (expand: each wave's hidden chunk
  // over the input tile), reused as the accumulator slabs after it.  The
  // decoder's main loop needs no scratch: its slabs go into the input tile
  // xt (dead once the main loop is done) when they fit, and its low-res src
  // region (read only in the prologue) then shares the work region with the
  // epilogue's stats scratch (int64 pairs, 1024 floats); the decoder stages
  // the src's norm slots in xt before the input tile is committed.  (Slabs in
  // xt: d2 50 -> 39 KB of LDS, four workgroups per CU instead of three.)
  const bool slab_in_xt = mode == 2 && L.CS * L.slab_stride <= xt_floats;
  L.work = o;
  L.lr = o;
  const int hid_floats = L.HPL ? 4 * 4 * L.HPL : 4 * L.P_in_pad * hid_stride(stride);  // 4 waves
  o += cmax(cmax(cmax(mode == 0 ? hid_floats : 1024, slab_in_xt ? 0 : L.CS * L.slab_stride),
                 mode == 2 ? r4(L.SR * L.SC * cin) : 0),
            stem_in ? stem_in_lds(L.IH, L.IW) : 0);
  L.nrm = o; o += mode == 2 ? r4(2 * cin) : 0;
  // decoder: per input-tile pixel, its 2x-upsample taps (four lr offsets as
  // u16 pairs, ly1, lx1), built while the prologue loads are in flight — only
  // for tiles with an odd side; even tiles upsample by 2x2 quads (dec_quads)
  L.uc = o;  o += (mode == 2 && (!VSS_QUADS || TH % 2 || TW % 2)) ? 4 * L.P_in_pad : 0;
  L.slab = slab_in_xt ? L.xt : L.work;
  L.stt = slab_in_xt ? L.work : L.xt;
  L.total = o;
  return L;
}

// Fused block: [prologue: stage X tile (or upsample+concat)] ->
//   for each 16-channel chunk c0 of the hidden/concat dim:
//     (expand pw on MFMA) -> dw3x3 (VALU) -> project pw accumulate (MFMA)
//   -> epilogue (bias, residual, store, instance-norm partial stats)
// Opt-in phase trace (make trace -> libvss_trace.so; never in the product
// build): thread 0 of every workgroup stamps s_memrealtime (100 MHz, one
// clock for the whole device) at: 0 start, 1 prologue committed, 2 main
// done, 3 end, 4 every prologue load landed, 5 decoder src norm ready, 6
// every prologue load issued; slots 8-15 the same points in shader clocks
// (s_memtime), so the trace also gives the core clock.
// (Layer launches only: the persistent forward, COH = true, stamps nothing.)
#ifdef VSS_TRACE
#define VSS_TRACE_FIELD unsigned long long* trace;
#define VSS_STAMP(k)                                                                                  \
  do {                                                                                                \
    if constexpr (!COH) {                                                                             \
      if (threadIdx.x == 0 && p.trace) {                                                              \
        unsigned long long* t_ = p.trace + (((long)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x) * 16; \
        t_[(k)] = __builtin_amdgcn_s_memrealtime();                                                   \
        t_[8 + (k)] = __builtin_amdgcn_s_memtime();                                                   \
        if ((k) == 0) {                                                                               \
          /* where the workgroup runs: HW_ID (cu, sh, se, ...) and XCC_ID */                          \
          t_[7] = __builtin_amdgcn_s_getreg((31 << 11) | 4);                                          \
          t_[15] = __builtin_amdgcn_s_getreg((15 << 11) | 20);                                        \
        }                                                                                             \
      }                                                                                               \
    }                                                                                                 \
  } while (0)
#else
#define VSS_TRACE_FIELD
#define VSS_STAMP(k) \
  do {               \
  } while (0)
#endif

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
  unsigned long long* acc_zero;  // all decoder norm accumulators [N][acc_stride]: zeroed here
  int acc_stride;
  VSS_TRACE_FIELD
};

struct BlockParams {
  const float* wimg;     // the layer's LDS weight image (block_lds regions w1..b2), built by the host;
                         // with KS > 1 one image per hidden slice, wimg_stride floats apart
  long wimg_stride;
  long x_part_stride;    // floats between the parts of x / skip / y (see block_flags)
  long skip_part_stride;
  long y_part_stride;
  const float* x;        // IR input [N][H][W][cin]   | DEC low-res src [N][h][w][cin]
  const float* skip;     // DEC skip [N][Ho][Wo][cskip]
  float* y;              // output [N][Ho][Wo][cout]
  // Instance norm, exact and order-free: every decoder workgroup adds the
  // fixed-point sums of its tile's outputs (sum v*2^32, sum v^2*2^24, int64)
  // to its frame's accumulator with device-scope atomics; the consumer (the
  // next kernel) turns the totals into scale/shift.  The stem kernel zeroes
  // the accumulators of every frame at the start of each forward.
  const unsigned long long* in_acc;  // DEC with norm_in: src accumulator [N][acc_stride] + src offset,
                                     // kAccSlots slots of [2][cin] (sum, sum of squares)
  const float* in_gamma;             // src layer's norm affine [cin]
  const float* in_beta;
  int in_hw;                         // pixels per frame of the src
  double in_inv_hw;                  // 1 / in_hw
  unsigned long long* out_acc;       // DEC: this layer's accumulator [N][acc_stride] + offset
                                     // (kAccSlots slots of [2][cout]; workgroup -> slot tile % kAccSlots)
  int acc_stride;                    // int64 elements per frame over all decoder layers
  float eps;
  int N, H, W;           // input spatial (IR: x dims; DEC: skip/output dims)
  int Ho, Wo;            // output spatial
  int cin, cskip, chid, cout;   // chid = hidden (IR expand) or channels fed to dw
  int stride;
  int relu6_dw;          // IR: relu6 after dw; DEC: none
  int residual;
  int TH, TW;            // output tile
  int tiles_x, tiles_y;
  int norm_in;           // DEC: src needs norm+relu
  StemParams stem;       // STEM_IN: the fused stem (frames of this call, stem weights, its output y)
  VSS_TRACE_FIELD
};

using BlockFn = void (*)(BlockParams);

// One compiled k_block shape (tools/gen_registry.py -> vss_registry.inc).
// flags: block_flags().
struct BlockEntry {
  int mode, stride, TH, TW, cin, cskip, chid, cout, flags;
  BlockFn fn[2];  // [PREC_F32, PREC_BF16X2]
  int threads = kThreads;  // workgroup size
  int variant = 0;         // BlockVariant: k_block or k_stem_b1 (wide)
};

// b1 with the stem fused on a wide workgroup (k_stem_b1, 16 waves): LDS
// carve in floats — the resized region x0 [3][2*IH+1][2*IW+2], the stem
// weights [27][16] + bias, the stem output tile xt [P_IN_PAD][16 + pad] and the
// block's weight image (block_lds regions w1..b2 of the same shape).
constexpr int kWideThreads = 1024;
struct StemB1Lds {
  int IH, IW, P_IN, P_IN_PAD, XS, XH, XW, XWP, x0, sw, sb, xt, wim, total;
};
__host__ __device__ constexpr StemB1Lds stem_b1_lds(int TH, int TW) {
  StemB1Lds L{};
  L.IH = TH + 2;
  L.IW = TW + 2;
  L.P_IN = L.IH * L.IW;
  L.P_IN_PAD = (L.P_IN + 15) & ~15;
  L.XS = 16 + VSS_XS_PAD;
  L.XH = 2 * L.IH + 1;
  L.XW = 2 * L.IW + 1;
  L.XWP = L.XW + 1;
  int o = 0;
  L.x0 = o;  o += r4(3 * L.XH * L.XWP);
  L.sw = o;  o += 27 * 16;
  L.sb = o;  o += 16;
  L.xt = o;  o += r4(L.P_IN_PAD * L.XS);
  const BlockLds B = block_lds(1 /*MODE_IR_DIRECT*/, 1, TH, TW, 16, 0, 16, 16, 1);
  L.wim = o; o += B.wimg_end - B.w1;
  L.total = o;
  return L;
}
// BlockEntry::variant
enum BlockVariant : int { VAR_BLOCK = 0, VAR_STEM_B1_WIDE = 1 };

const BlockEntry* block_registry(int* count);


struct HeadParams {
  const float* x;        // pre-norm dec output [N][h][w][cin]
  const unsigned long long* in_acc;  // its norm accumulator (see BlockParams), frame stride acc_stride
  int acc_stride;
  const float* gamma;    // its norm affine [cin]
  const float* beta;
  float eps;
  double inv_hw;         // 1 / (h * w_)
  const float* w;        // [cin]
  float b;
  float* mask;           // [N][Hm][Wm] f32
  int N, h, w_, cin;
  int Hm, Wm;
  VSS_TRACE_FIELD
};

// Fixed LDS of the stem and head bodies (floats; dynamic shared memory, so the
// persistent forward can run them from its own carve).
constexpr int kStemTH = 8, kStemTW = 32, kStemIH = 2 * kStemTH + 1, kStemIWP = 2 * kStemTW + 2;
constexpr int kStemLds = r4(3 * kStemIH * kStemIWP) + 27 * 16 + 16;
constexpr int kHeadTH = 16, kHeadTW = 64, kHeadZR = 10, kHeadZC = 34, kHeadZCP = 35;
constexpr int kHeadLds = kAccSlots * 2 * 16 * 2 + r4(kHeadZR * kHeadZCP) + 3 * 16;

// Instance-norm scale/shift of one channel from the exact fixed-point totals.
// inv_hw = 1 / (pixels per frame), computed by the host: the mean and E[x^2]
// take one f64 multiply each instead of an f64 division, and 1/sqrt(var + eps)
// is v_rsq_f64 refined by two Newton steps (~2^-50 relative; rounded to f32
// after) instead of an f64 sqrt and division — the norm's setup runs on the
// prologue's critical path of every decoder workgroup and the head.
__host__ __device__ inline void norm_affine(unsigned long long s_fx, unsigned long long q_fx, double inv_hw,
                                            float eps, float gamma, float beta, float* scale, float* shift) {
  const double mean = (double)(long long)s_fx * (0x1p-32 * inv_hw);
  const double ex2 = (double)(long long)q_fx * (0x1p-24 * inv_hw);
  const double var = ex2 - mean * mean > 0.0 ? ex2 - mean * mean : 0.0;
  const double x = var + (double)eps;
#ifdef __HIP_DEVICE_COMPILE__
  double r = __builtin_amdgcn_rsq(x);
  r = r * __builtin_fma(-0.5 * x * r, r, 1.5);
  r = r * __builtin_fma(-0.5 * x * r, r, 1.5);
#else
  const double r = 1.0 / __builtin_sqrt(x);
#endif
  const float rstd = (float)r;
  const float sc = rstd * gamma;
  *scale = sc;
  *shift = beta - (float)mean * sc;
}

struct PrepParams {      // standalone preprocess: frames -> [N][3][Hm][Wm] f32
  const uint8_t* frames;
  long row_stride, frame_stride;
  int fh, fw, fc;
  int Hm, Wm;
  float ry, rx;
  float* out;
  int N;
};

// Post-processing chain (vss_post.hip)
struct PostEmaParams {
  const float* masks;  // [n][P] raw seam masks
  float* ema;          // [n][P] EMA outputs
  float* state;        // [P] prevAlpha
  const int* valid;    // 0 before the stream's first frame
  int n;
  long P;
  double a;            // config.EMA
};

// Per-frame face inputs of the post chain (the same layout as vss_face_frame, include/vss.h)
struct FaceFrame {
  int has_affine;
  double affine[6];
  int has_box;
  double box[4];
  int video_w, video_h;
};

// One frame of the stabilised EMA: base = mask (+ 0.3 * warp(prevAlpha) when the
// frame has an affine), then the EMA; prevAlpha double-buffered (the warp reads
// other pixels' prevAlpha).
struct PostFaceEmaParams {
  const float* mask;     // [P] this frame's raw mask
  const float* prev;     // [P] prevAlpha
  float* next;           // [P] the new prevAlpha (= this frame's EMA)
  float* ema;            // [P] this frame's EMA output
  const int* valid;      // 0 before the stream's first frame
  int first;             // this is the call's first frame
  const FaceFrame* face; // this frame's face inputs (device)
  int H, W;
  double a;
};
void launch_post_face_ema(const PostFaceEmaParams& p, hipStream_t s);

struct PostFilterParams {
  const FaceFrame* faces;  // [n] per-frame face inputs (device) or null: no prior
  const float* ema;      // [n][H][W]
  const uint8_t* frames; // the n source frames (guide)
  long row_stride, frame_stride;
  int fh, fw, fc;
  float ry, rx;
  int H, W;
  const double* rtab;    // exp(-r / (2 sigma_r^2)), r = 0 .. 3*255^2
  double sw[3];          // exp(-s / (2 sigma_s^2)), s = 0, 1, 2
  double lo, hi, denom, gamma;
  int use_bilateral;
  float* alpha;          // [n][H][W] refined (may be null)
  uint8_t* alpha_u8;     // [n][H][W] (may be null)
};

// §8(f) row 3: destination-in compositing of the frame by the upscaled mask alpha
struct CompositeParams {
  const uint8_t* frames;  // [n] frames, row_stride / frame_stride bytes, fc = 3 or 4
  long row_stride, frame_stride;
  int fh, fw, fc;
  const uint8_t* alpha;   // [n][H][W] u8 (the post chain's alpha bytes)
  int H, W;
  float sy, sx;           // (float)H / fh, (float)W / fw
  uint8_t* out;           // [n] RGBA frames, out_row_stride / out_frame_stride bytes
  long out_row_stride, out_frame_stride;
};
void launch_composite(const CompositeParams& p, int n, hipStream_t s);

// VSS_OUT_FRAME: the f32 model-res masks upsampled to frame resolution with
// the same half-pixel bilinear as the compositing alpha (k_composite).
struct UpmaskParams {
  const float* masks;  // [n][H][W]
  int H, W;
  float sy, sx;        // (float)H / fh, (float)W / fw
  float* out;          // [n][fh][fw]
  int fh, fw;
};
void launch_upmask(const UpmaskParams& p, int n, hipStream_t s);

// Queued host path: only the frame rows the resize reads, pinned host -> HBM
// (vss_stage.hip).  rows: device list of the row indices; src / dst = frame 0.
struct FetchRowsParams {
  const uint8_t* src;    // pinned host staging (device-accessible)
  uint8_t* dst;          // the slot's HBM frame buffer (same layout)
  const int* rows;       // [nrows] rows to move
  long row_stride, frame_stride;
  int row_bytes;         // width * channels
  int vec16;             // 1: every row start and row_bytes are multiples of 16 B
};
void launch_fetch_rows(const FetchRowsParams& p, int nrows, int nframes, hipStream_t s);

void launch_post_ema(const PostEmaParams& p, hipStream_t s);
void launch_post_filter(const PostFilterParams& p, int n, hipStream_t s);

// XCD-aware tile order of the layer launches and the head.  Workgroups are
// dealt round-robin over the 8 XCDs (block b shares an XCD, and its L2, with
// b + 8; MI355X_MICROARCH.md, workgroup dispatch), so with the grid's natural
// order horizontally adjacent tiles — which read the same halo columns of the
// input and, in the decoders, the same low-res src columns — sit on different
// XCDs and each XCD fetches the shared lines again.  Remap: the workgroups of
// one XCD (b % 8) take one contiguous eighth of the logical (x, y, z) tile
// order, i.e. whole rows of tiles of one frame (with 8 frames, one frame per
// XCD), so neighbours share an L2.  A bijection on the grid (any remainder
// past the last full eighth keeps its own index); results do not depend on
// which workgroup computes which tile (tile-invariant, order-free norm sums).
// Measured: the post filter and the frame-resolution kernels gain nothing
// from it (profiles/NOTES.md), so they keep the natural order.
#ifndef VSS_XCD_REMAP
#define VSS_XCD_REMAP 1
#endif
struct TileIdx {
  int x, y, z;
};
__device__ __forceinline__ TileIdx xcd_tile() {
  if constexpr (VSS_XCD_REMAP) {
    const int gx = (int)gridDim.x, gy = (int)gridDim.y;
    const int L = (int)blockIdx.x + gx * ((int)blockIdx.y + gy * (int)blockIdx.z);
    const int per = (gx * gy * (int)gridDim.z) >> 3;
    const int T = L < (per << 3) ? (L & 7) * per + (L >> 3) : L;
    const int zy = T / gx;
    return {T - zy * gx, zy % gy, zy / gy};
  } else {
    return {(int)blockIdx.x, (int)blockIdx.y, (int)blockIdx.z};
  }
}

}  // namespace vss
