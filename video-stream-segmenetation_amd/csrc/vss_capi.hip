// vss_capi.hip — the C ABI (include/vss.h) over the gfx950 kernels.
//
// One handle = one GPU + one private HIP stream, mirroring one ORT
// InferenceSession (/root/reference/client/src/core/model.ts:12-29).  The
// handle parses the weights blob's layer table once, plans per-layer tiles for
// its model resolution, keeps every activation NHWC f32 in HBM for max_batch
// frames, and replays one captured hipGraph per (shape, buffers) key.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <string>
#include <tuple>
#include <vector>

#include "../../include/vss.h"
#include "vss_kernels.h"

namespace vss {
void (*stem_kernel16())(StemParams);
void (*head_kernel16())(HeadParams);
void (*prep_kernel())(PrepParams);
}  // namespace vss

using namespace vss;

namespace {

constexpr uint32_t kMagic = 0x57535356u, kNone = 0xFFFFFFFFu;
enum { K_STEM = 1, K_IR = 2, K_DEC = 3, K_HEAD = 4 };
enum { F_EXPAND = 1, F_RESIDUAL = 2 };
enum { O_W1, O_B1, O_WDW, O_BDW, O_W2, O_B2, O_GAMMA, O_BETA };

struct Rec {
  uint32_t kind, cin, chid, cout, stride, flags, src, skip, off[8];
};

struct LayerPlan {
  Rec rec{};
  int C = 0, H = 0, W = 0;     // output shape
  int inH = 0, inW = 0;        // shape of rec.src's output (x)
  int mode = -1, stride = 1, chid = 0;
  int TH = 0, TW = 0, tiles_x = 0, tiles_y = 0, grid_x = 0, grid_y = 0;
  int flags = 0;
  int ks = 1, xp = 1, sp = 1;  // hidden split of this layer, parts of its x / skip (block_flags)
  size_t part_stride = 0;      // floats between the parts of act
  long wimg_stride = 0;        // floats between the slices' weight images
  size_t lds = 0;
  const BlockEntry* entry = nullptr;  // compiled shape (registry)
  bool fused = false;          // computed inside its only consumer's prologue (no launch of its own)
  float* act = nullptr;        // [max_batch][H][W][C]
  int acc_off = -1;            // DEC: offset of its [2][C] norm accumulator in a frame's row of d_acc
  const float* wimg = nullptr;  // LDS weight image (block_lds regions w1..b2)
  int wimg_f4 = 0;
  const float *gamma = nullptr, *beta = nullptr;
  const float *stem_w = nullptr, *stem_b = nullptr, *head_w = nullptr;
  float head_b = 0.f;
};

using GraphKey = std::tuple<const void*, const void*, int, int, int, int, size_t, size_t>;

thread_local std::string g_tls_error;

}  // namespace

constexpr long kDefaultKsplitPixels = 256;
// expand layers whose unsplit LDS weight image exceeds this also split their
// hidden channels (keeps every layer within the persistent forward's LDS
// budget of two workgroups per CU; mirrors KSPLIT_WEIGHT_BYTES in
// tools/gen_registry.py)
constexpr size_t kKsplitWeightBytes = 40 * 1024;

struct vss_handle {
  vss_config cfg{};
  std::string weights_path;
  std::string err;
  int device = 0;
  hipStream_t stream = nullptr;
  std::vector<Rec> recs;
  std::vector<float> hdata;
  float eps = 1e-5f;
  std::vector<LayerPlan> L;
  unsigned long long* d_acc = nullptr;  // decoder instance-norm accumulators [max_batch][acc_stride]
  int acc_stride = 0;
  std::vector<void*> dev_allocs;
  size_t dev_bytes = 0;
  uint8_t* d_frames = nullptr;
  float* d_masks = nullptr;
  size_t frame_cap = 0;
  uint8_t* h_frames = nullptr;  // pinned staging
  float* h_masks = nullptr;
  float* d_fmasks = nullptr;  // VSS_OUT_FRAME: masks at frame resolution (allocated on first use)
  float* h_fmasks = nullptr;
  size_t fmask_cap = 0;       // floats
  const float* out_src = nullptr;  // what the last staged call left for the host copy
  size_t out_bytes = 0;
#ifdef VSS_TRACE
  std::vector<unsigned long long*> trace;  // per layer, [grid][4] stamps
  std::vector<int> trace_wgs;              // workgroups of the layer's last launch
#endif
  uint8_t* d_comp = nullptr;      // vss_segment_composite output, allocated on first use
  float* d_post_alpha = nullptr;  // vss_segment_post outputs [max_batch][P]
  uint8_t* d_post_u8 = nullptr;
  std::atomic<int> busy{0};
  int use_graph = 1;
  int profile = 0;
  static constexpr int kMaxBranches = 8;
  int branches = 1;  // parallel sub-batch chains inside the captured graph
  // expand layers with at most this many output pixels per frame split their
  // hidden channels over ks_max() workgroups (env VSS_KSPLIT_PIXELS overrides)
  long ksplit_pixels = kDefaultKsplitPixels;
  hipStream_t branch_streams[kMaxBranches] = {};
  hipEvent_t fork_ev = nullptr, join_ev[kMaxBranches] = {};
  std::map<GraphKey, hipGraphExec_t> graphs;
  // profiling: ring of event pairs per layer
  static constexpr int kSlots = 32;
  std::vector<hipEvent_t> ev;  // [slot][layer][2]
  std::vector<int> slot_pending;
  int prof_next = 0;
  std::vector<double> prof_sum;
  int prof_count = 0;
  double fwd_prof_sum = 0.0;
  int fwd_prof_count = 0;
  int last_n = 0;
  // persistent forward (k_forward): the whole network in one launch
  int want_forward = 0;          // env VSS_FORWARD=1 at create: plan for the persistent forward
  bool fwd_ok = false;           // every layer of the plan has a k_forward case
  int use_forward = 0;           // VSS_OPT_FORWARD
  FwdLayer* d_fwd_layers = nullptr;
  unsigned* d_fwd_ctl = nullptr;   // kFwdCtlWords (FwdParams::ctl)
  unsigned* d_fwd_done = nullptr;  // [n_layers][max_batch]
  int fwd_lds_floats = 0;
  int fwd_grid = 0;
  int fwd_order = 0;             // 0 layer-major, 1 diagonal (env VSS_FWD_ORDER=diag)
  int fuse_stem = 1;             // env VSS_FUSE_STEM=0: launch the stem on its own
  int keep_stem = 0;             // VSS_OPT_KEEP_STEM: the fused stem also stores its activation
  std::map<int, std::pair<FwdTask*, int>> fwd_tasks;  // per batch size n
  unsigned* fwd_dbg = nullptr;   // env VSS_FWD_DEBUG: host-mapped per-workgroup state
  unsigned long long* fwd_trace = nullptr;  // env VSS_FWD_TRACE: per-task stamps of the last launch
  size_t fwd_trace_cap = 0;                 // tasks
  int fwd_trace_n = 0;                      // tasks of the last traced launch
};

namespace {

int fail(vss_handle* h, int code, const std::string& msg) {
  if (h) h->err = msg;
  else g_tls_error = msg;
  return code;
}

#define HIP_TRY(h, expr)                                                                  \
  do {                                                                                    \
    hipError_t e_ = (expr);                                                               \
    if (e_ != hipSuccess)                                                                 \
      return fail((h), e_ == hipErrorOutOfMemory ? VSS_E_OOM : VSS_E_HIP,                \
                  std::string(#expr) + ": " + hipGetErrorString(e_));                     \
  } while (0)

template <class T>
int dalloc(vss_handle* h, T** p, size_t bytes) {
  void* q = nullptr;
  bytes = std::max<size_t>(bytes, 16);
  hipError_t e = hipMalloc(&q, bytes);
  if (e != hipSuccess) return fail(h, VSS_E_OOM, "hipMalloc(" + std::to_string(bytes) + ") failed");
  h->dev_allocs.push_back(q);
  h->dev_bytes += bytes;
  *p = static_cast<T*>(q);
  return VSS_OK;
}

uint16_t bf16_bits(float f) {  // pointwise weights are bf16-exact: truncation is exact
  uint32_t u;
  std::memcpy(&u, &f, 4);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

size_t block_lds_bytes(const LayerPlan& l, int TH, int TW) {
  const int cskip = l.mode == MODE_DEC ? (int)l.rec.chid : 0;
  return (size_t)block_lds(l.mode, l.stride, TH, TW, (int)l.rec.cin, cskip, l.chid / l.ks, l.C,
                           flags_stem_in(l.flags)).total * 4;
}

// Largest hidden split of an expand layer that leaves every wave >= 1 chunk of
// 16 channels (mirrors ks_max() in tools/gen_registry.py, which compiles the
// split variants).
int ks_max(const LayerPlan& l) {
  if (l.mode != MODE_IR_EXPAND) return 1;
  const int nchunk = l.chid / 16;
  for (int k : {4, 3, 2})
    if (nchunk % k == 0 && nchunk / k >= 4) return k;
  return 1;
}

void set_tile(LayerPlan& l, const BlockEntry* e) {
  l.entry = e;
  l.TH = e->TH;
  l.TW = e->TW;
  l.tiles_x = (l.W + l.TW - 1) / l.TW;
  l.tiles_y = (l.H + l.TH - 1) / l.TH;
  l.lds = block_lds_bytes(l, l.TH, l.TW);
}

// Tile choice among the compiled shapes for this layer (csrc/vss_registry.inc):
// the largest tile that still gives >= 2 workgroups per CU (256 CUs) at
// max_batch, preferring <= 64 KiB of LDS; otherwise the most workgroups.
int choose_tile(vss_handle* h, LayerPlan& l, int N, bool mk_only) {
  int count = 0;
  const BlockEntry* reg = block_registry(&count);
  const int cskip = l.mode == MODE_DEC ? (int)l.rec.chid : 0;
  const BlockEntry* best = nullptr;
  long best_score = -1;
  for (int i = 0; i < count; ++i) {
    const BlockEntry& e = reg[i];
    if (e.mode != l.mode || e.stride != l.stride || e.cin != (int)l.rec.cin || e.cskip != cskip ||
        e.chid != l.chid / l.ks || e.cout != l.C || e.flags != l.flags || (mk_only && e.mk < 0))
      continue;
    const long blocks = (long)((l.H + e.TH - 1) / e.TH) * ((l.W + e.TW - 1) / e.TW) * N;
    const size_t lds = block_lds_bytes(l, e.TH, e.TW);
    // score: enough blocks first, then bigger tiles, then less LDS
    long score = (blocks >= 512 ? 1L << 40 : blocks << 20) + (long)e.TH * e.TW * 1024 - (long)(lds / 1024);
    if (blocks >= 512 && lds > 64 * 1024) score -= 1L << 39;
    if (score > best_score) { best_score = score; best = &e; }
  }
  if (!best)
    return fail(h, VSS_E_UNSUPPORTED,
                "no compiled kernel for this layer shape (regenerate csrc/vss_registry.inc with "
                "tools/gen_registry.py and rebuild)");
  set_tile(l, best);
  return VSS_OK;
}

std::vector<const BlockEntry*> tile_candidates(const LayerPlan& l) {
  int count = 0;
  const BlockEntry* reg = block_registry(&count);
  const int cskip = l.mode == MODE_DEC ? (int)l.rec.chid : 0;
  std::vector<const BlockEntry*> out;
  for (int i = 0; i < count; ++i) {
    const BlockEntry& e = reg[i];
    if (e.mode == l.mode && e.stride == l.stride && e.cin == (int)l.rec.cin && e.cskip == cskip && e.chid == l.chid / l.ks &&
        e.cout == l.C && e.flags == l.flags)
      out.push_back(&e);
  }
  return out;
}

int load_weights(vss_handle* h) {
  std::ifstream f(h->weights_path, std::ios::binary);
  if (!f) return fail(h, VSS_E_IO, "cannot open weights blob '" + h->weights_path + "'");
  std::vector<char> blob((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  if (blob.size() < 32) return fail(h, VSS_E_IO, "weights blob too short");
  uint32_t hd[8];
  std::memcpy(hd, blob.data(), 32);
  if (hd[0] != kMagic || hd[1] != 1) return fail(h, VSS_E_IO, "bad weights blob magic/version");
  const uint32_t nl = hd[2], nf = hd[3];
  std::memcpy(&h->eps, &hd[4], 4);
  if (32 + 64ull * nl + 4ull * nf > blob.size()) return fail(h, VSS_E_IO, "weights blob truncated");
  h->recs.resize(nl);
  std::memcpy(h->recs.data(), blob.data() + 32, 64ull * nl);
  h->hdata.resize(nf);
  std::memcpy(h->hdata.data(), blob.data() + 32 + 64ull * nl, 4ull * nf);
  for (const Rec& r : h->recs)
    for (uint32_t o : r.off)
      if (o != kNone && o >= nf) return fail(h, VSS_E_IO, "weights offset out of range");
  return VSS_OK;
}

// Bytes of an unsplit expand layer's LDS weight image (block_lds regions w1..b2).
size_t weight_image_bytes(const LayerPlan& l) {
  const BlockLds B = block_lds(l.mode, l.stride, 1, 16, (int)l.rec.cin, 0, l.chid, l.C);
  return (size_t)(B.wimg_end - B.w1) * 4;
}

int plan_once(vss_handle* h, bool mk_only) {
  const int Hm = h->cfg.model_h, Wm = h->cfg.model_w, N = h->cfg.max_batch;
  const int nl = (int)h->recs.size();
  h->L.assign(nl, LayerPlan{});
  std::vector<int> consumers(nl, 0);
  for (const Rec& r : h->recs) {
    if (r.kind != K_STEM && r.src < (uint32_t)nl) consumers[r.src]++;
    if (r.kind == K_DEC && r.skip < (uint32_t)nl) consumers[r.skip]++;
  }
  for (int i = 0; i < nl; ++i) {
    LayerPlan& l = h->L[i];
    const Rec& r = h->recs[i];
    l.rec = r;
    l.C = (int)r.cout;
    auto bad = [&](const char* why) {
      return fail(h, VSS_E_UNSUPPORTED, "layer " + std::to_string(i) + ": " + why);
    };
    if (r.kind != K_STEM && (r.src >= (uint32_t)i)) return bad("src must precede layer");
    if (r.kind == K_STEM) {
      if (r.cin != 3 || r.cout != 16 || r.stride != 2) return bad("stem must be 3->16 stride 2");
      l.H = Hm / 2; l.W = Wm / 2;
    } else if (r.kind == K_IR) {
      const LayerPlan& s = h->L[r.src];
      if ((int)r.cin != s.C) return bad("ir cin != src channels");
      l.inH = s.H; l.inW = s.W;
      l.stride = (int)r.stride;
      if (l.stride != 1 && l.stride != 2) return bad("stride must be 1 or 2");
      l.H = l.stride == 2 ? (s.H + 1) / 2 : s.H;
      l.W = l.stride == 2 ? (s.W + 1) / 2 : s.W;
      l.mode = (r.flags & F_EXPAND) ? MODE_IR_EXPAND : MODE_IR_DIRECT;
      l.chid = (r.flags & F_EXPAND) ? (int)r.chid : (int)r.cin;
      if (r.cin % 16 || l.chid % 16 || r.cout % 16) return bad("channels must be multiples of 16");
      if ((r.flags & F_EXPAND) && r.cin > 64) return bad("expand cin > 64");
      if (l.mode == MODE_IR_DIRECT && l.stride != 1) return bad("direct ir needs stride 1");
      if ((r.flags & F_RESIDUAL) && (l.stride != 1 || r.cin != r.cout)) return bad("residual shape");
    } else if (r.kind == K_DEC) {
      const LayerPlan& s = h->L[r.src];
      const LayerPlan& k = h->L[r.skip];
      if (r.skip >= (uint32_t)i) return bad("skip must precede layer");
      if ((int)r.cin != s.C || (int)r.chid != k.C) return bad("dec channels");
      if (2 * s.H != k.H || 2 * s.W != k.W) return bad("dec src must be half the skip res");
      l.inH = s.H; l.inW = s.W;
      l.H = k.H; l.W = k.W;
      l.mode = MODE_DEC;
      l.chid = (int)(r.cin + r.chid);
      if (r.cin % 16 || r.chid % 16 || r.cout % 16) return bad("channels must be multiples of 16");
      if (r.off[O_GAMMA] == kNone || r.off[O_BETA] == kNone) return bad("dec needs gamma/beta");
    } else if (r.kind == K_HEAD) {
      const LayerPlan& s = h->L[r.src];
      if (s.rec.kind != K_DEC) return bad("head src must be a dec layer");
      if (2 * s.H != Hm || 2 * s.W != Wm) return bad("head src must be half model res");
      if (r.cin != 16 || (int)r.cin != s.C || r.cout != 1) return bad("head must be 16 -> 1");
      l.inH = s.H; l.inW = s.W;
      l.H = Hm; l.W = Wm; l.C = 1;
    } else {
      return bad("unknown kind");
    }
    // hidden split: expand layers whose output has at most ksplit_pixels
    // pixels per frame (a function of the model resolution only, so results
    // never depend on the batch or the autotuner)
    if (l.mode == MODE_IR_EXPAND &&
        ((long)l.H * l.W <= h->ksplit_pixels || weight_image_bytes(l) > kKsplitWeightBytes))
      l.ks = ks_max(l);
    if (r.kind == K_IR || r.kind == K_DEC) l.xp = h->L[r.src].ks;
    if (r.kind == K_DEC) l.sp = h->L[r.skip].ks;
    if (r.kind == K_IR) l.flags = block_flags(0, (r.flags & F_RESIDUAL) != 0, l.xp, 1, l.ks);
    // the stem fused into its only consumer, a stride-1 direct block (STEM_IN)
    if (r.kind == K_IR && !mk_only && h->fuse_stem && l.mode == MODE_IR_DIRECT && l.stride == 1 &&
        h->L[r.src].rec.kind == K_STEM && consumers[r.src] == 1 && r.cin == 16) {
      l.flags |= block_flags(0, 0, 1, 1, 1, 1);
      h->L[r.src].fused = true;
    }
    if (r.kind == K_DEC) l.flags = block_flags(h->L[r.src].rec.kind == K_DEC, 0, l.xp, l.sp, 1);
    if (l.mode >= 0) {
      int rc = choose_tile(h, l, N, mk_only);
      if (rc) return rc;
    }
  }
  if (nl == 0 || h->recs.back().kind != K_HEAD) return fail(h, VSS_E_UNSUPPORTED, "last layer must be the head");
  return VSS_OK;
}

// Plan for the persistent forward when every layer has a k_forward case
// (csrc/vss_mk.inc), else for per-layer launches.
int plan(vss_handle* h) {
  h->fwd_ok = h->want_forward != 0;
  int rc = plan_once(h, h->fwd_ok);
  if (rc == VSS_E_UNSUPPORTED && h->fwd_ok) {
    h->fwd_ok = false;
    rc = plan_once(h, false);
  }
  return rc;
}

int upload(vss_handle* h) {
  const int N = h->cfg.max_batch;
  float* d_data = nullptr;
  int rc = dalloc(h, &d_data, h->hdata.size() * 4);
  if (rc) return rc;
  HIP_TRY(h, hipMemcpy(d_data, h->hdata.data(), h->hdata.size() * 4, hipMemcpyHostToDevice));
  auto dp = [&](uint32_t off) -> const float* { return off == kNone ? nullptr : d_data + off; };
  // Per-layer LDS weight images: the exact bytes of block_lds regions w1..b2
  // (pointwise weights as bf16 rows padded to LD1/LD2, dw weights [9][C],
  // biases), so the kernel prologue is one flat 16-B copy.
  std::vector<float> img;
  std::vector<size_t> img_off(h->L.size(), 0), img_len(h->L.size(), 0);
  for (size_t i = 0; i < h->L.size(); ++i) {
    const LayerPlan& l = h->L[i];
    const Rec& r = l.rec;
    if (r.kind != K_IR && r.kind != K_DEC) continue;
    // the kernels keep pointwise weights as bf16: require bf16-exact values
    auto exact = [&](uint32_t off, size_t cnt) {
      for (size_t k = 0; k < cnt; ++k) {
        uint32_t u;
        std::memcpy(&u, &h->hdata[off + k], 4);
        if (u & 0xFFFFu) return false;
      }
      return true;
    };
    const bool expand = l.mode == MODE_IR_EXPAND;
    if ((expand && !exact(r.off[O_W1], (size_t)r.chid * r.cin)) || !exact(r.off[O_W2], (size_t)r.cout * l.chid))
      return fail(h, VSS_E_UNSUPPORTED, "layer " + std::to_string(i) + ": pointwise weights must be bf16-exact");
    const int cskip = l.mode == MODE_DEC ? (int)r.chid : 0;
    const int cs = l.chid / l.ks;  // hidden channels per slice
    const BlockLds B = block_lds(l.mode, l.stride, 1, 16, (int)r.cin, cskip, cs, l.C);
    const size_t span = (size_t)(B.wimg_end - B.w1);  // one slice's image (floats, multiple of 4)
    img_off[i] = img.size();
    img_len[i] = span;
    for (int sl = 0; sl < l.ks; ++sl) {
      const int h0 = sl * cs;  // first hidden channel of the slice
      const size_t base = img.size();
      img.resize(base + span, 0.f);
      float* im = img.data() + base;
      auto bf = [&](uint32_t off, size_t k) { return bf16_bits(h->hdata[off + k]); };
      if (expand) {
        uint16_t* d = reinterpret_cast<uint16_t*>(im + (B.w1 - B.w1));
        for (int a = 0; a < cs; ++a)
          for (int b = 0; b < (int)r.cin; ++b) d[(size_t)a * B.LD1 + b] = bf(r.off[O_W1], (size_t)(h0 + a) * r.cin + b);
        for (int c = 0; c < cs; ++c) im[B.b1 - B.w1 + c] = h->hdata[r.off[O_B1] + h0 + c];
      }
      uint16_t* d2 = reinterpret_cast<uint16_t*>(im + (B.w2 - B.w1));
      for (int a = 0; a < l.C; ++a)
        for (int b = 0; b < cs; ++b) d2[(size_t)a * B.LD2 + b] = bf(r.off[O_W2], (size_t)a * l.chid + h0 + b);
      for (int t = 0; t < 9; ++t)
        for (int c = 0; c < cs; ++c) im[B.wdw - B.w1 + t * cs + c] = h->hdata[r.off[O_WDW] + (size_t)(h0 + c) * 9 + t];
      for (int c = 0; c < cs; ++c) im[B.bdw - B.w1 + c] = h->hdata[r.off[O_BDW] + h0 + c];
      for (int c = 0; c < l.C; ++c) im[B.b2 - B.w1 + c] = h->hdata[r.off[O_B2] + c];
    }
  }
  float* d_img = nullptr;
  if ((rc = dalloc(h, &d_img, img.size() * 4))) return rc;
  int acc_total = 0;
  for (const LayerPlan& l : h->L)
    if (l.rec.kind == K_DEC) acc_total += kAccSlots * 2 * l.C;
  if ((rc = dalloc(h, &h->d_acc, (size_t)N * std::max(acc_total, 2) * 8))) return rc;
  HIP_TRY(h, hipMemset(h->d_acc, 0, (size_t)N * std::max(acc_total, 2) * 8));
  if (!img.empty()) HIP_TRY(h, hipMemcpy(d_img, img.data(), img.size() * 4, hipMemcpyHostToDevice));
  for (size_t i = 0; i < h->L.size(); ++i) {
    LayerPlan& l = h->L[i];
    const Rec& r = l.rec;
    l.part_stride = (size_t)N * l.H * l.W * l.C;
    if ((rc = dalloc(h, &l.act, l.part_stride * l.ks * 4))) return rc;
    HIP_TRY(h, hipMemset(l.act, 0, l.part_stride * l.ks * 4));
#ifdef VSS_TRACE
    if (h->trace.size() != h->L.size()) {
      h->trace.assign(h->L.size(), nullptr);
      h->trace_wgs.assign(h->L.size(), 0);
    }
    if ((rc = dalloc(h, &h->trace[i], (size_t)N * l.H * l.W * 16 * 8))) return rc;
    HIP_TRY(h, hipMemset(h->trace[i], 0, (size_t)N * l.H * l.W * 16 * 8));
#endif
    if (r.kind == K_STEM) {
      l.stem_w = dp(r.off[O_W1]);
      l.stem_b = dp(r.off[O_B1]);
    } else if (r.kind == K_IR || r.kind == K_DEC) {
      l.wimg = d_img + img_off[i];
      l.wimg_f4 = (int)(img_len[i] / 4);
      l.wimg_stride = (long)img_len[i];
      if (r.kind == K_DEC) {
        l.gamma = dp(r.off[O_GAMMA]);
        l.beta = dp(r.off[O_BETA]);
        l.acc_off = h->acc_stride;
        h->acc_stride += kAccSlots * 2 * l.C;
      }
    } else if (r.kind == K_HEAD) {
      l.head_w = dp(r.off[O_W2]);
      l.head_b = h->hdata[r.off[O_B2]];
    }
  }
  return VSS_OK;
}

int check_frames(vss_handle* h, int n, int fh, int fw, int fc, size_t rs, size_t fs) {
  if (n < 1 || n > h->cfg.max_batch) return fail(h, VSS_E_INVALID_ARG, "n must be in [1, max_batch]");
  if (fh < 1 || fw < 1) return fail(h, VSS_E_INVALID_ARG, "bad frame size");
  if (fc != 3 && fc != 4) return fail(h, VSS_E_INVALID_ARG, "channels must be 3 or 4");
  if (rs < (size_t)fw * fc) return fail(h, VSS_E_INVALID_ARG, "row_stride < width*channels");
  if (fs < rs * (size_t)fh) return fail(h, VSS_E_INVALID_ARG, "frame_stride < height*row_stride");
  return VSS_OK;
}

size_t frame_elems(const LayerPlan& l) { return (size_t)l.H * l.W * l.C; }

// The stem's parameters for this call's frames (frames point at frame f0).
StemParams stem_params(const vss_handle* h, const LayerPlan& l, const uint8_t* frames, size_t rs, size_t fs, int fh,
                       int fw, int fc, int f0) {
  const int Hm = h->cfg.model_h, Wm = h->cfg.model_w;
  StemParams p{};
  p.frames = frames; p.row_stride = (long)rs; p.frame_stride = (long)fs;
  p.fh = fh; p.fw = fw; p.fc = fc; p.Hm = Hm; p.Wm = Wm;
  p.ry = (float)((double)fh / (double)Hm);
  p.rx = (float)((double)fw / (double)Wm);
  p.w = l.stem_w; p.b = l.stem_b; p.y = l.act + (size_t)f0 * l.H * l.W * l.C;
  p.Ho = l.H; p.Wo = l.W; p.cout = l.C;
  p.acc_zero = h->d_acc + (size_t)f0 * h->acc_stride;
  p.acc_stride = h->acc_stride;
  return p;
}

// Kernel parameters of block layer l for frames [f0, f0 + n) of the batch.
BlockParams block_params(const vss_handle* h, const LayerPlan& l, int n, int f0 = 0) {
  const Rec& r = l.rec;
  const LayerPlan& src = h->L[r.src];
  const size_t fa = (size_t)f0 * h->acc_stride;
  BlockParams p{};
  p.wimg = l.wimg;
  p.wimg_stride = l.wimg_stride;
  p.x_part_stride = (long)src.part_stride;
  p.y_part_stride = (long)l.part_stride;
  p.x = src.act + f0 * frame_elems(src);
  p.y = l.act + f0 * frame_elems(l);
  p.eps = h->eps;
  p.N = n; p.H = l.inH; p.W = l.inW; p.Ho = l.H; p.Wo = l.W;
  p.cin = (int)r.cin; p.cout = l.C; p.chid = l.chid; p.stride = l.stride;
  p.TH = l.TH; p.TW = l.TW; p.tiles_x = l.tiles_x; p.tiles_y = l.tiles_y;
  p.acc_stride = h->acc_stride;
  if (r.kind == K_IR) {
    p.relu6_dw = 1;
    p.residual = (r.flags & F_RESIDUAL) ? 1 : 0;
  } else {
    const LayerPlan& sk = h->L[r.skip];
    p.skip = sk.act + f0 * frame_elems(sk);
    p.skip_part_stride = (long)sk.part_stride;
    p.cskip = (int)r.chid;
    p.relu6_dw = 0;
    p.out_acc = h->d_acc + fa + l.acc_off;
    p.norm_in = src.rec.kind == K_DEC ? 1 : 0;
    if (p.norm_in) {
      p.in_acc = h->d_acc + fa + src.acc_off;
      p.in_gamma = src.gamma;
      p.in_beta = src.beta;
      p.in_hw = src.H * src.W;
    }
  }
  return p;
}

int n_tasks_per_frame(const LayerPlan& l, int Hm, int Wm) {
  if (l.rec.kind == K_STEM) return ((l.W + kStemTW - 1) / kStemTW) * ((l.H + kStemTH - 1) / kStemTH);
  if (l.rec.kind == K_HEAD) return ((Wm + kHeadTW - 1) / kHeadTW) * ((Hm + kHeadTH - 1) / kHeadTH);
  return l.tiles_x * l.tiles_y * l.ks;
}

// The persistent forward's layer table (device), counters and launch shape.
int setup_forward(vss_handle* h) {
  if (!h->fwd_ok) return VSS_OK;
  const int Hm = h->cfg.model_h, Wm = h->cfg.model_w, N = h->cfg.max_batch;
  const int nl = (int)h->L.size();
  std::vector<FwdLayer> fl(nl);
  size_t lds = 0;
  for (int i = 0; i < nl; ++i) {
    const LayerPlan& l = h->L[i];
    const Rec& r = l.rec;
    FwdLayer& f = fl[i];
    std::memset(&f, 0, sizeof(f));
    f.dep[0] = f.dep[1] = -1;
    f.ks = 1;
    if (r.kind == K_STEM) {
      f.kind = FWD_STEM;
      f.tiles_x = (l.W + kStemTW - 1) / kStemTW;
      f.tiles_y = (l.H + kStemTH - 1) / kStemTH;
      StemParams& p = f.stem;
      p.Hm = Hm; p.Wm = Wm;
      p.w = l.stem_w; p.b = l.stem_b; p.y = l.act;
      p.Ho = l.H; p.Wo = l.W; p.cout = l.C;
      p.acc_zero = h->d_acc;
      p.acc_stride = h->acc_stride;
      lds = std::max(lds, (size_t)kStemLds * 4);
    } else if (r.kind == K_IR || r.kind == K_DEC) {
      f.kind = FWD_BLOCK;
      f.mk = l.entry->mk;
      f.tiles_x = l.tiles_x;
      f.tiles_y = l.tiles_y;
      f.ks = l.ks;
      f.block = block_params(h, l, N);
      f.dep[0] = (int)r.src;
      if (r.kind == K_DEC) f.dep[1] = (int)r.skip;
      lds = std::max(lds, l.lds);
    } else {
      const LayerPlan& src = h->L[r.src];
      f.kind = FWD_HEAD;
      f.tiles_x = (Wm + kHeadTW - 1) / kHeadTW;
      f.tiles_y = (Hm + kHeadTH - 1) / kHeadTH;
      HeadParams& p = f.head;
      p.x = src.act;
      p.in_acc = h->d_acc + src.acc_off;
      p.acc_stride = h->acc_stride;
      p.gamma = src.gamma; p.beta = src.beta; p.eps = h->eps;
      p.w = l.head_w; p.b = l.head_b;
      p.N = N; p.h = src.H; p.w_ = src.W; p.cin = src.C; p.Hm = Hm; p.Wm = Wm;
      f.dep[0] = (int)r.src;
      lds = std::max(lds, (size_t)kHeadLds * 4);
    }
    for (int k = 0; k < 2; ++k)
      if (f.dep[k] >= 0) f.need[k] = n_tasks_per_frame(h->L[f.dep[k]], Hm, Wm);
  }
  h->fwd_lds_floats = (int)((lds + 15) / 16 * 4) + 16;  // + the control words
  int rc = dalloc(h, &h->d_fwd_layers, sizeof(FwdLayer) * nl);
  if (!rc) rc = dalloc(h, &h->d_fwd_ctl, kFwdCtlWords * sizeof(unsigned));
  if (!rc) rc = dalloc(h, &h->d_fwd_done, sizeof(unsigned) * nl * N * kFwdLine);
  if (rc) return rc;
  HIP_TRY(h, hipMemcpy(h->d_fwd_layers, fl.data(), sizeof(FwdLayer) * nl, hipMemcpyHostToDevice));
  HIP_TRY(h, hipMemset(h->d_fwd_ctl, 0, kFwdCtlWords * sizeof(unsigned)));
  HIP_TRY(h, hipMemset(h->d_fwd_done, 0, sizeof(unsigned) * nl * N * kFwdLine));
  const int prec = h->cfg.dtype == VSS_DTYPE_F32 ? PREC_F32 : PREC_BF16X2;
  const FwdFn fn = forward_kernel(prec);
  const int bytes = h->fwd_lds_floats * 4;
  HIP_TRY(h, hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
  int per_cu = 0;
  HIP_TRY(h, hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kThreads, bytes));
  hipDeviceProp_t prop{};
  HIP_TRY(h, hipGetDeviceProperties(&prop, h->device));
  if (per_cu < 1) {  // cannot be resident: fall back to layer launches
    h->fwd_ok = false;
    return VSS_OK;
  }
  h->fwd_grid = per_cu * prop.multiProcessorCount / kFwdQueues * kFwdQueues;
  if (h->fwd_grid < kFwdQueues) {
    h->fwd_ok = false;
    return VSS_OK;
  }
  if (const char* ev = std::getenv("VSS_FWD_ORDER")) h->fwd_order = std::strcmp(ev, "diag") == 0 ? 1 : 0;
  h->use_forward = 1;
  if (std::getenv("VSS_FWD_DEBUG")) {
    HIP_TRY(h, hipHostMalloc((void**)&h->fwd_dbg, (size_t)h->fwd_grid * 4 * sizeof(unsigned), hipHostMallocCoherent));
    std::memset(h->fwd_dbg, 0xFF, (size_t)h->fwd_grid * 4 * sizeof(unsigned));
  }
  return VSS_OK;
}

// Task list of a forward over n frames, in an order where every task's
// dependencies come earlier (the ticket order is the only scheduling).
//   layer-major: layer by layer, frame by frame within a layer, tiles in
//                (slice, row, column) order;
//   diagonal   : by layer + frame, so frame f runs layer L beside frame f+1's
//                layer L-1.
int forward_tasks(vss_handle* h, int n, FwdTask** out, int* count) {
  auto it = h->fwd_tasks.find(n);
  if (it == h->fwd_tasks.end()) {
    const int Hm = h->cfg.model_h, Wm = h->cfg.model_w;
    const int nl = (int)h->L.size();
    std::vector<FwdTask> t;
    auto emit = [&](int li, int f) {
      const int k = n_tasks_per_frame(h->L[li], Hm, Wm);
      for (int j = 0; j < k; ++j) t.push_back(FwdTask{li, f, j, 0});
    };
    const char* only = std::getenv("VSS_FWD_ONLY");  // debug: one layer's tasks, no waits
    if (only) {
      for (int f = 0; f < n; ++f) emit(std::atoi(only), f);
    } else if (h->fwd_order == 1) {
      for (int d = 0; d < nl + n - 1; ++d)
        for (int f = std::max(0, d - nl + 1); f <= std::min(n - 1, d); ++f) emit(d - f, f);
    } else {
      for (int li = 0; li < nl; ++li)
        for (int f = 0; f < n; ++f) emit(li, f);
    }
    FwdTask* d = nullptr;
    int rc = dalloc(h, &d, t.size() * sizeof(FwdTask));
    if (rc) return rc;
    HIP_TRY(h, hipMemcpy(d, t.data(), t.size() * sizeof(FwdTask), hipMemcpyHostToDevice));
    it = h->fwd_tasks.emplace(n, std::make_pair(d, (int)t.size())).first;
  }
  *out = it->second.first;
  *count = it->second.second;
  return VSS_OK;
}

// Enqueue the whole forward for frames [f0, f0 + n) on stream s (frames and
// masks point at frame f0; no sync, no alloc: graph-capturable).
int enqueue_forward(vss_handle* h, const uint8_t* frames, int n, int fh, int fw, int fc, size_t rs,
                    size_t fs, float* masks, hipStream_t s, int prof_slot, int f0 = 0) {
  const int Hm = h->cfg.model_h, Wm = h->cfg.model_w;
  const int prec = h->cfg.dtype == VSS_DTYPE_F32 ? PREC_F32 : PREC_BF16X2;
  const int nl = (int)h->L.size();
  if (h->use_forward && f0 == 0) {
    FwdParams fp{};
    int rc = forward_tasks(h, n, const_cast<FwdTask**>(&fp.tasks), &fp.ntasks);
    if (rc) return rc;
    fp.layers = h->d_fwd_layers;
    fp.max_batch = h->cfg.max_batch;
    fp.n_layers = nl;
    fp.ctl = h->d_fwd_ctl;
    fp.done = h->d_fwd_done;
    fp.spin_limit = 20000000;  // 200 ms of s_memrealtime (100 MHz)
    fp.lds_floats = h->fwd_lds_floats;
    fp.frames = frames; fp.row_stride = (long)rs; fp.frame_stride = (long)fs;
    fp.fh = fh; fp.fw = fw; fp.fc = fc;
    fp.ry = (float)((double)fh / (double)Hm);
    fp.rx = (float)((double)fw / (double)Wm);
    fp.mask = masks;
    fp.dbg = h->fwd_dbg;
    fp.nowait = std::getenv("VSS_FWD_ONLY") ? 1 : 0;
    if (std::getenv("VSS_FWD_TRACE")) {
      if ((size_t)fp.ntasks > h->fwd_trace_cap) {
        if ((rc = dalloc(h, &h->fwd_trace, (size_t)fp.ntasks * 4 * 8))) return rc;
        h->fwd_trace_cap = (size_t)fp.ntasks;
      }
      fp.ttrace = h->fwd_trace;
      h->fwd_trace_n = fp.ntasks;
    }
    // every queue needs a workgroup: round the grid to a multiple of kFwdQueues
    const dim3 grid(std::min(h->fwd_grid, (fp.ntasks + kFwdQueues - 1) / kFwdQueues * kFwdQueues));
    const size_t lds = (size_t)h->fwd_lds_floats * 4;
    if (prof_slot >= 0)
      hipExtLaunchKernelGGL(forward_kernel(prec), grid, dim3(kThreads), (uint32_t)lds, s,
                            h->ev[(size_t)prof_slot * nl * 2], h->ev[(size_t)prof_slot * nl * 2 + 1], 0, fp);
    else
      hipLaunchKernelGGL(forward_kernel(prec), grid, dim3(kThreads), lds, s, fp);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(h, VSS_E_HIP, std::string("k_forward launch: ") + hipGetErrorString(e));
    return VSS_OK;
  }
  for (int i = 0; i < nl; ++i) {
    LayerPlan& l = h->L[i];
    const Rec& r = l.rec;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (prof_slot >= 0) {
      e0 = h->ev[((size_t)prof_slot * nl + i) * 2];
      e1 = h->ev[((size_t)prof_slot * nl + i) * 2 + 1];
    }
    auto go = [&](auto fn, dim3 grid, size_t lds, auto prm) {
      if (prof_slot >= 0)
        hipExtLaunchKernelGGL(fn, grid, dim3(kThreads), (uint32_t)lds, s, e0, e1, 0, prm);
      else
        hipLaunchKernelGGL(fn, grid, dim3(kThreads), lds, s, prm);
    };
    if (l.fused) {  // runs inside its consumer's launch
#ifdef VSS_TRACE
      h->trace_wgs[i] = 0;
#endif
      continue;
    }
    if (r.kind == K_STEM) {
      StemParams p = stem_params(h, l, frames, rs, fs, fh, fw, fc, f0);
#ifdef VSS_TRACE
      p.trace = h->trace[i];
      h->trace_wgs[i] = ((l.W + 31) / 32) * ((l.H + 7) / 8) * n;
#endif
      go(stem_kernel16(), dim3((l.W + kStemTW - 1) / kStemTW, (l.H + kStemTH - 1) / kStemTH, n), kStemLds * 4, p);
    } else if (r.kind == K_IR || r.kind == K_DEC) {
      BlockParams p = block_params(h, l, n, f0);
      if (flags_stem_in(l.flags)) {
        p.stem = stem_params(h, h->L[r.src], frames, rs, fs, fh, fw, fc, f0);
        if (!h->keep_stem) p.stem.y = nullptr;  // no layer reads it (vss_read_layer(0) only)
      }
#ifdef VSS_TRACE
      p.trace = h->trace[i];
      h->trace_wgs[i] = l.tiles_x * l.tiles_y * n * l.ks;
#endif
      go(l.entry->fn[prec == PREC_F32 ? 0 : 1], dim3(l.tiles_x, l.tiles_y, n * l.ks), l.lds, p);
    } else if (r.kind == K_HEAD) {
      const LayerPlan& src = h->L[r.src];
      HeadParams p{};
      p.x = src.act + f0 * frame_elems(src);
      p.in_acc = h->d_acc + (size_t)f0 * h->acc_stride + src.acc_off;
      p.acc_stride = h->acc_stride;
      p.gamma = src.gamma; p.beta = src.beta; p.eps = h->eps;
      p.w = l.head_w; p.b = l.head_b; p.mask = masks;
      p.N = n; p.h = src.H; p.w_ = src.W; p.cin = src.C; p.Hm = Hm; p.Wm = Wm;
#ifdef VSS_TRACE
      p.trace = h->trace[i];
      h->trace_wgs[i] = ((Wm + 63) / 64) * ((Hm + 15) / 16) * n;
#endif
      go(head_kernel16(), dim3((Wm + kHeadTW - 1) / kHeadTW, (Hm + kHeadTH - 1) / kHeadTH, n), kHeadLds * 4, p);
    }
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(h, VSS_E_HIP, std::string("kernel launch: ") + hipGetErrorString(e));
  return VSS_OK;
}

int harvest_slot(vss_handle* h, int slot) {
  const int nl = (int)h->L.size();
  if (h->slot_pending[slot] == 2) {  // one k_forward launch
    float ms = 0.f;
    HIP_TRY(h, hipEventSynchronize(h->ev[(size_t)slot * nl * 2 + 1]));
    HIP_TRY(h, hipEventElapsedTime(&ms, h->ev[(size_t)slot * nl * 2], h->ev[(size_t)slot * nl * 2 + 1]));
    h->fwd_prof_sum += ms;
    h->fwd_prof_count++;
    h->slot_pending[slot] = 0;
    return VSS_OK;
  }
  for (int i = 0; i < nl; ++i) {
    float ms = 0.f;
    if (h->L[i].fused) continue;  // timed inside its consumer's launch
    HIP_TRY(h, hipEventSynchronize(h->ev[((size_t)slot * nl + i) * 2 + 1]));
    HIP_TRY(h, hipEventElapsedTime(&ms, h->ev[((size_t)slot * nl + i) * 2], h->ev[((size_t)slot * nl + i) * 2 + 1]));
    h->prof_sum[i] += ms;
  }
  h->prof_count++;
  h->slot_pending[slot] = 0;
  return VSS_OK;
}

int forward(vss_handle* h, const uint8_t* frames, int n, int fh, int fw, int fc, size_t rs, size_t fs,
            float* masks, hipStream_t s) {
  h->last_n = n;
  if (h->profile) {
    const int slot = h->prof_next;
    h->prof_next = (h->prof_next + 1) % vss_handle::kSlots;
    if (h->slot_pending[slot]) {
      int rc = harvest_slot(h, slot);
      if (rc) return rc;
    }
    int rc = enqueue_forward(h, frames, n, fh, fw, fc, rs, fs, masks, s, slot);
    if (!rc) h->slot_pending[slot] = h->use_forward ? 2 : 1;
    return rc;
  }
  if (!h->use_graph) return enqueue_forward(h, frames, n, fh, fw, fc, rs, fs, masks, s, -1);
  GraphKey key{frames, masks, n, fh, fw, fc, rs, fs};
  auto it = h->graphs.find(key);
  if (it == h->graphs.end()) {
    if (h->use_forward) {  // the task table is uploaded outside the capture
      FwdTask* t = nullptr;
      int cnt = 0;
      int rc = forward_tasks(h, n, &t, &cnt);
      if (rc) return rc;
    }
    hipGraph_t g = nullptr;
    hipGraphExec_t ge = nullptr;
    HIP_TRY(h, hipStreamBeginCapture(h->stream, hipStreamCaptureModeRelaxed));
    // Independent sub-batches on forked streams: their kernels overlap, which
    // fills the GPU while each chain waits on memory latency.
    const int nb = h->use_forward ? 1 : std::max(1, std::min(h->branches, n));
    int rc = VSS_OK;
    if (nb == 1) {
      rc = enqueue_forward(h, frames, n, fh, fw, fc, rs, fs, masks, h->stream, -1);
    } else {
      (void)hipEventRecord(h->fork_ev, h->stream);
      const int Hm = h->cfg.model_h, Wm = h->cfg.model_w;
      for (int b = 0; b < nb && !rc; ++b) {
        const int f0 = (int)((long)n * b / nb), f1 = (int)((long)n * (b + 1) / nb);
        hipStream_t bs = h->branch_streams[b];
        (void)hipStreamWaitEvent(bs, h->fork_ev, 0);
        rc = enqueue_forward(h, frames + (size_t)f0 * fs, f1 - f0, fh, fw, fc, rs, fs,
                             masks + (size_t)f0 * Hm * Wm, bs, -1, f0);
        (void)hipEventRecord(h->join_ev[b], bs);
        (void)hipStreamWaitEvent(h->stream, h->join_ev[b], 0);
      }
    }
    hipError_t e = hipStreamEndCapture(h->stream, &g);
    if (rc) {
      if (g) (void)hipGraphDestroy(g);
      return rc;
    }
    if (e != hipSuccess) return fail(h, VSS_E_HIP, std::string("hipStreamEndCapture: ") + hipGetErrorString(e));
    e = hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    if (e != hipSuccess) return fail(h, VSS_E_HIP, std::string("hipGraphInstantiate: ") + hipGetErrorString(e));
    if (h->graphs.size() >= 16) {  // bound the cache
      (void)hipGraphExecDestroy(h->graphs.begin()->second);
      h->graphs.erase(h->graphs.begin());
    }
    it = h->graphs.emplace(key, ge).first;
  }
  HIP_TRY(h, hipGraphLaunch(it->second, s));
  return VSS_OK;
}

struct Busy {
  vss_handle* h;
  bool ok;
  explicit Busy(vss_handle* hh) : h(hh) {
    int z = 0;
    ok = h->busy.compare_exchange_strong(z, 1);
  }
  void release() { if (ok) { h->busy.store(0); ok = false; } }
  ~Busy() { release(); }
};

void enqueue_upmask(const vss_handle* h, const float* d_masks, int n, int fh, int fw, float* d_out, hipStream_t s) {
  UpmaskParams p{};
  p.masks = d_masks;
  p.H = h->cfg.model_h;
  p.W = h->cfg.model_w;
  p.sy = (float)p.H / (float)fh;
  p.sx = (float)p.W / (float)fw;
  p.out = d_out;
  p.fh = fh;
  p.fw = fw;
  launch_upmask(p, n, s);
}

int stage_in(vss_handle* h, const uint8_t* frames, int n, int fh, int fw, int fc, size_t rs, float* masks_out,
             int out_mode) {
  if (!frames || !masks_out) return fail(h, VSS_E_INVALID_ARG, "null frames/masks_out");
  if (out_mode != VSS_OUT_MODEL && out_mode != VSS_OUT_FRAME)
    return fail(h, VSS_E_INVALID_ARG, "out_mode must be VSS_OUT_MODEL or VSS_OUT_FRAME");
  int rc = check_frames(h, n, fh, fw, fc, rs, rs * (size_t)fh);
  if (rc) return rc;
  const size_t bytes = (size_t)n * fh * rs;
  if (bytes > h->frame_cap)
    return fail(h, VSS_E_INVALID_ARG, "frames exceed the handle's staging capacity (max_frame_h/w)");
  if (out_mode == VSS_OUT_FRAME && !h->d_fmasks) {  // sized for max_batch frames of the largest size
    const size_t cap = (size_t)h->cfg.max_batch * h->cfg.max_frame_h * h->cfg.max_frame_w;
    if ((rc = dalloc(h, &h->d_fmasks, cap * 4))) return rc;
    HIP_TRY(h, hipHostMalloc((void**)&h->h_fmasks, cap * 4, hipHostMallocDefault));
    h->fmask_cap = cap;
  }
  if (out_mode == VSS_OUT_FRAME && (size_t)n * fh * fw > h->fmask_cap)
    return fail(h, VSS_E_INVALID_ARG, "frame-size masks exceed max_batch * max_frame_h * max_frame_w");
  // staged in 1 MiB pieces, each piece's DMA queued as soon as it is in the
  // pinned buffer, so the copy engine runs under the next piece's memcpy
  // (the staging buffer is free: the previous call on this handle has
  // finished — Busy — before this one starts)
  constexpr size_t kStageChunk = size_t(1) << 20;
  for (size_t off = 0; off < bytes; off += kStageChunk) {
    const size_t len = std::min(kStageChunk, bytes - off);
    std::memcpy(h->h_frames + off, frames + off, len);
    HIP_TRY(h, hipMemcpyAsync(h->d_frames + off, h->h_frames + off, len, hipMemcpyHostToDevice, h->stream));
  }
  rc = forward(h, h->d_frames, n, fh, fw, fc, rs, rs * (size_t)fh, h->d_masks, h->stream);
  if (rc) return rc;
  if (out_mode == VSS_OUT_FRAME) {
    enqueue_upmask(h, h->d_masks, n, fh, fw, h->d_fmasks, h->stream);
    h->out_src = h->h_fmasks;
    h->out_bytes = (size_t)n * fh * fw * 4;
    HIP_TRY(h, hipMemcpyAsync(h->h_fmasks, h->d_fmasks, h->out_bytes, hipMemcpyDeviceToHost, h->stream));
  } else {
    h->out_src = h->h_masks;
    h->out_bytes = (size_t)n * h->cfg.model_h * h->cfg.model_w * 4;
    HIP_TRY(h, hipMemcpyAsync(h->h_masks, h->d_masks, h->out_bytes, hipMemcpyDeviceToHost, h->stream));
  }
  return VSS_OK;
}

struct AsyncCtx {
  vss_handle* h;
  float* out;
  const float* src;
  size_t bytes;
  vss_callback cb;
  void* user;
};

void async_done(void* p) {
  AsyncCtx* c = static_cast<AsyncCtx*>(p);
  std::memcpy(c->out, c->src, c->bytes);
  c->h->busy.store(0);
  if (c->cb) c->cb(c->user, VSS_OK);
  delete c;
}

// Autotune: time every compiled tile of every block layer at max_batch on
// this device and keep the fastest.  The kernels' arithmetic does not depend
// on the tile (see block_lds), so this changes speed only, never results.
int autotune(vss_handle* h) {
  if (h->fwd_ok) return VSS_OK;  // the persistent forward's tiles are fixed (vss_mk.inc)
  const int N = h->cfg.max_batch;
  const int pi = h->cfg.dtype == VSS_DTYPE_F32 ? 0 : 1;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  HIP_TRY(h, hipEventCreate(&e0));
  HIP_TRY(h, hipEventCreate(&e1));
  int rc = VSS_OK;
  for (LayerPlan& l : h->L) {
    if (l.mode < 0) continue;
    const std::vector<const BlockEntry*> cands = tile_candidates(l);
    if (cands.size() < 2) continue;
    // three rounds over the candidates, each candidate's best round kept: one
    // timing per candidate let clock / cache noise pick a different tile per
    // run (a +-2% spread of the whole forward between runs)
    std::vector<float> best_of(cands.size(), 1e30f);
    std::vector<char> usable(cands.size(), 1);
    for (int round = 0; round < 3 && rc == VSS_OK; ++round) {
      for (size_t c = 0; c < cands.size(); ++c) {
        if (!usable[c]) continue;
        const BlockEntry* e = cands[c];
        set_tile(l, e);
        if (hipFuncSetAttribute((const void*)e->fn[pi], hipFuncAttributeMaxDynamicSharedMemorySize, (int)l.lds) !=
            hipSuccess) {
          usable[c] = 0;
          continue;
        }
        BlockParams p = block_params(h, l, N);
        if (flags_stem_in(l.flags))  // the staging buffer as frames: any bytes, valid memory
          p.stem = stem_params(h, h->L[l.rec.src], h->d_frames, (size_t)h->cfg.max_frame_w * 3,
                               (size_t)h->cfg.max_frame_w * 3 * h->cfg.max_frame_h, h->cfg.max_frame_h,
                               h->cfg.max_frame_w, 3, 0);
        if (flags_stem_in(l.flags)) p.stem.y = nullptr;  // timed as the forward runs it by default
        const dim3 grid(l.tiles_x, l.tiles_y, N * l.ks);
        for (int k = 0; k < 2; ++k) hipLaunchKernelGGL(e->fn[pi], grid, dim3(kThreads), l.lds, h->stream, p);
        (void)hipEventRecord(e0, h->stream);
        for (int k = 0; k < 8; ++k) hipLaunchKernelGGL(e->fn[pi], grid, dim3(kThreads), l.lds, h->stream, p);
        (void)hipEventRecord(e1, h->stream);
        float ms = 0.f;
        if (hipEventSynchronize(e1) != hipSuccess || hipEventElapsedTime(&ms, e0, e1) != hipSuccess ||
            hipGetLastError() != hipSuccess) {
          rc = fail(h, VSS_E_HIP, "autotune launch failed");
          break;
        }
        best_of[c] = std::min(best_of[c], ms);
      }
    }
    const BlockEntry* best = l.entry;
    float best_ms = 1e30f;
    for (size_t c = 0; c < cands.size(); ++c)
      if (usable[c] && best_of[c] < best_ms * 0.98f) {  // ties keep the earlier (planner-preferred) shape
        best_ms = best_of[c];
        best = cands[c];
      }
    set_tile(l, best);
    if (rc) break;
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return rc;
}

// Pin layers to given compiled tiles (after the planner and the autotuner):
// the tile-invariance tests run every compiled tile of every layer this way.
int force_tiles(vss_handle* h, const char* spec) {
  if (h->fwd_ok) return VSS_OK;  // the persistent forward's tiles are fixed (vss_mk.inc)
  const int pi = h->cfg.dtype == VSS_DTYPE_F32 ? 0 : 1;
  const char* s = spec;
  while (*s) {
    int layer = -1, th = 0, tw = 0, used = 0;
    if (std::sscanf(s, "%d:%dx%d%n", &layer, &th, &tw, &used) != 3 || layer < 0 || layer >= (int)h->L.size())
      return fail(h, VSS_E_INVALID_ARG, std::string("VSS_TILE: bad entry in '") + spec + "'");
    LayerPlan& l = h->L[layer];
    const BlockEntry* pick = nullptr;
    if (l.mode >= 0)
      for (const BlockEntry* e : tile_candidates(l))
        if (e->TH == th && e->TW == tw) pick = e;
    if (!pick)
      return fail(h, VSS_E_UNSUPPORTED, "VSS_TILE: layer " + std::to_string(layer) + " has no compiled " +
                                            std::to_string(th) + "x" + std::to_string(tw) + " tile");
    set_tile(l, pick);
    HIP_TRY(h, hipFuncSetAttribute((const void*)pick->fn[pi], hipFuncAttributeMaxDynamicSharedMemorySize, (int)l.lds));
    s += used;
    if (*s == ',') ++s;
  }
  return VSS_OK;
}

}  // namespace

extern "C" {

int vss_version(void) { return VSS_VERSION; }

const char* vss_last_error(const vss_handle* h) { return h ? h->err.c_str() : g_tls_error.c_str(); }

int vss_create(const vss_config* cfg, vss_handle** out) {
  if (!cfg || !out) return fail(nullptr, VSS_E_INVALID_ARG, "null cfg/out");
  *out = nullptr;
  if (cfg->model_h <= 0 || cfg->model_w <= 0 || cfg->model_h % 16 || cfg->model_w % 16)
    return fail(nullptr, VSS_E_INVALID_ARG, "model_h/model_w must be positive multiples of 16");
  if (cfg->dtype != VSS_DTYPE_F32 && cfg->dtype != VSS_DTYPE_BF16X2)
    return fail(nullptr, VSS_E_INVALID_ARG, "unknown dtype");
  if (cfg->max_batch < 1 || cfg->max_frame_h < 1 || cfg->max_frame_w < 1)
    return fail(nullptr, VSS_E_INVALID_ARG, "max_batch/max_frame_h/max_frame_w must be >= 1");
  if (!cfg->weights_path) return fail(nullptr, VSS_E_INVALID_ARG, "weights_path is required");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
    return fail(nullptr, VSS_E_HIP, "no HIP device available");
  if (cfg->device_id < 0 || cfg->device_id >= ndev) return fail(nullptr, VSS_E_INVALID_ARG, "bad device_id");
  vss_handle* h = new vss_handle();
  h->cfg = *cfg;
  h->weights_path = cfg->weights_path;
  h->cfg.weights_path = nullptr;
  h->device = cfg->device_id;
  auto bail = [&](int rc) {
    g_tls_error = h->err;
    vss_destroy(h);
    return rc;
  };
  if (hipSetDevice(h->device) != hipSuccess) return bail(fail(h, VSS_E_HIP, "hipSetDevice failed"));
  if (const char* ev = std::getenv("VSS_KSPLIT_PIXELS")) h->ksplit_pixels = std::atol(ev);
  if (const char* ev = std::getenv("VSS_FORWARD")) h->want_forward = std::atoi(ev) != 0;
  if (const char* ev = std::getenv("VSS_FUSE_STEM")) h->fuse_stem = std::atoi(ev) != 0;
  int rc = load_weights(h);
  if (!rc) rc = plan(h);
  if (!rc) rc = upload(h);
  if (rc) return bail(rc);
  if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess)
    return bail(fail(h, VSS_E_HIP, "hipStreamCreate failed"));
  for (int b = 0; b < vss_handle::kMaxBranches; ++b)
    if (hipStreamCreateWithFlags(&h->branch_streams[b], hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&h->join_ev[b], hipEventDisableTiming) != hipSuccess)
      return bail(fail(h, VSS_E_HIP, "branch stream/event create failed"));
  if (hipEventCreateWithFlags(&h->fork_ev, hipEventDisableTiming) != hipSuccess)
    return bail(fail(h, VSS_E_HIP, "hipEventCreate failed"));
  h->frame_cap = (size_t)cfg->max_batch * cfg->max_frame_h * cfg->max_frame_w * 4;
  if ((rc = dalloc(h, &h->d_frames, h->frame_cap))) return bail(rc);
  if ((rc = dalloc(h, &h->d_masks, (size_t)cfg->max_batch * cfg->model_h * cfg->model_w * 4))) return bail(rc);
  if ((rc = dalloc(h, &h->d_post_alpha, (size_t)cfg->max_batch * cfg->model_h * cfg->model_w * 4))) return bail(rc);
  if ((rc = dalloc(h, &h->d_post_u8, (size_t)cfg->max_batch * cfg->model_h * cfg->model_w))) return bail(rc);
  if (hipHostMalloc((void**)&h->h_frames, h->frame_cap, hipHostMallocDefault) != hipSuccess ||
      hipHostMalloc((void**)&h->h_masks, (size_t)cfg->max_batch * cfg->model_h * cfg->model_w * 4,
                    hipHostMallocDefault) != hipSuccess)
    return bail(fail(h, VSS_E_OOM, "hipHostMalloc staging failed"));
  for (const LayerPlan& l : h->L)
    if (l.entry)
      for (BlockFn fn : l.entry->fn)
        if (hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)l.lds) != hipSuccess)
          return bail(fail(h, VSS_E_HIP, "hipFuncSetAttribute(max dynamic LDS) failed"));
  const int nl = (int)h->L.size();
  h->ev.resize((size_t)vss_handle::kSlots * nl * 2);
  for (auto& e : h->ev)
    if (hipEventCreate(&e) != hipSuccess) return bail(fail(h, VSS_E_HIP, "hipEventCreate failed"));
  h->slot_pending.assign(vss_handle::kSlots, 0);
  h->prof_sum.assign(nl, 0.0);
  if ((rc = setup_forward(h))) return bail(rc);
  if (!(cfg->flags & VSS_CREATE_NO_AUTOTUNE) && (rc = autotune(h))) return bail(rc);
  if (const char* ev = std::getenv("VSS_TILE"))  // tests / scans: "layer:THxTW[,layer:THxTW...]"
    if ((rc = force_tiles(h, ev))) return bail(rc);
  *out = h;
  return VSS_OK;
}

void vss_destroy(vss_handle* h) {
  if (!h) return;
  (void)hipSetDevice(h->device);
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  for (auto& kv : h->graphs) (void)hipGraphExecDestroy(kv.second);
  for (auto e : h->ev)
    if (e) (void)hipEventDestroy(e);
  for (int b = 0; b < vss_handle::kMaxBranches; ++b) {
    if (h->branch_streams[b]) (void)hipStreamDestroy(h->branch_streams[b]);
    if (h->join_ev[b]) (void)hipEventDestroy(h->join_ev[b]);
  }
  if (h->fork_ev) (void)hipEventDestroy(h->fork_ev);
  for (void* p : h->dev_allocs) (void)hipFree(p);
  if (h->h_frames) (void)hipHostFree(h->h_frames);
  if (h->h_masks) (void)hipHostFree(h->h_masks);
  if (h->h_fmasks) (void)hipHostFree(h->h_fmasks);
  if (h->fwd_dbg) (void)hipHostFree(h->fwd_dbg);
  if (h->stream) (void)hipStreamDestroy(h->stream);
  delete h;
}

int vss_get_info(const vss_handle* h, vss_info* info) {
  if (!h || !info) return VSS_E_INVALID_ARG;
  info->mask_h = h->cfg.model_h;
  info->mask_w = h->cfg.model_w;
  info->n_layers = (int)h->L.size();
  info->dtype = h->cfg.dtype;
  info->device_bytes = h->dev_bytes;
  return VSS_OK;
}

int vss_segment(vss_handle* h, const uint8_t* frames, int n, int height, int width, int channels,
                size_t row_stride, float* masks_out, int out_mode) {
  if (!h) return fail(nullptr, VSS_E_INVALID_ARG, "null handle");
  Busy b(h);
  if (!b.ok) return fail(h, VSS_E_BUSY, "a call is already in flight on this handle");
  HIP_TRY(h, hipSetDevice(h->device));
  int rc = stage_in(h, frames, n, height, width, channels, row_stride, masks_out, out_mode);
  if (rc) return rc;
  HIP_TRY(h, hipStreamSynchronize(h->stream));
  std::memcpy(masks_out, h->out_src, h->out_bytes);
  return VSS_OK;
}

int vss_segment_async(vss_handle* h, const uint8_t* frames, int n, int height, int width, int channels,
                      size_t row_stride, float* masks_out, int out_mode, vss_callback cb, void* user) {
  if (!h) return fail(nullptr, VSS_E_INVALID_ARG, "null handle");
  Busy b(h);
  if (!b.ok) return fail(h, VSS_E_BUSY, "a call is already in flight on this handle");
  HIP_TRY(h, hipSetDevice(h->device));
  int rc = stage_in(h, frames, n, height, width, channels, row_stride, masks_out, out_mode);
  if (rc) return rc;
  AsyncCtx* c = new AsyncCtx{h, masks_out, h->out_src, h->out_bytes, cb, user};
  hipError_t e = hipLaunchHostFunc(h->stream, async_done, c);
  if (e != hipSuccess) {
    delete c;
    return fail(h, VSS_E_HIP, std::string("hipLaunchHostFunc: ") + hipGetErrorString(e));
  }
  b.ok = false;  // released by async_done
  return VSS_OK;
}

int vss_segment_device(vss_handle* h, const uint8_t* d_frames, int n, int height, int width, int channels,
                       size_t row_stride, size_t frame_stride, float* d_masks, void* stream) {
  if (!h) return fail(nullptr, VSS_E_INVALID_ARG, "null handle");
  if (!d_frames || !d_masks) return fail(h, VSS_E_INVALID_ARG, "null device pointer");
  Busy b(h);
  if (!b.ok) return fail(h, VSS_E_BUSY, "a call is already in flight on this handle");
  int rc = check_frames(h, n, height, width, channels, row_stride, frame_stride);
  if (rc) return rc;
  HIP_TRY(h, hipSetDevice(h->device));
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : h->stream;
  return forward(h, d_frames, n, height, width, channels, row_stride, frame_stride, d_masks, s);
}

int vss_mask_to_frame_device(vss_handle* h, const float* d_masks, int n, int frame_h, int frame_w, float* d_out,
                             void* stream) {
  if (!h) return fail(nullptr, VSS_E_INVALID_ARG, "null handle");
  if (!d_masks || !d_out) return fail(h, VSS_E_INVALID_ARG, "null device pointer");
  if (n < 1 || n > h->cfg.max_batch || frame_h < 1 || frame_w < 1)
    return fail(h, VSS_E_INVALID_ARG, "n must be 1..max_batch and the frame size positive");
  HIP_TRY(h, hipSetDevice(h->device));
  enqueue_upmask(h, d_masks, n, frame_h, frame_w, d_out, stream ? static_cast<hipStream_t>(stream) : h->stream);
  HIP_TRY(h, hipGetLastError());
  return VSS_OK;
}

int vss_preprocess_device(vss_handle* h, const uint8_t* d_frames, int n, int height, int width, int channels,
                          size_t row_stride, size_t frame_stride, float* d_out, void* stream) {
  if (!h) return fail(nullptr, VSS_E_INVALID_ARG, "null handle");
  if (!d_frames || !d_out) return fail(h, VSS_E_INVALID_ARG, "null device pointer");
  int rc = check_frames(h, n, height, width, channels, row_stride, frame_stride);
  if (rc) return rc;
  HIP_TRY(h, hipSetDevice(h->device));
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : h->stream;
  PrepParams p{};
  p.frames = d_frames; p.row_stride = (long)row_stride; p.frame_stride = (long)frame_stride;
  p.fh = height; p.fw = width; p.fc = channels; p.Hm = h->cfg.model_h; p.Wm = h->cfg.model_w;
  p.ry = (float)((double)height / (double)p.Hm);
  p.rx = (float)((double)width / (double)p.Wm);
  p.out = d_out; p.N = n;
  const long total = (long)n * p.Hm * p.Wm;
  const int grid = (int)std::min<long>((total + 255) / 256, 4096);
  hipLaunchKernelGGL(prep_kernel(), dim3(grid), dim3(256), 0, s, p);
  HIP_TRY(h, hipGetLastError());
  return VSS_OK;
}

int vss_synchronize(vss_handle* h) {
  if (!h) return fail(nullptr, VSS_E_INVALID_ARG, "null handle");
  HIP_TRY(h, hipSetDevice(h->device));
  HIP_TRY(h, hipStreamSynchronize(h->stream));
  return VSS_OK;
}

int vss_set_option(vss_handle* h, int option, int value) {
  if (!h) return fail(nullptr, VSS_E_INVALID_ARG, "null handle");
  if (option == VSS_OPT_FORWARD) {
    if (value && !h->fwd_ok)
      return fail(h, VSS_E_UNSUPPORTED, "this plan has no persistent forward (a layer shape outside vss_mk.inc)");
    if ((value ? 1 : 0) != h->use_forward) {
      for (auto& kv : h->graphs) (void)hipGraphExecDestroy(kv.second);
      h->graphs.clear();
    }
    h->use_forward = value ? 1 : 0;
    return VSS_OK;
  }
  if (option == VSS_OPT_KEEP_STEM) {
    if ((value ? 1 : 0) != h->keep_stem) {  // the captured graphs hold the stem pointer
      for (auto& kv : h->graphs) (void)hipGraphExecDestroy(kv.second);
      h->graphs.clear();
    }
    h->keep_stem = value ? 1 : 0;
    return VSS_OK;
  }
  if (option == VSS_OPT_USE_GRAPH) h->use_graph = value ? 1 : 0;
  else if (option == VSS_OPT_PROFILE) h->profile = value ? 1 : 0;
  else if (option == VSS_OPT_BRANCHES) {
    if (value < 1 || value > vss_handle::kMaxBranches) return fail(h, VSS_E_INVALID_ARG, "branches must be 1..8");
    if (value != h->branches) {
      for (auto& kv : h->graphs) (void)hipGraphExecDestroy(kv.second);
      h->graphs.clear();
    }
    h->branches = value;
  }
  else return fail(h, VSS_E_INVALID_ARG, "unknown option");
  return VSS_OK;
}

int vss_get_option(vss_handle* h, int option, int* value) {
  if (!h) return fail(nullptr, VSS_E_INVALID_ARG, "null handle");
  if (!value) return fail(h, VSS_E_INVALID_ARG, "null value");
  switch (option) {
    case VSS_OPT_USE_GRAPH: *value = h->use_graph; return VSS_OK;
    case VSS_OPT_PROFILE: *value = h->profile; return VSS_OK;
    case VSS_OPT_BRANCHES: *value = h->branches; return VSS_OK;
    case VSS_OPT_FORWARD: *value = h->use_forward; return VSS_OK;
    case VSS_OPT_KEEP_STEM: *value = h->keep_stem; return VSS_OK;
    case VSS_OPT_FORWARD_FAULTS: {
      *value = 0;
      if (!h->d_fwd_ctl) return VSS_OK;
      HIP_TRY(h, hipSetDevice(h->device));
      HIP_TRY(h, hipDeviceSynchronize());
      unsigned w = 0;
      unsigned* fw = h->d_fwd_ctl + kFwdQueues * kFwdLine + 1;
      HIP_TRY(h, hipMemcpy(&w, fw, sizeof(w), hipMemcpyDeviceToHost));
      HIP_TRY(h, hipMemset(fw, 0, sizeof(unsigned)));
      *value = (int)w;
      return VSS_OK;
    }
    default: return fail(h, VSS_E_INVALID_ARG, "unknown option");
  }
}

int vss_forward_kernel(const vss_handle* h, char* buf, int cap) {
  if (!h || !buf || cap < 1) return VSS_E_INVALID_ARG;
  if (!h->fwd_ok) return VSS_E_UNSUPPORTED;
  char tmp[96];
  std::snprintf(tmp, sizeof(tmp), "void vss::k_forward<%d>(vss::FwdParams)",
                h->cfg.dtype == VSS_DTYPE_F32 ? PREC_F32 : PREC_BF16X2);
  std::snprintf(buf, (size_t)cap, "%s", tmp);
  return (int)std::strlen(tmp);
}

int vss_profile_read_forward(vss_handle* h, double* ms, int* count) {
  if (!h || !ms) return fail(h, VSS_E_INVALID_ARG, "null handle/ms");
  HIP_TRY(h, hipSetDevice(h->device));
  for (int s = 0; s < vss_handle::kSlots; ++s)
    if (h->slot_pending[s]) {
      int rc = harvest_slot(h, s);
      if (rc) return rc;
    }
  *ms = h->fwd_prof_count ? h->fwd_prof_sum / h->fwd_prof_count : 0.0;
  if (count) *count = h->fwd_prof_count;
  h->fwd_prof_sum = 0.0;
  h->fwd_prof_count = 0;
  return VSS_OK;
}

// Debug (not in vss.h): per-task stamps of the last VSS_FWD_TRACE launch, [n][4]
// {taken, deps met, body done, workgroup}; returns the task count.
int vss_fwd_trace_read(vss_handle* h, unsigned long long* out, int cap) {
  if (!h || !out || !h->fwd_trace) return VSS_E_INVALID_ARG;
  HIP_TRY(h, hipDeviceSynchronize());
  const int n = std::min(cap, h->fwd_trace_n);
  HIP_TRY(h, hipMemcpy(out, h->fwd_trace, (size_t)n * 4 * 8, hipMemcpyDeviceToHost));
  return n;
}

// Debug (not in vss.h): the k_forward per-workgroup state words (VSS_FWD_DEBUG),
// read WITHOUT synchronising, so a stuck launch can be inspected.
int vss_fwd_debug(const vss_handle* h, unsigned* out, int cap, int* grid) {
  if (!h || !out || !h->fwd_dbg) return VSS_E_INVALID_ARG;
  const int n = std::min(cap, h->fwd_grid * 4);
  for (int i = 0; i < n; ++i) out[i] = __atomic_load_n(h->fwd_dbg + i, __ATOMIC_RELAXED);
  if (grid) *grid = h->fwd_grid;
  return n;
}

int vss_layer_shape(const vss_handle* h, int layer, int* c, int* hh, int* ww) {
  if (!h || layer < 0 || layer >= (int)h->L.size()) return VSS_E_INVALID_ARG;
  if (c) *c = h->L[layer].C;
  if (hh) *hh = h->L[layer].H;
  if (ww) *ww = h->L[layer].W;
  return VSS_OK;
}

int vss_layer_tiles(const vss_handle* h, int layer, int* th, int* tw, int cap) {
  if (!h || layer < 0 || layer >= (int)h->L.size() || cap < 0 || (cap > 0 && (!th || !tw))) return VSS_E_INVALID_ARG;
  const LayerPlan& l = h->L[layer];
  if (l.mode < 0) return 0;
  int n = 0;
  for (const BlockEntry* e : tile_candidates(l)) {
    if (n < cap) {
      th[n] = e->TH;
      tw[n] = e->TW;
    }
    ++n;
  }
  return std::min(n, cap);
}

int vss_layer_kernel(const vss_handle* h, int layer, char* buf, int cap) {
  if (!h || layer < 0 || layer >= (int)h->L.size() || !buf || cap < 1) return VSS_E_INVALID_ARG;
  const LayerPlan& l = h->L[layer];
  const int prec = h->cfg.dtype == VSS_DTYPE_F32 ? PREC_F32 : PREC_BF16X2;
  char tmp[160];
  if (l.fused) std::snprintf(tmp, sizeof(tmp), "(fused into layer %d)", layer + 1);
  else if (l.rec.kind == K_STEM) std::snprintf(tmp, sizeof(tmp), "void vss::k_stem<16>(vss::StemParams)");
  else if (l.rec.kind == K_HEAD) std::snprintf(tmp, sizeof(tmp), "void vss::k_head<16>(vss::HeadParams)");
  else {
    const BlockEntry* e = l.entry;
    std::snprintf(tmp, sizeof(tmp), "void vss::k_block<%d, %d, %d, %d, %d, %d, %d, %d, %d, %d>(vss::BlockParams)",
                  e->mode, e->stride, e->TH, e->TW, e->cin, e->cskip, e->chid, e->cout, e->flags, prec);
  }
  const int len = (int)std::strlen(tmp);
  std::snprintf(buf, (size_t)cap, "%s", tmp);
  return len;
}

int vss_read_layer(vss_handle* h, int layer, int n, float* host_out) {
  if (!h) return fail(nullptr, VSS_E_INVALID_ARG, "null handle");
  if (layer < 0 || layer >= (int)h->L.size() || !host_out || n < 1 || n > h->cfg.max_batch)
    return fail(h, VSS_E_INVALID_ARG, "bad layer/n/out");
  const LayerPlan& l = h->L[layer];
  if (l.rec.kind == K_HEAD) return fail(h, VSS_E_INVALID_ARG, "the head's output is the mask buffer");
  if (l.rec.kind == K_STEM && !h->keep_stem)
    for (const LayerPlan& c : h->L)
      if (flags_stem_in(c.flags))
        return fail(h, VSS_E_INVALID_ARG,
                    "the stem is fused into layer 1 and not stored: set VSS_OPT_KEEP_STEM before the forward");
  HIP_TRY(h, hipSetDevice(h->device));
  HIP_TRY(h, hipDeviceSynchronize());
  const size_t cnt = (size_t)n * l.H * l.W * l.C;
  HIP_TRY(h, hipMemcpy(host_out, l.act, cnt * 4, hipMemcpyDeviceToHost));
  if (l.ks > 1) {  // a split layer's value = its parts summed in part order, as its consumers do
    std::vector<float> part(cnt);
    for (int q = 1; q < l.ks; ++q) {
      HIP_TRY(h, hipMemcpy(part.data(), l.act + q * l.part_stride, cnt * 4, hipMemcpyDeviceToHost));
      for (size_t k = 0; k < cnt; ++k) host_out[k] += part[k];
    }
  }
  return VSS_OK;
}

int vss_profile_read(vss_handle* h, double* ms_per_layer, int cap, int* count) {
  if (!h) return fail(nullptr, VSS_E_INVALID_ARG, "null handle");
  const int nl = (int)h->L.size();
  if (!ms_per_layer || cap < nl) return fail(h, VSS_E_INVALID_ARG, "cap < n_layers");
  HIP_TRY(h, hipSetDevice(h->device));
  for (int s = 0; s < vss_handle::kSlots; ++s)
    if (h->slot_pending[s]) {
      int rc = harvest_slot(h, s);
      if (rc) return rc;
    }
  for (int i = 0; i < nl; ++i) ms_per_layer[i] = h->prof_count ? h->prof_sum[i] / h->prof_count : 0.0;
  if (count) *count = h->prof_count;
  std::fill(h->prof_sum.begin(), h->prof_sum.end(), 0.0);
  h->prof_count = 0;
  return VSS_OK;
}

}  // extern "C"

// ---- post-processing chain (vss_post.hip) ----------------------------------
struct vss_post_state {
  vss_handle* h = nullptr;
  vss_post_config cfg{};
  float* state = nullptr;   // [P] prevAlpha
  int* valid = nullptr;     // device flag: 0 before the stream's first frame
  float* ema = nullptr;     // [max_batch][P]
  float* state2 = nullptr;  // [P] the other prevAlpha buffer (the stabilised EMA reads one, writes the other)
  FaceFrame* d_faces = nullptr;       // [max_batch] face inputs set by vss_post_set_faces
  const FaceFrame* faces = nullptr;   // the next call's face inputs (d_faces or a caller's device array)
  int faces_n = 0;                    // ... for this many frames (0: none)
  double* rtab = nullptr;   // exp(-r / (2 sigma_r^2)), r in [0, 3*255^2]
  double sw[3] = {0, 0, 0};
  double tab_sigma = -1.0;
  std::string err;
};

namespace {

constexpr int kRangeTab = 3 * 255 * 255 + 1;

int post_fail(vss_post_state* st, int code, const std::string& msg) {
  st->err = msg;
  if (st->h) st->h->err = msg;
  return code;
}

// Bilateral weights as the reference computes them (Math.exp of the same
// double quotients); built on the host so they are the exact doubles the
// oracle's libm produces.
int post_tables(vss_post_state* st) {
  const vss_post_config& c = st->cfg;
  const double ts2 = 2.0 * c.sigma_spatial * c.sigma_spatial, tr2 = 2.0 * c.sigma_range * c.sigma_range;
  for (int k = 0; k < 3; ++k) st->sw[k] = std::exp(-(double)k / ts2);
  if (st->tab_sigma != c.sigma_range) {
    std::vector<double> t(kRangeTab);
    for (int r = 0; r < kRangeTab; ++r) t[r] = std::exp(-(double)r / tr2);
    if (hipMemcpy(st->rtab, t.data(), t.size() * 8, hipMemcpyHostToDevice) != hipSuccess)
      return post_fail(st, VSS_E_HIP, "post: table upload failed");
    st->tab_sigma = c.sigma_range;
  }
  return VSS_OK;
}

int post_enqueue(vss_post_state* st, const uint8_t* d_frames, int n, int fh, int fw, int fc, size_t rs, size_t fs,
                 const float* d_masks, float* d_alpha, uint8_t* d_u8, hipStream_t s) {
  vss_handle* h = st->h;
  const int H = h->cfg.model_h, W = h->cfg.model_w;
  const FaceFrame* faces = nullptr;
  if (st->faces_n) {
    if (st->faces_n != n)
      return post_fail(st, VSS_E_INVALID_ARG, "vss_post_set_faces was given " + std::to_string(st->faces_n) +
                                                  " frames, this call has " + std::to_string(n));
    faces = st->faces;
    st->faces_n = 0;  // consumed
    st->faces = nullptr;
  }
  if (faces) {
    // the stabilised EMA, one frame at a time (the warp reads prevAlpha at other pixels)
    for (int t = 0; t < n; ++t) {
      PostFaceEmaParams pe{};
      pe.mask = d_masks + (long)t * H * W;
      pe.prev = st->state;
      pe.next = st->state2;
      pe.ema = st->ema + (long)t * H * W;
      pe.valid = st->valid;
      pe.first = t == 0;
      pe.face = faces + t;
      pe.H = H;
      pe.W = W;
      pe.a = st->cfg.ema;
      launch_post_face_ema(pe, s);
      std::swap(st->state, st->state2);
    }
  } else {
    PostEmaParams pe{};
    pe.masks = d_masks;
    pe.ema = st->ema;
    pe.state = st->state;
    pe.valid = st->valid;
    pe.n = n;
    pe.P = (long)H * W;
    pe.a = st->cfg.ema;
    launch_post_ema(pe, s);
  }
  HIP_TRY(h, hipMemsetAsync(st->valid, 1, sizeof(int), s));  // the stream has seen its first frame
  PostFilterParams pf{};
  pf.faces = faces;
  pf.ema = st->ema;
  pf.frames = d_frames;
  pf.row_stride = (long)rs;
  pf.frame_stride = (long)fs;
  pf.fh = fh; pf.fw = fw; pf.fc = fc;
  pf.ry = (float)((double)fh / (double)H);
  pf.rx = (float)((double)fw / (double)W);
  pf.H = H; pf.W = W;
  pf.rtab = st->rtab;
  for (int k = 0; k < 3; ++k) pf.sw[k] = st->sw[k];
  pf.lo = st->cfg.noise_cutoff;
  pf.hi = st->cfg.high_threshold;
  pf.denom = std::max(1e-6, st->cfg.high_threshold - st->cfg.noise_cutoff);
  pf.gamma = st->cfg.gamma;
  pf.use_bilateral = st->cfg.use_bilateral;
  pf.alpha = d_alpha;
  pf.alpha_u8 = d_u8;
  launch_post_filter(pf, n, s);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return post_fail(st, VSS_E_HIP, std::string("post launch: ") + hipGetErrorString(e));
  return VSS_OK;
}

}  // namespace

extern "C" {

void vss_post_config_default(vss_post_config* c) {
  if (!c) return;
  c->ema = 0.55;
  c->noise_cutoff = 0.06;
  c->high_threshold = 0.95;
  c->gamma = 0.4;
  c->sigma_spatial = 1.0;
  c->sigma_range = 12.0;
  c->use_bilateral = 1;
}

int vss_post_create(vss_handle* h, const vss_post_config* cfg, vss_post_state** out) {
  if (!h || !out) return fail(h, VSS_E_INVALID_ARG, "null handle/out");
  *out = nullptr;
  if (h->cfg.model_h < 3 || h->cfg.model_w < 3) return fail(h, VSS_E_UNSUPPORTED, "mask too small for post");
  vss_post_state* st = new vss_post_state();
  st->h = h;
  if (cfg) st->cfg = *cfg;
  else vss_post_config_default(&st->cfg);
  const size_t P = (size_t)h->cfg.model_h * h->cfg.model_w;
  auto bail = [&](int rc) {
    vss_post_destroy(st);
    return rc;
  };
  HIP_TRY(h, hipSetDevice(h->device));
  if (hipMalloc(&st->state, P * 4) != hipSuccess || hipMalloc(&st->valid, 16) != hipSuccess ||
      hipMalloc(&st->ema, P * 4 * h->cfg.max_batch) != hipSuccess || hipMalloc(&st->state2, P * 4) != hipSuccess ||
      hipMalloc(&st->d_faces, sizeof(FaceFrame) * h->cfg.max_batch) != hipSuccess ||
      hipMalloc(&st->rtab, (size_t)kRangeTab * 8) != hipSuccess)
    return bail(fail(h, VSS_E_OOM, "post: hipMalloc failed"));
  if (hipMemset(st->valid, 0, 16) != hipSuccess || hipMemset(st->state, 0, P * 4) != hipSuccess)
    return bail(fail(h, VSS_E_HIP, "post: hipMemset failed"));
  int rc = post_tables(st);
  if (rc) return bail(rc);
  *out = st;
  return VSS_OK;
}

void vss_post_destroy(vss_post_state* st) {
  if (!st) return;
  if (st->h) {
    (void)hipSetDevice(st->h->device);
    (void)hipStreamSynchronize(st->h->stream);
  }
  if (st->state) (void)hipFree(st->state);
  if (st->valid) (void)hipFree(st->valid);
  if (st->ema) (void)hipFree(st->ema);
  if (st->state2) (void)hipFree(st->state2);
  if (st->d_faces) (void)hipFree(st->d_faces);
  if (st->rtab) (void)hipFree(st->rtab);
  delete st;
}

int vss_post_reset(vss_post_state* st) {
  if (!st) return VSS_E_INVALID_ARG;
  HIP_TRY(st->h, hipSetDevice(st->h->device));
  HIP_TRY(st->h, hipStreamSynchronize(st->h->stream));
  HIP_TRY(st->h, hipMemset(st->valid, 0, sizeof(int)));
  st->faces_n = 0;
  st->faces = nullptr;
  return VSS_OK;
}

static_assert(sizeof(FaceFrame) == sizeof(vss_face_frame), "FaceFrame mirrors vss_face_frame");

int vss_post_set_faces(vss_post_state* st, const vss_face_frame* faces, int n) {
  if (!st) return VSS_E_INVALID_ARG;
  if (!faces || n < 1 || n > st->h->cfg.max_batch) return post_fail(st, VSS_E_INVALID_ARG, "faces: 1..max_batch frames");
  HIP_TRY(st->h, hipSetDevice(st->h->device));
  HIP_TRY(st->h, hipMemcpyAsync(st->d_faces, faces, sizeof(FaceFrame) * n, hipMemcpyHostToDevice, st->h->stream));
  st->faces = st->d_faces;
  st->faces_n = n;
  return VSS_OK;
}

int vss_post_set_faces_device(vss_post_state* st, const vss_face_frame* d_faces, int n) {
  if (!st) return VSS_E_INVALID_ARG;
  if (!d_faces || n < 1 || n > st->h->cfg.max_batch)
    return post_fail(st, VSS_E_INVALID_ARG, "faces: a device array of 1..max_batch frames");
  st->faces = reinterpret_cast<const FaceFrame*>(d_faces);
  st->faces_n = n;
  return VSS_OK;
}

int vss_post_set_config(vss_post_state* st, const vss_post_config* cfg) {
  if (!st || !cfg) return VSS_E_INVALID_ARG;
  if (cfg->sigma_spatial <= 0 || cfg->sigma_range <= 0) return post_fail(st, VSS_E_INVALID_ARG, "sigmas must be > 0");
  HIP_TRY(st->h, hipSetDevice(st->h->device));
  HIP_TRY(st->h, hipStreamSynchronize(st->h->stream));
  st->cfg = *cfg;
  return post_tables(st);
}

int vss_postprocess_device(vss_post_state* st, const uint8_t* d_frames, int n, int height, int width, int channels,
                           size_t row_stride, size_t frame_stride, const float* d_masks, float* d_alpha,
                           uint8_t* d_alpha_u8, void* stream) {
  if (!st) return fail(nullptr, VSS_E_INVALID_ARG, "null post state");
  vss_handle* h = st->h;
  if (!d_masks || (!d_frames && st->cfg.use_bilateral)) return fail(h, VSS_E_INVALID_ARG, "null device pointer");
  int rc = check_frames(h, n, height, width, channels, row_stride, frame_stride);
  if (rc) return rc;
  HIP_TRY(h, hipSetDevice(h->device));
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : h->stream;
  return post_enqueue(st, d_frames, n, height, width, channels, row_stride, frame_stride, d_masks, d_alpha,
                      d_alpha_u8, s);
}

int vss_segment_post(vss_handle* h, vss_post_state* st, const uint8_t* frames, int n, int height, int width,
                     int channels, size_t row_stride, float* alpha_out, uint8_t* alpha_u8_out) {
  if (!h || !st || st->h != h) return fail(h, VSS_E_INVALID_ARG, "handle / post state mismatch");
  if (!alpha_out && !alpha_u8_out) return fail(h, VSS_E_INVALID_ARG, "no output requested");
  Busy b(h);
  if (!b.ok) return fail(h, VSS_E_BUSY, "a call is already in flight on this handle");
  HIP_TRY(h, hipSetDevice(h->device));
  const size_t P = (size_t)h->cfg.model_h * h->cfg.model_w;
  int rc = stage_in(h, frames, n, height, width, channels, row_stride, h->h_masks, VSS_OUT_MODEL);
  if (rc) return rc;
  // outputs: alpha into d_masks' tail is not allowed (masks are the input): use the post scratch
  float* d_alpha = alpha_out ? h->d_post_alpha : nullptr;
  uint8_t* d_u8 = alpha_u8_out ? h->d_post_u8 : nullptr;
  rc = post_enqueue(st, h->d_frames, n, height, width, channels, row_stride, row_stride * (size_t)height,
                    h->d_masks, d_alpha, d_u8, h->stream);
  if (rc) return rc;
  if (alpha_out) HIP_TRY(h, hipMemcpyAsync(alpha_out, d_alpha, (size_t)n * P * 4, hipMemcpyDeviceToHost, h->stream));
  if (alpha_u8_out)
    HIP_TRY(h, hipMemcpyAsync(alpha_u8_out, d_u8, (size_t)n * P, hipMemcpyDeviceToHost, h->stream));
  HIP_TRY(h, hipStreamSynchronize(h->stream));
  return VSS_OK;
}

}  // extern "C"

#ifdef VSS_TRACE
// Trace build only: the stamps of `layer`'s last launch, [wgs][16] u64
// (s_memrealtime ticks, 100 MHz).  Returns the workgroup count.
extern "C" int vss_trace_read(vss_handle* h, int layer, unsigned long long* out, int cap) {
  if (!h || layer < 0 || layer >= (int)h->L.size() || !out) return VSS_E_INVALID_ARG;
  HIP_TRY(h, hipStreamSynchronize(h->stream));
  const int wgs = std::min(h->trace_wgs[layer], cap);
  HIP_TRY(h, hipMemcpy(out, h->trace[layer], (size_t)wgs * 16 * 8, hipMemcpyDeviceToHost));
  return wgs;
}
#endif

// ---- compositing (vss_post.hip k_composite) ---------------------------------
namespace {

int composite_enqueue(vss_handle* h, const uint8_t* d_frames, int n, int fh, int fw, int fc, size_t rs, size_t fs,
                      const uint8_t* d_alpha, uint8_t* d_out, size_t ors, size_t ofs, hipStream_t s) {
  CompositeParams p{};
  p.frames = d_frames;
  p.row_stride = (long)rs;
  p.frame_stride = (long)fs;
  p.fh = fh; p.fw = fw; p.fc = fc;
  p.alpha = d_alpha;
  p.H = h->cfg.model_h; p.W = h->cfg.model_w;
  p.sy = (float)p.H / (float)fh;
  p.sx = (float)p.W / (float)fw;
  p.out = d_out;
  p.out_row_stride = (long)ors;
  p.out_frame_stride = (long)ofs;
  launch_composite(p, n, s);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(h, VSS_E_HIP, std::string("composite launch: ") + hipGetErrorString(e));
  return VSS_OK;
}

}  // namespace

extern "C" {

int vss_composite_device(vss_handle* h, const uint8_t* d_frames, int n, int height, int width, int channels,
                         size_t row_stride, size_t frame_stride, const uint8_t* d_alpha_u8, uint8_t* d_out_rgba,
                         size_t out_row_stride, size_t out_frame_stride, void* stream) {
  if (!h) return fail(nullptr, VSS_E_INVALID_ARG, "null handle");
  if (!d_frames || !d_alpha_u8 || !d_out_rgba) return fail(h, VSS_E_INVALID_ARG, "null device pointer");
  int rc = check_frames(h, n, height, width, channels, row_stride, frame_stride);
  if (rc) return rc;
  if (out_row_stride < (size_t)width * 4 || out_row_stride % 4 || out_frame_stride < out_row_stride * height ||
      (reinterpret_cast<uintptr_t>(d_out_rgba) & 3))
    return fail(h, VSS_E_INVALID_ARG, "bad RGBA output geometry (row stride >= 4*width, multiple of 4)");
  HIP_TRY(h, hipSetDevice(h->device));
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : h->stream;
  return composite_enqueue(h, d_frames, n, height, width, channels, row_stride, frame_stride, d_alpha_u8,
                           d_out_rgba, out_row_stride, out_frame_stride, s);
}

int vss_segment_composite(vss_handle* h, vss_post_state* st, const uint8_t* frames, int n, int height, int width,
                          int channels, size_t row_stride, uint8_t* out_rgba) {
  if (!h || !st || st->h != h) return fail(h, VSS_E_INVALID_ARG, "handle / post state mismatch");
  if (!out_rgba) return fail(h, VSS_E_INVALID_ARG, "null output");
  Busy b(h);
  if (!b.ok) return fail(h, VSS_E_BUSY, "a call is already in flight on this handle");
  HIP_TRY(h, hipSetDevice(h->device));
  if (!h->d_comp) {
    const size_t cap = (size_t)h->cfg.max_batch * h->cfg.max_frame_h * h->cfg.max_frame_w * 4;
    int rc = dalloc(h, &h->d_comp, cap);
    if (rc) return rc;
  }
  int rc = stage_in(h, frames, n, height, width, channels, row_stride, h->h_masks, VSS_OUT_MODEL);
  if (rc) return rc;
  const size_t fs = row_stride * (size_t)height, ors = (size_t)width * 4, ofs = ors * height;
  if ((size_t)n * ofs > (size_t)h->cfg.max_batch * h->cfg.max_frame_h * h->cfg.max_frame_w * 4)
    return fail(h, VSS_E_INVALID_ARG, "RGBA output exceeds the handle's capacity (max_batch, max_frame_h/w)");
  rc = post_enqueue(st, h->d_frames, n, height, width, channels, row_stride, fs, h->d_masks, nullptr, h->d_post_u8,
                    h->stream);
  if (rc) return rc;
  rc = composite_enqueue(h, h->d_frames, n, height, width, channels, row_stride, fs, h->d_post_u8, h->d_comp, ors,
                         ofs, h->stream);
  if (rc) return rc;
  HIP_TRY(h, hipMemcpyAsync(out_rgba, h->d_comp, (size_t)n * ofs, hipMemcpyDeviceToHost, h->stream));
  HIP_TRY(h, hipStreamSynchronize(h->stream));
  return VSS_OK;
}

}  // extern "C"
