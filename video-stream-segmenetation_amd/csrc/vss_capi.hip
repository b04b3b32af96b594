// vss_capi.hip — the C ABI (include/vss.h) over the gfx950 kernels.
//
// One engine per GPU mirrors one ORT InferenceSession
// (/root/reference/client/src/core/model.ts:12-29): it parses the weights
// blob's layer table once, plans per-layer tiles for its model resolution and
// uploads the per-layer LDS weight images.  Unlike the reference, which
// serialises every session.run (client/src/core/main.ts:18-22), an engine owns
// `queue_depth` slots — each its own NHWC f32 activations for max_batch
// frames, decoder-norm accumulators, HIP stream, captured hipGraphs and
// (allocated on first use) pinned staging — so consecutive batches run
// concurrently: batch i+1's H2D overlaps batch i's forward (BASELINE config 5).
//
// A handle = engine 0 (device_ids[0], the masks' consumer) + peer engines for
// the other GPUs.  Host calls shard a batch contiguously over the engines and
// all-gather the masks over RCCL (one communicator per device and slot, so
// concurrent slots never share one); one-GPU-per-process callers join a
// clique with vss_comm_init_rank instead.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <immintrin.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <fstream>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
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
constexpr int kDefaultQueueDepth = 4, kMaxQueueDepth = 16, kDefaultStagingThreads = 8;

struct Rec {
  uint32_t kind, cin, chid, cout, stride, flags, src, skip, off[8];
};

struct LayerPlan {
  Rec rec{};
  int C = 0, H = 0, W = 0;     // output shape
  int inH = 0, inW = 0;        // shape of rec.src's output (x)
  int mode = -1, stride = 1, chid = 0;
  int TH = 0, TW = 0, tiles_x = 0, tiles_y = 0;
  int flags = 0;
  int ks = 1, xp = 1, sp = 1;  // hidden split of this layer, parts of its x / skip (block_flags)
  size_t part_stride = 0;      // floats between the parts of an activation
  long wimg_stride = 0;        // floats between the slices' weight images
  size_t lds = 0;
  const BlockEntry* entry = nullptr;  // compiled shape (registry)
  const BlockEntry* small = nullptr;  // the autotuner's batch-1 pick, for forwards of <= small_tile_n frames
  bool fused = false;          // computed inside its only consumer's prologue (no launch of its own)
  int acc_off = -1;            // DEC: offset of its [kAccSlots][2][C] norm accumulator in a frame's row
  const float* wimg = nullptr;  // LDS weight image (block_lds regions w1..b2)
  const float *gamma = nullptr, *beta = nullptr;
  const float *stem_w = nullptr, *stem_b = nullptr, *head_w = nullptr;
  float head_b = 0.f;
};

// One kernel launch of the forward: function, grid, LDS and its parameter
// block (every kernel takes one parameter struct by value).
struct Launch {
  const void* fn = nullptr;
  dim3 grid;
  int threads = kThreads;
  size_t lds = 0;
  int layer = 0;
  union Prm {
    StemParams stem;
    BlockParams block;
    HeadParams head;
  } prm;
};

// A forward's executable graphs per (slot, shape): up to kExecPerShape
// executables, each bound to the caller buffers (frames, masks) it last ran
// with.  A call whose buffers match one replays it as is; otherwise a new
// executable is built while the set has room, and after that the least
// recently used one is patched (hipGraphExecKernelNodeSetParams on the kernel
// nodes whose parameters differ — the first layer reads the frames, the head
// writes the masks) once ITS last launch is done (its own event: the wait is
// normally over already, since three newer launches were issued after it).
// So callers rotating up to kExecPerShape buffer pairs through a slot never
// patch in steady state, and no caller ever waits for the slot's latest work
// here (the round-3 single executable waited on every call of a
// caller rotating 3 buffers over 4 slots, holding the handle's lock).
using GraphKey = std::tuple<int, int, int, int, size_t, size_t>;  // n, fh, fw, fc, row / frame stride
constexpr int kExecPerShape = 4;
struct GraphEntry {
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
  hipEvent_t last = nullptr;          // recorded after this executable's latest launch
  bool launched = false;
  unsigned long long tick = 0;        // LRU clock of its latest launch
  std::vector<hipGraphNode_t> nodes;  // one kernel node per launch, in order
  std::vector<Launch> launches;       // the parameters the executable graph holds now
};

// The rows of an fh-row frame that the tfjs-legacy resize to the model's rows
// reads (prep_tap's y0 / y1, the same float arithmetic), for the queued host
// path's row staging (vss_stage.hip).
struct RowPlan {
  std::vector<int> rows;                    // sorted, distinct
  std::vector<std::pair<int, int>> runs;    // [first, last + 1) runs of consecutive rows
  int* d_rows = nullptr;                    // device copy of rows
};

// One batch in flight on one GPU: everything a forward writes.
struct Slot {
  std::vector<float*> act;            // per layer: [ks][max_batch][H][W][C]
  unsigned long long* acc = nullptr;  // decoder instance-norm accumulators [max_batch][acc_stride]
  float* d_masks = nullptr;           // [max_batch][P]: host paths' masks (the all-gather's send buffer)
  float* d_gather = nullptr;          // RCCL handles: [nranks * max_batch][P]
  hipStream_t stream = nullptr;       // the slot's stream (queued host calls)
  hipEvent_t done = nullptr;          // recorded after the slot's latest work (host or device call)
  hipStream_t done_stream = nullptr;  // the stream `done` was last recorded on
  hipEvent_t host_done = nullptr;     // engine 0: recorded after the latest host batch's D2H
  bool used = false;
  // Host-side state of the slot's latest host batch (guarded by the handle's mu):
  bool leased = false;                // reserved by vss_staging_acquire for its holder's next call
  bool host_busy = false;             // a host batch whose completion (copy / callback /
                                      // synchronous wait) has not finished; the slot's pinned
                                      // buffers belong to it until then
  int status = VSS_OK;                // of the latest host batch
  vss_ticket ticket = ~0ull;          // latest host ticket that ran in this slot (device calls
                                      // take no ticket and leave it alone)
  bool stem_stored = false;           // the latest forward stored the fused stem (VSS_OPT_KEEP_STEM)
  std::map<GraphKey, std::vector<GraphEntry>> graphs;
  std::map<GraphKey, unsigned long long> shape_tick;  // per shape: graph_tick of its latest use
  unsigned long long graph_tick = 0;
#ifdef VSS_TRACE
  std::vector<unsigned long long*> trace;  // per layer, [workgroups][16] stamps of this slot's latest forward
#endif
  ncclComm_t comm = nullptr;          // this GPU's communicator of the slot (RCCL handles)
  // host-path staging, allocated on the slot's first host call
  uint8_t* d_frames = nullptr;
  uint8_t* h_frames = nullptr;        // pinned
  float* h_masks = nullptr;           // pinned [max_batch][P] (engine 0: the whole batch)
  float* d_fmasks = nullptr;          // VSS_OUT_FRAME: [max_batch][frame] masks
  float* h_fmasks = nullptr;
};

thread_local std::string g_tls_error;
// The handle whose completion thread this is (null on every other thread): a
// callback runs there, and only that thread clears host_busy, so a call from a
// callback that would wait for a host_busy slot returns VSS_E_BUSY instead of
// waiting for itself.
thread_local const ::vss_handle* g_tls_completing = nullptr;

// Host threads for the pinned staging copies: a copy is cut into 256 KiB
// pieces that the pool's threads and the caller take in turn.  Measured on the
// MI355X box's host (tools/micro/pinned_copy.cpp, 7.4 MB into pinned memory):
// one thread 39 GB/s, two to four 58-61 GB/s when the copy runs alone; inside
// the queued pipeline (DMA engines reading the other slots' staging at the
// same time) 8 threads sustained ~29 GB/s against ~25 GB/s for 4 (spinning
// idle workers measured slower still).  The zero-copy lease
// (vss_staging_acquire) avoids the copy altogether.
// A copy into pinned staging with non-temporal 32-byte stores (AVX2): the
// destination is only read again by the DMA engine, so the stores skip the
// read-for-ownership of each destination line and do not evict the source
// frames from the caches.  Plain memcpy where AVX2 is absent or the
// destination is not 32-byte aligned (env VSS_PLAIN_MEMCPY=1 forces it).
// Measured on the box's 16-CPU share (noisy): VGA copy path ~26k -> ~29k
// frames/s, 1080p ~17k -> ~20k; the zero-copy path does not copy.  Since the
// staging copies only the rows the resize reads, a VGA batch is ~1150 row runs
// of 3840 B each (two rows): the streaming path takes pieces from 512 B on
// (it was 4 KiB, which sent every VGA run through plain memcpy and its
// read-for-ownership of the destination).
__attribute__((target("avx2"))) static void stream_copy_avx2(void* dst, const void* src, size_t len) {
  char* d = static_cast<char*>(dst);
  const char* s = static_cast<const char*>(src);
  size_t i = 0;
  for (; i + 128 <= len; i += 128) {
    const __m256i a = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i));
    const __m256i b = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i + 32));
    const __m256i c = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i + 64));
    const __m256i e = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i + 96));
    _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i), a);
    _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i + 32), b);
    _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i + 64), c);
    _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i + 96), e);
  }
  if (i < len) std::memcpy(d + i, s + i, len - i);
  _mm_sfence();  // the streamed lines are visible before this copy counts as done
}

static void staging_copy(void* dst, const void* src, size_t len) {
  static const bool avx2 = __builtin_cpu_supports("avx2") && !getenv("VSS_PLAIN_MEMCPY");
  if (avx2 && (reinterpret_cast<uintptr_t>(dst) & 31) == 0 && len >= 512) stream_copy_avx2(dst, src, len);
  else std::memcpy(dst, src, len);
}

class CopyPool {
 public:
  explicit CopyPool(int threads) {
    for (int i = 0; i < threads; ++i) workers_.emplace_back([this] { loop(); });
  }
  ~CopyPool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }
  struct Job {
    void* dst;
    const void* src;
    size_t len;
  };
  // Copies every job; returns as soon as every piece is in place.  A copy's
  // pieces live in a generation object that the workers share (shared_ptr), so
  // a worker that wakes after the copy is done finds no piece left and touches
  // nothing: the caller never waits for a sleeping worker's wake-up (round 5
  // waited for every worker to leave the generation — for one VGA frame, ~144
  // row runs of 3.8 KB, the slowest wake-up of 7 threads set the call's time,
  // 36 us at p50 where the caller alone copies it in ~14; tools/ts_prof.js).
  void run(const std::vector<Job>& jobs) {
    constexpr size_t kPiece = size_t(256) << 10;
    auto g = std::make_shared<Gen>();
    for (const Job& j : jobs)
      for (size_t off = 0; off < j.len; off += kPiece)
        g->pieces.push_back({static_cast<char*>(j.dst) + off, static_cast<const char*>(j.src) + off,
                             std::min(kPiece, j.len - off)});
    const size_t n = g->pieces.size();
    // a small copy (one VGA frame's rows: ~0.55 MB) on the calling thread
    // alone: waking the workers costs more than they save (VSS_COPY_INLINE_BYTES)
    static const size_t inline_bytes = [] {
      const char* e = std::getenv("VSS_COPY_INLINE_BYTES");
      return e ? (size_t)std::atoll(e) : (size_t(1) << 20);
    }();
    size_t total = 0;
    for (const Job& j : jobs) total += j.len;
    if (n <= 1 || workers_.empty() || total < inline_bytes) {
      for (const Job& p : g->pieces) staging_copy(p.dst, p.src, p.len);
      return;
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      cur_ = g;
      ++gen_;
    }
    cv_.notify_all();
    work(*g);
    // (VSS_COPY_WAIT_ALL=1, an A/B knob: also wait for every worker to have
    // taken and left this copy, round 5's protocol)
    static const bool wait_all = std::getenv("VSS_COPY_WAIT_ALL") && std::getenv("VSS_COPY_WAIT_ALL")[0] == '1';
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [&] { return g->done.load() == n && (!wait_all || g->left.load() == workers_.size()); });
    if (cur_ == g) cur_.reset();
  }

 private:
  struct Gen {
    std::vector<Job> pieces;
    std::atomic<size_t> next{0}, done{0}, left{0};
  };
  void work(Gen& g) {
    const size_t n = g.pieces.size();
    for (size_t i = g.next.fetch_add(1); i < n; i = g.next.fetch_add(1)) {
      staging_copy(g.pieces[i].dst, g.pieces[i].src, g.pieces[i].len);
      if (g.done.fetch_add(1) + 1 == n) {  // the last piece: wake the caller (under mu_: no lost wake-up)
        std::lock_guard<std::mutex> lk(mu_);
        done_cv_.notify_all();
      }
    }
  }
  void loop() {
    unsigned long seen = 0;
    for (;;) {
      std::shared_ptr<Gen> g;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
        g = cur_;
      }
      if (g) {
        work(*g);
        if (g->left.fetch_add(1) + 1 == workers_.size()) {
          std::lock_guard<std::mutex> lk(mu_);
          done_cv_.notify_all();
        }
      }
    }
  }
  std::vector<std::thread> workers_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  std::shared_ptr<Gen> cur_;
  unsigned long gen_ = 0;
  bool stop_ = false;
};

}  // namespace

constexpr long kDefaultKsplitPixels = 256;
// expand layers whose unsplit LDS weight image exceeds this also split their
// hidden channels (keeps every layer's LDS small enough for two workgroups per
// CU; mirrors KSPLIT_WEIGHT_BYTES in tools/gen_registry.py)
constexpr size_t kKsplitWeightBytes = 40 * 1024;

struct vss_handle {
  vss_config cfg{};            // this engine's config (max_batch = its share of the handle's)
  std::string weights_path;
  // the last error: written by any thread that fails a call (several may
  // submit at once) and by the completion thread; read by vss_last_error,
  // which copies it under err_mu into the caller's thread-local buffer
  std::string err;
  mutable std::mutex err_mu;
  int device = 0;
  hipStream_t stream = nullptr;          // NULL-stream device calls, post / composite, autotune
  std::vector<Rec> recs;
  std::vector<float> hdata;
  float eps = 1e-5f;
  std::vector<LayerPlan> L;
  int acc_stride = 0;
  std::vector<void*> dev_allocs;
  std::vector<void*> host_allocs;
  size_t dev_bytes = 0;
  size_t frame_cap = 0;        // staging bytes per slot
  std::vector<Slot> slots;
  int last_slot = -1;          // slot of the latest forward (vss_read_layer)
  std::map<int, RowPlan> row_plans;  // by frame height
  int row_fetch = 1;           // VSS_OPT_ROW_FETCH
#ifdef VSS_TRACE
  std::vector<int> trace_wgs;              // workgroups of the layer's last launch
#endif
  uint8_t* d_comp = nullptr;      // vss_segment_composite output, allocated on first use
  float* d_post_alpha = nullptr;  // vss_segment_post outputs [max_batch][P]
  uint8_t* d_post_u8 = nullptr;
  int use_graph = 1;
  int profile = 0;
  int fuse_stem = 1;              // env VSS_FUSE_STEM=0: launch the stem on its own
  int keep_stem = 0;              // VSS_OPT_KEEP_STEM: the fused stem also stores its activation
  // expand layers with at most this many output pixels per frame split their
  // hidden channels over ks_max() workgroups (env VSS_KSPLIT_PIXELS overrides)
  long ksplit_pixels = kDefaultKsplitPixels;
  // The hidden-channel split (KS workgroups per tile of a deep low-res expand
  // layer, consumers summing the parts) buys latency with one batch in flight
  // and costs throughput with four: measured round 4 (profiles/r04a/session.txt,
  // two interleaved pairs): headline 206.9 / 206.1k without against 194.7 /
  // 203.7k with, batch sweep at 4 in flight +4 % (b8), +7.5 % (b32), +6 % (b64),
  // at 1 in flight -3 % (b8).  Off by default; env VSS_KSPLIT=1 turns it on.
  bool ksplit_on = false;
  // profiling: ring of event pairs per layer
  static constexpr int kProfRing = 32;
  std::vector<hipEvent_t> ev;  // [ring][layer][2]
  std::vector<int> ring_pending;
  int prof_next = 0;
  std::vector<double> prof_sum;
  int prof_count = 0;
  int last_n = 0;
  // ---- the handle (engine 0 only) ----
  std::vector<vss_handle*> peers;  // engines 1..R-1 (device_ids[1..])
  int user_max_batch = 0;          // the handle's max_batch (all GPUs)
  bool rccl = false;               // host calls all-gather over RCCL (device_ids given)
  int nranks = 1, rank = 0;        // vss_comm_init_rank clique (one GPU per process)
  // set (release) once every communicator of the clique exists: the lock-free
  // vss_comm_status reads the communicators only after seeing it (acquire)
  std::atomic<bool> clique{false};
  // VSS_OPT_GATHER_FORM, fixed at vss_comm_init_rank.  VSS_GATHER_ORDERED (the
  // default): the clique's all-gathers on one communicator (slot 0's, the only
  // one created) and one stream, events ordering each gather after its forward
  // and the caller's stream after the gather — one total order of collectives
  // per rank.  VSS_GATHER_CONCURRENT: each slot's own communicator on the
  // slot's stream (vss_segment_gather_device)
  int gather_form = VSS_GATHER_ORDERED;
  std::vector<hipEvent_t> gather_ev;  // the ordered form's gather-done events, a ring of 2 x depth (call % size)
  // Submissions (slot choice, staging, enqueue) are serialised by mu; no
  // thread holds it while it waits for the GPU (waiters drop it first).
  std::mutex mu;
  std::condition_variable slot_cv;   // a slot's host_busy went false
  std::mutex post_mu;              // the synchronous post / composite calls share scratch
  vss_ticket next_ticket = 0;      // host batches (vss_submit*, vss_segment*)
  unsigned long long device_calls = 0;  // vss_segment_device: slot = count % depth
  int small_tile_n = 0;            // forwards of at most this many frames use LayerPlan::small
  std::atomic<unsigned long long> gather_calls{0};  // vss_segment_gather_device: slot = count % depth
                                                   // (atomic: vss_comm_status reads it lock-free)
  long graph_builds = 0, graph_patches = 0;  // VSS_OPT_GRAPH_BUILDS / _PATCHES
  CopyPool* pool = nullptr;
  // The completion thread (started on the first host batch that needs one):
  // waits for the queued host batches in ticket order, copies their masks
  // from the slot's pinned buffer into the caller's memory, fires callbacks.
  struct Completion {
    vss_ticket ticket;
    int slot;
    float* out;          // null: the D2H already went to the caller's pinned block
    const float* src;
    size_t bytes;
    vss_callback cb;
    void* user;
  };
  std::thread done_thread;
  std::mutex done_mu;
  std::condition_variable done_cv;
  std::deque<Completion> done_q;
  bool done_stop = false;
};

namespace {

void set_err(vss_handle* h, const std::string& msg) {
  std::lock_guard<std::mutex> lk(h->err_mu);
  h->err = msg;
}

int fail(vss_handle* h, int code, const std::string& msg) {
  if (h) set_err(h, msg);
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

#define NCCL_TRY(h, expr)                                                                 \
  do {                                                                                    \
    ncclResult_t r_ = (expr);                                                             \
    if (r_ != ncclSuccess)                                                                \
      return fail((h), VSS_E_RCCL, std::string(#expr) + ": " + ncclGetErrorString(r_));   \
  } while (0)

// A communicator's asynchronous error (ncclCommGetAsyncError): RCCL reports a
// failed collective — a peer gone, a network or device error — there, not at
// the enqueue.  Every gather polls it on the communicator it is about to use
// and fails with VSS_E_RCCL instead of enqueueing behind a broken one (a
// stuck collective with no error shows up only as no progress: bench.py's
// watchdog, which reads vss_comm_status).
int comm_healthy(vss_handle* h, ncclComm_t c, int slot) {
  if (!c) return VSS_OK;
  ncclResult_t ae = ncclSuccess;
  const ncclResult_t q = ncclCommGetAsyncError(c, &ae);
  if (q != ncclSuccess) return fail(h, VSS_E_RCCL, std::string("ncclCommGetAsyncError: ") + ncclGetErrorString(q));
  if (ae != ncclSuccess && ae != ncclInProgress)
    return fail(h, VSS_E_RCCL, "communicator of slot " + std::to_string(slot) + ": asynchronous error " +
                                   ncclGetErrorString(ae));
  return VSS_OK;
}

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

template <class T>
int halloc(vss_handle* h, T** p, size_t bytes) {
  void* q = nullptr;
  bytes = std::max<size_t>(bytes, 16);
  if (hipHostMalloc(&q, bytes, hipHostMallocDefault) != hipSuccess)
    return fail(h, VSS_E_OOM, "hipHostMalloc(" + std::to_string(bytes) + ") failed");
  h->host_allocs.push_back(q);
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

// LDS bytes of one workgroup of compiled shape e for layer l.
size_t entry_lds_bytes(const LayerPlan& l, const BlockEntry& e) {
  if (e.variant == VAR_STEM_B1_WIDE) return (size_t)stem_b1_lds(e.TH, e.TW).total * 4;
  return block_lds_bytes(l, e.TH, e.TW);
}

void set_tile(LayerPlan& l, const BlockEntry* e) {
  l.entry = e;
  l.TH = e->TH;
  l.TW = e->TW;
  l.tiles_x = (l.W + l.TW - 1) / l.TW;
  l.tiles_y = (l.H + l.TH - 1) / l.TH;
  l.lds = entry_lds_bytes(l, *e);
}

// Tile choice among the compiled shapes for this layer (csrc/vss_registry.inc):
// the largest tile that still gives >= 2 workgroups per CU (256 CUs) at
// max_batch, preferring <= 64 KiB of LDS; otherwise the most workgroups.
int choose_tile(vss_handle* h, LayerPlan& l, int N) {
  int count = 0;
  const BlockEntry* reg = block_registry(&count);
  const int cskip = l.mode == MODE_DEC ? (int)l.rec.chid : 0;
  const BlockEntry* best = nullptr;
  long best_score = -1;
  for (int i = 0; i < count; ++i) {
    const BlockEntry& e = reg[i];
    if (e.mode != l.mode || e.stride != l.stride || e.cin != (int)l.rec.cin || e.cskip != cskip ||
        e.chid != l.chid / l.ks || e.cout != l.C || e.flags != l.flags)
      continue;
    if (e.variant != VAR_BLOCK) continue;  // the stem + b1 kernels are candidates of the autotuner only
    const long blocks = (long)((l.H + e.TH - 1) / e.TH) * ((l.W + e.TW - 1) / e.TW) * N;
    const size_t lds = entry_lds_bytes(l, e);
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

int plan(vss_handle* h) {
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
      // the decoder's 2x upsample taps (block_body's tap records) are exact for
      // skip == 2 x src only (model_h / model_w multiples of 16 give that for
      // the spec's four stride-2 levels); anything else is refused here
      if (2 * s.H != k.H || 2 * s.W != k.W) return bad("dec skip must be exactly 2x its src");
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
    // (only with VSS_KSPLIT=1: see ksplit_on)
    if (l.mode == MODE_IR_EXPAND && h->ksplit_on &&
        ((long)l.H * l.W <= h->ksplit_pixels || weight_image_bytes(l) > kKsplitWeightBytes))
      l.ks = ks_max(l);
    if (r.kind == K_IR || r.kind == K_DEC) l.xp = h->L[r.src].ks;
    if (r.kind == K_DEC) l.sp = h->L[r.skip].ks;
    if (r.kind == K_IR) l.flags = block_flags(0, (r.flags & F_RESIDUAL) != 0, l.xp, 1, l.ks);
    // the stem fused into its only consumer, a stride-1 direct block (STEM_IN)
    if (r.kind == K_IR && h->fuse_stem && l.mode == MODE_IR_DIRECT && l.stride == 1 &&
        h->L[r.src].rec.kind == K_STEM && consumers[r.src] == 1 && r.cin == 16) {
      l.flags |= block_flags(0, 0, 1, 1, 1, 1);
      h->L[r.src].fused = true;
    }
    if (r.kind == K_DEC) l.flags = block_flags(h->L[r.src].rec.kind == K_DEC, 0, l.xp, l.sp, 1);
    if (l.mode >= 0) {
      int rc = choose_tile(h, l, N);
      if (rc) return rc;
    }
  }
  if (nl == 0 || h->recs.back().kind != K_HEAD) return fail(h, VSS_E_UNSUPPORTED, "last layer must be the head");
  return VSS_OK;
}

int upload(vss_handle* h) {
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
  if (!img.empty()) HIP_TRY(h, hipMemcpy(d_img, img.data(), img.size() * 4, hipMemcpyHostToDevice));
  h->acc_stride = 0;
  for (size_t i = 0; i < h->L.size(); ++i) {
    LayerPlan& l = h->L[i];
    const Rec& r = l.rec;
    l.part_stride = (size_t)h->cfg.max_batch * l.H * l.W * l.C;
    if (r.kind == K_STEM) {
      l.stem_w = dp(r.off[O_W1]);
      l.stem_b = dp(r.off[O_B1]);
    } else if (r.kind == K_IR || r.kind == K_DEC) {
      l.wimg = d_img + img_off[i];
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
#ifdef VSS_TRACE
  h->trace_wgs.assign(h->L.size(), 0);
#endif
  return VSS_OK;
}

// A slot's device buffers (activations, norm accumulators, masks), stream and
// completion event; the host staging comes on its first host call.
int make_slot(vss_handle* h, Slot& s, int gather_ranks) {
  const int N = h->cfg.max_batch;
  const size_t P = (size_t)h->cfg.model_h * h->cfg.model_w;
  int rc;
  s.act.assign(h->L.size(), nullptr);
  for (size_t i = 0; i < h->L.size(); ++i) {
    const LayerPlan& l = h->L[i];
    if (l.rec.kind == K_HEAD) continue;  // the head writes the caller's masks
    if ((rc = dalloc(h, &s.act[i], l.part_stride * l.ks * 4))) return rc;
    HIP_TRY(h, hipMemset(s.act[i], 0, l.part_stride * l.ks * 4));
  }
  const size_t acc = (size_t)N * std::max(h->acc_stride, 2) * 8;
  if ((rc = dalloc(h, &s.acc, acc))) return rc;
  HIP_TRY(h, hipMemset(s.acc, 0, acc));
  if ((rc = dalloc(h, &s.d_masks, (size_t)N * P * 4))) return rc;
  if (gather_ranks > 0 && (rc = dalloc(h, &s.d_gather, (size_t)gather_ranks * N * P * 4))) return rc;
  // VSS_SLOT_QUEUES=cumask: the slot's stream carries a CU mask of every CU,
  // which gives it a hardware queue of its own (the runtime shares its pooled
  // queues between plain streams — GPU_MAX_HW_QUEUES of them — so two slots
  // could land on one queue and run one after the other)
  static const char* q = std::getenv("VSS_SLOT_QUEUES");
  if (q && !std::strcmp(q, "cumask")) {
    int cus = 0;
    HIP_TRY(h, hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, h->device));
    std::vector<uint32_t> mask((cus + 31) / 32, 0u);
    for (int c = 0; c < cus; ++c) mask[c / 32] |= 1u << (c % 32);
    HIP_TRY(h, hipExtStreamCreateWithCUMask(&s.stream, (uint32_t)mask.size(), mask.data()));
  } else {
    HIP_TRY(h, hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking));
  }
  // host waits on it sleep instead of spinning: several waiting threads (the
  // N-API addon's libuv workers, vss_wait callers) would otherwise take the
  // cores the staging copies run on
  HIP_TRY(h, hipEventCreateWithFlags(&s.done, hipEventDisableTiming | hipEventBlockingSync));
  HIP_TRY(h, hipEventCreateWithFlags(&s.host_done, hipEventDisableTiming | hipEventBlockingSync));
#ifdef VSS_TRACE
  s.trace.assign(h->L.size(), nullptr);
  for (size_t i = 0; i < h->L.size(); ++i) {
    const LayerPlan& l = h->L[i];
    const size_t bytes = (size_t)h->cfg.max_batch * l.H * l.W * 16 * 8;  // >= one record per workgroup
    if ((rc = dalloc(h, &s.trace[i], bytes))) return rc;
    HIP_TRY(h, hipMemset(s.trace[i], 0, bytes));
  }
#endif
  return VSS_OK;
}

int ensure_staging(vss_handle* h, Slot& s) {
  if (s.h_frames) return VSS_OK;
  const size_t P = (size_t)h->cfg.model_h * h->cfg.model_w;
  int rc;
  if ((rc = dalloc(h, &s.d_frames, h->frame_cap))) return rc;
  if ((rc = halloc(h, &s.h_frames, h->frame_cap))) return rc;
  // engine 0 receives the whole batch's masks (gathered from every GPU)
  const size_t nm = (size_t)std::max(h->cfg.max_batch, h->user_max_batch);
  if ((rc = halloc(h, &s.h_masks, nm * P * 4))) return rc;
  return VSS_OK;
}

int ensure_frame_masks(vss_handle* h, Slot& s) {
  if (s.h_fmasks) return VSS_OK;
  const size_t cap = (size_t)std::max(h->cfg.max_batch, h->user_max_batch) * h->cfg.max_frame_h * h->cfg.max_frame_w;
  int rc;
  if ((rc = dalloc(h, &s.d_fmasks, cap * 4))) return rc;
  if ((rc = halloc(h, &s.h_fmasks, cap * 4))) return rc;
  return VSS_OK;
}

// prep_tap's rows, computed exactly as the kernel computes them (f32, no contraction).
#pragma clang fp contract(off)
int row_plan(vss_handle* h, int fh, const RowPlan** out) {
  auto it = h->row_plans.find(fh);
  if (it == h->row_plans.end()) {
    const int Hm = h->cfg.model_h;
    const float ry = (float)((double)fh / (double)Hm);
    std::vector<char> need(fh, 0);
    for (int y = 0; y < Hm; ++y) {
      const float fy = (float)y * ry;
      const int y0 = (int)std::floor(std::max(fy, 0.f));
      const int y1 = std::min(fh - 1, (int)std::ceil(fy));
      need[std::min(y0, fh - 1)] = 1;
      need[y1] = 1;
    }
    RowPlan rp;
    for (int r = 0; r < fh; ++r)
      if (need[r]) {
        rp.rows.push_back(r);
        if (!rp.runs.empty() && rp.runs.back().second == r) rp.runs.back().second = r + 1;
        else rp.runs.push_back({r, r + 1});
      }
    int rc = dalloc(h, &rp.d_rows, rp.rows.size() * sizeof(int));
    if (rc) return rc;
    HIP_TRY(h, hipMemcpy(rp.d_rows, rp.rows.data(), rp.rows.size() * sizeof(int), hipMemcpyHostToDevice));
    it = h->row_plans.emplace(fh, std::move(rp)).first;
  }
  *out = &it->second;
  return VSS_OK;
}
#pragma clang fp contract(on)

int check_frames(vss_handle* h, int n, int fh, int fw, int fc, size_t rs, size_t fs, int max_n) {
  if (n < 1 || n > max_n) return fail(h, VSS_E_INVALID_ARG, "n must be in [1, max_batch]");
  if (fh < 1 || fw < 1) return fail(h, VSS_E_INVALID_ARG, "bad frame size");
  if (fc != 3 && fc != 4) return fail(h, VSS_E_INVALID_ARG, "channels must be 3 or 4");
  if (rs < (size_t)fw * fc) return fail(h, VSS_E_INVALID_ARG, "row_stride < width*channels");
  if (fs < rs * (size_t)fh) return fail(h, VSS_E_INVALID_ARG, "frame_stride < height*row_stride");
  return VSS_OK;
}

// The stem's parameters for this call's frames (frames point at frame 0 of the call).
StemParams stem_params(const vss_handle* h, const Slot& s, int li, const uint8_t* frames, size_t rs, size_t fs,
                       int fh, int fw, int fc) {
  const LayerPlan& l = h->L[li];
  const int Hm = h->cfg.model_h, Wm = h->cfg.model_w;
  StemParams p{};
  p.frames = frames; p.row_stride = (long)rs; p.frame_stride = (long)fs;
  p.fh = fh; p.fw = fw; p.fc = fc; p.Hm = Hm; p.Wm = Wm;
  p.ry = (float)((double)fh / (double)Hm);
  p.rx = (float)((double)fw / (double)Wm);
  p.w = l.stem_w; p.b = l.stem_b; p.y = s.act[li];
  p.Ho = l.H; p.Wo = l.W; p.cout = l.C;
  p.acc_zero = s.acc;
  p.acc_stride = h->acc_stride;
  return p;
}

// Kernel parameters of block layer li for the call's n frames.
BlockParams block_params(const vss_handle* h, const Slot& s, int li, int n, const LayerPlan* lp = nullptr) {
  const LayerPlan& l = lp ? *lp : h->L[li];
  const Rec& r = l.rec;
  const LayerPlan& src = h->L[r.src];
  BlockParams p{};
  p.wimg = l.wimg;
  p.wimg_stride = l.wimg_stride;
  p.x_part_stride = (long)src.part_stride;
  p.y_part_stride = (long)l.part_stride;
  p.x = s.act[r.src];
  p.y = s.act[li];
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
    p.skip = s.act[r.skip];
    p.skip_part_stride = (long)sk.part_stride;
    p.cskip = (int)r.chid;
    p.relu6_dw = 0;
    p.out_acc = s.acc + l.acc_off;
    p.norm_in = src.rec.kind == K_DEC ? 1 : 0;
    if (p.norm_in) {
      p.in_acc = s.acc + src.acc_off;
      p.in_gamma = src.gamma;
      p.in_beta = src.beta;
      p.in_hw = src.H * src.W;
      p.in_inv_hw = 1.0 / (double)p.in_hw;
    }
  }
  return p;
}

// The forward of n frames with slot s's buffers as a list of launches (no
// sync, no alloc): the eager path launches them, the graph path adds them as
// kernel nodes.
void forward_launches(vss_handle* h, Slot& s, const uint8_t* frames, int n, int fh, int fw, int fc, size_t rs,
                      size_t fs, float* masks, std::vector<Launch>* out) {
  const int Hm = h->cfg.model_h, Wm = h->cfg.model_w;
  const int prec = h->cfg.dtype == VSS_DTYPE_F32 ? PREC_F32 : PREC_BF16X2;
  const int nl = (int)h->L.size();
  out->clear();
  for (int i = 0; i < nl; ++i) {
    LayerPlan& l = h->L[i];
    const Rec& r = l.rec;
    if (l.fused) {  // runs inside its consumer's launch
#ifdef VSS_TRACE
      h->trace_wgs[i] = 0;
#endif
      continue;
    }
    Launch L{};
    L.layer = i;
    if (r.kind == K_STEM) {
      StemParams p = stem_params(h, s, i, frames, rs, fs, fh, fw, fc);
#ifdef VSS_TRACE
      p.trace = s.trace[i];
      h->trace_wgs[i] = ((l.W + kStemTW - 1) / kStemTW) * ((l.H + kStemTH - 1) / kStemTH) * n;
#endif
      L.fn = (const void*)stem_kernel16();
      L.grid = dim3((l.W + kStemTW - 1) / kStemTW, (l.H + kStemTH - 1) / kStemTH, n);
      L.lds = kStemLds * 4;
      L.prm.stem = p;
    } else if (r.kind == K_IR || r.kind == K_DEC) {
      // a small batch on the batch-1 tile (autotune): bitwise the same results
      LayerPlan small_plan;
      const bool use_small = l.small && n <= h->small_tile_n;
      if (use_small) {
        small_plan = l;
        set_tile(small_plan, l.small);
      }
      const LayerPlan& lt = use_small ? small_plan : l;
      BlockParams p = block_params(h, s, i, n, &lt);
      if (flags_stem_in(l.flags)) {
        p.stem = stem_params(h, s, (int)r.src, frames, rs, fs, fh, fw, fc);
        if (!h->keep_stem) p.stem.y = nullptr;  // no layer reads it (vss_read_layer(0) only)
      }
#ifdef VSS_TRACE
      p.trace = s.trace[i];
      h->trace_wgs[i] = lt.tiles_x * lt.tiles_y * n * lt.ks;
#endif
      L.fn = (const void*)lt.entry->fn[prec == PREC_F32 ? 0 : 1];
      L.grid = dim3(lt.tiles_x, lt.tiles_y, n * lt.ks);
      L.threads = lt.entry->threads;
      L.lds = lt.lds;
      L.prm.block = p;
    } else if (r.kind == K_HEAD) {
      const LayerPlan& src = h->L[r.src];
      HeadParams p{};
      p.x = s.act[r.src];
      p.in_acc = s.acc + src.acc_off;
      p.acc_stride = h->acc_stride;
      p.gamma = src.gamma; p.beta = src.beta; p.eps = h->eps;
      p.w = l.head_w; p.b = l.head_b; p.mask = masks;
      p.N = n; p.h = src.H; p.w_ = src.W; p.cin = src.C; p.Hm = Hm; p.Wm = Wm;
      p.inv_hw = 1.0 / ((double)src.H * src.W);
#ifdef VSS_TRACE
      p.trace = s.trace[i];
      h->trace_wgs[i] = ((Wm + kHeadTW - 1) / kHeadTW) * ((Hm + kHeadTH - 1) / kHeadTH) * n;
#endif
      L.fn = (const void*)head_kernel16();
      L.grid = dim3((Wm + kHeadTW - 1) / kHeadTW, (Hm + kHeadTH - 1) / kHeadTH, n);
      L.lds = kHeadLds * 4;
      L.prm.head = p;
    } else {
      continue;
    }
    out->push_back(L);
  }
}

hipKernelNodeParams node_params(const Launch& L, void** args) {
  hipKernelNodeParams kp{};
  args[0] = const_cast<Launch::Prm*>(&L.prm);
  kp.func = const_cast<void*>(L.fn);
  kp.gridDim = L.grid;
  kp.blockDim = dim3(L.threads);
  kp.sharedMemBytes = (unsigned)L.lds;
  kp.kernelParams = args;
  kp.extra = nullptr;
  return kp;
}

// Eager launches on stream st; prof_slot >= 0: each launch records its layer's
// event pair of that profiling ring entry (hipExtLaunchKernel).
int launch_eager(vss_handle* h, const std::vector<Launch>& ls, hipStream_t st, int prof_slot) {
  const int nl = (int)h->L.size();
  for (const Launch& L : ls) {
    void* args[1] = {const_cast<Launch::Prm*>(&L.prm)};
    if (prof_slot >= 0) {
      hipEvent_t e0 = h->ev[((size_t)prof_slot * nl + L.layer) * 2];
      hipEvent_t e1 = h->ev[((size_t)prof_slot * nl + L.layer) * 2 + 1];
      HIP_TRY(h, hipExtLaunchKernel(L.fn, L.grid, dim3(L.threads), args, L.lds, st, e0, e1, 0));
    } else {
      HIP_TRY(h, hipLaunchKernel(L.fn, L.grid, dim3(L.threads), args, L.lds, st));
    }
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(h, VSS_E_HIP, std::string("kernel launch: ") + hipGetErrorString(e));
  return VSS_OK;
}

int harvest_ring(vss_handle* h, int slot) {
  const int nl = (int)h->L.size();
  for (int i = 0; i < nl; ++i) {
    float ms = 0.f;
    if (h->L[i].fused) continue;  // timed inside its consumer's launch
    HIP_TRY(h, hipEventSynchronize(h->ev[((size_t)slot * nl + i) * 2 + 1]));
    HIP_TRY(h, hipEventElapsedTime(&ms, h->ev[((size_t)slot * nl + i) * 2], h->ev[((size_t)slot * nl + i) * 2 + 1]));
    h->prof_sum[i] += ms;
  }
  h->prof_count++;
  h->ring_pending[slot] = 0;
  return VSS_OK;
}

bool has_fused_stem(const vss_handle* h) {
  for (const LayerPlan& l : h->L)
    if (flags_stem_in(l.flags)) return true;
  return false;
}

void destroy_graph(GraphEntry& g) {
  if (g.last && g.launched) (void)hipEventSynchronize(g.last);  // never destroy an executable in flight
  if (g.exec) (void)hipGraphExecDestroy(g.exec);
  if (g.graph) (void)hipGraphDestroy(g.graph);
  if (g.last) (void)hipEventDestroy(g.last);
  g = GraphEntry();
}

void destroy_graph_set(std::vector<GraphEntry>& v) {
  for (GraphEntry& g : v) destroy_graph(g);
  v.clear();
}

// Build slot s's executable graph for these launches: one kernel node per
// launch, each depending on the previous one (a linear chain).
int build_graph(vss_handle* h, const std::vector<Launch>& ls, GraphEntry* out) {
  GraphEntry g;
  HIP_TRY(h, hipGraphCreate(&g.graph, 0));
  g.launches = ls;
  for (const Launch& L : g.launches) {
    void* args[1];
    const hipKernelNodeParams kp = node_params(L, args);
    hipGraphNode_t node = nullptr;
    const hipError_t e = hipGraphAddKernelNode(&node, g.graph, g.nodes.empty() ? nullptr : &g.nodes.back(),
                                               g.nodes.empty() ? 0 : 1, &kp);
    if (e != hipSuccess) {
      destroy_graph(g);
      return fail(h, VSS_E_HIP, std::string("hipGraphAddKernelNode: ") + hipGetErrorString(e));
    }
    g.nodes.push_back(node);
  }
  hipError_t e = hipGraphInstantiate(&g.exec, g.graph, nullptr, nullptr, 0);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&g.last, hipEventDisableTiming);
  if (e != hipSuccess) {
    destroy_graph(g);
    return fail(h, VSS_E_HIP, std::string("hipGraphInstantiate: ") + hipGetErrorString(e));
  }
  h->graph_builds++;
  *out = std::move(g);
  return VSS_OK;
}

// Kernel nodes of g whose parameter blocks differ from this call's launches.
int graph_diff(const GraphEntry& g, const std::vector<Launch>& ls) {
  int d = 0;
  for (size_t i = 0; i < ls.size(); ++i) d += std::memcmp(&ls[i].prm, &g.launches[i].prm, sizeof(Launch::Prm)) != 0;
  return d;
}

// Point executable g at this call's launches: the kernel nodes whose parameter
// blocks differ are updated.  An update must not race a launch of the same
// executable still in flight, so it first waits for g's own latest launch.
int patch_graph(vss_handle* h, GraphEntry& g, const std::vector<Launch>& ls) {
  bool waited = false;
  for (size_t i = 0; i < ls.size(); ++i) {
    if (std::memcmp(&ls[i].prm, &g.launches[i].prm, sizeof(Launch::Prm)) == 0) continue;
    if (!waited && g.launched) HIP_TRY(h, hipEventSynchronize(g.last));
    waited = true;
    void* args[1];
    const hipKernelNodeParams kp = node_params(ls[i], args);
    HIP_TRY(h, hipGraphExecKernelNodeSetParams(g.exec, g.nodes[i], &kp));
    g.launches[i] = ls[i];
  }
  if (waited) h->graph_patches++;
  return VSS_OK;
}

// The executable of slot s for this call (see GraphEntry): one bound to the
// same buffers, else a new one while the shape's set has room, else the least
// recently used one patched.
// Bound the cache at kMaxShapes shapes per slot: before a new shape's graphs
// are added, the least recently used shape's (by shape_tick: its latest
// prepare or launch) are destroyed.
constexpr size_t kMaxShapes = 16;
void make_room_for_shape(Slot& s) {
  if (s.graphs.size() < kMaxShapes) return;
  auto victim = s.graphs.begin();
  unsigned long long oldest = ~0ull;
  for (auto it = s.graphs.begin(); it != s.graphs.end(); ++it) {
    const auto t = s.shape_tick.find(it->first);
    const unsigned long long tick = t == s.shape_tick.end() ? 0ull : t->second;
    if (tick < oldest) {
      oldest = tick;
      victim = it;
    }
  }
  destroy_graph_set(victim->second);
  s.shape_tick.erase(victim->first);
  s.graphs.erase(victim);
}

int pick_graph(vss_handle* h, Slot& s, const GraphKey& key, const std::vector<Launch>& ls, GraphEntry** out) {
  auto it = s.graphs.find(key);
  if (it == s.graphs.end()) {
    make_room_for_shape(s);
    it = s.graphs.emplace(key, std::vector<GraphEntry>()).first;
  }
  s.shape_tick[key] = s.graph_tick + 1;  // (the launch below takes this tick)
  std::vector<GraphEntry>& v = it->second;
  GraphEntry* lru = nullptr;
  for (GraphEntry& g : v) {
    if (graph_diff(g, ls) == 0) {
      *out = &g;
      return VSS_OK;
    }
    if (!lru || !g.launched || (lru->launched && g.tick < lru->tick)) lru = &g;  // never-launched first
  }
  if ((int)v.size() < kExecPerShape && !(lru && !lru->launched)) {
    v.emplace_back();
    if (int rc = build_graph(h, ls, &v.back())) {
      v.pop_back();
      return rc;
    }
    *out = &v.back();
    return VSS_OK;
  }
  if (int rc = patch_graph(h, *lru, ls)) return rc;
  *out = lru;
  return VSS_OK;
}

// VSS_TIME_DEVICE=1: host-clock stamps of each phase of vss_segment_device
// (entry, lock, claim, launch list, pick_graph, hipGraphLaunch, event,
// release), the last 256 calls printed to stderr when the handle is destroyed
// (tools/window_trace.py: where the short window's first call goes).
struct DeviceClock {
  static constexpr int kPts = 8, kRing = 256;
  bool on = std::getenv("VSS_TIME_DEVICE") != nullptr;
  double t[kRing][kPts] = {};
  long calls = 0;
  double* cur = nullptr;
  static double now() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
  }
  void begin() {
    if (!on) return;
    cur = t[calls++ % kRing];
    cur[0] = now();
  }
  void mark(int k) {
    if (on && cur) cur[k] = now();
  }
  void dump() {
    if (!on || !calls) return;
    const long n = std::min<long>(calls, kRing);
    std::fprintf(stderr, "vss device calls (us from entry: lock claim list pick launch event release):\n");
    for (long i = calls - n; i < calls; ++i) {
      const double* c = t[i % kRing];
      std::fprintf(stderr, "  call %ld at %.1f:", i, c[0]);
      for (int k = 1; k < kPts; ++k) std::fprintf(stderr, " %.1f", c[k] - c[0]);
      std::fprintf(stderr, "\n");
    }
  }
};
DeviceClock g_device_clock;

// The forward of n frames with slot `si`'s buffers, on stream st: one of the
// slot's executable graphs for this shape replayed (pick_graph), or eager
// launches.
int forward(vss_handle* h, int si, const uint8_t* frames, int n, int fh, int fw, int fc, size_t rs, size_t fs,
            float* masks, hipStream_t st) {
  Slot& s = h->slots[si];
  h->last_n = n;
  h->last_slot = si;
  s.stem_stored = !has_fused_stem(h) || h->keep_stem;
  std::vector<Launch> ls;
  forward_launches(h, s, frames, n, fh, fw, fc, rs, fs, masks, &ls);
  g_device_clock.mark(3);
  if (h->profile) {
    const int ring = h->prof_next;
    h->prof_next = (h->prof_next + 1) % vss_handle::kProfRing;
    if (h->ring_pending[ring]) {
      int rc = harvest_ring(h, ring);
      if (rc) return rc;
    }
    int rc = launch_eager(h, ls, st, ring);
    if (!rc) h->ring_pending[ring] = 1;
    return rc;
  }
  if (!h->use_graph) return launch_eager(h, ls, st, -1);
  GraphEntry* g = nullptr;
  if (int rc = pick_graph(h, s, GraphKey{n, fh, fw, fc, rs, fs}, ls, &g)) return rc;
  g_device_clock.mark(4);
  HIP_TRY(h, hipGraphLaunch(g->exec, st));
  g_device_clock.mark(5);
  HIP_TRY(h, hipEventRecord(g->last, st));
  g_device_clock.mark(6);
  g->launched = true;
  g->tick = ++s.graph_tick;
  return VSS_OK;
}

void drop_graphs(vss_handle* h) {
  for (Slot& s : h->slots) {
    for (auto& kv : s.graphs) destroy_graph_set(kv.second);
    s.graphs.clear();
    s.shape_tick.clear();
  }
}

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

// Every engine of the handle: engine 0 then the peers.
std::vector<vss_handle*> engines(vss_handle* h) {
  std::vector<vss_handle*> e{h};
  e.insert(e.end(), h->peers.begin(), h->peers.end());
  return e;
}

// Stream-order a slot's next user after its previous one (device side): the
// caller's stream waits for the slot's done event — except when both this
// call and the slot's previous work are on the slot's OWN stream
// (vss_slot_stream), which the handle created and destroys, so no other
// stream can ever carry its address while the handle lives: stream order then
// already holds (5 us of host time per device call saved, 14 -> 9 us,
// tools/window_probe.py).  Round 3 compared any caller stream by address,
// which a destroyed-and-recreated stream or two threads' hipStreamPerThread
// could fool; caller streams now always wait.
int claim_slot(vss_handle* e, Slot& s, hipStream_t st) {
  // (VSS_TEST_NO_CLAIM=1: no wait at all — a diagnostic for callers that keep
  // one stream per slot, tools/window_trace.py; never set in the product)
  static const bool no_claim = std::getenv("VSS_TEST_NO_CLAIM") && std::getenv("VSS_TEST_NO_CLAIM")[0] == '1';
  if (no_claim) return VSS_OK;
  if (s.used && !(st == s.stream && s.done_stream == s.stream)) HIP_TRY(e, hipStreamWaitEvent(st, s.done, 0));
  return VSS_OK;
}

int release_slot(vss_handle* e, Slot& s, hipStream_t st) {
  HIP_TRY(e, hipEventRecord(s.done, st));
  s.used = true;
  s.done_stream = st;
  return VSS_OK;
}

// Is slot k free for a host batch on every GPU of the handle: no lease, no
// host batch still completing, its latest work done?  (mu held)
int slot_free(vss_handle* h, int k, bool* free_) {
  *free_ = !h->slots[k].leased && !h->slots[k].host_busy;
  if (!*free_) return VSS_OK;
  for (vss_handle* e : engines(h)) {
    Slot& s = e->slots[k];
    if (!s.used) continue;
    HIP_TRY(e, hipSetDevice(e->device));
    const hipError_t q = hipEventQuery(s.done);
    if (q == hipErrorNotReady) {
      *free_ = false;
      return VSS_OK;
    }
    if (q != hipSuccess) return fail(h, VSS_E_HIP, std::string("hipEventQuery: ") + hipGetErrorString(q));
  }
  return VSS_OK;
}

// Wait for events with mu released (lk is relocked before returning).
int wait_events_unlocked(vss_handle* h, std::unique_lock<std::mutex>& lk,
                         const std::vector<std::pair<int, hipEvent_t>>& evs) {
  lk.unlock();
  hipError_t e = hipSuccess;
  for (const auto& de : evs) {
    e = hipSetDevice(de.first);
    if (e == hipSuccess) e = hipEventSynchronize(de.second);
    if (e != hipSuccess) break;
  }
  lk.lock();
  if (e != hipSuccess) return fail(h, VSS_E_HIP, std::string("hipEventSynchronize: ") + hipGetErrorString(e));
  return VSS_OK;
}

// The slot for the next host batch (mu held through lk): the first free one
// from the round-robin slot on; if every slot is in flight, VSS_E_BUSY — or,
// with wait_free, wait for the round-robin slot (mu released meanwhile) and
// look again.
int pick_slot(vss_handle* h, std::unique_lock<std::mutex>& lk, bool wait_free, int* out) {
  const int S = (int)h->slots.size();
  for (;;) {
    const int k0 = (int)(h->next_ticket % S);
    for (int j = 0; j < S; ++j) {
      bool fr = false;
      if (int rc = slot_free(h, (k0 + j) % S, &fr)) return rc;
      if (fr) {
        *out = (k0 + j) % S;
        return VSS_OK;
      }
    }
    if (!wait_free) return fail(h, VSS_E_BUSY, "queue full: " + std::to_string(S) + " batches in flight");
    int k = -1;
    for (int j = 0; j < S && k < 0; ++j)
      if (!h->slots[(k0 + j) % S].leased) k = (k0 + j) % S;
    if (k < 0) return fail(h, VSS_E_BUSY, "every slot is leased (vss_staging_acquire)");
    if (h->slots[k].host_busy) {  // its completion is still running: wait for it
      if (g_tls_completing == h)
        return fail(h, VSS_E_BUSY, "called from a completion callback: every slot is still completing");
      h->slot_cv.wait(lk);
      continue;
    }
    std::vector<std::pair<int, hipEvent_t>> evs;
    for (vss_handle* e : engines(h))
      if (e->slots[k].used) evs.push_back({e->device, e->slots[k].done});
    if (int rc = wait_events_unlocked(h, lk, evs)) return rc;
  }
}

// a batch of n frames over R GPUs in contiguous shards of
// per = ceil(n / R); rank r takes [first, first + count) (the last ranks may
// get fewer frames, or none).  Every rank all-gathers `per` rows, so the
// gathered [R][per] rows hold frame i at row i and the padding rows after the
// last frame (only the last non-empty shard can be short).
void shard_plan(int n, int R, int r, int* first, int* count, int* per) {
  const int m = R > 0 ? (n + R - 1) / R : 0;
  const int f0 = r * m;
  *first = std::min(f0, n);
  *count = std::max(0, std::min(n - f0, m));
  *per = m;
}

// The gathered [R][per] rows -> frame order (vss_gather_runs): rank r's
// count frames sit at gathered rows r * per .. r * per + count - 1 and belong
// at output rows first .. first + count - 1; adjacent runs merge (with
// contiguous shards of per frames they all do: one run of n rows).
int gather_runs(int n, int R, int* src_row, int* dst_row, int* rows) {
  int nr = 0;
  for (int r = 0; r < R; ++r) {
    int first, count, per;
    shard_plan(n, R, r, &first, &count, &per);
    if (count == 0) continue;
    const int src = r * per;
    if (nr > 0 && src_row[nr - 1] + rows[nr - 1] == src && dst_row[nr - 1] + rows[nr - 1] == first) {
      rows[nr - 1] += count;
    } else {
      src_row[nr] = src;
      dst_row[nr] = first;
      rows[nr] = count;
      ++nr;
    }
  }
  return nr;
}

// Completion thread of a handle: host batches that need host work when they
// finish (a copy out of the slot's pinned buffer, a callback) are queued in
// ticket order; the thread waits for each batch's D2H, copies, marks the
// slot free for reuse and fires the callback (outside every lock, so a
// callback may call vss_* functions — except vss_destroy of its own handle).
void completion_loop(vss_handle* h) {
  (void)hipSetDevice(h->device);
  g_tls_completing = h;
  for (;;) {
    vss_handle::Completion c;
    {
      std::unique_lock<std::mutex> dl(h->done_mu);
      h->done_cv.wait(dl, [&] { return h->done_stop || !h->done_q.empty(); });
      if (h->done_q.empty()) return;  // stopping, and every queued batch completed
      c = h->done_q.front();
      h->done_q.pop_front();
    }
    Slot& s = h->slots[c.slot];
    hipError_t e = hipEventSynchronize(s.host_done);  // not re-recorded while host_busy
    const int st = e == hipSuccess ? VSS_OK : VSS_E_HIP;
    if (st == VSS_OK && c.out) std::memcpy(c.out, c.src, c.bytes);
    // the slot counts as free once its done event has fired on every GPU too
    // (recorded right after host_done): a submit after this completion finds it free
    for (vss_handle* en : engines(h))
      if (e == hipSuccess && hipSetDevice(en->device) == hipSuccess) e = hipEventSynchronize(en->slots[c.slot].done);
    (void)hipSetDevice(h->device);
    {
      std::lock_guard<std::mutex> lk(h->mu);
      if (st != VSS_OK) set_err(h, std::string("batch failed: ") + hipGetErrorString(e));
      s.status = st;
      s.host_busy = false;
    }
    h->slot_cv.notify_all();
    if (c.cb) c.cb(c.user, st);
  }
}

void push_completion(vss_handle* h, const vss_handle::Completion& c) {  // mu held
  if (!h->done_thread.joinable()) h->done_thread = std::thread(completion_loop, h);
  {
    std::lock_guard<std::mutex> dl(h->done_mu);
    h->done_q.push_back(c);
  }
  h->done_cv.notify_one();
}

void stop_completions(vss_handle* h) {
  if (!h->done_thread.joinable()) return;
  {
    std::lock_guard<std::mutex> dl(h->done_mu);
    h->done_stop = true;
  }
  h->done_cv.notify_all();
  h->done_thread.join();
}

// VSS_TIME_SUBMIT=1: host time of each phase of the queued submit, summed over
// the calls and printed when the handle is destroyed (where the calling
// thread's time goes; tools/ts_prof.js showed the N-API call dominating).
// Every call's phases are kept too (up to 8192 calls) and printed as per-phase
// medians by batch size.
struct SubmitClock {
  static constexpr int kPhases = 8;
  bool on = std::getenv("VSS_TIME_SUBMIT") != nullptr;
  double ns[kPhases] = {};
  long calls = 0;
  std::chrono::steady_clock::time_point t;
  std::vector<std::pair<int, std::vector<double>>> rows;  // (frames, per-phase ns)
  void start() {
    if (on) t = std::chrono::steady_clock::now();
  }
  void mark(int k) {
    if (!on) return;
    const auto n = std::chrono::steady_clock::now();
    const double d = std::chrono::duration<double, std::nano>(n - t).count();
    ns[k] += d;
    if (k == 0 && rows.size() < 8192) rows.push_back({0, std::vector<double>(kPhases, 0.0)});
    if (!rows.empty()) rows.back().second[k] = d;
    t = n;
  }
  void frames(int n) {
    if (on && !rows.empty()) rows.back().first = n;
  }
};
SubmitClock g_submit_clock;

// Pinned result buffers (vss_host_alloc): a masks_out inside one of these
// receives the batch's D2H directly, so the completion copies nothing.  The
// registry is process-wide (any handle, any GPU), keyed by start address.
std::mutex g_pin_mu;
std::map<uintptr_t, size_t> g_pinned;

bool pinned_range(const void* p, size_t bytes) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  std::lock_guard<std::mutex> lk(g_pin_mu);
  auto it = g_pinned.upper_bound(a);
  if (it == g_pinned.begin()) return false;
  --it;
  return a >= it->first && a + bytes <= it->first + it->second;
}

// A queued host call: stage n host frames (each GPU its contiguous shard),
// then on every GPU's slot stream H2D -> forward -> [RCCL all-gather] and on
// engine 0's: [frame-size upsample] -> D2H -> host_done.  What happens on the
// host when the batch is done:
//   * masks_out inside a vss_host_alloc block and no callback: nothing — the
//     D2H wrote them there, the event is the completion (vss_wait syncs it);
//   * otherwise the completion thread copies out of the slot's pinned buffer
//     and fires the callback, in ticket order;
//   * sync (vss_segment): the calling thread waits and copies, mu released.
//   wait_free: block until a slot is free (else VSS_E_BUSY);
//   list: frame i at list[i] instead of frames + i * height * row_stride;
//   lease: the slot a vss_staging_acquire reserved (-1: pick a free one).
int submit_host(vss_handle* h, const uint8_t* frames, const uint8_t* const* list, int n, int fh, int fw, int fc,
                size_t rs, float* masks_out, int out_mode, bool wait_free, bool sync, vss_callback cb, void* user,
                vss_ticket* ticket, int lease = -1) {
  if ((!frames && !list) || !masks_out) return fail(h, VSS_E_INVALID_ARG, "null frames/masks_out");
  if (list)
    for (int i = 0; i < n; ++i)
      if (!list[i]) return fail(h, VSS_E_INVALID_ARG, "null frame pointer in the list");
  if (out_mode != VSS_OUT_MODEL && out_mode != VSS_OUT_FRAME)
    return fail(h, VSS_E_INVALID_ARG, "out_mode must be VSS_OUT_MODEL or VSS_OUT_FRAME");
  int rc = check_frames(h, n, fh, fw, fc, rs, rs * (size_t)fh, h->user_max_batch);
  if (rc) return rc;
  const std::vector<vss_handle*> E = engines(h);
  const int R = (int)E.size();
  int m = 0, f0_, n0_;
  shard_plan(n, R, 0, &f0_, &n0_, &m);  // frames per GPU
  const size_t fbytes = (size_t)fh * rs;
  if ((size_t)m * fbytes > h->frame_cap)
    return fail(h, VSS_E_INVALID_ARG, "frames exceed the handle's staging capacity (max_frame_h/w)");
  if (out_mode == VSS_OUT_FRAME && (size_t)n * fh * fw > (size_t)h->user_max_batch * h->cfg.max_frame_h * h->cfg.max_frame_w)
    return fail(h, VSS_E_INVALID_ARG, "frame-size masks exceed max_batch * max_frame_h * max_frame_w");
  const size_t P = (size_t)h->cfg.model_h * h->cfg.model_w;
  SubmitClock& clk = g_submit_clock;
  clk.start();
  const int clk_n = n;
  std::unique_lock<std::mutex> lk(h->mu);
  clk.mark(0);
  // a free slot: its previous batch is done on every GPU, so its staging may be rewritten
  int k = lease;
  if (lease >= 0) {
    if (lease >= (int)h->slots.size() || !h->slots[lease].leased)
      return fail(h, VSS_E_INVALID_ARG, "not a leased slot (vss_staging_acquire)");
    h->slots[lease].leased = false;  // its batch runs now
  } else if ((rc = pick_slot(h, lk, wait_free, &k))) {
    return rc;
  }
  for (vss_handle* e : E) {
    HIP_TRY(e, hipSetDevice(e->device));
    if ((rc = ensure_staging(e, e->slots[k]))) return fail(h, rc, e->err);
  }
  Slot& s0 = h->slots[k];
  if (out_mode == VSS_OUT_FRAME && (rc = ensure_frame_masks(h, s0))) return rc;
  clk.mark(1);
  // only the rows the resize reads cross PCIe when that skips 60 % of them or
  // more (measured: 1080p, 20 % of the rows, 8.7k -> 23-29k frames/s; at
  // 640x480, 50 %, the kernel's reads of pinned memory lost to one DMA of the
  // whole frames, 38-46k -> 31-39k)
  //   Whatever moves the rows across PCIe, only the rows the resize reads are
  // copied into the staging (the other rows of the staged frames are never
  // read: the fused stem, k_prep and the post chain's guide all sample the
  // same rows): at 640x480 that halves the host memcpy of the copy path.
  // (VSS_FETCH_SINGLE=k, an A/B knob, default 0: batches of at most k
  // frames move their rows with k_fetch_rows whatever their share.  For one
  // 640x480 frame it depends on the box: the TS segmentFrame p50 0.146-0.152
  // against 0.155-0.198 ms on one (profiles/r06/r06an), 0.182-0.185 against
  // 0.155-0.191 on another (r06aq) — the kernel's reads of pinned host
  // memory are slower on some hosts than one DMA of the whole frame)
  static const int fetch_single = [] {
    const char* e = std::getenv("VSS_FETCH_SINGLE");
    return e ? std::atoi(e) : 0;
  }();
  std::vector<const RowPlan*> plans(R, nullptr);  // the rows (row_fetch on)
  std::vector<bool> fetch(R, false);              // move them with k_fetch_rows (else one DMA)
  for (int r = 0; r < R; ++r) {
    HIP_TRY(E[r], hipSetDevice(E[r]->device));
    if (!h->row_fetch) continue;
    if ((rc = row_plan(E[r], fh, &plans[r]))) return fail(h, rc, E[r]->err);
    fetch[r] = plans[r]->rows.size() * 5 <= (size_t)fh * 2 || (n <= fetch_single && n >= 1);
  }
  // stage every GPU's shard (zero-copy when the caller wrote into this slot's buffer)
  std::vector<CopyPool::Job> jobs;
  for (int r = 0; r < R; ++r) {
    int f0, nr, per;
    shard_plan(n, R, r, &f0, &nr, &per);
    uint8_t* dst = E[r]->slots[k].h_frames;
    for (int i = 0; i < nr; ++i) {
      const uint8_t* src = list ? list[f0 + i] : frames + (size_t)(f0 + i) * fbytes;
      uint8_t* d = dst + (size_t)i * fbytes;
      if (src == d) continue;
      if (plans[r]) {
        for (const auto& run : plans[r]->runs)
          jobs.push_back({d + (size_t)run.first * rs, src + (size_t)run.first * rs, (size_t)(run.second - run.first) * rs});
      } else if (list) {
        jobs.push_back({d, src, fbytes});
      } else {  // contiguous: the shard in one job
        jobs.push_back({d, src, (size_t)(nr - i) * fbytes});
        break;
      }
    }
  }
  clk.mark(2);
  h->pool->run(jobs);
  clk.mark(3);
  // From the first claim on, every exit records each claimed slot's done event
  // (so the slot's next user is ordered after whatever was enqueued) and a
  // failure leaves the slot free with the error as its status.
  int claimed = 0;
  auto abort_batch = [&](int code) {
    for (int r = 0; r < claimed; ++r) {
      (void)hipSetDevice(E[r]->device);
      (void)hipEventRecord(E[r]->slots[k].done, E[r]->slots[k].stream);
      E[r]->slots[k].used = true;
      E[r]->slots[k].done_stream = E[r]->slots[k].stream;
    }
    (void)hipSetDevice(h->device);
    s0.status = code;
    return code;
  };
  for (int r = 0; r < R; ++r) {
    vss_handle* e = E[r];
    Slot& s = e->slots[k];
    int f0, nr, per;
    shard_plan(n, R, r, &f0, &nr, &per);
    HIP_TRY(e, hipSetDevice(e->device));
    if ((rc = claim_slot(e, s, s.stream))) return abort_batch(fail(h, rc, e->err));
    ++claimed;
    if (nr > 0) {
      if (fetch[r]) {
        FetchRowsParams fp{};
        fp.src = s.h_frames;
        fp.dst = s.d_frames;
        fp.rows = plans[r]->d_rows;
        fp.row_stride = (long)rs;
        fp.frame_stride = (long)fbytes;
        fp.row_bytes = fw * fc;
        fp.vec16 = (rs % 16 == 0 && fbytes % 16 == 0 && (fw * fc) % 16 == 0) ? 1 : 0;
        launch_fetch_rows(fp, (int)plans[r]->rows.size(), nr, s.stream);
        const hipError_t e_ = hipGetLastError();
        if (e_ != hipSuccess) return abort_batch(fail(h, VSS_E_HIP, std::string("k_fetch_rows: ") + hipGetErrorString(e_)));
      } else {
        const hipError_t e_ = hipMemcpyAsync(s.d_frames, s.h_frames, (size_t)nr * fbytes, hipMemcpyHostToDevice, s.stream);
        if (e_ != hipSuccess) return abort_batch(fail(h, VSS_E_HIP, std::string("H2D: ") + hipGetErrorString(e_)));
      }
      if ((rc = forward(e, k, s.d_frames, nr, fh, fw, fc, rs, fbytes, s.d_masks, s.stream)))
        return abort_batch(fail(h, rc, e->err));
    }
  }
  clk.mark(4);
  const float* res = s0.d_masks;
  if (h->rccl) {
    for (int r = 0; r < R; ++r)
      if ((rc = comm_healthy(E[r], E[r]->slots[k].comm, k))) return abort_batch(fail(h, rc, E[r]->err));
    // one all-gather of f32 masks per GPU, m frames each (padding rows of the
    // last shards are gathered and dropped): [rank][m][P] = frame order
    ncclResult_t nr_ = ncclGroupStart();
    for (int r = 0; r < R && nr_ == ncclSuccess; ++r) {
      Slot& s = E[r]->slots[k];
      nr_ = ncclAllGather(s.d_masks, s.d_gather, (size_t)m * P, ncclFloat32, s.comm, s.stream);
    }
    const ncclResult_t ne = ncclGroupEnd();
    if (nr_ == ncclSuccess) nr_ = ne;
    if (nr_ != ncclSuccess) return abort_batch(fail(h, VSS_E_RCCL, std::string("ncclAllGather: ") + ncclGetErrorString(nr_)));
    res = s0.d_gather;
  }
  HIP_TRY(h, hipSetDevice(h->device));
  const float* src = s0.h_masks;
  size_t bytes = (size_t)n * P * 4;
  if (out_mode == VSS_OUT_FRAME) bytes = (size_t)n * fh * fw * 4;
  // masks_out from vss_host_alloc: the D2H lands there, nothing to copy after
  const bool direct = pinned_range(masks_out, bytes);
  hipError_t e_ = hipSuccess;
  // gathered rows -> frame order (one run per rank at most; for the plain
  // handle and contiguous shards a single run of n rows from row 0)
  std::vector<int> run_src(R), run_dst(R), run_rows(R);
  const int nruns = h->rccl ? gather_runs(n, R, run_src.data(), run_dst.data(), run_rows.data()) : (n > 0 ? 1 : 0);
  if (!h->rccl && nruns) run_src[0] = run_dst[0] = 0, run_rows[0] = n;
  if (out_mode == VSS_OUT_FRAME) {
    const size_t F = (size_t)fh * fw;
    for (int j = 0; j < nruns && e_ == hipSuccess; ++j) {
      enqueue_upmask(h, res + (size_t)run_src[j] * P, run_rows[j], fh, fw, s0.d_fmasks + (size_t)run_dst[j] * F,
                     s0.stream);
      e_ = hipGetLastError();
    }
    src = s0.h_fmasks;
    if (e_ == hipSuccess)
      e_ = hipMemcpyAsync(direct ? masks_out : s0.h_fmasks, s0.d_fmasks, bytes, hipMemcpyDeviceToHost, s0.stream);
  } else {
    float* dst = direct ? masks_out : s0.h_masks;
    for (int j = 0; j < nruns && e_ == hipSuccess; ++j)
      e_ = hipMemcpyAsync(dst + (size_t)run_dst[j] * P, res + (size_t)run_src[j] * P, (size_t)run_rows[j] * P * 4,
                          hipMemcpyDeviceToHost, s0.stream);
  }
  if (e_ == hipSuccess) e_ = hipEventRecord(s0.host_done, s0.stream);
  if (e_ != hipSuccess) return abort_batch(fail(h, VSS_E_HIP, std::string("D2H: ") + hipGetErrorString(e_)));
  clk.mark(5);
  for (vss_handle* e : E) {
    HIP_TRY(e, hipSetDevice(e->device));
    if ((rc = release_slot(e, e->slots[k], e->slots[k].stream))) return abort_batch(fail(h, rc, e->err));
  }
  HIP_TRY(h, hipSetDevice(h->device));
  const vss_ticket t = h->next_ticket++;
  s0.ticket = t;
  s0.status = VSS_OK;
  clk.mark(6);
  if (sync) {
    // the slot's pinned buffers stay ours until the copy below: host_busy
    s0.host_busy = true;
    std::vector<std::pair<int, hipEvent_t>> evs{{h->device, s0.host_done}};
    for (vss_handle* e : E) evs.push_back({e->device, e->slots[k].done});
    rc = wait_events_unlocked(h, lk, evs);
    if (!rc && !direct) std::memcpy(masks_out, src, bytes);
    s0.status = rc;
    s0.host_busy = false;
    lk.unlock();
    h->slot_cv.notify_all();
    return rc;
  }
  if (!direct || cb) {
    s0.host_busy = true;
    s0.status = 1;  // pending until the completion thread has run
    push_completion(h, {t, k, direct ? nullptr : masks_out, src, bytes, cb, user});
  }
  clk.mark(7);
  clk.frames(clk_n);
  clk.calls += clk.on ? 1 : 0;
  if (ticket) *ticket = t;
  return VSS_OK;
}

// Autotune: time every compiled tile of every block layer at max_batch on
// this device and keep the fastest.  The kernels' arithmetic does not depend
// on the tile (see block_lds), so this changes speed only, never results.
//   Default: one launch at a time (latency).  VSS_AUTOTUNE=throughput times
// a candidate as the engine runs it in steady state instead — one launch per
// slot, all slots' streams at once (each slot's own buffers) — where a tile's
// LDS x lifetime per output decides, not its latency alone (at 4 batches in
// flight the CUs hold ~3.3 workgroups each, LDS-full, ~4 % idle:
// tools/trace_inflight.py).  Measured (round 3, 2 x 2 interleaved runs):
// 179.6k / 193.6k frames/s throughput-tuned against 192.5k / 188.9k — its
// picks vary between runs, so latency stays the default.
//   small: time the candidates at batch N (1) and keep the pick as the layer's
// small-batch tile (LayerPlan::small), the layer's own tile restored.
int autotune_at(vss_handle* h, int N, bool small) {
  const int pi = h->cfg.dtype == VSS_DTYPE_F32 ? 0 : 1;
  Slot& s = h->slots[0];
  if (int rc = ensure_staging(h, s)) return rc;  // the stem reads the staging buffer as frames
  static const char* mode_env = std::getenv("VSS_AUTOTUNE");
  const bool concurrent = h->slots.size() > 1 && mode_env && !std::strcmp(mode_env, "throughput");
  // VSS_AUTOTUNE=lds: the latency timings, but the pick minimises the layer's
  // LDS x lifetime (workgroups x allocated LDS x latency / rounds of
  // workgroups: what one batch costs the LDS-full chip at 4 batches in flight,
  // tools/lds_time.py) instead of its latency.  VSS_AUTOTUNE_DUMP=1: every
  // candidate's numbers on stderr.
  const bool lds_obj = mode_env && !std::strcmp(mode_env, "lds");
  static const bool dump = std::getenv("VSS_AUTOTUNE_DUMP") != nullptr;
  const int S = concurrent ? (int)h->slots.size() : 1;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  HIP_TRY(h, hipEventCreate(&e0));
  HIP_TRY(h, hipEventCreate(&e1));
  std::vector<hipEvent_t> ends(S, nullptr);
  for (auto& e : ends) HIP_TRY(h, hipEventCreateWithFlags(&e, hipEventDisableTiming));
  int rc = VSS_OK;
  for (size_t li = 0; li < h->L.size(); ++li) {
    LayerPlan& l = h->L[li];
    if (l.mode < 0) continue;
    const std::vector<const BlockEntry*> cands = tile_candidates(l);
    if (cands.size() < 2) continue;
    const BlockEntry* own = l.entry;
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
        std::vector<BlockParams> prm(S);
        for (int k = 0; k < S; ++k) {
          prm[k] = block_params(h, h->slots[k], (int)li, N);
          if (flags_stem_in(l.flags)) {  // slot 0's staging buffer as frames: any bytes, valid memory
            prm[k].stem = stem_params(h, h->slots[k], (int)l.rec.src, s.d_frames, (size_t)h->cfg.max_frame_w * 3,
                                      (size_t)h->cfg.max_frame_w * 3 * h->cfg.max_frame_h, h->cfg.max_frame_h,
                                      h->cfg.max_frame_w, 3);
            prm[k].stem.y = nullptr;  // timed as the forward runs it by default
          }
        }
        const dim3 grid(l.tiles_x, l.tiles_y, N * l.ks);
        auto run = [&](int reps) {
          for (int k = 0; k < S; ++k) {
            hipStream_t st = S > 1 ? h->slots[k].stream : h->stream;
            if (S > 1) (void)hipStreamWaitEvent(st, e0, 0);
            for (int q = 0; q < reps; ++q)
              hipLaunchKernelGGL(e->fn[pi], grid, dim3(e->threads), l.lds, st, prm[k]);
            if (S > 1) {
              (void)hipEventRecord(ends[k], st);
              (void)hipStreamWaitEvent(h->stream, ends[k], 0);
            }
          }
        };
        (void)hipEventRecord(e0, h->stream);
        run(2);
        (void)hipEventRecord(e0, h->stream);
        run(8);
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
    double best_obj = 1e30;
    for (size_t c = 0; c < cands.size(); ++c) {
      if (!usable[c]) continue;
      double obj = best_of[c];
      if (lds_obj || dump) {
        set_tile(l, cands[c]);
        int occ = 0;
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void*)cands[c]->fn[pi], cands[c]->threads,
                                                            (int)l.lds);
        occ = std::max(1, std::min(occ, lds_wg_per_cu((int)l.lds)));
        int cus = 256;
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, h->device);
        const long wgs = (long)l.tiles_x * l.tiles_y * N * l.ks;
        const long rounds = (wgs + (long)cus * occ - 1) / ((long)cus * occ);
        const double alloc = (double)((l.lds + kLdsGranule - 1) / kLdsGranule * kLdsGranule);
        const double lt = (double)wgs * alloc * (best_of[c] / 8.0 * 1e3) / (double)rounds / 1e6;  // MB x us
        if (dump)
          std::fprintf(stderr, "autotune batch %d layer %zu cand %zu %dx%d var %d: %.2f us/launch, %ld WGs, %d/CU, %zu B LDS, "
                       "%ld rounds, LDS x life %.1f MB*us\n", N, li, c, cands[c]->TH, cands[c]->TW, cands[c]->variant,
                       best_of[c] / 8.0 * 1e3, wgs, occ, (size_t)l.lds, rounds, lt);
        if (lds_obj) obj = lt;
      }
      if (obj < best_obj * 0.98) {  // ties keep the earlier (planner-preferred) shape
        best_obj = obj;
        best = cands[c];
      }
    }
    if (small) {
      l.small = best != own ? best : nullptr;
      set_tile(l, own);
    } else {
      set_tile(l, best);
    }
    if (rc) break;
  }
  for (auto e : ends) (void)hipEventDestroy(e);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return rc;
}

// Tiles for max_batch, then (max_batch >= 4) a second pick at batch 1 that
// the forwards of at most max_batch / 4 frames use (small_tile_n): one batch
// of 8 and one frame want different tiles — at batch 1 the batch-8 tiles leave
// most CUs idle (b1's 4x16 tile: 144 workgroups).  Results do not depend on
// the tile (block_lds), so a forward's masks are bitwise the same either way.
// VSS_SMALL_TILES=0: the max_batch tiles for every batch size.
int autotune(vss_handle* h) {
  if (int rc = autotune_at(h, h->cfg.max_batch, false)) return rc;
  static const bool small_on = !(std::getenv("VSS_SMALL_TILES") && std::getenv("VSS_SMALL_TILES")[0] == '0');
  if (small_on && h->cfg.max_batch >= 4) {
    if (int rc = autotune_at(h, 1, true)) return rc;
    h->small_tile_n = h->cfg.max_batch / 4;
  }
  return VSS_OK;
}

// Pin layers to given compiled tiles (after the planner and the autotuner):
// the tile-invariance tests run every compiled tile of every layer this way.
int force_tiles(vss_handle* h, const char* spec) {
  const int pi = h->cfg.dtype == VSS_DTYPE_F32 ? 0 : 1;
  const char* s = spec;
  while (*s) {
    // "layer:THxTW" (the first compiled shape with that tile) or "layer:#k"
    // (candidate k of vss_layer_tiles' list: tiles can repeat across variants)
    int layer = -1, th = 0, tw = 0, idx = -1, used = 0;
    if (std::sscanf(s, "%d:#%d%n", &layer, &idx, &used) != 2 &&
        std::sscanf(s, "%d:%dx%d%n", &layer, &th, &tw, &used) != 3)
      return fail(h, VSS_E_INVALID_ARG, std::string("VSS_TILE: bad entry in '") + spec + "'");
    if (layer < 0 || layer >= (int)h->L.size())
      return fail(h, VSS_E_INVALID_ARG, std::string("VSS_TILE: bad layer in '") + spec + "'");
    LayerPlan& l = h->L[layer];
    const BlockEntry* pick = nullptr;
    if (l.mode >= 0) {
      const std::vector<const BlockEntry*> c = tile_candidates(l);
      if (idx >= 0) {
        if (idx < (int)c.size()) pick = c[idx];
      } else {
        for (const BlockEntry* e : c)
          if (!pick && e->TH == th && e->TW == tw) pick = e;
      }
    }
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

void destroy_engine(vss_handle* h);

// One engine on one GPU: weights, plan, slots (gather_ranks > 0: each slot
// holds a gather buffer for that many GPUs' masks).
int create_engine(const vss_config* cfg, int device, int max_batch, int user_max_batch, int depth, int gather_ranks,
                  vss_handle** out) {
  vss_handle* h = new vss_handle();
  *out = h;
  h->cfg = *cfg;
  h->cfg.max_batch = max_batch;
  h->cfg.device_id = device;
  h->cfg.device_ids = nullptr;
  h->weights_path = cfg->weights_path;
  h->cfg.weights_path = nullptr;
  h->device = device;
  h->user_max_batch = user_max_batch;
  if (hipSetDevice(h->device) != hipSuccess) return fail(h, VSS_E_HIP, "hipSetDevice failed");
  if (const char* ev = std::getenv("VSS_KSPLIT_PIXELS")) h->ksplit_pixels = std::atol(ev);
  if (const char* ev = std::getenv("VSS_KSPLIT")) h->ksplit_on = std::atoi(ev) != 0;
  if (const char* ev = std::getenv("VSS_FUSE_STEM")) h->fuse_stem = std::atoi(ev) != 0;
  // (the round-5 knob: VSS_GATHER_SERIAL=0 selects the concurrent form, =1 the ordered one)
  if (const char* ev = std::getenv("VSS_GATHER_SERIAL"))
    h->gather_form = ev[0] == '0' ? VSS_GATHER_CONCURRENT : VSS_GATHER_ORDERED;
  int rc = load_weights(h);
  if (!rc) rc = plan(h);
  if (!rc) rc = upload(h);
  if (rc) return rc;
  HIP_TRY(h, hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking));
  h->frame_cap = (size_t)max_batch * cfg->max_frame_h * cfg->max_frame_w * 4;
  h->slots.resize(depth);
  for (Slot& s : h->slots)
    if ((rc = make_slot(h, s, gather_ranks))) return rc;
  const size_t P = (size_t)cfg->model_h * cfg->model_w;
  if ((rc = dalloc(h, &h->d_post_alpha, (size_t)max_batch * P * 4))) return rc;
  if ((rc = dalloc(h, &h->d_post_u8, (size_t)max_batch * P))) return rc;
  for (const LayerPlan& l : h->L)
    if (l.entry)
      for (BlockFn fn : l.entry->fn)
        HIP_TRY(h, hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)l.lds));
  const int nl = (int)h->L.size();
  h->ev.resize((size_t)vss_handle::kProfRing * nl * 2);
  for (auto& e : h->ev) HIP_TRY(h, hipEventCreate(&e));
  h->ring_pending.assign(vss_handle::kProfRing, 0);
  h->prof_sum.assign(nl, 0.0);
  if (!(cfg->flags & VSS_CREATE_NO_AUTOTUNE) && (rc = autotune(h))) return rc;
  if (const char* ev = std::getenv("VSS_TILE"))  // tests / scans: "layer:THxTW[,layer:THxTW...]"
    if ((rc = force_tiles(h, ev))) return rc;
  return VSS_OK;
}

void destroy_engine(vss_handle* h) {
  if (!h) return;
  if (g_submit_clock.on && g_submit_clock.calls > 0) {
    static const char* names[SubmitClock::kPhases] = {"lock", "slot", "plan", "copy", "h2d+fwd", "d2h", "release",
                                                      "queue"};
    std::fprintf(stderr, "vss submit phases (us/call over %ld calls):", g_submit_clock.calls);
    for (int k = 0; k < SubmitClock::kPhases; ++k)
      std::fprintf(stderr, " %s %.1f", names[k], g_submit_clock.ns[k] / 1e3 / g_submit_clock.calls);
    std::fprintf(stderr, "\n");
    std::map<int, std::vector<std::vector<double>>> by_n;
    for (const auto& r : g_submit_clock.rows) by_n[r.first].push_back(r.second);
    for (auto& kv : by_n) {
      std::fprintf(stderr, "vss submit phases, %d-frame calls (%zu), median us:", kv.first, kv.second.size());
      for (int k = 0; k < SubmitClock::kPhases; ++k) {
        std::vector<double> v;
        for (const auto& r : kv.second) v.push_back(r[k]);
        std::nth_element(v.begin(), v.begin() + v.size() / 2, v.end());
        std::fprintf(stderr, " %s %.1f", names[k], v[v.size() / 2] / 1e3);
      }
      std::fprintf(stderr, "\n");
    }
    g_submit_clock = SubmitClock();
    g_submit_clock.on = true;
  }
  stop_completions(h);  // every queued batch completes (and its callback fires) first
  (void)hipSetDevice(h->device);
  (void)hipDeviceSynchronize();
  for (Slot& s : h->slots) {
    for (auto& kv : s.graphs) destroy_graph_set(kv.second);
    if (s.comm) (void)ncclCommDestroy(s.comm);
    if (s.stream) (void)hipStreamDestroy(s.stream);
    if (s.done) (void)hipEventDestroy(s.done);
    if (s.host_done) (void)hipEventDestroy(s.host_done);
  }
  for (auto e : h->ev)
    if (e) (void)hipEventDestroy(e);
  for (auto e : h->gather_ev)
    if (e) (void)hipEventDestroy(e);
  for (void* p : h->dev_allocs) (void)hipFree(p);
  for (void* p : h->host_allocs) (void)hipHostFree(p);
  if (h->stream) (void)hipStreamDestroy(h->stream);
  delete h->pool;
  delete h;
}


}  // namespace

extern "C" {

int vss_version(void) { return VSS_VERSION; }

const char* vss_last_error(const vss_handle* h) {
  // a handle's message is copied under its lock into this thread's buffer:
  // the pointer stays valid until this thread's next vss_last_error or failing
  // call, whatever other threads' calls on the handle write meanwhile
  if (!h) return g_tls_error.c_str();
  thread_local std::string copy;
  std::lock_guard<std::mutex> lk(h->err_mu);
  copy = h->err;
  return copy.c_str();
}

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
  if (cfg->queue_depth < 0 || cfg->queue_depth > kMaxQueueDepth)
    return fail(nullptr, VSS_E_INVALID_ARG, "queue_depth must be 0 (default) .. " + std::to_string(kMaxQueueDepth));
  if (cfg->staging_threads < 0 || cfg->staging_threads > 64)
    return fail(nullptr, VSS_E_INVALID_ARG, "staging_threads must be 0 (default) .. 64");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
    return fail(nullptr, VSS_E_HIP, "no HIP device available");
  std::vector<int> devs;
  if (cfg->device_ids) {
    if (cfg->n_gpus < 1) return fail(nullptr, VSS_E_INVALID_ARG, "n_gpus must be >= 1 with device_ids");
    for (int r = 0; r < cfg->n_gpus; ++r) {
      const int d = cfg->device_ids[r];
      if (d < 0 || d >= ndev)
        return fail(nullptr, VSS_E_INVALID_ARG, "device_ids[" + std::to_string(r) + "] = " + std::to_string(d) +
                                                    " is not a HIP device (0.." + std::to_string(ndev - 1) + ")");
      if (std::find(devs.begin(), devs.end(), d) != devs.end())
        return fail(nullptr, VSS_E_INVALID_ARG, "device_ids lists GPU " + std::to_string(d) + " twice");
      devs.push_back(d);
    }
  } else {
    if (cfg->n_gpus > 1) return fail(nullptr, VSS_E_INVALID_ARG, "n_gpus > 1 needs device_ids");
    if (cfg->device_id < 0 || cfg->device_id >= ndev) return fail(nullptr, VSS_E_INVALID_ARG, "bad device_id");
    devs.push_back(cfg->device_id);
  }
  const int R = (int)devs.size();
  if (cfg->max_batch < R) return fail(nullptr, VSS_E_INVALID_ARG, "max_batch must be >= n_gpus");
  const int depth = cfg->queue_depth ? cfg->queue_depth : kDefaultQueueDepth;
  const int per = (cfg->max_batch + R - 1) / R;  // frames per GPU
  const bool rccl = cfg->device_ids != nullptr;
  vss_handle* h = nullptr;
  auto bail = [&](vss_handle* bad, int rc) {
    g_tls_error = bad && !bad->err.empty() ? bad->err : g_tls_error;
    if (h) {
      stop_completions(h);
      for (vss_handle* p : h->peers) destroy_engine(p);
      h->peers.clear();
      if (bad && bad != h) destroy_engine(bad);
      destroy_engine(h);
    } else if (bad) {
      destroy_engine(bad);
    }
    return rc;
  };
  int rc = create_engine(cfg, devs[0], per, cfg->max_batch, depth, rccl ? R : 0, &h);
  if (rc) {
    vss_handle* bad = h;
    h = nullptr;
    return bail(bad, rc);
  }
  h->rccl = rccl;
  for (int r = 1; r < R; ++r) {
    vss_handle* p = nullptr;
    rc = create_engine(cfg, devs[r], per, per, depth, R, &p);
    if (rc) return bail(p, rc);
    h->peers.push_back(p);
  }
  if (rccl) {
    // one communicator per slot over the handle's GPUs (concurrent slots never share one)
    for (int k = 0; k < depth; ++k) {
      std::vector<ncclComm_t> comms(R, nullptr);
      const ncclResult_t nr = ncclCommInitAll(comms.data(), R, devs.data());
      if (nr != ncclSuccess)
        return bail(nullptr, fail(nullptr, VSS_E_RCCL, std::string("ncclCommInitAll: ") + ncclGetErrorString(nr)));
      std::vector<vss_handle*> E = engines(h);
      for (int r = 0; r < R; ++r) E[r]->slots[k].comm = comms[r];
    }
  }
  const int threads = cfg->staging_threads ? cfg->staging_threads : kDefaultStagingThreads;
  h->pool = new CopyPool(threads - 1);  // the submitting thread copies too
  (void)hipSetDevice(h->device);
  *out = h;
  return VSS_OK;
}

void vss_destroy(vss_handle* h) {
  if (!h) return;
  g_device_clock.dump();
  // drain the completion thread first: it reads h->peers and waits on the
  // peers' slot events, so every queued batch completes (and its callback
  // fires) while the peers still exist (use-after-free otherwise)
  stop_completions(h);
  for (vss_handle* p : h->peers) destroy_engine(p);
  h->peers.clear();
  destroy_engine(h);
}

int vss_get_info(const vss_handle* h, vss_info* info) {
  if (!h || !info) return VSS_E_INVALID_ARG;
  info->mask_h = h->cfg.model_h;
  info->mask_w = h->cfg.model_w;
  info->n_layers = (int)h->L.size();
  info->dtype = h->cfg.dtype;
  info->device_bytes = h->dev_bytes;
  for (const vss_handle* p : h->peers) info->device_bytes += p->dev_bytes;
  info->n_gpus = 1 + (int)h->peers.size();
  info->queue_depth = (int)h->slots.size();
  info->rccl = h->rccl ? 1 : 0;
  return VSS_OK;
}

int vss_segment(vss_handle* h, const uint8_t* frames, int n, int height, int width, int channels,
                size_t row_stride, float* masks_out, int out_mode) {
  if (!h) return fail(nullptr, VSS_E_INVALID_ARG, "null handle");
  return submit_host(h, frames, nullptr, n, height, width, channels, row_stride, masks_out, out_mode, true, true,
                     nullptr, nullptr, nullptr);
}

int vss_segment_async(vss_handle* h, const uint8_t* frames, int n, int height, int width, int channels,
                      size_t row_stride, float* masks_out, int out_mode, vss_callback cb, void* user) {
  if (!h) return fail(nullptr, VSS_E_INVALID_ARG, "null handle");
  return submit_host(h, frames, nullptr, n, height, width, channels, row_stride, masks_out, out_mode, false, false, cb,
                     user, nullptr);
}

int vss_submit(vss_handle* h, const uint8_t* frames, int n, int height, int width, int channels, size_t row_stride,
               float* masks_out, int out_mode, vss_ticket* ticket) {
  if (!h) return fail(nullptr, VSS_E_INVALID_ARG, "null handle");
  if (!ticket) return fail(h, VSS_E_INVALID_ARG, "null ticket");
  return submit_host(h, frames, nullptr, n, height, width, channels, row_stride, masks_out, out_mode, false, false,
                     nullptr, nullptr, ticket);
}

int vss_submit_list(vss_handle* h, const uint8_t* const* frames, int n, int height, int width, int channels,
                    size_t row_stride, float* masks_out, int out_mode, vss_ticket* ticket) {
  if (!h) return fail(nullptr, VSS_E_INVALID_ARG, "null handle");
  if (!ticket || !frames) return fail(h, VSS_E_INVALID_ARG, "null ticket/frames");
  return submit_host(h, nullptr, frames, n, height, width, channels, row_stride, masks_out, out_mode, false, false,
                     nullptr, nullptr, ticket);
}

int vss_submit_list_async(vss_handle* h, const uint8_t* const* frames, int n, int height, int width, int channels,
                          size_t row_stride, float* masks_out, int out_mode, vss_callback cb, void* user,
                          vss_ticket* ticket) {
  if (!h) return fail(nullptr, VSS_E_INVALID_ARG, "null handle");
  if (!frames || !cb) return fail(h, VSS_E_INVALID_ARG, "null frames/callback");
  return submit_host(h, nullptr, frames, n, height, width, channels, row_stride, masks_out, out_mode, true, false, cb,
                     user, ticket);
}

// The slot holding host ticket t, or -1 when no slot does any more: a slot
// takes a new host batch only once it is free (its previous batch done and
// completed), so a ticket no slot holds is done.  mu held.
static int ticket_slot(const vss_handle* h, vss_ticket t) {
  for (size_t k = 0; k < h->slots.size(); ++k)
    if (h->slots[k].ticket == t) return (int)k;
  return -1;
}

int vss_wait(vss_handle* h, vss_ticket ticket) {
  if (!h) return fail(nullptr, VSS_E_INVALID_ARG, "null handle");
  std::unique_lock<std::mutex> lk(h->mu);
  if (ticket >= h->next_ticket) return fail(h, VSS_E_INVALID_ARG, "unknown ticket");
  const int k = ticket_slot(h, ticket);
  if (k < 0) return VSS_OK;
  Slot& s = h->slots[k];
  // a batch with host work (copy / callback): the completion thread finishes it
  if (g_tls_completing == h && s.ticket == ticket && s.host_busy)
    return fail(h, VSS_E_BUSY, "vss_wait from a completion callback on a batch that completes after it");
  h->slot_cv.wait(lk, [&] { return s.ticket != ticket || !s.host_busy; });
  if (s.ticket != ticket) return VSS_OK;
  // otherwise its D2H into the caller's pinned block is the completion; the
  // slot's done events (recorded after it) too, so the slot is free on return
  std::vector<std::pair<int, hipEvent_t>> evs{{h->device, s.host_done}};
  for (vss_handle* e : engines(h)) evs.push_back({e->device, e->slots[k].done});
  if (int rc = wait_events_unlocked(h, lk, evs)) return rc;
  if (s.ticket != ticket) return VSS_OK;
  return s.status > 0 ? VSS_OK : s.status;
}

int vss_query(vss_handle* h, vss_ticket ticket) {
  if (!h) return fail(nullptr, VSS_E_INVALID_ARG, "null handle");
  std::lock_guard<std::mutex> lk(h->mu);
  if (ticket >= h->next_ticket) return fail(h, VSS_E_INVALID_ARG, "unknown ticket");
  const int k = ticket_slot(h, ticket);
  if (k < 0) return 1;
  Slot& s = h->slots[k];
  if (s.host_busy) return 0;
  HIP_TRY(h, hipSetDevice(h->device));
  const hipError_t q = hipEventQuery(s.host_done);
  if (q == hipErrorNotReady) return 0;
  if (q != hipSuccess) return fail(h, VSS_E_HIP, std::string("hipEventQuery: ") + hipGetErrorString(q));
  return s.status < 0 ? s.status : 1;
}

int vss_staging_acquire(vss_handle* h, int* slot, uint8_t** frames, size_t* capacity) {
  if (!h || !slot || !frames) return fail(h, VSS_E_INVALID_ARG, "null handle/slot/frames");
  std::unique_lock<std::mutex> lk(h->mu);
  if (!h->peers.empty())
    return fail(h, VSS_E_UNSUPPORTED, "zero-copy staging is per GPU: a multi-GPU handle stages its shards itself");
  int k = 0;
  int rc = pick_slot(h, lk, true, &k);  // a free slot (waits for one, mu released meanwhile)
  if (rc) return rc;
  HIP_TRY(h, hipSetDevice(h->device));
  if ((rc = ensure_staging(h, h->slots[k]))) return rc;
  h->slots[k].leased = true;
  *slot = k;
  *frames = h->slots[k].h_frames;
  if (capacity) *capacity = h->frame_cap;
  return VSS_OK;
}

int vss_staging_release(vss_handle* h, int slot) {
  if (!h) return fail(nullptr, VSS_E_INVALID_ARG, "null handle");
  std::lock_guard<std::mutex> lk(h->mu);
  if (slot < 0 || slot >= (int)h->slots.size() || !h->slots[slot].leased)
    return fail(h, VSS_E_INVALID_ARG, "not a leased slot");
  h->slots[slot].leased = false;
  return VSS_OK;
}

int vss_submit_staged(vss_handle* h, int slot, int n, int height, int width, int channels, size_t row_stride,
                      float* masks_out, int out_mode, vss_callback cb, void* user, vss_ticket* ticket) {
  if (!h) return fail(nullptr, VSS_E_INVALID_ARG, "null handle");
  if (slot < 0 || slot >= (int)h->slots.size()) return fail(h, VSS_E_INVALID_ARG, "bad slot");
  return submit_host(h, h->slots[slot].h_frames, nullptr, n, height, width, channels, row_stride, masks_out, out_mode,
                     false, false, cb, user, ticket, slot);
}

int vss_host_alloc(size_t bytes, void** ptr) {
  if (!ptr || bytes == 0) return VSS_E_INVALID_ARG;
  *ptr = nullptr;
  void* q = nullptr;
  if (hipHostMalloc(&q, bytes, hipHostMallocPortable) != hipSuccess || !q) return VSS_E_OOM;
  std::lock_guard<std::mutex> lk(g_pin_mu);
  g_pinned[reinterpret_cast<uintptr_t>(q)] = bytes;
  *ptr = q;
  return VSS_OK;
}

int vss_host_free(void* ptr) {
  if (!ptr) return VSS_OK;
  {
    std::lock_guard<std::mutex> lk(g_pin_mu);
    if (g_pinned.erase(reinterpret_cast<uintptr_t>(ptr)) == 0) return VSS_E_INVALID_ARG;
  }
  return hipHostFree(ptr) == hipSuccess ? VSS_OK : VSS_E_HIP;
}

int vss_segment_device(vss_handle* h, const uint8_t* d_frames, int n, int height, int width, int channels,
                       size_t row_stride, size_t frame_stride, float* d_masks, void* stream) {
  if (!h) return fail(nullptr, VSS_E_INVALID_ARG, "null handle");
  if (!d_frames || !d_masks) return fail(h, VSS_E_INVALID_ARG, "null device pointer");
  g_device_clock.begin();
  int rc = check_frames(h, n, height, width, channels, row_stride, frame_stride, h->cfg.max_batch);
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(h->mu);
  HIP_TRY(h, hipSetDevice(h->device));
  g_device_clock.mark(1);
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : h->stream;
  // round-robin slots, ordered on the device (no host wait): consecutive
  // calls on different streams run concurrently.  Device calls take no
  // ticket: a host batch in the same slot keeps its ticket and completion.
  const int k = (int)(h->device_calls++ % h->slots.size());
  Slot& sl = h->slots[k];
  if ((rc = claim_slot(h, sl, s))) return rc;
  g_device_clock.mark(2);
  rc = forward(h, k, d_frames, n, height, width, channels, row_stride, frame_stride, d_masks, s);
  const int rr = release_slot(h, sl, s);  // also after a failed enqueue: the next user orders after it
  g_device_clock.mark(7);
  return rc ? rc : rr;
}

int vss_comm_status(vss_handle* h, int* async_errors, int cap, int* nslots, unsigned long long* gather_calls) {
  if (!h) return fail(nullptr, VSS_E_INVALID_ARG, "null handle");
  // no handle lock: a watchdog calls this while another thread may be blocked
  // inside a call that holds it.  The communicators are read only once the
  // clique is published (vss_comm_init_rank's release store; they do not
  // change after it); before that every slot reports -1
  const int ns = (int)h->slots.size();
  if (nslots) *nslots = ns;
  if (gather_calls) *gather_calls = h->gather_calls.load(std::memory_order_relaxed);
  const bool ready = h->clique.load(std::memory_order_acquire) || h->rccl;
  for (int k = 0; k < ns && k < cap && async_errors; ++k) {
    ncclResult_t ae = ncclSuccess;
    const ncclComm_t c = ready ? h->slots[k].comm : nullptr;
    async_errors[k] = !c ? -1 : (ncclCommGetAsyncError(c, &ae) == ncclSuccess ? (int)ae : -2);
  }
  return VSS_OK;
}

int vss_comm_unique_id(vss_handle* h, void* ids, size_t cap, size_t* len) {
  if (!h || !ids) return fail(h, VSS_E_INVALID_ARG, "null handle/ids");
  const size_t need = h->slots.size() * sizeof(ncclUniqueId);
  if (len) *len = need;
  if (cap < need) return fail(h, VSS_E_INVALID_ARG, "ids buffer needs " + std::to_string(need) + " bytes");
  for (size_t k = 0; k < h->slots.size(); ++k)
    NCCL_TRY(h, ncclGetUniqueId(reinterpret_cast<ncclUniqueId*>(static_cast<char*>(ids) + k * sizeof(ncclUniqueId))));
  return VSS_OK;
}

int vss_comm_init_rank(vss_handle* h, int nranks, int rank, const void* ids, size_t len) {
  if (!h || !ids) return fail(h, VSS_E_INVALID_ARG, "null handle/ids");
  if (!h->peers.empty() || h->rccl)
    return fail(h, VSS_E_UNSUPPORTED, "a handle over several GPUs has its own communicators");
  if (h->clique) return fail(h, VSS_E_INVALID_ARG, "the handle already joined a clique");
  if (nranks < 1 || rank < 0 || rank >= nranks) return fail(h, VSS_E_INVALID_ARG, "bad nranks/rank");
  if (len != h->slots.size() * sizeof(ncclUniqueId))
    return fail(h, VSS_E_INVALID_ARG, "ids must be the " + std::to_string(h->slots.size() * sizeof(ncclUniqueId)) +
                                          " bytes of vss_comm_unique_id (same queue_depth on every rank)");
  std::lock_guard<std::mutex> lk(h->mu);
  HIP_TRY(h, hipSetDevice(h->device));
  HIP_TRY(h, hipDeviceSynchronize());
  // the ordered form uses slot 0's communicator alone: only it is created
  const size_t ncomm = h->gather_form == VSS_GATHER_ORDERED ? 1 : h->slots.size();
  for (size_t k = 0; k < ncomm; ++k) {
    ncclUniqueId id;
    std::memcpy(&id, static_cast<const char*>(ids) + k * sizeof(ncclUniqueId), sizeof(id));
    NCCL_TRY(h, ncclCommInitRank(&h->slots[k].comm, nranks, id, rank));
  }
  h->gather_ev.assign(2 * h->slots.size(), nullptr);
  for (hipEvent_t& e : h->gather_ev) HIP_TRY(h, hipEventCreateWithFlags(&e, hipEventDisableTiming));
  h->nranks = nranks;
  h->rank = rank;
  h->clique.store(true, std::memory_order_release);
  return VSS_OK;
}

int vss_segment_gather_device(vss_handle* h, const uint8_t* d_frames, int n, int height, int width, int channels,
                              size_t row_stride, size_t frame_stride, float* d_gathered, void* stream) {
  if (!h) return fail(nullptr, VSS_E_INVALID_ARG, "null handle");
  if (!h->clique) return fail(h, VSS_E_INVALID_ARG, "vss_comm_init_rank first");
  if (!d_frames || !d_gathered) return fail(h, VSS_E_INVALID_ARG, "null device pointer");
  int rc = check_frames(h, n, height, width, channels, row_stride, frame_stride, h->cfg.max_batch);
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(h->mu);
  HIP_TRY(h, hipSetDevice(h->device));
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : h->stream;
  // round-robin over the gather calls alone (a counter of their own), so every
  // rank uses the same slot's communicator for its i-th gather whatever other
  // device calls it interleaves
  const bool serial = h->gather_form == VSS_GATHER_ORDERED;
  const unsigned long long call = h->gather_calls.load(std::memory_order_relaxed);
  const int k = (int)(call % h->slots.size());
  if ((rc = comm_healthy(h, h->slots[serial ? 0 : k].comm, serial ? 0 : k))) return rc;
  h->gather_calls.fetch_add(1, std::memory_order_relaxed);
  Slot& sl = h->slots[k];
  if ((rc = claim_slot(h, sl, s))) return rc;
  if ((rc = forward(h, k, d_frames, n, height, width, channels, row_stride, frame_stride, sl.d_masks, s))) {
    (void)release_slot(h, sl, s);
    return rc;
  }
  const size_t P = (size_t)h->cfg.model_h * h->cfg.model_w;
  // VSS_GATHER_ORDERED (default): every gather on slot 0's
  // communicator, one at a time in call order — one total order of
  // collectives per rank, the same on every rank, whatever the runtime's
  // stream -> hardware queue mapping.  Each gather runs on the caller's
  // stream right behind its forward and first waits for the previous call's
  // gather (an event chain), so no two collectives of a rank are ever in
  // flight together; the forwards of the batches in flight still overlap
  // the gathers.  (Round 6 ran them on a gather stream of their own, two
  // cross-stream hops per call: each collective then held that stream ~57 us
  // at one rank, 141-145k frames/s against 198-205k, profiles/r06/r06ak.)
  // VSS_GATHER_CONCURRENT (opt-in until an 8-GPU record exists): each slot's
  // own communicator on the slot's stream, so the gathers of the batches in
  // flight overlap too; every rank uses slot k for its i-th call, so each
  // communicator sees its collectives in the same order on every rank.
  ncclResult_t nr = ncclSuccess;
  hipError_t he = hipSuccess;
  if (!serial) {
    nr = ncclAllGather(sl.d_masks, d_gathered, (size_t)n * P, ncclFloat32, sl.comm, s);
  } else {
    const size_t ne = h->gather_ev.size();
    if (call > 0) he = hipStreamWaitEvent(s, h->gather_ev[(call - 1) % ne], 0);  // the previous gather, done
    if (he == hipSuccess) nr = ncclAllGather(sl.d_masks, d_gathered, (size_t)n * P, ncclFloat32, h->slots[0].comm, s);
    if (he == hipSuccess && nr == ncclSuccess) he = hipEventRecord(h->gather_ev[call % ne], s);
  }
  const int rr = release_slot(h, sl, s);
  if (nr != ncclSuccess) return fail(h, VSS_E_RCCL, std::string("ncclAllGather: ") + ncclGetErrorString(nr));
  if (he != hipSuccess) return fail(h, VSS_E_HIP, std::string("gather ordering: ") + hipGetErrorString(he));
  return rr;
}

int vss_mask_to_frame_device(vss_handle* h, const float* d_masks, int n, int frame_h, int frame_w, float* d_out,
                             void* stream) {
  if (!h) return fail(nullptr, VSS_E_INVALID_ARG, "null handle");
  if (!d_masks || !d_out) return fail(h, VSS_E_INVALID_ARG, "null device pointer");
  if (n < 1 || n > h->user_max_batch || frame_h < 1 || frame_w < 1)
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
  int rc = check_frames(h, n, height, width, channels, row_stride, frame_stride, h->user_max_batch);
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
  for (vss_handle* e : engines(h)) {
    HIP_TRY(e, hipSetDevice(e->device));
    HIP_TRY(e, hipStreamSynchronize(e->stream));
    for (Slot& s : e->slots) {
      HIP_TRY(e, hipStreamSynchronize(s.stream));
      if (s.used) HIP_TRY(e, hipEventSynchronize(s.done));
    }
  }
  HIP_TRY(h, hipSetDevice(h->device));
  // and every host batch's completion (copy, callback) has run
  std::unique_lock<std::mutex> lk(h->mu);
  auto idle = [&] {
    for (const Slot& s : h->slots)
      if (s.host_busy) return false;
    return true;
  };
  if (g_tls_completing == h && !idle())
    return fail(h, VSS_E_BUSY, "vss_synchronize from a completion callback while later batches complete");
  h->slot_cv.wait(lk, idle);
  return VSS_OK;
}

int vss_set_option(vss_handle* h, int option, int value) {
  if (!h) return fail(nullptr, VSS_E_INVALID_ARG, "null handle");
  if (option == 3 || option == 4 || option == 5)
    return fail(h, VSS_E_UNSUPPORTED, "option removed (round-1 experiment measured slower; profiles/NOTES.md)");
  if (option == VSS_OPT_GRAPH_BUILDS || option == VSS_OPT_GRAPH_PATCHES || option == VSS_OPT_COMM_RANKS ||
      option == VSS_OPT_GATHER_CALLS)
    return fail(h, VSS_E_INVALID_ARG, "read-only option (vss_get_option)");
  if (option != VSS_OPT_KEEP_STEM && option != VSS_OPT_USE_GRAPH && option != VSS_OPT_PROFILE &&
      option != VSS_OPT_ROW_FETCH && option != VSS_OPT_GATHER_FORM)
    return fail(h, VSS_E_INVALID_ARG, "unknown option");
  std::lock_guard<std::mutex> lk(h->mu);
  if (option == VSS_OPT_GATHER_FORM) {
    if (value != VSS_GATHER_ORDERED && value != VSS_GATHER_CONCURRENT)
      return fail(h, VSS_E_INVALID_ARG, "gather form: VSS_GATHER_ORDERED or VSS_GATHER_CONCURRENT");
    if (h->clique && value != h->gather_form)
      return fail(h, VSS_E_INVALID_ARG, "the gather form is fixed at vss_comm_init_rank");
    h->gather_form = value;
    return VSS_OK;
  }
  for (vss_handle* e : engines(h)) {
    if (option == VSS_OPT_KEEP_STEM) {
      if ((value ? 1 : 0) != e->keep_stem) drop_graphs(e);  // the graphs hold the stem pointer
      e->keep_stem = value ? 1 : 0;
    } else if (option == VSS_OPT_USE_GRAPH) {
      e->use_graph = value ? 1 : 0;
    } else if (option == VSS_OPT_ROW_FETCH) {
      e->row_fetch = value ? 1 : 0;
    } else {
      e->profile = value ? 1 : 0;
    }
  }
  return VSS_OK;
}

int vss_get_option(vss_handle* h, int option, int* value) {
  if (!h) return fail(nullptr, VSS_E_INVALID_ARG, "null handle");
  if (!value) return fail(h, VSS_E_INVALID_ARG, "null value");
  std::lock_guard<std::mutex> lk(h->mu);
  switch (option) {
    case VSS_OPT_USE_GRAPH: *value = h->use_graph; return VSS_OK;
    case VSS_OPT_PROFILE: *value = h->profile; return VSS_OK;
    case VSS_OPT_KEEP_STEM: *value = h->keep_stem; return VSS_OK;
    case VSS_OPT_ROW_FETCH: *value = h->row_fetch; return VSS_OK;
    case VSS_OPT_GRAPH_BUILDS:
    case VSS_OPT_GRAPH_PATCHES: {
      long v = 0;
      for (const vss_handle* e : engines(h)) v += option == VSS_OPT_GRAPH_BUILDS ? e->graph_builds : e->graph_patches;
      *value = (int)std::min<long>(v, 0x7fffffff);
      return VSS_OK;
    }
    case VSS_OPT_GATHER_CALLS:
      *value = (int)(h->gather_calls.load() & 0x7FFFFFFF);
      return VSS_OK;
    case VSS_OPT_GATHER_FORM: *value = h->gather_form; return VSS_OK;
    case VSS_OPT_COMM_RANKS: {
      if (h->rccl) {
        *value = 1 + (int)h->peers.size();
      } else if (h->clique) {
        int c = 0;
        NCCL_TRY(h, ncclCommCount(h->slots[0].comm, &c));
        *value = c;
      } else {
        *value = 1;
      }
      return VSS_OK;
    }
    default: return fail(h, VSS_E_INVALID_ARG, "unknown option");
  }
}

int vss_prepare_device(vss_handle* h, int n, int height, int width, int channels, size_t row_stride,
                       size_t frame_stride) {
  if (!h) return fail(nullptr, VSS_E_INVALID_ARG, "null handle");
  int rc = check_frames(h, n, height, width, channels, row_stride, frame_stride, h->cfg.max_batch);
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(h->mu);
  HIP_TRY(h, hipSetDevice(h->device));
  if (!h->use_graph || h->profile) return VSS_OK;  // eager launches: nothing to build
  const GraphKey key{n, height, width, channels, row_stride, frame_stride};
  for (size_t k = 0; k < h->slots.size(); ++k) {
    Slot& s = h->slots[k];
    if (s.graphs.count(key)) {
      s.shape_tick[key] = ++s.graph_tick;
      continue;
    }
    make_room_for_shape(s);
    std::vector<Launch> ls;
    // null buffers: the first call patches in its own (the slot is idle then)
    forward_launches(h, s, nullptr, n, height, width, channels, row_stride, frame_stride, nullptr, &ls);
    GraphEntry g;
    if ((rc = build_graph(h, ls, &g))) return rc;
    // the executable's device-side state now, not at its first launch
    if (const hipError_t e = hipGraphUpload(g.exec, s.stream); e != hipSuccess) {
      destroy_graph(g);
      return fail(h, VSS_E_HIP, std::string("hipGraphUpload: ") + hipGetErrorString(e));
    }
    HIP_TRY(h, hipStreamSynchronize(s.stream));
    s.graphs[key].push_back(std::move(g));
    s.shape_tick[key] = ++s.graph_tick;
  }
  return VSS_OK;
}

int vss_slot_stream(vss_handle* h, int k, void** stream) {
  if (!h || !stream) return fail(h, VSS_E_INVALID_ARG, "null handle/stream");
  if (k < 0 || k >= (int)h->slots.size()) return fail(h, VSS_E_INVALID_ARG, "slot out of range");
  *stream = h->slots[k].stream;
  return VSS_OK;
}

int vss_shard_plan(int n, int nranks, int rank, int* first, int* count, int* per_rank) {
  if (n < 0 || nranks < 1 || rank < 0 || rank >= nranks || !first || !count || !per_rank) return VSS_E_INVALID_ARG;
  shard_plan(n, nranks, rank, first, count, per_rank);
  return VSS_OK;
}

int vss_gather_runs(int n, int nranks, int* src_row, int* dst_row, int* rows) {
  if (n < 0 || nranks < 1 || !src_row || !dst_row || !rows) return VSS_E_INVALID_ARG;
  return gather_runs(n, nranks, src_row, dst_row, rows);
}

int vss_layer_shape(const vss_handle* h, int layer, int* c, int* hh, int* ww) {
  if (!h || layer < 0 || layer >= (int)h->L.size()) return VSS_E_INVALID_ARG;
  if (c) *c = h->L[layer].C;
  if (hh) *hh = h->L[layer].H;
  if (ww) *ww = h->L[layer].W;
  return VSS_OK;
}

int vss_layer_occupancy(const vss_handle* h, int layer, int* wg_per_cu, int* lds_bytes) {
  if (!h || layer < 0 || layer >= (int)h->L.size() || !wg_per_cu) return VSS_E_INVALID_ARG;
  const LayerPlan& l = h->L[layer];
  *wg_per_cu = 0;
  if (lds_bytes) *lds_bytes = (int)l.lds;
  if (!l.entry) return VSS_OK;
  const int pi = h->cfg.dtype == VSS_DTYPE_F32 ? 0 : 1;
  HIP_TRY(const_cast<vss_handle*>(h), hipSetDevice(h->device));
  HIP_TRY(const_cast<vss_handle*>(h),
          hipOccupancyMaxActiveBlocksPerMultiprocessor(wg_per_cu, (const void*)l.entry->fn[pi], l.entry->threads,
                                                       l.lds));
  // the API assumes a finer LDS granule than gfx950 allocates (kLdsGranule)
  *wg_per_cu = std::min(*wg_per_cu, lds_wg_per_cu((int)l.lds));
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

// The demangled kernel name of layer l run as compiled shape e (rocprofv3's spelling).
static void entry_name(const vss_handle* h, const LayerPlan& l, int layer, const BlockEntry* e, char* tmp, size_t cap_) {
  const int prec = h->cfg.dtype == VSS_DTYPE_F32 ? PREC_F32 : PREC_BF16X2;
  if (l.fused) std::snprintf(tmp, cap_, "(fused into layer %d)", layer + 1);
  else if (l.rec.kind == K_STEM) std::snprintf(tmp, cap_, "void vss::k_stem<16>(vss::StemParams)");
  else if (l.rec.kind == K_HEAD) std::snprintf(tmp, cap_, "void vss::k_head<16>(vss::HeadParams)");
  else {
    if (e->variant == VAR_STEM_B1_WIDE)
      std::snprintf(tmp, cap_, "void vss::k_stem_b1<%d, %d, %d>(vss::BlockParams)", e->TH, e->TW, prec);
    else
      std::snprintf(tmp, cap_, "void vss::k_block<%d, %d, %d, %d, %d, %d, %d, %d, %d, %d>(vss::BlockParams)",
                    e->mode, e->stride, e->TH, e->TW, e->cin, e->cskip, e->chid, e->cout, e->flags, prec);
  }
}

int vss_layer_kernel(const vss_handle* h, int layer, char* buf, int cap) {
  if (!h || layer < 0 || layer >= (int)h->L.size() || !buf || cap < 1) return VSS_E_INVALID_ARG;
  const LayerPlan& l = h->L[layer];
  char tmp[160];
  entry_name(h, l, layer, l.entry, tmp, sizeof(tmp));
  const int len = (int)std::strlen(tmp);
  std::snprintf(buf, (size_t)cap, "%s", tmp);
  return len;
}

int vss_layer_tile_kernel(const vss_handle* h, int layer, int idx, char* buf, int cap) {
  if (!h || layer < 0 || layer >= (int)h->L.size() || !buf || cap < 1) return VSS_E_INVALID_ARG;
  const LayerPlan& l = h->L[layer];
  if (l.mode < 0) return VSS_E_INVALID_ARG;
  const std::vector<const BlockEntry*> c = tile_candidates(l);
  if (idx < 0 || idx >= (int)c.size()) return VSS_E_INVALID_ARG;
  char tmp[160];
  entry_name(h, l, layer, c[idx], tmp, sizeof(tmp));
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
  if (h->last_slot < 0) return fail(h, VSS_E_INVALID_ARG, "no forward has run on this handle");
  const Slot& s = h->slots[h->last_slot];
  if (l.rec.kind == K_STEM && !s.stem_stored)
    return fail(h, VSS_E_INVALID_ARG,
                "the stem is fused into layer 1 and the latest forward did not store it: set VSS_OPT_KEEP_STEM "
                "before the forward");
  HIP_TRY(h, hipSetDevice(h->device));
  HIP_TRY(h, hipDeviceSynchronize());
  const size_t cnt = (size_t)n * l.H * l.W * l.C;
  HIP_TRY(h, hipMemcpy(host_out, s.act[layer], cnt * 4, hipMemcpyDeviceToHost));
  if (l.ks > 1) {  // a split layer's value = its parts summed in part order, as its consumers do
    std::vector<float> part(cnt);
    for (int q = 1; q < l.ks; ++q) {
      HIP_TRY(h, hipMemcpy(part.data(), s.act[layer] + q * l.part_stride, cnt * 4, hipMemcpyDeviceToHost));
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
  for (int s = 0; s < vss_handle::kProfRing; ++s)
    if (h->ring_pending[s]) {
      int rc = harvest_ring(h, s);
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
  if (st->h) set_err(st->h, msg);
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

// The seam for the synchronous post / composite host calls on engine 0:
// stage the frames into a free slot, H2D and forward on the handle's stream
// (after that slot's previous work); returns the slot, claimed and marked
// host_busy — the caller enqueues its own work and ends with finish_seam.
// mu held through lk (released only while waiting for a slot).
int seam_on_stream(vss_handle* h, std::unique_lock<std::mutex>& lk, const uint8_t* frames, int n, int fh, int fw,
                   int fc, size_t rs, int* slot) {
  if (!frames) return fail(h, VSS_E_INVALID_ARG, "null frames");
  int rc = check_frames(h, n, fh, fw, fc, rs, rs * (size_t)fh, h->cfg.max_batch);
  if (rc) return rc;
  const size_t fbytes = (size_t)fh * rs;
  if ((size_t)n * fbytes > h->frame_cap)
    return fail(h, VSS_E_INVALID_ARG, "frames exceed the handle's staging capacity (max_frame_h/w)");
  HIP_TRY(h, hipSetDevice(h->device));
  int k = 0;
  if ((rc = pick_slot(h, lk, true, &k))) return rc;  // free: its staging is rewritten below
  Slot& s = h->slots[k];
  if ((rc = ensure_staging(h, s))) return rc;
  if (frames != s.h_frames) h->pool->run({{s.h_frames, frames, (size_t)n * fbytes}});
  if ((rc = claim_slot(h, s, h->stream))) return rc;
  const hipError_t e = hipMemcpyAsync(s.d_frames, s.h_frames, (size_t)n * fbytes, hipMemcpyHostToDevice, h->stream);
  if (e != hipSuccess) rc = fail(h, VSS_E_HIP, std::string("H2D: ") + hipGetErrorString(e));
  if (!rc) rc = forward(h, k, s.d_frames, n, fh, fw, fc, rs, fbytes, s.d_masks, h->stream);
  if (rc) {
    (void)release_slot(h, s, h->stream);
    return rc;
  }
  s.host_busy = true;
  *slot = k;
  return VSS_OK;
}

// End of a synchronous post / composite call on slot k (rc: its enqueue
// status): record the slot's done event, wait for the handle's stream with mu
// released, give the slot back.
int finish_seam(vss_handle* h, std::unique_lock<std::mutex>& lk, int k, int rc) {
  Slot& s = h->slots[k];
  const int rr = release_slot(h, s, h->stream);
  if (!rc) rc = rr;
  if (!rc) {
    lk.unlock();
    const hipError_t e = hipStreamSynchronize(h->stream);
    lk.lock();
    if (e != hipSuccess) rc = fail(h, VSS_E_HIP, std::string("hipStreamSynchronize: ") + hipGetErrorString(e));
  }
  s.host_busy = false;
  lk.unlock();
  h->slot_cv.notify_all();
  return rc;
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
  const size_t nb = (size_t)std::max(h->cfg.max_batch, h->user_max_batch);
  auto bail = [&](int rc) {
    vss_post_destroy(st);
    return rc;
  };
  HIP_TRY(h, hipSetDevice(h->device));
  if (hipMalloc(&st->state, P * 4) != hipSuccess || hipMalloc(&st->valid, 16) != hipSuccess ||
      hipMalloc(&st->ema, P * 4 * nb) != hipSuccess || hipMalloc(&st->state2, P * 4) != hipSuccess ||
      hipMalloc(&st->d_faces, sizeof(FaceFrame) * nb) != hipSuccess ||
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
    (void)hipDeviceSynchronize();
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
  HIP_TRY(st->h, hipDeviceSynchronize());
  HIP_TRY(st->h, hipMemset(st->valid, 0, sizeof(int)));
  st->faces_n = 0;
  st->faces = nullptr;
  return VSS_OK;
}

static_assert(sizeof(FaceFrame) == sizeof(vss_face_frame), "FaceFrame mirrors vss_face_frame");

int vss_post_set_faces(vss_post_state* st, const vss_face_frame* faces, int n) {
  if (!st) return VSS_E_INVALID_ARG;
  if (!faces || n < 1 || n > std::max(st->h->cfg.max_batch, st->h->user_max_batch))
    return post_fail(st, VSS_E_INVALID_ARG, "faces: 1..max_batch frames");
  HIP_TRY(st->h, hipSetDevice(st->h->device));
  HIP_TRY(st->h, hipMemcpyAsync(st->d_faces, faces, sizeof(FaceFrame) * n, hipMemcpyHostToDevice, st->h->stream));
  HIP_TRY(st->h, hipStreamSynchronize(st->h->stream));  // consumers may run on any stream
  st->faces = st->d_faces;
  st->faces_n = n;
  return VSS_OK;
}

int vss_post_set_faces_device(vss_post_state* st, const vss_face_frame* d_faces, int n) {
  if (!st) return VSS_E_INVALID_ARG;
  if (!d_faces || n < 1 || n > std::max(st->h->cfg.max_batch, st->h->user_max_batch))
    return post_fail(st, VSS_E_INVALID_ARG, "faces: a device array of 1..max_batch frames");
  st->faces = reinterpret_cast<const FaceFrame*>(d_faces);
  st->faces_n = n;
  return VSS_OK;
}

int vss_post_set_config(vss_post_state* st, const vss_post_config* cfg) {
  if (!st || !cfg) return VSS_E_INVALID_ARG;
  if (cfg->sigma_spatial <= 0 || cfg->sigma_range <= 0) return post_fail(st, VSS_E_INVALID_ARG, "sigmas must be > 0");
  HIP_TRY(st->h, hipSetDevice(st->h->device));
  HIP_TRY(st->h, hipDeviceSynchronize());
  st->cfg = *cfg;
  return post_tables(st);
}

int vss_postprocess_device(vss_post_state* st, const uint8_t* d_frames, int n, int height, int width, int channels,
                           size_t row_stride, size_t frame_stride, const float* d_masks, float* d_alpha,
                           uint8_t* d_alpha_u8, void* stream) {
  if (!st) return fail(nullptr, VSS_E_INVALID_ARG, "null post state");
  vss_handle* h = st->h;
  if (!d_masks || (!d_frames && st->cfg.use_bilateral)) return fail(h, VSS_E_INVALID_ARG, "null device pointer");
  int rc = check_frames(h, n, height, width, channels, row_stride, frame_stride,
                        std::max(h->cfg.max_batch, h->user_max_batch));
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
  std::lock_guard<std::mutex> pl(h->post_mu);
  std::unique_lock<std::mutex> lk(h->mu);
  int k = 0;
  int rc = seam_on_stream(h, lk, frames, n, height, width, channels, row_stride, &k);
  if (rc) return rc;
  Slot& s = h->slots[k];
  const size_t P = (size_t)h->cfg.model_h * h->cfg.model_w;
  float* d_alpha = alpha_out ? h->d_post_alpha : nullptr;
  uint8_t* d_u8 = alpha_u8_out ? h->d_post_u8 : nullptr;
  rc = post_enqueue(st, s.d_frames, n, height, width, channels, row_stride, row_stride * (size_t)height, s.d_masks,
                    d_alpha, d_u8, h->stream);
  hipError_t e = hipSuccess;
  if (!rc && alpha_out) e = hipMemcpyAsync(alpha_out, d_alpha, (size_t)n * P * 4, hipMemcpyDeviceToHost, h->stream);
  if (!rc && e == hipSuccess && alpha_u8_out)
    e = hipMemcpyAsync(alpha_u8_out, d_u8, (size_t)n * P, hipMemcpyDeviceToHost, h->stream);
  if (!rc && e != hipSuccess) rc = fail(h, VSS_E_HIP, std::string("D2H: ") + hipGetErrorString(e));
  return finish_seam(h, lk, k, rc);
}

}  // extern "C"

#ifdef VSS_TRACE
// Trace build only: the stamps of `layer`'s last launch, [wgs][16] u64
// (s_memrealtime ticks, 100 MHz).  Returns the workgroup count.
// vss_trace_read_slot: the same for slot `slot`'s latest forward (several
// batches in flight: tools/trace_inflight.py).  Stamp 7 holds the workgroup's
// HW_ID register (cu, shader array, shader engine), stamp 15 its XCC_ID.
extern "C" int vss_trace_read_slot(vss_handle* h, int slot, int layer, unsigned long long* out, int cap) {
  if (!h || layer < 0 || layer >= (int)h->L.size() || !out || slot < 0 || slot >= (int)h->slots.size())
    return VSS_E_INVALID_ARG;
  HIP_TRY(h, hipDeviceSynchronize());
  const int wgs = std::min(h->trace_wgs[layer], cap);
  HIP_TRY(h, hipMemcpy(out, h->slots[slot].trace[layer], (size_t)wgs * 16 * 8, hipMemcpyDeviceToHost));
  return wgs;
}

extern "C" int vss_trace_read(vss_handle* h, int layer, unsigned long long* out, int cap) {
  if (!h || h->last_slot < 0) return VSS_E_INVALID_ARG;
  return vss_trace_read_slot(h, h->last_slot, layer, out, cap);
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
  int rc = check_frames(h, n, height, width, channels, row_stride, frame_stride,
                        std::max(h->cfg.max_batch, h->user_max_batch));
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
  std::lock_guard<std::mutex> pl(h->post_mu);
  std::unique_lock<std::mutex> lk(h->mu);
  HIP_TRY(h, hipSetDevice(h->device));
  const size_t cap = (size_t)h->cfg.max_batch * h->cfg.max_frame_h * h->cfg.max_frame_w * 4;
  if (!h->d_comp) {
    int rc = dalloc(h, &h->d_comp, cap);
    if (rc) return rc;
  }
  const size_t fs = row_stride * (size_t)height, ors = (size_t)width * 4, ofs = ors * height;
  if ((size_t)n * ofs > cap)
    return fail(h, VSS_E_INVALID_ARG, "RGBA output exceeds the handle's capacity (max_batch, max_frame_h/w)");
  int k = 0;
  int rc = seam_on_stream(h, lk, frames, n, height, width, channels, row_stride, &k);
  if (rc) return rc;
  Slot& s = h->slots[k];
  rc = post_enqueue(st, s.d_frames, n, height, width, channels, row_stride, fs, s.d_masks, nullptr, h->d_post_u8,
                    h->stream);
  if (!rc)
    rc = composite_enqueue(h, s.d_frames, n, height, width, channels, row_stride, fs, h->d_post_u8, h->d_comp, ors,
                           ofs, h->stream);
  if (!rc) {
    const hipError_t e = hipMemcpyAsync(out_rgba, h->d_comp, (size_t)n * ofs, hipMemcpyDeviceToHost, h->stream);
    if (e != hipSuccess) rc = fail(h, VSS_E_HIP, std::string("D2H: ") + hipGetErrorString(e));
  }
  return finish_seam(h, lk, k, rc);
}

}  // extern "C"

// Introspection for the registry generator's LDS mirror (tests/test_registry.py):
// the bytes of LDS block_lds() carves for one k_block shape.
extern "C" int vss_block_lds_bytes(int mode, int stride, int th, int tw, int cin, int cskip, int chid, int cout,
                                   int stem_in) {
  return block_lds(mode, stride, th, tw, cin, cskip, chid, cout, stem_in).total * 4;
}
