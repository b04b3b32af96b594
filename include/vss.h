/*
 * vss.h — C ABI of the MI355X-native per-frame person-segmentation path.
 *
 * Drop-in boundary for steps 1-2 of processFrame
 * (/root/reference/client/src/core/frameProcessorTest.ts:78-97): frame pixels
 * in, the seam triple (alphaRaw: Float32Array(maskH*maskW), maskW, maskH) out.
 * Plain pointers and sizes only.  Each entry point names the reference
 * interface it replaces; the Node-API and ctypes bindings that sit on top of
 * it are in INTEGRATION.md.
 *
 * Errors: every int-returning call returns VSS_OK (0) or a negative VSS_E_*
 * code; the message is in vss_last_error(handle) (thread-local when handle is
 * NULL, e.g. after a failed vss_create).  This mirrors ORT-web's
 * _OrtGetLastError(code*, msg**) (client/public/ort-wasm-simd-threaded.mjs:50)
 * behind the rejecting `session.run` promise.
 *
 * Threading / queueing: the reference serialises every session.run behind one
 * promise chain (runModnetExclusive, client/src/core/main.ts:18-22), so one
 * batch is ever in flight.  A handle here owns `queue_depth` slots — each its
 * own activations, HIP stream, captured hipGraphs and pinned staging — and up
 * to that many batches run at once: batch i+1's host->device copy overlaps
 * batch i's forward and batch i-1's device->host copy (the steady-state
 * decode -> infer loop of BASELINE config 5).  Callbacks fire, and tickets
 * complete, in submission order; a queued call beyond the depth gets
 * VSS_E_BUSY (vss_segment_async) or waits (the synchronous calls).  Calls may
 * come from several host threads (submission is serialised inside).
 *
 * Multi-GPU: a handle created with n_gpus / device_ids owns
 * one engine per GPU; the host-memory calls shard a batch contiguously over
 * them and all-gather the masks over RCCL (ncclAllGather inside one
 * ncclGroupStart/End, one communicator per device and slot).  Processes that
 * each own one GPU (torchrun) join one RCCL clique instead through
 * vss_comm_unique_id / vss_comm_init_rank and vss_segment_gather_device.
 */
#ifndef VSS_H_
#define VSS_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VSS_VERSION 30000 /* 3.0.0: graphs patched per call, completion thread, shard plan */

enum {
  VSS_OK = 0,
  VSS_E_INVALID_ARG = -1,
  VSS_E_HIP = -2,
  VSS_E_RCCL = -3,
  VSS_E_BUSY = -4,
  VSS_E_OOM = -5,
  VSS_E_IO = -6,
  VSS_E_UNSUPPORTED = -7
};

/* Pointwise-GEMM arithmetic (activations are f32 in HBM in every mode). */
enum {
  VSS_DTYPE_F32 = 0,    /* v_mfma_f32_16x16x4_f32, exact f32 fma chains            */
  VSS_DTYPE_BF16X2 = 1  /* v_mfma_f32_16x16x32_bf16 on a hi+lo bf16 split (default) */
};

/* Mask resolution: model (the reference's seam, frameProcessorTest.ts:96-97). */
/* out_mode of vss_segment / vss_segment_async: masks at model resolution
 * (the seam triple, n * mask_h * mask_w floats), or upsampled on the GPU to
 * the frames' resolution (n * height * width floats; half-pixel bilinear —
 * the canvas drawImage upscale of :177 defined as in vss_composite_device). */
enum { VSS_OUT_MODEL = 0, VSS_OUT_FRAME = 1 };

/* Options for vss_set_option.  (Values 3-5 belonged to round-1 experiments —
 * sub-batch graph branches and the persistent k_forward — measured slower and
 * removed; profiles/NOTES.md keeps the numbers.  Setting them fails with
 * VSS_E_UNSUPPORTED.) */
enum {
  VSS_OPT_USE_GRAPH = 1, /* 1: replay a hipGraph per (slot, shape) (default 1): up to 4 executables
                            per (slot, shape), each bound to one (frames, masks) buffer pair; a
                            call with a fifth pair patches the least recently used executable's
                            first and last kernel nodes (hipGraphExecKernelNodeSetParams) */
  VSS_OPT_PROFILE = 2,   /* 1: time every kernel with HIP events (eager launches)         */
  VSS_OPT_KEEP_STEM = 6, /* 1: the stem fused into layer 1 also stores its activation, so
                            vss_read_layer(0) can report it (a debugging aid: 4.7 MB of HBM
                            writes per batch of 8 at 144x256 that no layer reads).  Default 0:
                            the forward writes only what a later layer or the caller reads;
                            vss_read_layer(0) fails with VSS_E_INVALID_ARG unless the latest
                            forward ran with the option set. */
  VSS_OPT_ROW_FETCH = 7, /* 1 (default): the queued host calls move only the frame rows the
                            tfjs-legacy resize reads (frameProcessorTest.ts:80) across PCIe —
                            staged host-side and fetched by a kernel from pinned memory — when
                            that skips 60 % of the rows or more (four fifths at 720p and 1080p
                            for 144 model rows; at 640x480 half, where one DMA of the whole
                            frames is faster); 0: whole frames by DMA.  Masks are identical
                            either way. */
  /* Read-only counters (vss_get_option; vss_set_option fails): */
  VSS_OPT_GRAPH_BUILDS = 8,  /* executable graphs built (per slot and shape, one per buffer pair,
                                at most 4)                                                   */
  VSS_OPT_GRAPH_PATCHES = 9, /* graph replays that patched their buffers' kernel parameters */
  VSS_OPT_COMM_RANKS = 10,   /* ranks of the handle's RCCL clique (ncclCommCount; the GPUs of a
                                multi-GPU handle; 1 without a clique)                        */
  VSS_OPT_GATHER_CALLS = 11, /* vss_segment_gather_device calls so far: call i runs on slot i %
                                queue_depth, counted apart from the other device calls, so ranks
                                that interleave different vss_segment_device calls still agree on
                                every collective (read-only) */
  VSS_OPT_GATHER_FORM = 12   /* how vss_segment_gather_device issues its all-gathers (VSS_GATHER_*);
                                settable until vss_comm_init_rank, fixed after it.  Default
                                VSS_GATHER_ORDERED (environment VSS_GATHER_SERIAL=0 at vss_create:
                                VSS_GATHER_CONCURRENT) */
};

/* VSS_OPT_GATHER_FORM values. */
enum {
  VSS_GATHER_ORDERED = 0,    /* one communicator (slot 0's, the only one created); each gather on
                                the caller's stream behind its forward, after the previous call's
                                gather has completed (an event chain): every rank runs one
                                collective at a time in its call order, which no stream ->
                                hardware-queue mapping can reorder; the forwards of the batches in
                                flight still overlap the gathers */
  VSS_GATHER_CONCURRENT = 1  /* one communicator per slot, each gather on its slot's stream: the
                                gathers of the batches in flight overlap each other too */
};

typedef struct vss_handle vss_handle;

typedef struct vss_config {
  int model_h, model_w;    /* model input resolution; multiples of 16. Reference: 288x512
                              (MODEL_INPUT_SIZE, frameProcessorTest.ts:10); default 144x256 */
  int dtype;               /* VSS_DTYPE_* */
  int device_id;           /* HIP device ordinal when device_ids is NULL (one GPU) */
  int max_batch;           /* frames per call (over all the handle's GPUs) */
  int max_frame_h, max_frame_w; /* host-staging capacity for vss_segment (channels <= 4) */
  const char* weights_path;     /* vss weights blob (model/make_weights.py) */
  int flags;                    /* VSS_CREATE_* */
  /* one handle over n_gpus distinct GPUs device_ids[0..n_gpus-1]
   * (the masks' consumer is device_ids[0]).  With device_ids != NULL the host
   * calls always go through the RCCL path, n_gpus == 1 included. */
  int n_gpus;
  const int* device_ids;
  int queue_depth;              /* batches in flight (slots per GPU); 0 = default 4, max 16 */
  int staging_threads;          /* host threads for the pinned staging copies; 0 = default 8 */
} vss_config;

/* vss_config.flags */
enum {
  VSS_CREATE_NO_AUTOTUNE = 1 /* keep the planner's tile per layer instead of timing every compiled
                                tile at max_batch during vss_create (results are identical either way) */
};

typedef struct vss_info {
  int mask_h, mask_w;      /* (maskH, maskW) of the seam */
  int n_layers;
  int dtype;
  size_t device_bytes;     /* HBM held by the handle (all its GPUs) */
  int n_gpus;              /* GPUs of the handle */
  int queue_depth;         /* slots (batches in flight) */
  int rccl;                /* 1: the host calls all-gather the masks over RCCL */
} vss_info;

/* status callback for vss_segment_async: called on the handle's completion
 * thread once the masks are in masks_out (status = VSS_OK) or the batch
 * failed; in submission order.  No lock is held: the callback may call vss_*
 * functions of its handle (a new submit, vss_query), except vss_destroy.
 * Only this thread completes host batches, so a call from a callback that
 * would have to wait for a later batch's completion (vss_wait on it,
 * vss_synchronize, a blocking vss_segment / vss_staging_acquire when every
 * slot is still completing) returns VSS_E_BUSY instead of deadlocking. */
typedef void (*vss_callback)(void* user, int status);

/* Submission ticket of a queued batch (vss_submit, vss_wait). */
typedef uint64_t vss_ticket;

/* Library version (VSS_VERSION). */
int vss_version(void);

/* Replaces initializeModnet (client/src/core/model.ts:12-29) /
 * _OrtCreateSession (ort-wasm-simd-threaded.mjs:51). */
int vss_create(const vss_config* cfg, vss_handle** out);

/* Replaces InferenceSession.release. */
void vss_destroy(vss_handle* h);

/* Replaces _OrtGetLastError (ort-wasm-simd-threaded.mjs:50).  Thread-safe: the
 * handle's last message is copied into a buffer of the calling thread, valid
 * until that thread's next vss_last_error call (NULL handle: the calling
 * thread's last failure without a handle, e.g. vss_create's). */
const char* vss_last_error(const vss_handle* h);

int vss_get_info(const vss_handle* h, vss_info* info);

/* The model-res masks of vss_segment_device upsampled to frame_h x frame_w
 * (what VSS_OUT_FRAME returns): d_out [n][frame_h][frame_w] f32, enqueued on
 * `stream`.  Replaces the canvas scaling of the mask, frameProcessorTest.ts:177. */
int vss_mask_to_frame_device(vss_handle* h, const float* d_masks, int n, int frame_h, int frame_w, float* d_out,
                             void* stream);

/* Synchronous host-memory call.  Replaces frameProcessorTest.ts:79-97
 * (fromPixels .. session.run .. squeezeMaskTo2D) for n frames at once:
 * frames: n frames of h rows, row_stride bytes per row, frames packed
 *         back to back (frame stride = h*row_stride), channels 3 (RGB) or 4
 *         (RGBA; alpha dropped as tf.browser.fromPixels does, :79);
 * masks_out: n * mask_h * mask_w floats (VSS_OUT_MODEL) or n * height * width
 *            (VSS_OUT_FRAME), row-major per frame, in [0,1]. */
int vss_segment(vss_handle* h, const uint8_t* frames, int n, int height, int width, int channels,
                size_t row_stride, float* masks_out, int out_mode);

/* Same as vss_segment but queued: returns once the frames are staged (the
 * caller may reuse `frames` then); cb fires when masks_out is filled, in
 * submission order.  VSS_E_BUSY when queue_depth batches are already in
 * flight.  The caller keeps masks_out alive until the callback (replaces the
 * async `await session.run`, frameProcessorTest.ts:91). */
int vss_segment_async(vss_handle* h, const uint8_t* frames, int n, int height, int width,
                      int channels, size_t row_stride, float* masks_out, int out_mode,
                      vss_callback cb, void* user);

/* The queued call without a callback: *ticket identifies the batch for
 * vss_wait / vss_query.  VSS_E_BUSY when the queue is full. */
int vss_submit(vss_handle* h, const uint8_t* frames, int n, int height, int width, int channels,
               size_t row_stride, float* masks_out, int out_mode, vss_ticket* ticket);

/* vss_submit for frames that are not one contiguous buffer: frames[i] points
 * at frame i (each height rows of row_stride bytes); each is copied straight
 * into the pinned staging (no packing copy on the caller's side). */
int vss_submit_list(vss_handle* h, const uint8_t* const* frames, int n, int height, int width, int channels,
                    size_t row_stride, float* masks_out, int out_mode, vss_ticket* ticket);

/* vss_submit_list with a completion callback instead of a wait, for a host
 * that must not block a thread per batch (the N-API addon's one submit thread
 * per handle: its calls are queued in call order, and cb resolves the batch's
 * promise): waits for a free slot instead of returning VSS_E_BUSY (from a
 * completion callback, where that wait could not end: VSS_E_BUSY).  cb fires
 * on the handle's completion thread once masks_out is filled or the batch
 * failed, in submission order; *ticket (may be NULL) as vss_submit's. */
int vss_submit_list_async(vss_handle* h, const uint8_t* const* frames, int n, int height, int width, int channels,
                          size_t row_stride, float* masks_out, int out_mode, vss_callback cb, void* user,
                          vss_ticket* ticket);

/* Block until batch `ticket` is done (its masks_out filled); returns that
 * batch's status.  vss_query: 1 done, 0 still running, < 0 an error. */
int vss_wait(vss_handle* h, vss_ticket ticket);
int vss_query(vss_handle* h, vss_ticket ticket);

/* Zero-copy staging (the decode -> infer loop of BASELINE config 5): reserve
 * a free slot (waits for one) and get its pinned host buffer (capacity
 * bytes); decode the frames straight into it (frame i at i * height *
 * row_stride) and queue them with vss_submit_staged — no staging copy.  The
 * lease holds the slot until then (vss_staging_release gives it back
 * unused); other calls skip leased slots.  cb may be NULL (then vss_wait on
 * *ticket). */
int vss_staging_acquire(vss_handle* h, int* slot, uint8_t** frames, size_t* capacity);
int vss_staging_release(vss_handle* h, int slot);
int vss_submit_staged(vss_handle* h, int slot, int n, int height, int width, int channels, size_t row_stride,
                      float* masks_out, int out_mode, vss_callback cb, void* user, vss_ticket* ticket);

/* Pinned host memory for results (process-wide, any handle / GPU): a
 * masks_out of vss_segment / vss_submit* / vss_segment_async that lies inside
 * a vss_host_alloc block receives the batch's D2H directly — the completion
 * copies nothing (otherwise the masks land in the slot's pinned buffer and the
 * completion thread copies them to masks_out).  The JS side of the reference
 * gets a fresh Float32Array per frame (squeezeMaskTo2D,
 * frameProcessorTest.ts:190-201); the N-API addon hands out these blocks as
 * its result ArrayBuffers.  vss_host_free: VSS_E_INVALID_ARG for a pointer
 * vss_host_alloc did not return; freeing a block a batch still writes into is
 * the caller's error, as for any masks_out. */
int vss_host_alloc(size_t bytes, void** ptr);
int vss_host_free(void* ptr);

/* Device-resident variant: d_frames and d_masks are HBM pointers of the
 * handle's first GPU; the work is enqueued on `stream` (a hipStream_t; NULL =
 * the handle's stream) and not waited for.  frame_stride = bytes between
 * frames.  Consecutive calls take consecutive slots, so calls on different
 * streams run concurrently (each stream sees its own calls in order).  Any
 * caller stream may be used and destroyed at any time: a call waits on the
 * device for its slot's previous work (an event wait), unless both are on that
 * slot's own stream (vss_slot_stream), where stream order suffices. */
int vss_segment_device(vss_handle* h, const uint8_t* d_frames, int n, int height, int width,
                       int channels, size_t row_stride, size_t frame_stride, float* d_masks,
                       void* stream);

/* Build the executable graphs of every slot for this batch shape now (no
 * launch), so the first calls of a steady loop replay instead of building
 * (the graph is otherwise built by the slot's first call of that shape).
 * The device pointers are bound by the first call.  Only the handle's first
 * GPU is prepared: device calls (vss_segment_device, _gather_device) run
 * there; a multi-GPU handle's peers run host batches, whose per-GPU shard
 * shapes build their graphs on first use.  A slot keeps graphs for at most 16
 * shapes (past that, the graphs of the shape least recently prepared or run
 * are dropped), and up to 4 executables per shape,
 * each bound to one (frames, masks) buffer pair. */
int vss_prepare_device(vss_handle* h, int n, int height, int width, int channels, size_t row_stride,
                       size_t frame_stride);

/* Slot k's HIP stream (a hipStream_t; k < queue_depth).  Device calls whose
 * `stream` is the stream of the slot they take (device calls take slots
 * round-robin: call i -> slot i % queue_depth) order after that slot's
 * previous work for free, and the handle's slot streams sit on distinct
 * hardware queues, so batches in flight on them run concurrently. */
int vss_slot_stream(vss_handle* h, int k, void** stream);

/* The batch sharding of SURVEY.md §8(e), host-only (no GPU needed): a batch
 * of n frames over nranks GPUs in contiguous shards of *per_rank =
 * ceil(n / nranks) frames; rank `rank` takes frames [*first, *first + *count)
 * (the last ranks may get fewer, or none).  Every rank all-gathers *per_rank
 * rows, so the gathered [nranks][per_rank] rows hold frame i at row i (only
 * the last non-empty shard can be short; its padding rows follow frame n-1).
 * The multi-GPU handle and vss_segment_gather_device callers use this plan. */
int vss_shard_plan(int n, int nranks, int rank, int* first, int* count, int* per_rank);

/* The multi-GPU handle's copy-out, host-only (no GPU needed): after the
 * all-gather of a batch of n frames over nranks GPUs (vss_shard_plan), the
 * gathered buffer holds nranks blocks of per_rank rows, rank r's block being
 * its shard's frames then padding.  Writes the runs that move every frame's
 * row to frame order in the caller's buffer — run j copies rows[j] rows from
 * gathered row src_row[j] to output row dst_row[j]; runs never read a padding
 * row — and returns their number (at most nranks; each array needs nranks
 * entries), or VSS_E_INVALID_ARG.  submit_host's D2H (VSS_OUT_MODEL) and the
 * frame-size upsample (VSS_OUT_FRAME) both follow these runs. */
int vss_gather_runs(int n, int nranks, int* src_row, int* dst_row, int* rows);

/* ---- one GPU per process (torchrun): an RCCL clique over the processes ------
 * Rank 0 calls vss_comm_unique_id (ids for every slot; *len bytes, at most
 * cap), hands the bytes to every rank, and each rank calls vss_comm_init_rank
 * on its own handle.  Then vss_segment_gather_device runs the rank's n frames
 * and all-gathers every rank's masks into d_gathered [nranks * n][mask_h *
 * mask_w] in rank order, on `stream`; every rank must make the same sequence
 * of calls with the same n. */
int vss_comm_unique_id(vss_handle* h, void* ids, size_t cap, size_t* len);
int vss_comm_init_rank(vss_handle* h, int nranks, int rank, const void* ids, size_t len);
int vss_segment_gather_device(vss_handle* h, const uint8_t* d_frames, int n, int height, int width,
                              int channels, size_t row_stride, size_t frame_stride, float* d_gathered,
                              void* stream);

/* Health of the handle's communicators, for a watchdog (takes no handle lock:
 * safe while another thread is blocked in a call).  async_errors[k] = slot k's
 * ncclCommGetAsyncError result (0 = ncclSuccess, 7 = ncclInProgress, any other
 * = an RCCL error code; -1 = the slot has no communicator, -2 = the query
 * failed) for k < min(cap, *nslots); *gather_calls = vss_segment_gather_device
 * calls so far (call i runs on slot i % *nslots).  Every gather also checks
 * its communicator first and fails with VSS_E_RCCL on an asynchronous error.
 * No reference counterpart (the reference runs on one device). */
int vss_comm_status(vss_handle* h, int* async_errors, int cap, int* nslots, unsigned long long* gather_calls);

/* Preprocessing alone (frameProcessorTest.ts:79-85): d_out = [n][3][mask_h][mask_w]
 * f32, the exact ORT input tensor. Enqueued on `stream`. */
int vss_preprocess_device(vss_handle* h, const uint8_t* d_frames, int n, int height, int width,
                          int channels, size_t row_stride, size_t frame_stride, float* d_out,
                          void* stream);

/* Wait for all work enqueued by this handle. */
int vss_synchronize(vss_handle* h);

int vss_set_option(vss_handle* h, int option, int value);
int vss_get_option(vss_handle* h, int option, int* value);

/* Per-layer output shape (C, H, W) at the handle's model resolution. */
int vss_layer_shape(const vss_handle* h, int layer, int* c, int* hh, int* ww);

/* Copy layer `layer`'s output of the most recent forward to host as NHWC f32
 * [n][H][W][C] (debug / per-layer parity; synchronises the handle). */
int vss_read_layer(vss_handle* h, int layer, int n, float* host_out);

/* The kernel that runs layer `layer` as rocprofv3 names it, e.g.
 * "void vss::k_block<2, 1, 8, 8, 32, 16, 48, 16, 1, 1>(vss::BlockParams)"
 * (template arguments: mode, stride, tile h, tile w, cin, cskip, chid, cout,
 * flags, precision).  Returns the string length, or a negative code. */
int vss_layer_kernel(const vss_handle* h, int layer, char* buf, int cap);

/* The output tiles compiled for `layer`'s shape (csrc/vss_registry.inc), as
 * (tile h, tile w) pairs in th[k], tw[k]; returns how many (0 for the stem
 * and the head), at most `cap` written.  Any of them can be pinned with the
 * environment variable VSS_TILE="layer:THxTW[,...]" at vss_create, or by
 * index, VSS_TILE="layer:#k" (a tile can be compiled as more than one kernel:
 * b1's k_block and the wide k_stem_b1); results do not depend on the tile
 * (bitwise). */
int vss_layer_tiles(const vss_handle* h, int layer, int* th, int* tw, int cap);

/* The kernel name (as vss_layer_kernel) of candidate `idx` of vss_layer_tiles'
 * list for `layer`.  Returns the string length, or a negative code. */
int vss_layer_tile_kernel(const vss_handle* h, int layer, int idx, char* buf, int cap);

/* Workgroups of `layer`'s kernel that fit one CU at once (registers, from
 * hipOccupancyMaxActiveBlocksPerMultiprocessor, and the layer's dynamic LDS in
 * gfx950's 2 KiB allocation granules) and its LDS bytes per workgroup; 0 for
 * the fused stem and the head. */
int vss_layer_occupancy(const vss_handle* h, int layer, int* wg_per_cu, int* lds_bytes);

/* Kernel times from VSS_OPT_PROFILE runs: per layer, the mean over `count`
 * forwards (ms).  Resets the accumulators. */
int vss_profile_read(vss_handle* h, double* ms_per_layer, int cap, int* count);

/* Bytes of LDS one k_block workgroup of this shape carves (block_lds in
 * csrc/vss_kernels.h); no GPU needed.  tools/gen_registry.py mirrors it. */
int vss_block_lds_bytes(int mode, int stride, int th, int tw, int cin, int cskip, int chid, int cout, int stem_in);

/* ---- §8(f) row 1: the reference's mask post-processing, on the GPU ----------
 * processFrame's steps after the seam (frameProcessorTest.ts:115-169):
 * temporalEMA (:218) -> morphologicalOpening (:644) -> jointBilateral3x3 with the
 * guide image (:230, :315) -> refineAlphaOnce (:270) -> alphaToImageData (:204),
 * computed in doubles with f32 stores as the reference's JS does.  The guide
 * (a browser-canvas resample in the reference) is the frame's tfjs-legacy
 * bilinear resample at mask resolution, rounded half up to u8. */
typedef struct vss_post_config {
  double ema;            /* config.EMA                      (0.55, frameProcessorTest.ts:12) */
  double noise_cutoff;   /* config.NOISE_CUTOFF             (0.06, :13) */
  double high_threshold; /* config.HIGH_THRESHOLD           (0.95, :14) */
  double gamma;          /* config.GAMMA                    (0.4,  :15) */
  double sigma_spatial;  /* config.BILATERAL_SIGMA_SPATIAL  (1.0,  :17) */
  double sigma_range;    /* config.BILATERAL_SIGMA_RANGE    (12.0, :18) */
  int use_bilateral;     /* config.USE_BILATERAL            (1,    :16) */
} vss_post_config;

/* The reference's defaultConfig (frameProcessorTest.ts:20-28). */
void vss_post_config_default(vss_post_config* cfg);

/* Post-processing state of ONE video stream: prevAlpha (frameProcessorTest.ts:47),
 * reset = the stream's next frame is its first.  One call in flight per state. */
typedef struct vss_post_state vss_post_state;
int vss_post_create(vss_handle* h, const vss_post_config* cfg, vss_post_state** out);
void vss_post_destroy(vss_post_state* st);
int vss_post_reset(vss_post_state* st);
/* Live knob changes, like the settings sliders (client/script.ts:16-25). */
int vss_post_set_config(vss_post_state* st, const vss_post_config* cfg);

/* n CONSECUTIVE frames of the state's stream (HBM pointers, enqueued on `stream`):
 * d_masks = the seam's masks [n][mask_h][mask_w] (e.g. from vss_segment_device),
 * d_frames = the same frames (for the guide); outputs (either may be NULL):
 * d_alpha [n][mask_h][mask_w] f32 = refinedAlpha (:166), d_alpha_u8 = the
 * ImageData alpha bytes (:169, :213). */
int vss_postprocess_device(vss_post_state* st, const uint8_t* d_frames, int n, int height, int width,
                           int channels, size_t row_stride, size_t frame_stride, const float* d_masks,
                           float* d_alpha, uint8_t* d_alpha_u8, void* stream);

/* §8(f) row 4: the face stabiliser's inputs to the post chain, per frame
 * (processFrame's opts.lastAffine and its face detection,
 * frameProcessorTest.ts:99-114, :131-166):
 *   has_affine: warp prevAlpha by the affine (warpAffineNearest :335 with
 *               invertAffine :323) and blend it 0.3 / 0.7 into the mask
 *               before the EMA (:102-113);
 *   has_box:    the elliptical face prior of the detection box (facePriorMask
 *               :697-741) -> a 3x3 closing inside it after the opening
 *               (morphologicalClosingInPrior :743-787) and the prior's clamp
 *               in refineAlphaOnce (:297-307).
 * Doubles, as the reference's JS numbers; video_w/h = the video size the box
 * is in (0 = the frames' size). */
typedef struct vss_face_frame {
  int has_affine;
  double affine[6];   /* a11, a12, tx, a21, a22, ty (estimateAffineFromLandmarks's form, :455-563) */
  int has_box;
  double box[4];      /* x0, y0, x1, y1 in video pixels (runFaceDetector's box, :396-452) */
  int video_w, video_h;
} vss_face_frame;

/* The face inputs of the NEXT vss_postprocess_device / vss_segment_post call on
 * this state, one per frame of that call (n must match it); consumed by it.
 * d_faces: the same from device memory (e.g. written by the GPU face stage). */
int vss_post_set_faces(vss_post_state* st, const vss_face_frame* faces, int n);
int vss_post_set_faces_device(vss_post_state* st, const vss_face_frame* d_faces, int n);

/* Host-memory convenience: seam + post chain for n consecutive frames of the
 * state's stream (replaces frameProcessorTest.ts:78-169 up to putImageData). */
int vss_segment_post(vss_handle* h, vss_post_state* st, const uint8_t* frames, int n, int height, int width,
                     int channels, size_t row_stride, float* alpha_out, uint8_t* alpha_u8_out);

/* ---- §8(f) row 3: compositing (frameProcessorTest.ts:170-178) ----------------
 * The output canvas (= the video's size, client/src/core/main.ts:43-44) after
 * drawImage(video) and 'destination-in' drawImage(maskCanvas): RGBA u8
 * (ImageData layout, not premultiplied), colour = the frame's, alpha = the
 * mask's alpha bytes upscaled to the frame (half-pixel bilinear in f32, rounded
 * half up — a definition: browser canvas filtering is not reproducible), colour
 * 0 where alpha is 0.  d_alpha_u8 = [n][mask_h][mask_w] (vss_postprocess_device).
 * out_row_stride: multiple of 4 bytes, >= 4 * width. */
int vss_composite_device(vss_handle* h, const uint8_t* d_frames, int n, int height, int width, int channels,
                         size_t row_stride, size_t frame_stride, const uint8_t* d_alpha_u8, uint8_t* d_out_rgba,
                         size_t out_row_stride, size_t out_frame_stride, void* stream);

/* Host-memory convenience: seam + post chain + compositing for n consecutive
 * frames of the state's stream -> out_rgba [n][height][width][4]
 * (replaces processFrame frameProcessorTest.ts:78-178). */
int vss_segment_composite(vss_handle* h, vss_post_state* st, const uint8_t* frames, int n, int height, int width,
                          int channels, size_t row_stride, uint8_t* out_rgba);

#ifdef __cplusplus
}
#endif

#endif /* VSS_H_ */
