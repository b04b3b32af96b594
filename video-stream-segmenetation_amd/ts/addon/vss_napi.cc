// vss_napi.cc — thin Node-API addon over the C ABI (include/vss.h).
//
// Replaces, for the TypeScript host, ORT-web's JS<->WASM glue
// (/root/reference/client/public/ort-wasm-simd-threaded.mjs:50-53, the
// _OrtCreateSession/_OrtRun/_OrtGetLastError exports behind
// InferenceSession.run).  Exports:
//   version() -> number
//   create(opts) -> handle            (opts: modelH, modelW, dtype, deviceId, deviceIds, maxBatch,
//                                       maxFrameH, maxFrameW, weightsPath, autotune, queueDepth,
//                                       stagingThreads)
//   info(handle) -> {maskW, maskH, nLayers, deviceBytes, nGpus, queueDepth, rccl}
//   segment(handle, frames: Uint8Array | Uint8Array[], n, height, width, channels, rowStride, outMode?)
//       -> Promise<Float32Array>      (n * maskH * maskW masks, or n * height * width with
//                                      outMode 1 = VSS_OUT_FRAME; rejects with Error(vss_last_error)).
//       Queued: returns at once; the handle's submit thread submits the batches in call
//       order (vss_submit_list_async: the frames copied frame by frame into the pinned
//       staging, no packing) and the completion callback settles the promise through a
//       thread-safe function (no thread waits per batch).  segment.ts keeps at most
//       queueDepth batches in flight (beyond that the submit waits for a free slot).
//   stagingAcquire(handle) -> {slot, data: Uint8Array}   zero-copy input: a free slot's pinned
//       staging buffer (valid until the handle is destroyed; waits for a free slot)
//   segmentStaged(handle, slot, n, height, width, channels, rowStride, outMode?) -> Promise<Float32Array>
//       queue the frames decoded into that slot's buffer (no staging copy)
//   stagingRelease(handle, slot)      give a lease back unused
//   destroy(handle)
//   postCreate(handle, config?) -> post     (config keys as the reference's `config`:
//                                             EMA, NOISE_CUTOFF, HIGH_THRESHOLD, GAMMA,
//                                             USE_BILATERAL, BILATERAL_SIGMA_SPATIAL,
//                                             BILATERAL_SIGMA_RANGE; frameProcessorTest.ts:12-30)
//   postSetConfig(post, config), postReset(post), postDestroy(post)
//   postSetFaces(post, faces: {affine?: number[6], box?: number[4], videoW?, videoH?}[])
//       the face stabiliser's inputs of the next segmentPost / segmentComposite call, one per frame
//       (processFrame's opts.lastAffine and detection box, :99-166)
//   segmentPost(handle, post, frames, n, height, width, channels, rowStride)
//       -> Promise<{alpha: Float32Array, alphaU8: Uint8Array}>   (processFrame :78-169)
//   segmentComposite(handle, post, frames, n, height, width, channels, rowStride)
//       -> Promise<Uint8Array>   RGBA output canvases, n * height * width * 4 (:78-178)
//   ortCreate(modelBytes: Uint8Array, inputDims: number[] | null, deviceId, convPrecision) -> session
//       ONNX sessions (include/vso.h) behind InferenceSession.create (model.ts:14, :38, :61)
//   ortInfo(session) -> {inputNames, outputNames, inputShapes, outputShapes}
//   ortRun(session, inputs: Float32Array[]) -> Promise<Float32Array[]>   (session.run)
//   ortDestroy(session)              (throws while a face tracker uses the session)
//   faceCreate(detector, landmarks, config?, deviceId?) -> tracker
//       the GPU face stage (include/vsf.h) over two ONNX sessions; config keys
//       interval, warpGain, faceScoreThresh, landmarkScoreThresh, roiPad
//   faceTrack(tracker, frames, n, height, width, channels, rowStride, maskW, maskH)
//       -> Promise<{affine: number[6] | null, box: number[4] | null, videoW, videoH}[]>
//       (the postSetFaces form, one entry per frame)
//   faceReset(tracker), faceDestroy(tracker)
//   traceDump() -> Float64Array   VSS_NAPI_TRACE=1: per-batch phase stamps (see TracePoint)
//   poolStats() -> {hits, carves, slabs, fallbacks, pinnedBytes}   the result blocks' allocator
// Nothing blocks the event loop while a batch runs — as `await session.run` does not block.
#include <node_api.h>

#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <deque>
#include <string>
#include <thread>
#include <vector>

#include "../../../include/vsf.h"
#include "../../../include/vso.h"
#include "../../../include/vss.h"

namespace {

#define NAPI_OK(env, call)                                                   \
  do {                                                                       \
    if ((call) != napi_ok) {                                                 \
      napi_throw_error((env), nullptr, "node-api call failed: " #call);      \
      return nullptr;                                                        \
    }                                                                        \
  } while (0)

// Set by the environment's cleanup hook: finalizers that run during teardown
// make no more N-API calls (the env is going away).
std::atomic<bool> g_env_closing{false};

struct Post;
struct Submitter;

struct Handle {
  vss_handle* h = nullptr;
  int mask_h = 0, mask_w = 0;
  std::vector<Post*> posts;  // destroyed before the handle, whatever order the GC finalizes in
  // Queued batches whose libuv work still holds h (JS thread only): destroy()
  // or the GC finalizer while some are pending defers vss_destroy to the last
  // one's completion, so no worker ever waits on a destroyed handle.
  int pending = 0;
  bool closing = false;    // destroy() / finalizer ran: no new work; release when pending == 0
  bool finalized = false;  // the JS external is gone: the last completion deletes this
  Submitter* sub = nullptr;  // segment()'s submit thread + result delivery (created on first use)
};

void stop_submitter(Handle* hd);  // (pending == 0: joins the thread, releases the delivery)

struct Post {
  Handle* hd = nullptr;
  vss_post_state* st = nullptr;
};

void release_handle(Handle* hd) {
  hd->closing = true;
  if (hd->pending > 0) return;  // work_done() of the last queued batch finishes the release
  for (Post* p : hd->posts) {
    if (p->st) vss_post_destroy(p->st);
    p->st = nullptr;
    p->hd = nullptr;
  }
  hd->posts.clear();
  stop_submitter(hd);
  if (hd->h) vss_destroy(hd->h);
  hd->h = nullptr;
}

void finalize_handle(napi_env, void* data, void*) {
  Handle* hd = static_cast<Handle*>(data);
  release_handle(hd);
  if (hd->pending > 0) hd->finalized = true;
  else delete hd;
}

// A queued batch's async work finished (its Complete callback, JS thread).
void work_done(Handle* hd) {
  if (--hd->pending > 0 || !hd->closing) return;
  const bool del = hd->finalized;
  release_handle(hd);
  if (del) delete hd;
}

void release_post(Post* p) {
  if (p->st) vss_post_destroy(p->st);
  p->st = nullptr;
  if (p->hd) p->hd->posts.erase(std::remove(p->hd->posts.begin(), p->hd->posts.end(), p), p->hd->posts.end());
  p->hd = nullptr;
}

void finalize_post(napi_env, void* data, void*) {
  Post* p = static_cast<Post*>(data);
  release_post(p);
  delete p;
}

Handle* get_handle(napi_env env, napi_value v) {
  void* p = nullptr;
  if (napi_get_value_external(env, v, &p) != napi_ok || !p) {
    napi_throw_type_error(env, nullptr, "expected a vss handle");
    return nullptr;
  }
  Handle* hd = static_cast<Handle*>(p);
  if (!hd->h || hd->closing) {
    napi_throw_error(env, nullptr, "vss handle already destroyed");
    return nullptr;
  }
  return hd;
}

bool get_int_prop(napi_env env, napi_value obj, const char* key, int* out) {
  bool has = false;
  if (napi_has_named_property(env, obj, key, &has) != napi_ok || !has) return false;
  napi_value v;
  napi_get_named_property(env, obj, key, &v);
  napi_valuetype t;
  napi_typeof(env, v, &t);
  if (t == napi_boolean) {
    bool b = false;
    napi_get_value_bool(env, v, &b);
    *out = b ? 1 : 0;
    return true;
  }
  return napi_get_value_int32(env, v, out) == napi_ok;
}

bool get_str_prop(napi_env env, napi_value obj, const char* key, std::string* out) {
  bool has = false;
  if (napi_has_named_property(env, obj, key, &has) != napi_ok || !has) return false;
  napi_value v;
  napi_get_named_property(env, obj, key, &v);
  size_t len = 0;
  if (napi_get_value_string_utf8(env, v, nullptr, 0, &len) != napi_ok) return false;
  out->resize(len);
  napi_get_value_string_utf8(env, v, &(*out)[0], len + 1, &len);
  return true;
}

napi_value Version(napi_env env, napi_callback_info) {
  napi_value r;
  NAPI_OK(env, napi_create_int32(env, vss_version(), &r));
  return r;
}

napi_value Create(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_OK(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  vss_config cfg{};
  cfg.model_h = 144; cfg.model_w = 256; cfg.dtype = VSS_DTYPE_BF16X2; cfg.device_id = 0;
  cfg.max_batch = 8; cfg.max_frame_h = 1080; cfg.max_frame_w = 1920;
  std::string weights, dtype;
  std::vector<int> device_ids;
  int autotune = 1;
  if (argc >= 1) {
    get_int_prop(env, argv[0], "modelH", &cfg.model_h);
    get_int_prop(env, argv[0], "modelW", &cfg.model_w);
    get_int_prop(env, argv[0], "deviceId", &cfg.device_id);
    get_int_prop(env, argv[0], "maxBatch", &cfg.max_batch);
    get_int_prop(env, argv[0], "maxFrameH", &cfg.max_frame_h);
    get_int_prop(env, argv[0], "maxFrameW", &cfg.max_frame_w);
    get_int_prop(env, argv[0], "autotune", &autotune);
    get_int_prop(env, argv[0], "queueDepth", &cfg.queue_depth);
    get_int_prop(env, argv[0], "stagingThreads", &cfg.staging_threads);
    get_str_prop(env, argv[0], "weightsPath", &weights);
    bool has = false;
    if (napi_has_named_property(env, argv[0], "deviceIds", &has) == napi_ok && has) {
      napi_value arr;
      napi_get_named_property(env, argv[0], "deviceIds", &arr);
      bool is_arr = false;
      napi_is_array(env, arr, &is_arr);
      if (is_arr) {
        uint32_t len = 0;
        napi_get_array_length(env, arr, &len);
        for (uint32_t i = 0; i < len; ++i) {
          napi_value v;
          int d = -1;
          napi_get_element(env, arr, i, &v);
          if (napi_get_value_int32(env, v, &d) != napi_ok) {
            napi_throw_type_error(env, nullptr, "deviceIds must be an array of GPU ordinals");
            return nullptr;
          }
          device_ids.push_back(d);
        }
        cfg.n_gpus = (int)device_ids.size();
        cfg.device_ids = device_ids.data();
      }
    }
    if (get_str_prop(env, argv[0], "dtype", &dtype)) {
      if (dtype == "f32") cfg.dtype = VSS_DTYPE_F32;
      else if (dtype == "bf16x2") cfg.dtype = VSS_DTYPE_BF16X2;
      else {
        napi_throw_range_error(env, nullptr, "dtype must be 'f32' or 'bf16x2'");
        return nullptr;
      }
    }
  }
  cfg.weights_path = weights.c_str();
  cfg.flags = autotune ? 0 : VSS_CREATE_NO_AUTOTUNE;
  vss_handle* h = nullptr;
  const int rc = vss_create(&cfg, &h);
  if (rc != VSS_OK) {
    const std::string msg = "vss_create failed (" + std::to_string(rc) + "): " + vss_last_error(nullptr);
    napi_throw_error(env, std::to_string(rc).c_str(), msg.c_str());
    return nullptr;
  }
  Handle* hd = new Handle();
  hd->h = h;
  vss_info inf{};
  vss_get_info(h, &inf);
  hd->mask_h = inf.mask_h;
  hd->mask_w = inf.mask_w;
  napi_value ext;
  NAPI_OK(env, napi_create_external(env, hd, finalize_handle, nullptr, &ext));
  return ext;
}

napi_value Info(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_OK(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  Handle* hd = get_handle(env, argv[0]);
  if (!hd) return nullptr;
  vss_info inf{};
  vss_get_info(hd->h, &inf);
  napi_value o, v;
  NAPI_OK(env, napi_create_object(env, &o));
  napi_create_int32(env, inf.mask_w, &v);
  napi_set_named_property(env, o, "maskW", v);
  napi_create_int32(env, inf.mask_h, &v);
  napi_set_named_property(env, o, "maskH", v);
  napi_create_int32(env, inf.n_layers, &v);
  napi_set_named_property(env, o, "nLayers", v);
  napi_create_double(env, (double)inf.device_bytes, &v);
  napi_set_named_property(env, o, "deviceBytes", v);
  napi_create_int32(env, inf.n_gpus, &v);
  napi_set_named_property(env, o, "nGpus", v);
  napi_create_int32(env, inf.queue_depth, &v);
  napi_set_named_property(env, o, "queueDepth", v);
  napi_get_boolean(env, inf.rccl != 0, &v);
  napi_set_named_property(env, o, "rccl", v);
  return o;
}

napi_value Destroy(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_OK(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  void* p = nullptr;
  if (napi_get_value_external(env, argv[0], &p) == napi_ok && p) release_handle(static_cast<Handle*>(p));
  return nullptr;
}

bool get_double_prop(napi_env env, napi_value obj, const char* key, double* out) {
  bool has = false;
  if (napi_has_named_property(env, obj, key, &has) != napi_ok || !has) return false;
  napi_value v;
  napi_get_named_property(env, obj, key, &v);
  napi_valuetype t;
  napi_typeof(env, v, &t);
  if (t == napi_boolean) {
    bool b = false;
    napi_get_value_bool(env, v, &b);
    *out = b ? 1.0 : 0.0;
    return true;
  }
  return napi_get_value_double(env, v, out) == napi_ok;
}

// The reference's config object (frameProcessorTest.ts:12-18) -> vss_post_config.
void read_post_config(napi_env env, napi_value obj, vss_post_config* c) {
  double ub = c->use_bilateral;
  get_double_prop(env, obj, "EMA", &c->ema);
  get_double_prop(env, obj, "NOISE_CUTOFF", &c->noise_cutoff);
  get_double_prop(env, obj, "HIGH_THRESHOLD", &c->high_threshold);
  get_double_prop(env, obj, "GAMMA", &c->gamma);
  get_double_prop(env, obj, "BILATERAL_SIGMA_SPATIAL", &c->sigma_spatial);
  get_double_prop(env, obj, "BILATERAL_SIGMA_RANGE", &c->sigma_range);
  if (get_double_prop(env, obj, "USE_BILATERAL", &ub)) c->use_bilateral = ub != 0.0 ? 1 : 0;
}

void throw_vss(napi_env env, const char* what, int rc, const char* msg) {
  const std::string m = std::string(what) + " failed (" + std::to_string(rc) + "): " + (msg ? msg : "");
  napi_throw_error(env, std::to_string(rc).c_str(), m.c_str());
}

Post* get_post(napi_env env, napi_value v) {
  void* p = nullptr;
  if (napi_get_value_external(env, v, &p) != napi_ok || !p) {
    napi_throw_type_error(env, nullptr, "expected a vss post state");
    return nullptr;
  }
  Post* ps = static_cast<Post*>(p);
  if (!ps->st) {
    napi_throw_error(env, nullptr, "vss post state already destroyed");
    return nullptr;
  }
  return ps;
}

napi_value PostCreate(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  NAPI_OK(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  Handle* hd = argc >= 1 ? get_handle(env, argv[0]) : nullptr;
  if (!hd) return nullptr;
  vss_post_config cfg;
  vss_post_config_default(&cfg);
  if (argc >= 2) read_post_config(env, argv[1], &cfg);
  vss_post_state* st = nullptr;
  const int rc = vss_post_create(hd->h, &cfg, &st);
  if (rc != VSS_OK) {
    throw_vss(env, "vss_post_create", rc, vss_last_error(hd->h));
    return nullptr;
  }
  Post* p = new Post();
  p->hd = hd;
  p->st = st;
  hd->posts.push_back(p);
  napi_value ext;
  NAPI_OK(env, napi_create_external(env, p, finalize_post, nullptr, &ext));
  return ext;
}

napi_value PostSetConfig(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  NAPI_OK(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  Post* p = argc >= 2 ? get_post(env, argv[0]) : nullptr;
  if (!p) return nullptr;
  vss_post_config cfg;
  vss_post_config_default(&cfg);
  read_post_config(env, argv[1], &cfg);
  const int rc = vss_post_set_config(p->st, &cfg);
  if (rc != VSS_OK) throw_vss(env, "vss_post_set_config", rc, vss_last_error(p->hd->h));
  return nullptr;
}

napi_value PostReset(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_OK(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  Post* p = argc >= 1 ? get_post(env, argv[0]) : nullptr;
  if (!p) return nullptr;
  const int rc = vss_post_reset(p->st);
  if (rc != VSS_OK) throw_vss(env, "vss_post_reset", rc, vss_last_error(p->hd->h));
  return nullptr;
}

bool get_doubles(napi_env env, napi_value obj, const char* key, double* out, uint32_t n) {
  bool has = false;
  if (napi_has_named_property(env, obj, key, &has) != napi_ok || !has) return false;
  napi_value v;
  napi_get_named_property(env, obj, key, &v);
  bool is_arr = false;
  uint32_t len = 0;
  if (napi_is_array(env, v, &is_arr) != napi_ok || !is_arr || napi_get_array_length(env, v, &len) != napi_ok ||
      len != n)
    return false;
  for (uint32_t k = 0; k < n; ++k) {
    napi_value e;
    napi_get_element(env, v, k, &e);
    if (napi_get_value_double(env, e, out + k) != napi_ok) return false;
  }
  return true;
}

napi_value PostSetFaces(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  NAPI_OK(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  Post* p = argc >= 2 ? get_post(env, argv[0]) : nullptr;
  if (!p) return nullptr;
  bool is_arr = false;
  uint32_t n = 0;
  if (napi_is_array(env, argv[1], &is_arr) != napi_ok || !is_arr || napi_get_array_length(env, argv[1], &n) != napi_ok) {
    napi_throw_type_error(env, nullptr, "postSetFaces(post, faces[]): an array, one entry per frame");
    return nullptr;
  }
  std::vector<vss_face_frame> faces(n);
  for (uint32_t k = 0; k < n; ++k) {
    napi_value f;
    napi_get_element(env, argv[1], k, &f);
    vss_face_frame& o = faces[k];
    std::memset(&o, 0, sizeof(o));
    napi_valuetype t;
    napi_typeof(env, f, &t);
    if (t != napi_object) continue;  // null / undefined: no face inputs for this frame
    o.has_affine = get_doubles(env, f, "affine", o.affine, 6) ? 1 : 0;
    o.has_box = get_doubles(env, f, "box", o.box, 4) ? 1 : 0;
    get_int_prop(env, f, "videoW", &o.video_w);
    get_int_prop(env, f, "videoH", &o.video_h);
  }
  const int rc = vss_post_set_faces(p->st, faces.data(), (int)n);
  if (rc != VSS_OK) throw_vss(env, "vss_post_set_faces", rc, vss_last_error(p->hd->h));
  return nullptr;
}

napi_value PostDestroy(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_OK(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  void* p = nullptr;
  if (argc >= 1 && napi_get_value_external(env, argv[0], &p) == napi_ok && p) release_post(static_cast<Post*>(p));
  return nullptr;
}

// ---- queued segment ----------------------------------------------------------
// segment(): the JS thread validates the call, takes a result block and
// queues the batch on the handle's submit thread (Submitter), then returns
// its promise.  That one thread submits the batches in call order
// (vss_submit_list_async: the staging copy of the frames into the slot's
// pinned memory, on the handle's staging_threads pool, then H2D -> forward ->
// D2H enqueued), so ticket order is call order and no two threads submit on a
// handle at once (several libuv workers submitted concurrently).
// The batch's completion callback, on the library's completion thread, hands
// the batch to the JS thread through a thread-safe function that settles the
// promise — no libuv worker is blocked in vss_wait per batch in flight.
// VSS_NAPI_SYNC_STAGE=1 (the round-4 form): the submit (staging copy) runs
// inside the call and a libuv worker waits for the batch.
// VSS_NAPI_TRACE=1: per batch, CLOCK_MONOTONIC stamps (ns) of each phase for
// traceDump() (tools/ts_prof.js: the phase table of profiles/r06*/).
enum TracePoint : int {
  TP_CALL = 0,      // segment() entered (JS thread)
  TP_QUEUED,        // segment() returns: the batch is queued for the submit thread
  TP_SUBMIT,        // the submit thread starts vss_submit_list_async
  TP_SUBMITTED,     // it returned: frames staged, H2D / forward / D2H enqueued
  TP_DONE,          // completion callback (the library's completion thread)
  TP_JS,            // the JS thread runs the delivery
  TP_RESOLVED,      // the promise is resolved
  TP_COUNT
};
const bool g_trace = [] {
  const char* e = std::getenv("VSS_NAPI_TRACE");
  return e && e[0] == '1';
}();
std::mutex& g_trace_mu = *new std::mutex;
std::vector<double>& g_trace_rows = *new std::vector<double>;  // [batch][TP_COUNT + 1] (+ frames)

double now_ns() {
  return (double)std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct QueuedWork {
  napi_async_work work = nullptr;  // (the synchronous-stage form only)
  napi_deferred deferred = nullptr;
  napi_ref out_ref = nullptr;
  Handle* hd = nullptr;  // pending counted until the promise is settled
  vss_handle* h = nullptr;
  vss_ticket ticket = 0;
  size_t out_count = 0;
  int rc = 0;
  std::string err, what = "vss_wait";
  // the submit thread's inputs; the frames' arrays are referenced until the batch is done
  std::vector<const uint8_t*> list;
  int slot = -1;  // segmentStaged: the leased slot whose pinned staging holds the frames
  int n = 0, height = 0, width = 0, channels = 0, out_mode = VSS_OUT_MODEL;
  size_t rs = 0;
  float* out = nullptr;
  std::vector<napi_ref> frame_refs;
  double t[TP_COUNT] = {};
};

struct Submitter {
  std::thread th;
  std::mutex mu;
  std::condition_variable cv;
  std::deque<QueuedWork*> q;
  bool stop = false;
  napi_threadsafe_function tsfn = nullptr;
  int owed = 0;  // (JS thread) batches whose delivery is still due: the tsfn keeps the loop alive while > 0
};

napi_value make_error(napi_env env, const std::string& what, int rc, const std::string& err) {
  napi_value msg, code, e;
  const std::string m = what + " failed (" + std::to_string(rc) + "): " + err;
  napi_create_string_utf8(env, m.c_str(), m.size(), &msg);
  napi_create_string_utf8(env, std::to_string(rc).c_str(), NAPI_AUTO_LENGTH, &code);
  napi_create_error(env, code, msg, &e);
  return e;
}

// Settle a batch's promise and drop its references (JS thread).
void settle(napi_env env, QueuedWork* w) {
  if (w->rc == VSS_OK) {
    napi_value ab = nullptr, arr;
    napi_get_reference_value(env, w->out_ref, &ab);
    napi_create_typedarray(env, napi_float32_array, w->out_count, ab, 0, &arr);
    napi_resolve_deferred(env, w->deferred, arr);
  } else {
    napi_reject_deferred(env, w->deferred, make_error(env, w->what, w->rc, w->err));
  }
  napi_delete_reference(env, w->out_ref);
  for (napi_ref r : w->frame_refs) napi_delete_reference(env, r);
  if (g_trace) {
    w->t[TP_RESOLVED] = now_ns();
    std::lock_guard<std::mutex> lk(g_trace_mu);
    g_trace_rows.insert(g_trace_rows.end(), w->t, w->t + TP_COUNT);
    g_trace_rows.push_back((double)w->n);
  }
  Handle* hd = w->hd;
  delete w;
  work_done(hd);
}

// The submit thread's delivery of a batch to the JS thread.
void deliver_js(napi_env env, napi_value, void* context, void* data) {
  QueuedWork* w = static_cast<QueuedWork*>(data);
  if (!env) {  // the environment is being torn down: nothing to settle
    delete w;
    return;
  }
  if (g_trace) w->t[TP_JS] = now_ns();
  Submitter* sub = static_cast<Submitter*>(context);
  if (--sub->owed == 0) napi_unref_threadsafe_function(env, sub->tsfn);
  settle(env, w);
}

// vss_callback: the batch is done (library completion thread).
void batch_done(void* user, int status) {
  QueuedWork* w = static_cast<QueuedWork*>(user);
  if (g_trace) w->t[TP_DONE] = now_ns();
  w->rc = status;
  if (status != VSS_OK) w->err = vss_last_error(w->h);
  napi_call_threadsafe_function(w->hd->sub->tsfn, w, napi_tsfn_nonblocking);
}

void submit_loop(Submitter* sub) {
  for (;;) {
    QueuedWork* w = nullptr;
    {
      std::unique_lock<std::mutex> lk(sub->mu);
      sub->cv.wait(lk, [&] { return sub->stop || !sub->q.empty(); });
      if (sub->q.empty()) return;
      w = sub->q.front();
      sub->q.pop_front();
    }
    if (g_trace) w->t[TP_SUBMIT] = now_ns();
    const int rc = w->slot >= 0 ? vss_submit_staged(w->h, w->slot, w->n, w->height, w->width, w->channels, w->rs,
                                                    w->out, w->out_mode, batch_done, w, &w->ticket)
                                : vss_submit_list_async(w->h, w->list.data(), w->n, w->height, w->width, w->channels,
                                                        w->rs, w->out, w->out_mode, batch_done, w, &w->ticket);
    if (g_trace) w->t[TP_SUBMITTED] = now_ns();
    if (rc != VSS_OK) {  // never queued: no callback will come
      w->rc = rc;
      w->what = w->slot >= 0 ? "vss_submit_staged" : "vss_submit";
      w->err = vss_last_error(w->h);
      napi_call_threadsafe_function(sub->tsfn, w, napi_tsfn_blocking);
    }
  }
}

Submitter* submitter(napi_env env, Handle* hd) {
  if (hd->sub) return hd->sub;
  Submitter* sub = new Submitter();
  napi_value name;
  napi_create_string_utf8(env, "vss_segment", NAPI_AUTO_LENGTH, &name);
  if (napi_create_threadsafe_function(env, nullptr, nullptr, name, 0, 1, nullptr, nullptr, sub, deliver_js,
                                      &sub->tsfn) != napi_ok) {
    delete sub;
    return nullptr;
  }
  napi_unref_threadsafe_function(env, sub->tsfn);  // referenced only while deliveries are owed
  sub->th = std::thread(submit_loop, sub);
  hd->sub = sub;
  return sub;
}

// Queue a batch on the submit thread (JS thread).
void enqueue(napi_env env, Handle* hd, QueuedWork* w) {
  Submitter* sub = hd->sub;
  if (sub->owed++ == 0) napi_ref_threadsafe_function(env, sub->tsfn);
  w->hd = hd;
  ++hd->pending;
  if (g_trace) w->t[TP_QUEUED] = now_ns();
  {
    std::lock_guard<std::mutex> lk(sub->mu);
    sub->q.push_back(w);
  }
  sub->cv.notify_one();
}

void stop_submitter(Handle* hd) {
  Submitter* sub = hd->sub;
  if (!sub) return;
  {
    std::lock_guard<std::mutex> lk(sub->mu);
    sub->stop = true;
  }
  sub->cv.notify_one();
  if (sub->th.joinable()) sub->th.join();
  // (at environment teardown Node finalizes the thread-safe function itself)
  if (!g_env_closing.load()) napi_release_threadsafe_function(sub->tsfn, napi_tsfn_release);
  delete sub;
  hd->sub = nullptr;
}

// The synchronous-stage form: a libuv worker waits for the batch.
void QueuedExecute(napi_env, void* data) {  // libuv worker thread: no JS calls here
  QueuedWork* w = static_cast<QueuedWork*>(data);
  w->rc = vss_wait(w->h, w->ticket);
  if (w->rc != VSS_OK) w->err = vss_last_error(w->h);
  if (g_trace) w->t[TP_DONE] = now_ns();
}

void QueuedComplete(napi_env env, napi_status, void* data) {
  QueuedWork* w = static_cast<QueuedWork*>(data);
  if (g_trace) w->t[TP_JS] = now_ns();
  napi_delete_async_work(env, w->work);
  settle(env, w);
}

// traceDump() -> Float64Array [batch][8]: the TracePoint stamps (ns, CLOCK_MONOTONIC
// — process.hrtime's clock) and the batch's frame count; clears the record.
napi_value TraceDump(napi_env env, napi_callback_info) {
  std::vector<double> rows;
  {
    std::lock_guard<std::mutex> lk(g_trace_mu);
    rows.swap(g_trace_rows);
  }
  napi_value ab, arr;
  void* d = nullptr;
  NAPI_OK(env, napi_create_arraybuffer(env, rows.size() * sizeof(double), &d, &ab));
  if (!rows.empty()) std::memcpy(d, rows.data(), rows.size() * sizeof(double));
  NAPI_OK(env, napi_create_typedarray(env, napi_float64_array, rows.size(), ab, 0, &arr));
  return arr;
}

// The masks' ArrayBuffer: a pinned block, so the batch's D2H lands in it
// directly and the completion copies nothing — before, the masks were copied
// out of the slot's pinned buffer into fresh malloc'd pages on the HIP
// completion thread, one batch after another.  Pinning (and unpinning:
// hipHostFree waits for the device) is far too slow for the per-call path:
// blocks are carved from 64 MiB pinned slabs (vss_host_alloc; the library's
// direct-D2H check accepts any range inside one) in 64 KiB size classes and
// recycled — the finalizer V8 runs when a result is collected puts its block
// on the free list of its class, and slabs are never unpinned while the
// process runs.  In steady state the live blocks are the results V8 has not
// collected yet (its external-memory pressure — napi_adjust_external_memory —
// sets the pace); past kPinnedCap bytes of slabs, results fall back to
// malloc'd memory (then the completion copies).  Round 5 pinned one block per
// size as it was first needed: a one-frame call (147 KB of masks) whose size
// had no free block paid a hipHostMalloc, 41 us at p50 of segment()'s 42
// (tools/ts_prof.js, profiles/r06a).  Not zero-filled (Node 12's
// napi_create_arraybuffer spent ~0.19 ms clearing 1.2 MB on the JS thread per
// call).
struct MaskBlock {
  size_t bytes;  // the size class
  bool pinned;
};

// Never destroyed: result ArrayBuffers can be finalized while the process
// exits (V8 tearing the environment down), after static destructors of this
// module could otherwise have run.
std::mutex& g_pool_mu = *new std::mutex;
std::multimap<size_t, void*>& g_pool = *new std::multimap<size_t, void*>;  // free pinned blocks by size class
char* g_slab = nullptr;                // the slab being carved
size_t g_slab_left = 0;
size_t g_pinned_bytes = 0;             // every slab
struct PoolStats {
  unsigned long long hits = 0, carves = 0, slabs = 0, fallbacks = 0;
};
PoolStats g_pool_stats;
constexpr size_t kPinnedCap = size_t(2) << 30;
constexpr size_t kSlab = size_t(64) << 20, kClass = size_t(64) << 10;

// VSS_NAPI_PINNED=0: malloc'd results (the completion copies), for A/B runs
const bool g_use_pinned = [] {
  const char* e = std::getenv("VSS_NAPI_PINNED");
  return !(e && e[0] == '0');
}();

size_t size_class(size_t bytes) { return (bytes + kClass - 1) / kClass * kClass; }

void* pool_get(size_t cls, bool* pinned) {
  *pinned = false;
  if (!g_use_pinned) return std::malloc(cls);
  std::lock_guard<std::mutex> lk(g_pool_mu);
  auto it = g_pool.find(cls);
  if (it != g_pool.end()) {
    void* p = it->second;
    g_pool.erase(it);
    *pinned = true;
    ++g_pool_stats.hits;
    return p;
  }
  if (g_slab_left < cls) {  // a new slab (the rest of the old one stays unused)
    const size_t sz = std::max(kSlab, cls);
    void* p = nullptr;
    if (g_pinned_bytes + sz > kPinnedCap || vss_host_alloc(sz, &p) != VSS_OK) {
      ++g_pool_stats.fallbacks;
      return std::malloc(cls);
    }
    g_pinned_bytes += sz;
    ++g_pool_stats.slabs;
    g_slab = static_cast<char*>(p);
    g_slab_left = sz;
  }
  void* p = g_slab;
  g_slab += cls;
  g_slab_left -= cls;
  ++g_pool_stats.carves;
  *pinned = true;
  return p;
}

void pool_put(void* p, size_t cls) {
  std::lock_guard<std::mutex> lk(g_pool_mu);
  g_pool.emplace(cls, p);
}

// poolStats() -> {hits, carves, slabs, fallbacks, pinnedBytes}: the result blocks' allocator
napi_value PoolStatsJs(napi_env env, napi_callback_info) {
  PoolStats st;
  size_t pinned = 0;
  {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    st = g_pool_stats;
    pinned = g_pinned_bytes;
  }
  napi_value o, v;
  NAPI_OK(env, napi_create_object(env, &o));
  const std::pair<const char*, double> kv[] = {{"hits", (double)st.hits}, {"carves", (double)st.carves},
                                               {"slabs", (double)st.slabs}, {"fallbacks", (double)st.fallbacks},
                                               {"pinnedBytes", (double)pinned}};
  for (const auto& e : kv) {
    napi_create_double(env, e.second, &v);
    napi_set_named_property(env, o, e.first, v);
  }
  return o;
}

void free_masks(napi_env env, void* data, void* hint) {
  MaskBlock* b = static_cast<MaskBlock*>(hint);
  if (b->pinned)
    pool_put(data, b->bytes);
  else
    std::free(data);
  if (!g_env_closing.load()) {
    int64_t adj = 0;
    napi_adjust_external_memory(env, -(int64_t)b->bytes, &adj);
  }
  delete b;
}

bool masks_buffer(napi_env env, size_t bytes, void** data, napi_value* ab) {
  MaskBlock* b = new MaskBlock{size_class(std::max<size_t>(bytes, 16)), false};
  void* p = pool_get(b->bytes, &b->pinned);
  if (!p) {
    delete b;
    return false;
  }
  if (napi_create_external_arraybuffer(env, p, bytes, free_masks, b, ab) != napi_ok) {
    if (b->pinned)
      pool_put(p, b->bytes);
    else
      std::free(p);
    delete b;
    return false;
  }
  int64_t adj = 0;
  napi_adjust_external_memory(env, (int64_t)b->bytes, &adj);
  *data = p;
  return true;
}

bool u8_view(napi_env env, napi_value v, const uint8_t** data, size_t* len) {
  bool is_ta = false;
  napi_is_typedarray(env, v, &is_ta);
  if (!is_ta) return false;
  napi_typedarray_type tt;
  void* d = nullptr;
  napi_value buf;
  size_t off = 0;
  if (napi_get_typedarray_info(env, v, &tt, len, &d, &buf, &off) != napi_ok) return false;
  if (tt != napi_uint8_array && tt != napi_uint8_clamped_array) return false;
  *data = static_cast<const uint8_t*>(d);
  return true;
}

// segment(handle, frames | frames[], n, height, width, channels, rowStride, outMode?)
napi_value Segment(napi_env env, napi_callback_info info) {
  size_t argc = 8;
  napi_value argv[8];
  NAPI_OK(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  if (argc < 7) {
    napi_throw_type_error(env, nullptr, "segment(handle, frames, n, height, width, channels, rowStride, outMode?)");
    return nullptr;
  }
  Handle* hd = get_handle(env, argv[0]);
  if (!hd) return nullptr;
  int n = 0, height = 0, width = 0, channels = 0, rs = 0, out_mode = VSS_OUT_MODEL;
  napi_get_value_int32(env, argv[2], &n);
  napi_get_value_int32(env, argv[3], &height);
  napi_get_value_int32(env, argv[4], &width);
  napi_get_value_int32(env, argv[5], &channels);
  napi_get_value_int32(env, argv[6], &rs);
  if (argc >= 8) napi_get_value_int32(env, argv[7], &out_mode);
  if (n < 1 || height < 1 || width < 1 || rs < 1) {
    napi_throw_range_error(env, nullptr, "segment: n, height, width and rowStride must be >= 1");
    return nullptr;
  }
  const size_t fbytes = (size_t)height * (size_t)rs;
  bool is_arr = false;
  napi_is_array(env, argv[1], &is_arr);
  const uint8_t* contiguous = nullptr;
  std::vector<const uint8_t*> list;
  if (is_arr) {
    uint32_t len = 0;
    napi_get_array_length(env, argv[1], &len);
    if (len != (uint32_t)n) {
      napi_throw_range_error(env, nullptr, "segment: the frame list must hold n frames");
      return nullptr;
    }
    for (uint32_t i = 0; i < len; ++i) {
      napi_value v;
      napi_get_element(env, argv[1], i, &v);
      const uint8_t* d = nullptr;
      size_t l = 0;
      if (!u8_view(env, v, &d, &l)) {
        napi_throw_type_error(env, nullptr, "frames must be Uint8Array or Uint8ClampedArray");
        return nullptr;
      }
      if (l < fbytes) {
        napi_throw_range_error(env, nullptr, "a frame buffer is smaller than height * rowStride");
        return nullptr;
      }
      list.push_back(d);
    }
  } else {
    size_t l = 0;
    if (!u8_view(env, argv[1], &contiguous, &l)) {
      napi_throw_type_error(env, nullptr, "frames must be a Uint8Array or Uint8ClampedArray");
      return nullptr;
    }
    if (l < (size_t)n * fbytes) {
      napi_throw_range_error(env, nullptr, "frames buffer smaller than n * height * rowStride");
      return nullptr;
    }
  }
  const double t_call = g_trace ? now_ns() : 0.0;
  static const bool sync_stage = [] {
    const char* e = std::getenv("VSS_NAPI_SYNC_STAGE");
    return e && e[0] == '1';
  }();
  if (!sync_stage && !submitter(env, hd)) {
    napi_throw_error(env, nullptr, "segment: cannot create the result delivery");
    return nullptr;
  }
  QueuedWork* w = new QueuedWork();
  w->t[TP_CALL] = t_call;
  w->h = hd->h;
  w->out_count = out_mode == VSS_OUT_FRAME ? (size_t)n * height * width : (size_t)n * hd->mask_h * hd->mask_w;
  napi_value ab, promise;
  void* out = nullptr;
  if (!masks_buffer(env, w->out_count * 4, &out, &ab)) {
    delete w;
    napi_throw_error(env, nullptr, "out of host memory for the masks");
    return nullptr;
  }
  NAPI_OK(env, napi_create_promise(env, &w->deferred, &promise));
  if (!is_arr)
    for (int i = 0; i < n; ++i) list.push_back(contiguous + (size_t)i * fbytes);
  if (!sync_stage) {
    // the submit thread stages the frames (the submit's cost: 3.7 MB per VGA
    // batch of 8 copied into pinned memory), so the JS thread only enqueues;
    // the frames' arrays are referenced until the batch is done, and the
    // caller must not modify them before the promise settles (ts/segment.ts)
    w->list = std::move(list);
    w->n = n;
    w->height = height;
    w->width = width;
    w->channels = channels;
    w->rs = (size_t)rs;
    w->out = static_cast<float*>(out);
    w->out_mode = out_mode;
    if (is_arr) {
      for (uint32_t i = 0; i < (uint32_t)n; ++i) {
        napi_value v;
        napi_ref r;
        napi_get_element(env, argv[1], i, &v);
        NAPI_OK(env, napi_create_reference(env, v, 1, &r));
        w->frame_refs.push_back(r);
      }
    } else {
      napi_ref r;
      NAPI_OK(env, napi_create_reference(env, argv[1], 1, &r));
      w->frame_refs.push_back(r);
    }
    napi_create_reference(env, ab, 1, &w->out_ref);
    w->n = n;
    enqueue(env, hd, w);
    return promise;
  }
  // staged here: the frames may be reused by the caller as soon as this returns
  w->n = n;
  if (g_trace) w->t[TP_QUEUED] = w->t[TP_SUBMIT] = now_ns();
  const int rc = vss_submit_list(hd->h, list.data(), n, height, width, channels, (size_t)rs, static_cast<float*>(out),
                                 out_mode, &w->ticket);
  if (g_trace) w->t[TP_SUBMITTED] = now_ns();
  if (rc != VSS_OK) {
    napi_reject_deferred(env, w->deferred, make_error(env, "vss_submit", rc, vss_last_error(hd->h)));
    delete w;
    return promise;
  }
  napi_create_reference(env, ab, 1, &w->out_ref);  // masks_out stays alive until the batch is done
  napi_value name;
  napi_create_string_utf8(env, "vss_wait", NAPI_AUTO_LENGTH, &name);
  NAPI_OK(env, napi_create_async_work(env, nullptr, name, QueuedExecute, QueuedComplete, w, &w->work));
  NAPI_OK(env, napi_queue_async_work(env, w->work));
  w->hd = hd;
  ++hd->pending;
  return promise;
}

void noop_finalize(napi_env, void*, void*) {}  // the pinned staging belongs to the handle

napi_value StagingAcquire(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_OK(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  Handle* hd = get_handle(env, argv[0]);
  if (!hd) return nullptr;
  int slot = -1;
  uint8_t* p = nullptr;
  size_t cap = 0;
  const int rc = vss_staging_acquire(hd->h, &slot, &p, &cap);
  if (rc != VSS_OK) {
    napi_throw(env, make_error(env, "vss_staging_acquire", rc, vss_last_error(hd->h)));
    return nullptr;
  }
  napi_value ab, arr, o, v;
  NAPI_OK(env, napi_create_external_arraybuffer(env, p, cap, noop_finalize, nullptr, &ab));
  NAPI_OK(env, napi_create_typedarray(env, napi_uint8_array, cap, ab, 0, &arr));
  NAPI_OK(env, napi_create_object(env, &o));
  napi_create_int32(env, slot, &v);
  napi_set_named_property(env, o, "slot", v);
  napi_set_named_property(env, o, "data", arr);
  return o;
}

napi_value StagingRelease(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  NAPI_OK(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  Handle* hd = get_handle(env, argv[0]);
  if (!hd) return nullptr;
  int slot = -1;
  napi_get_value_int32(env, argv[1], &slot);
  const int rc = vss_staging_release(hd->h, slot);
  if (rc != VSS_OK) napi_throw(env, make_error(env, "vss_staging_release", rc, vss_last_error(hd->h)));
  return nullptr;
}

// segmentStaged(handle, slot, n, height, width, channels, rowStride, outMode?)
napi_value SegmentStaged(napi_env env, napi_callback_info info) {
  size_t argc = 8;
  napi_value argv[8];
  NAPI_OK(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  if (argc < 7) {
    napi_throw_type_error(env, nullptr, "segmentStaged(handle, slot, n, height, width, channels, rowStride, outMode?)");
    return nullptr;
  }
  Handle* hd = get_handle(env, argv[0]);
  if (!hd) return nullptr;
  int slot = -1, n = 0, height = 0, width = 0, channels = 0, rs = 0, out_mode = VSS_OUT_MODEL;
  napi_get_value_int32(env, argv[1], &slot);
  napi_get_value_int32(env, argv[2], &n);
  napi_get_value_int32(env, argv[3], &height);
  napi_get_value_int32(env, argv[4], &width);
  napi_get_value_int32(env, argv[5], &channels);
  napi_get_value_int32(env, argv[6], &rs);
  if (argc >= 8) napi_get_value_int32(env, argv[7], &out_mode);
  if (n < 1 || height < 1 || width < 1 || rs < 1) {
    napi_throw_range_error(env, nullptr, "segmentStaged: n, height, width and rowStride must be >= 1");
    return nullptr;
  }
  const double t_call = g_trace ? now_ns() : 0.0;
  if (!submitter(env, hd)) {
    napi_throw_error(env, nullptr, "segmentStaged: cannot create the result delivery");
    return nullptr;
  }
  QueuedWork* w = new QueuedWork();
  w->t[TP_CALL] = t_call;
  w->h = hd->h;
  w->out_count = out_mode == VSS_OUT_FRAME ? (size_t)n * height * width : (size_t)n * hd->mask_h * hd->mask_w;
  napi_value ab, promise;
  void* out = nullptr;
  if (!masks_buffer(env, w->out_count * 4, &out, &ab)) {
    delete w;
    napi_throw_error(env, nullptr, "out of host memory for the masks");
    return nullptr;
  }
  NAPI_OK(env, napi_create_promise(env, &w->deferred, &promise));
  // submitted by the submit thread, after every earlier call's batch (call
  // order is ticket order); nothing to stage: the frames are in the slot
  w->slot = slot;
  w->n = n;
  w->height = height;
  w->width = width;
  w->channels = channels;
  w->rs = (size_t)rs;
  w->out = static_cast<float*>(out);
  w->out_mode = out_mode;
  napi_create_reference(env, ab, 1, &w->out_ref);
  enqueue(env, hd, w);
  return promise;
}

struct SegmentWork {
  napi_async_work work = nullptr;
  napi_deferred deferred = nullptr;
  napi_ref frames_ref = nullptr, out_ref = nullptr;
  napi_ref u8_ref = nullptr;             // segmentPost: the alpha bytes
  Handle* hd = nullptr;                  // pending counted until SegmentComplete
  vss_handle* h = nullptr;
  vss_post_state* post = nullptr;        // segmentPost / segmentComposite
  bool composite = false;                // segmentComposite: out_u8 holds the RGBA canvases
  const uint8_t* frames = nullptr;
  float* out = nullptr;
  uint8_t* out_u8 = nullptr;
  int n = 0, height = 0, width = 0, channels = 0, out_mode = VSS_OUT_MODEL;
  size_t row_stride = 0, out_count = 0;
  int rc = 0;
  std::string err;
};

void SegmentExecute(napi_env, void* data) {  // libuv worker thread: no JS calls here
  SegmentWork* w = static_cast<SegmentWork*>(data);
  if (w->composite)
    w->rc = vss_segment_composite(w->h, w->post, w->frames, w->n, w->height, w->width, w->channels, w->row_stride,
                                  w->out_u8);
  else
    w->rc = vss_segment_post(w->h, w->post, w->frames, w->n, w->height, w->width, w->channels, w->row_stride, w->out,
                             w->out_u8);
  if (w->rc != VSS_OK) w->err = vss_last_error(w->h);
}

void SegmentComplete(napi_env env, napi_status, void* data) {
  SegmentWork* w = static_cast<SegmentWork*>(data);
  napi_value ab = nullptr;
  napi_get_reference_value(env, w->out_ref, &ab);
  if (w->rc == VSS_OK && w->composite) {
    napi_value ab8 = nullptr, arr8;
    napi_get_reference_value(env, w->u8_ref, &ab8);
    napi_create_typedarray(env, napi_uint8_array, (size_t)w->n * w->height * w->width * 4, ab8, 0, &arr8);
    napi_resolve_deferred(env, w->deferred, arr8);
  } else if (w->rc == VSS_OK) {
    napi_value arr;
    napi_create_typedarray(env, napi_float32_array, w->out_count, ab, 0, &arr);
    if (w->post) {
      napi_value ab8 = nullptr, arr8, o;
      napi_get_reference_value(env, w->u8_ref, &ab8);
      napi_create_typedarray(env, napi_uint8_array, w->out_count, ab8, 0, &arr8);
      napi_create_object(env, &o);
      napi_set_named_property(env, o, "alpha", arr);
      napi_set_named_property(env, o, "alphaU8", arr8);
      napi_resolve_deferred(env, w->deferred, o);
    } else {
      napi_resolve_deferred(env, w->deferred, arr);
    }
  } else {
    napi_value msg, code, e;
    const std::string m = std::string(w->composite ? "vss_segment_composite" : "vss_segment_post") + " failed (" +
                          std::to_string(w->rc) + "): " + w->err;
    napi_create_string_utf8(env, m.c_str(), m.size(), &msg);
    napi_create_string_utf8(env, std::to_string(w->rc).c_str(), NAPI_AUTO_LENGTH, &code);
    napi_create_error(env, code, msg, &e);
    napi_reject_deferred(env, w->deferred, e);
  }
  napi_delete_reference(env, w->frames_ref);
  napi_delete_reference(env, w->out_ref);
  if (w->u8_ref) napi_delete_reference(env, w->u8_ref);
  napi_delete_async_work(env, w->work);
  Handle* hd = w->hd;
  delete w;
  work_done(hd);
}

// segmentPost(handle, post, frames, ...) and segmentComposite(handle, post, frames, ...)
napi_value SegmentImpl(napi_env env, napi_callback_info info, bool with_post, bool composite = false) {
  size_t argc = 9;
  napi_value all[9];
  NAPI_OK(env, napi_get_cb_info(env, info, &argc, all, nullptr, nullptr));
  const size_t need = with_post ? 8 : 7;
  if (argc < need) {
    napi_throw_type_error(env, nullptr,
                          with_post ? "segmentPost(handle, post, frames, n, height, width, channels, rowStride)"
                                    : "segment(handle, frames, n, height, width, channels, rowStride)");
    return nullptr;
  }
  Handle* hd = get_handle(env, all[0]);
  if (!hd) return nullptr;
  Post* ps = nullptr;
  if (with_post) {
    ps = get_post(env, all[1]);
    if (!ps) return nullptr;
    if (ps->hd != hd) {
      napi_throw_error(env, nullptr, "post state belongs to another handle");
      return nullptr;
    }
  }
  napi_value* argv = with_post ? all + 1 : all;
  bool is_ta = false;
  napi_is_typedarray(env, argv[1], &is_ta);
  if (!is_ta) {
    napi_throw_type_error(env, nullptr, "frames must be a Uint8Array or Uint8ClampedArray");
    return nullptr;
  }
  napi_typedarray_type tt;
  size_t len = 0, off = 0;
  void* data = nullptr;
  napi_value buf;
  NAPI_OK(env, napi_get_typedarray_info(env, argv[1], &tt, &len, &data, &buf, &off));
  if (tt != napi_uint8_array && tt != napi_uint8_clamped_array) {
    napi_throw_type_error(env, nullptr, "frames must be a Uint8Array or Uint8ClampedArray");
    return nullptr;
  }
  SegmentWork* w = new SegmentWork();
  int rs = 0;
  napi_get_value_int32(env, argv[2], &w->n);
  napi_get_value_int32(env, argv[3], &w->height);
  napi_get_value_int32(env, argv[4], &w->width);
  napi_get_value_int32(env, argv[5], &w->channels);
  napi_get_value_int32(env, argv[6], &rs);
  w->row_stride = (size_t)rs;
  if (w->n < 1 || w->height < 1 || rs < 1 || len < (size_t)w->n * w->height * w->row_stride) {
    delete w;
    napi_throw_range_error(env, nullptr, "frames buffer smaller than n * height * rowStride");
    return nullptr;
  }
  w->h = hd->h;
  w->post = ps ? ps->st : nullptr;
  w->frames = static_cast<const uint8_t*>(data);
  if (!with_post && argc >= 8) napi_get_value_int32(env, argv[7], &w->out_mode);
  w->out_count = w->out_mode == VSS_OUT_FRAME ? (size_t)w->n * w->height * w->width
                                              : (size_t)w->n * hd->mask_h * hd->mask_w;
  napi_value ab;
  void* out = nullptr;
  NAPI_OK(env, napi_create_arraybuffer(env, w->out_count * 4, &out, &ab));
  w->out = static_cast<float*>(out);
  w->composite = composite;
  if (ps) {
    napi_value ab8;
    void* out8 = nullptr;
    const size_t bytes8 = composite ? (size_t)w->n * w->height * w->width * 4 : w->out_count;
    NAPI_OK(env, napi_create_arraybuffer(env, bytes8, &out8, &ab8));
    w->out_u8 = static_cast<uint8_t*>(out8);
    napi_create_reference(env, ab8, 1, &w->u8_ref);
  }
  napi_create_reference(env, argv[1], 1, &w->frames_ref);  // keep the frames alive until done
  napi_create_reference(env, ab, 1, &w->out_ref);
  napi_value promise, name;
  NAPI_OK(env, napi_create_promise(env, &w->deferred, &promise));
  napi_create_string_utf8(env, ps ? "vss_segment_post" : "vss_segment", NAPI_AUTO_LENGTH, &name);
  NAPI_OK(env, napi_create_async_work(env, nullptr, name, SegmentExecute, SegmentComplete, w, &w->work));
  NAPI_OK(env, napi_queue_async_work(env, w->work));
  w->hd = hd;
  ++hd->pending;
  return promise;
}

napi_value SegmentPost(napi_env env, napi_callback_info info) { return SegmentImpl(env, info, true); }
napi_value SegmentComposite(napi_env env, napi_callback_info info) { return SegmentImpl(env, info, true, true); }

// ---- ONNX sessions (include/vso.h) -------------------------------------------
struct OrtSess {
  vso_session* s = nullptr;
  int users = 0;  // face trackers driving this session
  std::vector<std::string> in_names, out_names;
  std::vector<std::vector<int64_t>> in_shapes, out_shapes;
};

void finalize_ort(napi_env, void* data, void*) {
  OrtSess* o = static_cast<OrtSess*>(data);
  if (o->s) vso_destroy(o->s);
  delete o;
}

OrtSess* get_ort(napi_env env, napi_value v) {
  void* p = nullptr;
  if (napi_get_value_external(env, v, &p) != napi_ok || !p) {
    napi_throw_type_error(env, nullptr, "expected an ONNX session");
    return nullptr;
  }
  OrtSess* o = static_cast<OrtSess*>(p);
  if (!o->s) {
    napi_throw_error(env, nullptr, "ONNX session already released");
    return nullptr;
  }
  return o;
}

size_t elem_count(const std::vector<int64_t>& d) {
  size_t n = 1;
  for (int64_t v : d) n *= (size_t)v;
  return n;
}

napi_value OrtCreate(napi_env env, napi_callback_info info) {
  size_t argc = 4;
  napi_value argv[4];
  NAPI_OK(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  bool is_ta = false;
  if (argc < 1 || napi_is_typedarray(env, argv[0], &is_ta) != napi_ok || !is_ta) {
    napi_throw_type_error(env, nullptr,
                          "ortCreate(modelBytes: Uint8Array, inputDims?: number[], deviceId?: number, convPrecision?: number)");
    return nullptr;
  }
  napi_typedarray_type tt;
  size_t len = 0, off = 0;
  void* data = nullptr;
  napi_value buf;
  NAPI_OK(env, napi_get_typedarray_info(env, argv[0], &tt, &len, &data, &buf, &off));
  std::vector<int64_t> dims;
  bool is_arr = false;
  if (argc >= 2 && napi_is_array(env, argv[1], &is_arr) == napi_ok && is_arr) {
    uint32_t n = 0;
    napi_get_array_length(env, argv[1], &n);
    for (uint32_t k = 0; k < n; ++k) {
      napi_value e;
      double d = 0;
      napi_get_element(env, argv[1], k, &e);
      napi_get_value_double(env, e, &d);
      dims.push_back((int64_t)d);
    }
  }
  int device = 0;
  if (argc >= 3) napi_get_value_int32(env, argv[2], &device);
  vso_options opts;
  vso_options_default(&opts);
  if (argc >= 4) napi_get_value_int32(env, argv[3], &opts.conv_precision);
  vso_session* s = nullptr;
  const int rc = vso_create_ex(data, len, dims.empty() ? nullptr : dims.data(), (int)dims.size(), device, &opts, &s);
  if (rc != VSO_OK) {
    throw_vss(env, "vso_create", rc, vso_last_error(nullptr));
    return nullptr;
  }
  OrtSess* o = new OrtSess();
  o->s = s;
  int ni = 0, no = 0;
  vso_io_count(s, &ni, &no);
  char name[512];
  int64_t d[16];
  for (int k = 0; k < ni; ++k) {
    vso_input_name(s, k, name, sizeof(name));
    o->in_names.push_back(name);
    const int r = vso_input_shape(s, k, d, 16);
    o->in_shapes.emplace_back(d, d + std::max(0, std::min(r, 16)));
  }
  for (int k = 0; k < no; ++k) {
    vso_output_name(s, k, name, sizeof(name));
    o->out_names.push_back(name);
    const int r = vso_output_shape(s, k, d, 16);
    o->out_shapes.emplace_back(d, d + std::max(0, std::min(r, 16)));
  }
  napi_value ext;
  NAPI_OK(env, napi_create_external(env, o, finalize_ort, nullptr, &ext));
  return ext;
}

napi_value names_array(napi_env env, const std::vector<std::string>& v) {
  napi_value a, e;
  napi_create_array_with_length(env, v.size(), &a);
  for (size_t k = 0; k < v.size(); ++k) {
    napi_create_string_utf8(env, v[k].c_str(), NAPI_AUTO_LENGTH, &e);
    napi_set_element(env, a, (uint32_t)k, e);
  }
  return a;
}

napi_value shapes_array(napi_env env, const std::vector<std::vector<int64_t>>& v) {
  napi_value a, row, e;
  napi_create_array_with_length(env, v.size(), &a);
  for (size_t k = 0; k < v.size(); ++k) {
    napi_create_array_with_length(env, v[k].size(), &row);
    for (size_t j = 0; j < v[k].size(); ++j) {
      napi_create_double(env, (double)v[k][j], &e);
      napi_set_element(env, row, (uint32_t)j, e);
    }
    napi_set_element(env, a, (uint32_t)k, row);
  }
  return a;
}

napi_value OrtInfo(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_OK(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  OrtSess* o = argc >= 1 ? get_ort(env, argv[0]) : nullptr;
  if (!o) return nullptr;
  napi_value r;
  NAPI_OK(env, napi_create_object(env, &r));
  napi_set_named_property(env, r, "inputNames", names_array(env, o->in_names));
  napi_set_named_property(env, r, "outputNames", names_array(env, o->out_names));
  napi_set_named_property(env, r, "inputShapes", shapes_array(env, o->in_shapes));
  napi_set_named_property(env, r, "outputShapes", shapes_array(env, o->out_shapes));
  return r;
}

struct OrtWork {
  napi_async_work work = nullptr;
  napi_deferred deferred = nullptr;
  vso_session* s = nullptr;
  std::vector<napi_ref> in_refs, out_refs;  // inputs and output buffers held until done
  std::vector<const float*> ins;
  std::vector<float*> outs;
  std::vector<size_t> out_counts;
  int rc = 0;
  std::string err;
};

void OrtExecute(napi_env, void* data) {  // libuv worker thread: no JS calls here
  OrtWork* w = static_cast<OrtWork*>(data);
  w->rc = vso_run(w->s, w->ins.data(), w->outs.data());
  if (w->rc != VSO_OK) w->err = vso_last_error(w->s);
}

void OrtComplete(napi_env env, napi_status, void* data) {
  OrtWork* w = static_cast<OrtWork*>(data);
  if (w->rc == VSO_OK) {
    napi_value a;
    napi_create_array_with_length(env, w->outs.size(), &a);
    for (size_t k = 0; k < w->outs.size(); ++k) {
      napi_value ab, ta;
      napi_get_reference_value(env, w->out_refs[k], &ab);
      napi_create_typedarray(env, napi_float32_array, w->out_counts[k], ab, 0, &ta);
      napi_set_element(env, a, (uint32_t)k, ta);
    }
    napi_resolve_deferred(env, w->deferred, a);
  } else {
    napi_value msg, code, e;
    const std::string m = "vso_run failed (" + std::to_string(w->rc) + "): " + w->err;
    napi_create_string_utf8(env, m.c_str(), m.size(), &msg);
    napi_create_string_utf8(env, std::to_string(w->rc).c_str(), NAPI_AUTO_LENGTH, &code);
    napi_create_error(env, code, msg, &e);
    napi_reject_deferred(env, w->deferred, e);
  }
  for (napi_ref r : w->in_refs) napi_delete_reference(env, r);
  for (napi_ref r : w->out_refs) napi_delete_reference(env, r);
  napi_delete_async_work(env, w->work);
  delete w;
}

napi_value OrtRun(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  NAPI_OK(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  OrtSess* o = argc >= 1 ? get_ort(env, argv[0]) : nullptr;
  if (!o) return nullptr;
  bool is_arr = false;
  uint32_t n = 0;
  if (argc < 2 || napi_is_array(env, argv[1], &is_arr) != napi_ok || !is_arr ||
      napi_get_array_length(env, argv[1], &n) != napi_ok || n != o->in_names.size()) {
    napi_throw_type_error(env, nullptr, "ortRun(session, inputs: Float32Array[]): one array per model input");
    return nullptr;
  }
  // validate every input before anything is allocated or referenced
  std::vector<napi_value> elems(n);
  std::vector<const float*> ptrs(n);
  for (uint32_t k = 0; k < n; ++k) {
    napi_value buf;
    bool ta = false;
    napi_typedarray_type tt;
    size_t len = 0, off = 0;
    void* data = nullptr;
    napi_get_element(env, argv[1], k, &elems[k]);
    if (napi_is_typedarray(env, elems[k], &ta) != napi_ok || !ta ||
        napi_get_typedarray_info(env, elems[k], &tt, &len, &data, &buf, &off) != napi_ok ||
        tt != napi_float32_array || len != elem_count(o->in_shapes[k])) {
      const std::string m = "input '" + o->in_names[k] + "' must be a Float32Array of " +
                            std::to_string(elem_count(o->in_shapes[k])) + " elements";
      napi_throw_range_error(env, nullptr, m.c_str());
      return nullptr;
    }
    ptrs[k] = static_cast<const float*>(data);
  }
  OrtWork* w = new OrtWork();
  w->s = o->s;
  w->ins = ptrs;
  for (uint32_t k = 0; k < n; ++k) {
    napi_ref r;
    napi_create_reference(env, elems[k], 1, &r);
    w->in_refs.push_back(r);
  }
  for (size_t k = 0; k < o->out_names.size(); ++k) {
    const size_t cnt = elem_count(o->out_shapes[k]);
    napi_value ab;
    void* out = nullptr;
    NAPI_OK(env, napi_create_arraybuffer(env, cnt * 4, &out, &ab));
    napi_ref r;
    napi_create_reference(env, ab, 1, &r);
    w->out_refs.push_back(r);
    w->outs.push_back(static_cast<float*>(out));
    w->out_counts.push_back(cnt);
  }
  napi_value promise, name;
  NAPI_OK(env, napi_create_promise(env, &w->deferred, &promise));
  napi_create_string_utf8(env, "vso_run", NAPI_AUTO_LENGTH, &name);
  NAPI_OK(env, napi_create_async_work(env, nullptr, name, OrtExecute, OrtComplete, w, &w->work));
  NAPI_OK(env, napi_queue_async_work(env, w->work));
  return promise;
}

napi_value OrtDestroy(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_OK(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  void* p = nullptr;
  if (argc >= 1 && napi_get_value_external(env, argv[0], &p) == napi_ok && p) {
    OrtSess* o = static_cast<OrtSess*>(p);
    if (o->users > 0) {
      napi_throw_error(env, nullptr, "ONNX session in use by a face tracker: destroy the tracker first");
      return nullptr;
    }
    if (o->s) vso_destroy(o->s);
    o->s = nullptr;
  }
  return nullptr;
}

// ---- GPU face stage (include/vsf.h) ------------------------------------------
struct Face {
  vsf_tracker* t = nullptr;
  OrtSess* det = nullptr;
  OrtSess* lmk = nullptr;
  napi_ref det_ref = nullptr, lmk_ref = nullptr;  // the sessions outlive the tracker
  int inflight = 0;                                 // faceTrack calls not yet completed
};

void release_face(napi_env env, Face* f) {
  if (f->t) vsf_destroy(f->t);
  f->t = nullptr;
  if (f->det) f->det->users--;
  if (f->lmk) f->lmk->users--;
  f->det = f->lmk = nullptr;
  if (env && f->det_ref) napi_delete_reference(env, f->det_ref);
  if (env && f->lmk_ref) napi_delete_reference(env, f->lmk_ref);
  f->det_ref = f->lmk_ref = nullptr;
}

void finalize_face(napi_env env, void* data, void*) {
  Face* f = static_cast<Face*>(data);
  release_face(env, f);
  delete f;
}

Face* get_face(napi_env env, napi_value v) {
  void* p = nullptr;
  if (napi_get_value_external(env, v, &p) != napi_ok || !p) {
    napi_throw_type_error(env, nullptr, "expected a face tracker");
    return nullptr;
  }
  Face* f = static_cast<Face*>(p);
  if (!f->t) {
    napi_throw_error(env, nullptr, "face tracker already destroyed");
    return nullptr;
  }
  return f;
}

napi_value FaceCreate(napi_env env, napi_callback_info info) {
  size_t argc = 4;
  napi_value argv[4];
  NAPI_OK(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  if (argc < 2) {
    napi_throw_type_error(env, nullptr, "faceCreate(detector, landmarks, config?, deviceId?)");
    return nullptr;
  }
  OrtSess* det = get_ort(env, argv[0]);
  if (!det) return nullptr;
  OrtSess* lmk = get_ort(env, argv[1]);
  if (!lmk) return nullptr;
  vsf_config c;
  vsf_config_default(&c);
  napi_valuetype t = napi_undefined;
  if (argc >= 3) napi_typeof(env, argv[2], &t);
  if (t == napi_object) {
    get_int_prop(env, argv[2], "interval", &c.interval);
    get_double_prop(env, argv[2], "warpGain", &c.warp_gain);
    get_double_prop(env, argv[2], "faceScoreThresh", &c.face_score_thresh);
    get_double_prop(env, argv[2], "landmarkScoreThresh", &c.landmark_score_thresh);
    get_double_prop(env, argv[2], "roiPad", &c.roi_pad);
  }
  int device = 0;
  if (argc >= 4) napi_get_value_int32(env, argv[3], &device);
  vsf_tracker* tr = nullptr;
  const int rc = vsf_create(det->s, lmk->s, &c, device, &tr);
  if (rc != VSS_OK) {
    throw_vss(env, "vsf_create", rc, vsf_last_error(nullptr));
    return nullptr;
  }
  Face* f = new Face();
  f->t = tr;
  f->det = det;
  f->lmk = lmk;
  det->users++;
  lmk->users++;
  napi_create_reference(env, argv[0], 1, &f->det_ref);
  napi_create_reference(env, argv[1], 1, &f->lmk_ref);
  napi_value ext;
  NAPI_OK(env, napi_create_external(env, f, finalize_face, nullptr, &ext));
  return ext;
}

struct FaceWork {
  napi_async_work work = nullptr;
  napi_deferred deferred = nullptr;
  napi_ref frames_ref = nullptr, face_ref = nullptr;
  Face* f = nullptr;
  vsf_tracker* t = nullptr;
  const uint8_t* frames = nullptr;
  int n = 0, h = 0, w = 0, c = 0, mask_w = 0, mask_h = 0;
  size_t rs = 0;
  std::vector<vss_face_frame> out;
  int rc = 0;
  std::string err;
};

void FaceExecute(napi_env, void* data) {  // libuv worker thread
  FaceWork* w = static_cast<FaceWork*>(data);
  w->rc = vsf_track(w->t, w->frames, w->n, w->h, w->w, w->c, w->rs, w->mask_w, w->mask_h, w->out.data());
  if (w->rc != VSS_OK) w->err = vsf_last_error(w->t);
}

napi_value doubles_array(napi_env env, const double* v, int n) {
  napi_value a, e;
  napi_create_array_with_length(env, n, &a);
  for (int k = 0; k < n; ++k) {
    napi_create_double(env, v[k], &e);
    napi_set_element(env, a, (uint32_t)k, e);
  }
  return a;
}

void FaceComplete(napi_env env, napi_status, void* data) {
  FaceWork* w = static_cast<FaceWork*>(data);
  if (w->rc == VSS_OK) {
    napi_value a, nul;
    napi_get_null(env, &nul);
    napi_create_array_with_length(env, w->out.size(), &a);
    for (size_t k = 0; k < w->out.size(); ++k) {
      const vss_face_frame& f = w->out[k];
      napi_value o, v;
      napi_create_object(env, &o);
      napi_set_named_property(env, o, "affine", f.has_affine ? doubles_array(env, f.affine, 6) : nul);
      napi_set_named_property(env, o, "box", f.has_box ? doubles_array(env, f.box, 4) : nul);
      napi_create_int32(env, f.video_w, &v);
      napi_set_named_property(env, o, "videoW", v);
      napi_create_int32(env, f.video_h, &v);
      napi_set_named_property(env, o, "videoH", v);
      napi_set_element(env, a, (uint32_t)k, o);
    }
    napi_resolve_deferred(env, w->deferred, a);
  } else {
    napi_value msg, code, e;
    const std::string m = "vsf_track failed (" + std::to_string(w->rc) + "): " + w->err;
    napi_create_string_utf8(env, m.c_str(), m.size(), &msg);
    napi_create_string_utf8(env, std::to_string(w->rc).c_str(), NAPI_AUTO_LENGTH, &code);
    napi_create_error(env, code, msg, &e);
    napi_reject_deferred(env, w->deferred, e);
  }
  w->f->inflight--;
  napi_delete_reference(env, w->frames_ref);
  napi_delete_reference(env, w->face_ref);
  napi_delete_async_work(env, w->work);
  delete w;
}

napi_value FaceTrack(napi_env env, napi_callback_info info) {
  size_t argc = 9;
  napi_value argv[9];
  NAPI_OK(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  Face* f = argc >= 1 ? get_face(env, argv[0]) : nullptr;
  if (!f) return nullptr;
  int v[7] = {0, 0, 0, 0, 0, 0, 0};  // n, h, w, c, rowStride, maskW, maskH
  bool ta = false;
  napi_typedarray_type tt;
  size_t len = 0, off = 0;
  void* data = nullptr;
  napi_value buf;
  bool ok = argc >= 9 && napi_is_typedarray(env, argv[1], &ta) == napi_ok && ta &&
            napi_get_typedarray_info(env, argv[1], &tt, &len, &data, &buf, &off) == napi_ok &&
            (tt == napi_uint8_array || tt == napi_uint8_clamped_array);
  for (int k = 0; ok && k < 7; ++k) ok = napi_get_value_int32(env, argv[2 + k], &v[k]) == napi_ok;
  if (!ok) {
    napi_throw_type_error(env, nullptr,
                          "faceTrack(tracker, frames: Uint8Array, n, height, width, channels, rowStride, maskW, maskH)");
    return nullptr;
  }
  if (v[0] < 0 || v[1] < 1 || v[4] < 1 || (size_t)v[0] * v[1] * v[4] > len) {
    napi_throw_range_error(env, nullptr, "faceTrack: frames buffer smaller than n * height * rowStride");
    return nullptr;
  }
  FaceWork* w = new FaceWork();
  w->t = f->t;
  w->frames = static_cast<const uint8_t*>(data);
  w->n = v[0];
  w->h = v[1];
  w->w = v[2];
  w->c = v[3];
  w->rs = (size_t)v[4];
  w->mask_w = v[5];
  w->mask_h = v[6];
  w->out.resize((size_t)v[0]);
  w->f = f;
  f->inflight++;
  napi_create_reference(env, argv[1], 1, &w->frames_ref);
  napi_create_reference(env, argv[0], 1, &w->face_ref);  // the tracker outlives the call
  napi_value promise, name;
  NAPI_OK(env, napi_create_promise(env, &w->deferred, &promise));
  napi_create_string_utf8(env, "vsf_track", NAPI_AUTO_LENGTH, &name);
  NAPI_OK(env, napi_create_async_work(env, nullptr, name, FaceExecute, FaceComplete, w, &w->work));
  NAPI_OK(env, napi_queue_async_work(env, w->work));
  return promise;
}

napi_value FaceReset(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_OK(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  Face* f = argc >= 1 ? get_face(env, argv[0]) : nullptr;
  if (!f) return nullptr;
  const int rc = vsf_reset(f->t);
  if (rc != VSS_OK) throw_vss(env, "vsf_reset", rc, vsf_last_error(f->t));
  return nullptr;
}

napi_value FaceDestroy(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_OK(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  void* p = nullptr;
  if (argc >= 1 && napi_get_value_external(env, argv[0], &p) == napi_ok && p) {
    Face* f = static_cast<Face*>(p);
    if (f->inflight > 0) {
      napi_throw_error(env, nullptr, "faceDestroy: a faceTrack call is still running on this tracker");
      return nullptr;
    }
    release_face(env, f);
  }
  return nullptr;
}

// VSS_NAPI_SEGV_TRACE=1: a fatal signal prints the native backtrace to
// stderr before the process dies (diagnosing crashes at process exit).
void segv_trace(int sig) {
  void* fr[64];
  const int n = backtrace(fr, 64);
  const char msg[] = "vss_napi: fatal signal, native backtrace:\n";
  (void)!write(2, msg, sizeof(msg) - 1);
  backtrace_symbols_fd(fr, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}

void env_cleanup(void*) { g_env_closing.store(true); }

napi_value Init(napi_env env, napi_value exports) {
  napi_add_env_cleanup_hook(env, env_cleanup, nullptr);
  if (const char* e = std::getenv("VSS_NAPI_SEGV_TRACE"))
    if (e[0] == '1') {
      signal(SIGSEGV, segv_trace);
      signal(SIGABRT, segv_trace);
    }
  const napi_property_descriptor props[] = {
      {"version", nullptr, Version, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"create", nullptr, Create, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"info", nullptr, Info, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"segment", nullptr, Segment, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"stagingAcquire", nullptr, StagingAcquire, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"stagingRelease", nullptr, StagingRelease, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"segmentStaged", nullptr, SegmentStaged, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"traceDump", nullptr, TraceDump, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"poolStats", nullptr, PoolStatsJs, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"destroy", nullptr, Destroy, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"postCreate", nullptr, PostCreate, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"postSetConfig", nullptr, PostSetConfig, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"postReset", nullptr, PostReset, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"postDestroy", nullptr, PostDestroy, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"postSetFaces", nullptr, PostSetFaces, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"segmentPost", nullptr, SegmentPost, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"segmentComposite", nullptr, SegmentComposite, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"ortCreate", nullptr, OrtCreate, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"ortInfo", nullptr, OrtInfo, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"ortRun", nullptr, OrtRun, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"ortDestroy", nullptr, OrtDestroy, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"faceCreate", nullptr, FaceCreate, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"faceTrack", nullptr, FaceTrack, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"faceReset", nullptr, FaceReset, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"faceDestroy", nullptr, FaceDestroy, nullptr, nullptr, nullptr, napi_default, nullptr},
  };
  napi_define_properties(env, exports, sizeof(props) / sizeof(props[0]), props);
  return exports;
}

}  // namespace

NAPI_MODULE(NODE_GYP_MODULE_NAME, Init)
