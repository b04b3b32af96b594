// vss_face.hip — §8(f) row 4: the face detector -> ROI -> landmarks -> affine
// stage on the GPU (include/vsf.h), producing the post chain's per-frame
// vss_face_frame inputs in HBM.
//
// Per face frame (stream index % interval == 0), on the caller's stream:
//   k_face_letterbox : toSquareLetterbox (frameProcessorTest.ts:613-642) of the
//                      frame into the detector's S x S input, /255, NCHW.  The
//                      draw rectangle is resampled with the seam's tfjs-legacy
//                      bilinear (the same arithmetic as k_prep); outside it 0.
//   detector session : vso_run_device (MediaPipeFaceDetector.onnx).
//   k_face_decode    : runFaceDetector's first-best argmax over box_scores and
//                      the box mapped back by mapFromSquareToSrc and clamped
//                      (:408-452); cropFaceROI's rectangle (:451-473).
//   k_face_roi       : preprocessToNCHW (:357-391) of the ROI sub-image to the
//                      landmark input (the same bilinear), /255, NCHW.
//   landmark session : vso_run_device (MediaPipeFaceLandmarkDetector.onnx).
//   k_face_affine    : runLandmarks468's point scaling (:491-500) and
//                      estimateAffineFromLandmarks (:505-563).
// then once per call:
//   k_face_scan      : main.ts:76-94 in stream order: frame t gets lastAffine
//                      as it stood before t, and its own detection box; a new
//                      matrix is blended into lastAffine by WARP_GAIN.
// Geometry is JS-number arithmetic: doubles, no FMA contraction, Math.round
// / floor / ceil as JS defines them.  Nothing crosses to the host.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/vsf.h"

namespace vsf {

// decode record of one face frame (vsf_inspect what = 6)
enum {
  D_HAS_DET, D_SCORE, D_X0, D_Y0, D_X1, D_Y1, D_RX0, D_RY0, D_RW, D_RH, D_HAS_M,
  D_A11, D_A12, D_TX, D_A21, D_A22, D_TY, D_COUNT
};

struct Geometry {  // host-computed toSquareLetterbox geometry (JS doubles)
  double scale;
  int draw_w, draw_h, off_x, off_y;
};

// one bilinear sample of the tfjs-legacy resize of an (h x w) u8 image to a
// grid with ratios (ry, rx), output pixel (y, x), /255 — k_prep's arithmetic
// (vss_kernels.hip prep_tap/prep_finish; oracle/vss_oracle.c resize_px).
__device__ __forceinline__ void bilinear3(const uint8_t* __restrict__ f, long rs, int fc, int h, int w, float ry,
                                          float rx, int y, int x, float out[3]) {
#pragma clang fp contract(off)
  const float fy = (float)y * ry, fx = (float)x * rx;
  const int y0 = (int)floorf(fmaxf(fy, 0.f)), x0 = (int)floorf(fmaxf(fx, 0.f));
  const int y1 = min(h - 1, (int)ceilf(fy)), x1 = min(w - 1, (int)ceilf(fx));
  const float dy = fy - (float)y0, dx = fx - (float)x0;
  const uint8_t* r0 = f + (long)y0 * rs;
  const uint8_t* r1 = f + (long)y1 * rs;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float tl = r0[x0 * fc + c], tr = r0[x1 * fc + c], bl = r1[x0 * fc + c], br = r1[x1 * fc + c];
    const float top = __builtin_fmaf(tr - tl, dx, tl);
    const float bot = __builtin_fmaf(br - bl, dx, bl);
    out[c] = __builtin_fmaf(bot - top, dy, top) / 255.0f;
  }
}

struct LetterboxParams {
  const uint8_t* frame;
  long rs;
  int fc, h, w;
  int S;  // square side
  int draw_w, draw_h, off_x, off_y;
  float ry, rx;  // h / draw_h, w / draw_w
  float* out;    // [3][S][S]
};

__global__ __launch_bounds__(256) void k_face_letterbox(LetterboxParams p) {
  const int plane = p.S * p.S;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= plane) return;
  const int y = i / p.S, x = i - y * p.S;
  const int ly = y - p.off_y, lx = x - p.off_x;
  float v[3] = {0.f, 0.f, 0.f};
  if (ly >= 0 && ly < p.draw_h && lx >= 0 && lx < p.draw_w)
    bilinear3(p.frame, p.rs, p.fc, p.h, p.w, p.ry, p.rx, ly, lx, v);
  p.out[i] = v[0];
  p.out[plane + i] = v[1];
  p.out[2 * plane + i] = v[2];
}

struct DecodeParams {
  const float* coords;  // [A][cd]
  const float* scores;  // [A]
  int A, cd;
  int S;                // detector side (FD_INPUT)
  double scale;         // letterbox geometry
  int off_x, off_y;
  int w, h;             // video size
  double thresh, pad;
  double* det;          // [D_COUNT]
};

__device__ __forceinline__ double js_min(double a, double b) { return (a != a || b != b) ? NAN : (a < b ? a : b); }
__device__ __forceinline__ double js_max(double a, double b) { return (a != a || b != b) ? NAN : (a > b ? a : b); }

__global__ __launch_bounds__(256) void k_face_decode(DecodeParams p) {
#pragma clang fp contract(off)
  __shared__ float s_best[256];
  __shared__ int s_idx[256];
  // per thread: the first maximum of its strided subset (strict >, as the
  // reference's loop: a NaN never wins, -Infinity never beats the start)
  float best = -INFINITY;
  int idx = -1;
  for (int i = threadIdx.x; i < p.A; i += 256) {
    const float s = p.scores[i];
    if (s > best) { best = s; idx = i; }
  }
  s_best[threadIdx.x] = best;
  s_idx[threadIdx.x] = idx;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (threadIdx.x < off) {
      const float b = s_best[threadIdx.x + off];
      const int bi = s_idx[threadIdx.x + off];
      const int ai = s_idx[threadIdx.x];
      // the earliest index among the maxima == the sequential scan's answer
      if (bi >= 0 && (ai < 0 || b > s_best[threadIdx.x] || (b == s_best[threadIdx.x] && bi < ai))) {
        s_best[threadIdx.x] = b;
        s_idx[threadIdx.x] = bi;
      }
    }
    __syncthreads();
  }
  if (threadIdx.x != 0) return;
  double* d = p.det;
  for (int k = 0; k < D_COUNT; ++k) d[k] = 0.0;
  const int bi = s_idx[0];
  if (bi < 0) return;
  const double score = (double)s_best[0];
  const float* c = p.coords + (long)bi * p.cd;
  // p_letterbox = coords * FD_INPUT (:434-435); mapFromSquareToSrc (:638-641)
  const double S = (double)p.S;
  const double px0 = ((double)c[0] * S - (double)p.off_x) / p.scale;
  const double py0 = ((double)c[1] * S - (double)p.off_y) / p.scale;
  const double px1 = ((double)c[2] * S - (double)p.off_x) / p.scale;
  const double py1 = ((double)c[3] * S - (double)p.off_y) / p.scale;
  const double x0 = js_max(0.0, js_min((double)p.w, px0));
  const double y0 = js_max(0.0, js_min((double)p.h, py0));
  const double x1 = js_max(0.0, js_min((double)p.w, px1));
  const double y1 = js_max(0.0, js_min((double)p.h, py1));
  // :445 (a NaN box — only from NaN model outputs — is treated as no detection)
  if (!(x1 > x0) || !(y1 > y0)) return;
  d[D_HAS_DET] = 1.0;
  d[D_SCORE] = score;
  d[D_X0] = x0; d[D_Y0] = y0; d[D_X1] = x1; d[D_Y1] = y1;
  if (!(score >= p.thresh)) return;  // :134 — no prior, no ROI, no landmarks
  // cropFaceROI (:452-460)
  const double bw = x1 - x0, bh = y1 - y0;
  const double padX = bw * p.pad, padY = bh * p.pad;
  const double rx0 = fmax(0.0, floor(x0 - padX));
  const double ry0 = fmax(0.0, floor(y0 - padY));
  const double rx1 = fmin((double)p.w, ceil(x1 + padX));
  const double ry1 = fmin((double)p.h, ceil(y1 + padY));
  d[D_RX0] = rx0;
  d[D_RY0] = ry0;
  d[D_RW] = fmax(1.0, rx1 - rx0);
  d[D_RH] = fmax(1.0, ry1 - ry0);
}

struct RoiParams {
  const uint8_t* frame;
  long rs;
  int fc;
  const double* det;
  int LH, LW;
  float* out;  // [3][LH][LW]
};

__global__ __launch_bounds__(256) void k_face_roi(RoiParams p) {
  const int plane = p.LH * p.LW;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= plane) return;
  float v[3] = {0.f, 0.f, 0.f};
  if (p.det[D_RW] > 0.0) {  // a box at or above the threshold
    const int rx0 = (int)p.det[D_RX0], ry0 = (int)p.det[D_RY0];
    const int rw = (int)p.det[D_RW], rh = (int)p.det[D_RH];
    const float ry = (float)((double)rh / (double)p.LH), rx = (float)((double)rw / (double)p.LW);
    const int y = i / p.LW, x = i - y * p.LW;
    bilinear3(p.frame + (long)ry0 * p.rs + (long)rx0 * p.fc, p.rs, p.fc, rh, rw, ry, rx, y, x, v);
  }
  p.out[i] = v[0];
  p.out[plane + i] = v[1];
  p.out[2 * plane + i] = v[2];
}

struct AffineParams {
  const float* lm_scores;  // scores[0]
  const float* lm;         // [num][dim]
  int num, dim;
  double lthresh;
  int w, h;                // video
  int mask_w, mask_h;
  double* det;
};

__global__ void k_face_affine(AffineParams p) {
#pragma clang fp contract(off)
  if (threadIdx.x != 0) return;
  double* d = p.det;
  if (!(d[D_RW] > 0.0)) return;
  const double score = (double)p.lm_scores[0];
  if (!(score >= p.lthresh)) return;  // :143
  if (p.num < 300) return;            // :513
  const double rw = d[D_RW], rh = d[D_RH], rx0 = d[D_RX0], ry0 = d[D_RY0];
  const int idxs[5] = {33, 263, 1, 13, 14};
  const double refx[5] = {0.35, 0.65, 0.50, 0.58, 0.42};
  const double refy[5] = {0.4, 0.4, 0.55, 0.70, 0.70};
  double dx[5], dy[5], rxv[5], ryv[5];
  for (int k = 0; k < 5; ++k) {
    // runLandmarks468 (:494-498): ROI pixels; transformToFull (:471): + x0, y0
    const float* q = p.lm + (long)idxs[k] * p.dim;
    dx[k] = (double)q[0] * rw + rx0;
    dy[k] = (double)q[1] * rh + ry0;
    rxv[k] = refx[k] * (double)p.w;
    ryv[k] = refy[k] * (double)p.h;
  }
  // avg / sum (:565-572): left-to-right from 0
  double s;
  s = 0; for (int k = 0; k < 5; ++k) s += rxv[k]; const double cxRef = s / 5;
  s = 0; for (int k = 0; k < 5; ++k) s += ryv[k]; const double cyRef = s / 5;
  s = 0; for (int k = 0; k < 5; ++k) s += dx[k]; const double cxDst = s / 5;
  s = 0; for (int k = 0; k < 5; ++k) s += dy[k]; const double cyDst = s / 5;
  double rcx[5], rcy[5], dcx[5], dcy[5];
  for (int k = 0; k < 5; ++k) {
    rcx[k] = rxv[k] - cxRef; rcy[k] = ryv[k] - cyRef;
    dcx[k] = dx[k] - cxDst; dcy[k] = dy[k] - cyDst;
  }
  double refNormSum = 0, dstNormSum = 0, Sxx = 0, Sxy = 0;
  for (int k = 0; k < 5; ++k) refNormSum += rcx[k] * rcx[k] + rcy[k] * rcy[k];
  for (int k = 0; k < 5; ++k) dstNormSum += dcx[k] * dcx[k] + dcy[k] * dcy[k];
  if (refNormSum < 1e-6 || dstNormSum < 1e-6) return;  // :546
  for (int k = 0; k < 5; ++k) Sxx += rcx[k] * dcx[k] + rcy[k] * dcy[k];
  for (int k = 0; k < 5; ++k) Sxy += -rcy[k] * dcx[k] + rcx[k] * dcy[k];
  const double theta = atan2(Sxy, Sxx);
  const double cosT = cos(theta), sinT = sin(theta);
  const double sc = sqrt(dstNormSum / refNormSum);
  const double tx = cxDst - (sc * (cosT * cxRef - sinT * cyRef));
  const double ty = cyDst - (sc * (sinT * cxRef + cosT * cyRef));
  const double sx = (double)p.mask_w / (double)p.w, sy = (double)p.mask_h / (double)p.h;
  d[D_A11] = sc * cosT;
  d[D_A12] = -sc * sinT;
  d[D_TX] = tx * sx;
  d[D_A21] = sc * sinT;
  d[D_A22] = sc * cosT;
  d[D_TY] = ty * sy;
  d[D_HAS_M] = 1.0;
}

struct ScanParams {
  const double* dets;  // [k][D_COUNT], the face frames of this call in order
  double* state;       // [7]: has, a11, a12, tx, a21, a22, ty (lastAffine)
  vss_face_frame* out; // [n]
  int n;
  long long base;      // stream index of frame 0
  int interval;
  double gain;
  int w, h;
};

__global__ void k_face_scan(ScanParams p) {
#pragma clang fp contract(off)
  if (threadIdx.x != 0) return;
  double st[7];
  for (int k = 0; k < 7; ++k) st[k] = p.state[k];
  int slot = 0;
  for (int t = 0; t < p.n; ++t) {
    vss_face_frame f;
    memset(&f, 0, sizeof f);  // padding too: the output bytes are deterministic
    f.has_affine = st[0] != 0.0;
    for (int k = 0; k < 6; ++k) f.affine[k] = f.has_affine ? st[1 + k] : 0.0;
    f.has_box = 0;
    for (int k = 0; k < 4; ++k) f.box[k] = 0.0;
    f.video_w = p.w;
    f.video_h = p.h;
    if ((p.base + t) % p.interval == 0) {
      const double* d = p.dets + (long)slot * D_COUNT;
      ++slot;
      if (d[D_RW] > 0.0) {  // detection at or above FACE_SCORE_THRESH
        f.has_box = 1;
        f.box[0] = d[D_X0]; f.box[1] = d[D_Y0]; f.box[2] = d[D_X1]; f.box[3] = d[D_Y1];
      }
      if (d[D_HAS_M] != 0.0) {  // main.ts:77-89
        for (int k = 0; k < 6; ++k) {
          const double m = d[D_A11 + k];
          st[1 + k] = st[0] != 0.0 ? st[1 + k] * (1 - p.gain) + m * p.gain : m;
        }
        st[0] = 1.0;
      }
    }
    p.out[t] = f;
  }
  for (int k = 0; k < 7; ++k) p.state[k] = st[k];
}

}  // namespace vsf

using namespace vsf;

struct vsf_tracker {
  vso_session* det = nullptr;
  vso_session* lmk = nullptr;
  vsf_config cfg{};
  int device = 0;
  std::string err;
  int S = 0;             // detector input side
  int LH = 0, LW = 0;    // landmark input
  int A = 0, cd = 0;     // anchors, coords per anchor
  int out_coords = 0, out_scores = 0, n_det_out = 0;
  int out_lscore = 0, out_lm = 0, n_lmk_out = 0;
  long lscore_numel = 0;
  int lm_num = 0, lm_dim = 0;
  std::vector<long> det_out_numel, lmk_out_numel;
  long long frame_idx = 0;
  double* d_state = nullptr;
  // per face-slot arena
  int slots = 0;
  long slot_floats = 0;
  float* arena = nullptr;
  double* d_dets = nullptr;
  std::vector<float*> scratch;  // extra detector/landmark outputs (unused by the stage)
  int last_k = 0;
  long long last_base = 0;
  hipStream_t stream = nullptr;
  uint8_t* stage_frames = nullptr;  // vsf_track staging
  size_t stage_frames_cap = 0;
  vss_face_frame* stage_faces = nullptr;
  int stage_faces_cap = 0;
  bool busy = false;
  // slot layout (floats)
  long o_det_in = 0, o_coords = 0, o_scores = 0, o_lmk_in = 0, o_lscore = 0, o_lm = 0;
};

namespace {

thread_local std::string g_err;

int fail(vsf_tracker* t, int code, const std::string& msg) {
  (t ? t->err : g_err) = msg;
  return code;
}

#define VSF_HIP(t, x)                                                                     \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess)                                                                 \
      return fail((t), e_ == hipErrorOutOfMemory ? VSS_E_OOM : VSS_E_HIP,                 \
                  std::string(#x) + ": " + hipGetErrorString(e_));                         \
  } while (0)

long numel(const int64_t* d, int r) {
  long n = 1;
  for (int i = 0; i < r; ++i) n *= (long)d[i];
  return n;
}

int find_output(vso_session* s, const char* name, int n_out) {
  char buf[256];
  for (int i = 0; i < n_out; ++i)
    if (vso_output_name(s, i, buf, sizeof buf) >= 0 && std::strcmp(buf, name) == 0) return i;
  return -1;
}

double js_round(double x) {  // Math.round: nearest, ties toward +infinity
  const double f = std::floor(x);
  return x - f >= 0.5 ? f + 1.0 : f;
}

Geometry letterbox(int S, int w, int h) {
  // toSquareLetterbox :614-619
  Geometry g;
  g.scale = std::fmin((double)S / w, (double)S / h);
  g.draw_w = (int)std::fmax(1.0, js_round((double)w * g.scale));
  g.draw_h = (int)std::fmax(1.0, js_round((double)h * g.scale));
  g.off_x = (int)std::floor((double)(S - g.draw_w) / 2);
  g.off_y = (int)std::floor((double)(S - g.draw_h) / 2);
  return g;
}

int ensure_slots(vsf_tracker* t, int k) {
  if (k <= t->slots) return 0;
  VSF_HIP(t, hipDeviceSynchronize());  // earlier calls' kernels may still use the old arena
  if (t->arena) (void)hipFree(t->arena);
  if (t->d_dets) (void)hipFree(t->d_dets);
  t->arena = nullptr;
  t->d_dets = nullptr;
  t->slots = 0;
  VSF_HIP(t, hipMalloc(&t->arena, (size_t)k * t->slot_floats * sizeof(float)));
  VSF_HIP(t, hipMalloc(&t->d_dets, (size_t)k * D_COUNT * sizeof(double)));
  t->slots = k;
  return 0;
}

}  // namespace

extern "C" {

void vsf_config_default(vsf_config* c) {
  if (!c) return;
  c->interval = 6;
  c->warp_gain = 0.7;
  c->face_score_thresh = 0.6;
  c->landmark_score_thresh = 0.3;
  c->roi_pad = 0.25;
}

const char* vsf_last_error(const vsf_tracker* t) { return t ? t->err.c_str() : g_err.c_str(); }

int vsf_create(vso_session* detector, vso_session* landmarks, const vsf_config* cfg, int device_id,
               vsf_tracker** out) {
  if (!out) return fail(nullptr, VSS_E_INVALID_ARG, "out is NULL");
  *out = nullptr;
  if (!detector || !landmarks) return fail(nullptr, VSS_E_INVALID_ARG, "detector and landmark sessions required");
  vsf_config c;
  vsf_config_default(&c);
  if (cfg) c = *cfg;
  if (c.interval < 1) return fail(nullptr, VSS_E_INVALID_ARG, "interval must be >= 1");
  auto* t = new vsf_tracker();
  t->det = detector;
  t->lmk = landmarks;
  t->cfg = c;
  t->device = device_id;
  int ni = 0, no = 0;
  int64_t d[8];
  auto bad = [&](const std::string& m) {
    delete t;
    return fail(nullptr, VSS_E_INVALID_ARG, m);
  };
  // detector: image [1,3,S,S] -> box_coords [1,A,cd>=4], box_scores [1,A,1]
  if (vso_io_count(detector, &ni, &no) != 0 || ni != 1) return bad("detector: expected one input");
  if (vso_input_shape(detector, 0, d, 8) != 4 || d[0] != 1 || d[1] != 3 || d[2] != d[3] || d[2] < 1)
    return bad("detector: input must be [1,3,S,S]");
  t->S = (int)d[2];
  t->n_det_out = no;
  t->out_coords = find_output(detector, "box_coords", no);
  t->out_scores = find_output(detector, "box_scores", no);
  if (t->out_coords < 0 || t->out_scores < 0) return bad("detector: outputs box_coords and box_scores required");
  int r = vso_output_shape(detector, t->out_coords, d, 8);
  if (r != 3 || d[0] != 1 || d[2] < 4) return bad("detector: box_coords must be [1,A,>=4]");
  t->A = (int)d[1];
  t->cd = (int)d[2];
  r = vso_output_shape(detector, t->out_scores, d, 8);
  if (r < 2 || d[0] != 1 || d[1] != t->A || numel(d, r) != t->A) return bad("detector: box_scores must be [1,A,1]");
  for (int i = 0; i < no; ++i) {
    r = vso_output_shape(detector, i, d, 8);
    t->det_out_numel.push_back(numel(d, r));
  }
  // landmarks: image [1,3,LH,LW] -> scores [1], landmarks [1,num>=300,dim>=2]
  if (vso_io_count(landmarks, &ni, &no) != 0 || ni != 1) return bad("landmarks: expected one input");
  if (vso_input_shape(landmarks, 0, d, 8) != 4 || d[0] != 1 || d[1] != 3 || d[2] < 1 || d[3] < 1)
    return bad("landmarks: input must be [1,3,H,W]");
  t->LH = (int)d[2];
  t->LW = (int)d[3];
  t->n_lmk_out = no;
  t->out_lscore = find_output(landmarks, "scores", no);
  t->out_lm = find_output(landmarks, "landmarks", no);
  if (t->out_lscore < 0 || t->out_lm < 0) return bad("landmarks: outputs scores and landmarks required");
  r = vso_output_shape(landmarks, t->out_lscore, d, 8);
  t->lscore_numel = numel(d, r);
  if (t->lscore_numel < 1) return bad("landmarks: empty scores");
  r = vso_output_shape(landmarks, t->out_lm, d, 8);
  if (r != 3 || d[0] != 1 || d[2] < 2) return bad("landmarks: landmarks must be [1,N,>=2]");
  t->lm_num = (int)d[1];
  t->lm_dim = (int)d[2];
  if (t->lm_num < 264) return bad("landmarks: fewer than 264 points (index 263 is an anchor)");
  for (int i = 0; i < no; ++i) {
    r = vso_output_shape(landmarks, i, d, 8);
    t->lmk_out_numel.push_back(numel(d, r));
  }
  auto r4 = [](long n) { return (n + 3) & ~3L; };
  long o = 0;
  t->o_det_in = o; o += r4(3L * t->S * t->S);
  t->o_coords = o; o += r4((long)t->A * t->cd);
  t->o_scores = o; o += r4(t->A);
  t->o_lmk_in = o; o += r4(3L * t->LH * t->LW);
  t->o_lscore = o; o += r4(t->lscore_numel);
  t->o_lm = o; o += r4((long)t->lm_num * t->lm_dim);
  t->slot_floats = o;
  if (hipSetDevice(device_id) != hipSuccess) return bad("hipSetDevice failed");
  hipError_t e = hipStreamCreateWithFlags(&t->stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipMalloc(&t->d_state, 7 * sizeof(double));
  if (e == hipSuccess) e = hipMemset(t->d_state, 0, 7 * sizeof(double));
  // outputs the stage does not read still need somewhere to go
  for (int i = 0; e == hipSuccess && i < t->n_det_out; ++i)
    if (i != t->out_coords && i != t->out_scores) {
      float* p = nullptr;
      e = hipMalloc(&p, (size_t)t->det_out_numel[i] * 4);
      t->scratch.push_back(p);
    }
  for (int i = 0; e == hipSuccess && i < t->n_lmk_out; ++i)
    if (i != t->out_lscore && i != t->out_lm) {
      float* p = nullptr;
      e = hipMalloc(&p, (size_t)t->lmk_out_numel[i] * 4);
      t->scratch.push_back(p);
    }
  if (e != hipSuccess) {
    vsf_destroy(t);
    return fail(nullptr, VSS_E_HIP, std::string("vsf_create: ") + hipGetErrorString(e));
  }
  *out = t;
  return VSS_OK;
}

void vsf_destroy(vsf_tracker* t) {
  if (!t) return;
  (void)hipSetDevice(t->device);
  if (t->stream) (void)hipStreamSynchronize(t->stream);
  if (t->arena) (void)hipFree(t->arena);
  if (t->d_dets) (void)hipFree(t->d_dets);
  if (t->d_state) (void)hipFree(t->d_state);
  for (float* p : t->scratch) (void)hipFree(p);
  if (t->stage_frames) (void)hipFree(t->stage_frames);
  if (t->stage_faces) (void)hipFree(t->stage_faces);
  if (t->stream) (void)hipStreamDestroy(t->stream);
  delete t;
}

int vsf_reset(vsf_tracker* t) {
  if (!t) return fail(nullptr, VSS_E_INVALID_ARG, "null tracker");
  VSF_HIP(t, hipSetDevice(t->device));
  VSF_HIP(t, hipMemset(t->d_state, 0, 7 * sizeof(double)));
  t->frame_idx = 0;
  return VSS_OK;
}

int vsf_track_device(vsf_tracker* t, const uint8_t* d_frames, int n, int h, int w, int c, size_t rs, size_t fs,
                     int mask_w, int mask_h, vss_face_frame* d_faces, void* stream) {
  if (!t) return fail(nullptr, VSS_E_INVALID_ARG, "null tracker");
  if (t->busy) return fail(t, VSS_E_BUSY, "a call is already in flight on this tracker");
  if (n < 0 || (n > 0 && (!d_frames || !d_faces)) || h < 1 || w < 1 || (c != 3 && c != 4) ||
      rs < (size_t)w * c || (n > 1 && fs < rs * (size_t)h) || mask_w < 1 || mask_h < 1)
    return fail(t, VSS_E_INVALID_ARG, "bad frames / mask geometry");
  if (n == 0) return VSS_OK;
  struct Busy {
    bool& b;
    explicit Busy(bool& x) : b(x) { b = true; }
    ~Busy() { b = false; }
  } busy(t->busy);
  VSF_HIP(t, hipSetDevice(t->device));
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int iv = t->cfg.interval;
  // face frames of this call: stream indices base + i with (base + i) % iv == 0
  const long long base = t->frame_idx;
  const int first = (int)((iv - base % iv) % iv);
  const int k = first < n ? (n - 1 - first) / iv + 1 : 0;
  if (int rc = ensure_slots(t, k)) return rc;
  const Geometry g = letterbox(t->S, w, h);
  std::vector<float*> det_outs(t->n_det_out), lmk_outs(t->n_lmk_out);
  for (int s = 0; s < k; ++s) {
    const int f = first + s * iv;
    const uint8_t* frame = d_frames + (size_t)f * fs;
    float* slot = t->arena + (long)s * t->slot_floats;
    double* det = t->d_dets + (long)s * D_COUNT;
    LetterboxParams lp{frame, (long)rs, c, h, w, t->S, g.draw_w, g.draw_h, g.off_x, g.off_y,
                       (float)((double)h / g.draw_h), (float)((double)w / g.draw_w), slot + t->o_det_in};
    hipLaunchKernelGGL(k_face_letterbox, dim3((t->S * t->S + 255) / 256), dim3(256), 0, st, lp);
    VSF_HIP(t, hipGetLastError());
    int sc = 0;
    for (int i = 0; i < t->n_det_out; ++i)
      det_outs[i] = i == t->out_coords ? slot + t->o_coords : i == t->out_scores ? slot + t->o_scores
                                                                                 : t->scratch[sc++];
    const float* din = slot + t->o_det_in;
    if (vso_run_device(t->det, &din, det_outs.data(), st) != 0)
      return fail(t, VSS_E_HIP, std::string("detector: ") + vso_last_error(t->det));
    DecodeParams dp{slot + t->o_coords, slot + t->o_scores, t->A, t->cd, t->S, g.scale, g.off_x, g.off_y,
                    w, h, t->cfg.face_score_thresh, t->cfg.roi_pad, det};
    hipLaunchKernelGGL(k_face_decode, dim3(1), dim3(256), 0, st, dp);
    VSF_HIP(t, hipGetLastError());
    RoiParams rp{frame, (long)rs, c, det, t->LH, t->LW, slot + t->o_lmk_in};
    hipLaunchKernelGGL(k_face_roi, dim3((t->LH * t->LW + 255) / 256), dim3(256), 0, st, rp);
    VSF_HIP(t, hipGetLastError());
    for (int i = 0; i < t->n_lmk_out; ++i)
      lmk_outs[i] = i == t->out_lscore ? slot + t->o_lscore : i == t->out_lm ? slot + t->o_lm : t->scratch[sc++];
    const float* lin = slot + t->o_lmk_in;
    if (vso_run_device(t->lmk, &lin, lmk_outs.data(), st) != 0)
      return fail(t, VSS_E_HIP, std::string("landmarks: ") + vso_last_error(t->lmk));
    AffineParams ap{slot + t->o_lscore, slot + t->o_lm, t->lm_num, t->lm_dim, t->cfg.landmark_score_thresh,
                    w, h, mask_w, mask_h, det};
    hipLaunchKernelGGL(k_face_affine, dim3(1), dim3(64), 0, st, ap);
    VSF_HIP(t, hipGetLastError());
  }
  ScanParams sp{t->d_dets, t->d_state, d_faces, n, base, iv, t->cfg.warp_gain, w, h};
  hipLaunchKernelGGL(k_face_scan, dim3(1), dim3(64), 0, st, sp);
  VSF_HIP(t, hipGetLastError());
  t->frame_idx = base + n;
  t->last_k = k;
  t->last_base = base + first;
  return VSS_OK;
}

int vsf_track(vsf_tracker* t, const uint8_t* frames, int n, int h, int w, int c, size_t rs, int mask_w,
              int mask_h, vss_face_frame* faces) {
  if (!t) return fail(nullptr, VSS_E_INVALID_ARG, "null tracker");
  if (n < 0 || (n > 0 && (!frames || !faces)) || h < 1 || w < 1 || (c != 3 && c != 4) || rs < (size_t)w * c)
    return fail(t, VSS_E_INVALID_ARG, "bad frames");
  if (n == 0) return VSS_OK;
  VSF_HIP(t, hipSetDevice(t->device));
  const size_t fbytes = rs * (size_t)h * n;
  if (fbytes > t->stage_frames_cap) {
    if (t->stage_frames) (void)hipFree(t->stage_frames);
    t->stage_frames = nullptr;
    t->stage_frames_cap = 0;
    VSF_HIP(t, hipMalloc(&t->stage_frames, fbytes));
    t->stage_frames_cap = fbytes;
  }
  if (n > t->stage_faces_cap) {
    if (t->stage_faces) (void)hipFree(t->stage_faces);
    t->stage_faces = nullptr;
    t->stage_faces_cap = 0;
    VSF_HIP(t, hipMalloc(&t->stage_faces, (size_t)n * sizeof(vss_face_frame)));
    t->stage_faces_cap = n;
  }
  VSF_HIP(t, hipMemcpyAsync(t->stage_frames, frames, fbytes, hipMemcpyHostToDevice, t->stream));
  if (int rc = vsf_track_device(t, t->stage_frames, n, h, w, c, rs, rs * (size_t)h, mask_w, mask_h, t->stage_faces,
                                t->stream))
    return rc;
  VSF_HIP(t, hipMemcpyAsync(faces, t->stage_faces, (size_t)n * sizeof(vss_face_frame), hipMemcpyDeviceToHost,
                            t->stream));
  VSF_HIP(t, hipStreamSynchronize(t->stream));
  return VSS_OK;
}

int vsf_last_face_count(const vsf_tracker* t) { return t ? t->last_k : VSS_E_INVALID_ARG; }

int vsf_inspect(vsf_tracker* t, int k, int what, void* out, int cap, long long* frame_index) {
  if (!t) return fail(nullptr, VSS_E_INVALID_ARG, "null tracker");
  if (k < 0 || k >= t->last_k || what < 0 || what > 6 || cap < 0 || (cap > 0 && !out))
    return fail(t, VSS_E_INVALID_ARG, "bad face slot / field");
  VSF_HIP(t, hipSetDevice(t->device));
  VSF_HIP(t, hipDeviceSynchronize());
  if (frame_index) *frame_index = t->last_base + (long long)k * t->cfg.interval;
  const float* slot = t->arena + (long)k * t->slot_floats;
  const void* src;
  long count;
  size_t esz = 4;
  switch (what) {
    case 0: src = slot + t->o_det_in; count = 3L * t->S * t->S; break;
    case 1: src = slot + t->o_coords; count = (long)t->A * t->cd; break;
    case 2: src = slot + t->o_scores; count = t->A; break;
    case 3: src = slot + t->o_lmk_in; count = 3L * t->LH * t->LW; break;
    case 4: src = slot + t->o_lscore; count = t->lscore_numel; break;
    case 5: src = slot + t->o_lm; count = (long)t->lm_num * t->lm_dim; break;
    default: src = t->d_dets + (long)k * D_COUNT; count = D_COUNT; esz = 8; break;
  }
  const long m = count < cap ? count : cap;
  if (m > 0) VSF_HIP(t, hipMemcpy(out, src, (size_t)m * esz, hipMemcpyDeviceToHost));
  return (int)count;
}

}  // extern "C"
