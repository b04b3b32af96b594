/*
 * vsf.h — C ABI of the GPU face stage: the face
 * detector -> ROI -> 468-landmark -> similarity-affine branch of processFrame
 * (/root/reference/client/src/core/frameProcessorTest.ts:125-150) and the main
 * loop's lastAffine bookkeeping (client/src/core/main.ts:50-94), producing the
 * per-frame vss_face_frame inputs of the post chain (vss.h) in device memory.
 *
 * The two networks run as vso sessions (vso.h) on the reference's own ONNX
 * files (client/src/assets/MediaPipeFaceDetector.onnx,
 * MediaPipeFaceLandmarkDetector.onnx).  Everything between and after them is
 * HIP kernels on the caller's stream, with no host round trip:
 *   1. the detector input: toSquareLetterbox (:613-642) of the frame into the
 *      detector's square input, /255, NCHW;
 *   2. runFaceDetector's decode (:408-452): the first best box_scores entry,
 *      its box_coords[0..3] * side mapped back by mapFromSquareToSrc (the
 *      `letterboxMap` the reference destructures from preprocessToNCHW but never
 *      gets, SURVEY.md §0.5: the branch is dead there; this is the fix) and
 *      clamped to the frame;
 *   3. cropFaceROI (:451-473) + preprocessToNCHW (:357-391) of the ROI to the
 *      landmark input;
 *   4. runLandmarks468's point scaling (:475-503) and
 *      estimateAffineFromLandmarks (:505-563);
 *   5. main.ts:76-94's blend of the new matrix into lastAffine (WARP_GAIN).
 * The browser canvas resamples of 1 and 3 are defined as the seam's own
 * tfjs-legacy bilinear of the frame (1: into the
 * letterbox's draw rectangle, 0 outside; 3: of the ROI sub-image).
 *
 * Schedule (main.ts:56-59, frameProcessorTest.ts:125-130): the stage runs on
 * the frames whose stream index is a multiple of `interval`; frame t's
 * has_affine/affine is lastAffine as it stood before frame t, its has_box/box
 * the detection on frame t (face frames with score >= face_score_thresh only).
 * The wall-clock gate L_MIN_MS and the in-flight flag (main.ts:11,56-59) are
 * timing artefacts of the browser loop and are not modelled.
 *
 * Errors: 0 or a negative VSS_E_* code, message in vsf_last_error(t)
 * (thread-local when t is NULL).  One call in flight per tracker; the tracker
 * drives its two sessions, which must not be run concurrently elsewhere.
 */
#ifndef VSF_H_
#define VSF_H_

#include "vso.h"
#include "vss.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct vsf_config {
  int interval;                 /* LANDMARK_INTERVAL, main.ts:10 (6) */
  double warp_gain;             /* WARP_GAIN, main.ts:12 (0.7) */
  double face_score_thresh;     /* FACE_SCORE_THRESH, frameProcessorTest.ts:35 (0.6) */
  double landmark_score_thresh; /* lm.score >= 0.3, :143 */
  double roi_pad;               /* cropFaceROI padRatio, :139 (0.25) */
} vsf_config;

typedef struct vsf_tracker vsf_tracker;

void vsf_config_default(vsf_config* cfg);

/* Binds a detector session (input [1,3,S,S]; outputs box_coords [1,A,>=4],
 * box_scores [1,A,1]) and a landmark session (input [1,3,LH,LW]; outputs scores
 * [1], landmarks [1,>=300,>=2]) — model.ts:36-67's initializeFaceDetector /
 * initializeLandmarks.  Both sessions must live on device_id; the tracker does
 * not own them. */
int vsf_create(vso_session* detector, vso_session* landmarks, const vsf_config* cfg, int device_id,
               vsf_tracker** out);
void vsf_destroy(vsf_tracker* t);
const char* vsf_last_error(const vsf_tracker* t);

/* frameIdx = 0 and lastAffine = null (a new stream). */
int vsf_reset(vsf_tracker* t);

/* n consecutive frames of the stream (device memory, RGB or RGBA u8) ->
 * d_faces[n] (device memory), ready for vss_post_set_faces_device.  mask_w/h =
 * the seam's mask size (estimateAffineFromLandmarks scales tx/ty to it).
 * Asynchronous on `stream`. */
int vsf_track_device(vsf_tracker* t, const uint8_t* d_frames, int n, int height, int width, int channels,
                     size_t row_stride, size_t frame_stride, int mask_w, int mask_h, vss_face_frame* d_faces,
                     void* stream);

/* Host-memory convenience (synchronous). */
int vsf_track(vsf_tracker* t, const uint8_t* frames, int n, int height, int width, int channels,
              size_t row_stride, int mask_w, int mask_h, vss_face_frame* faces);

/* Inspection of the last call's k-th face frame (0-based among the frames the
 * stage ran on; synchronous).  what: 0 detector input, 1 box_coords,
 * 2 box_scores, 3 landmark input, 4 landmark scores, 5 landmarks (f32 each),
 * 6 the decode as 17 doubles: has_det, score, x0, y0, x1, y1, roi_x0, roi_y0,
 * roi_w, roi_h, has_m, a11, a12, tx, a21, a22, ty.  Returns
 * the element count (copies min(count, cap)); the stream index of that frame
 * via *frame_index when non-NULL. */
int vsf_inspect(vsf_tracker* t, int k, int what, void* out, int cap, long long* frame_index);

/* Face frames the last call ran the stage on. */
int vsf_last_face_count(const vsf_tracker* t);

#ifdef __cplusplus
}
#endif

#endif /* VSF_H_ */
