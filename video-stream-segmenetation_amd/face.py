"""The GPU face stage (include/vsf.h): face detector ->
ROI -> 468 landmarks -> similarity affine, per `interval`-th frame, producing
the post chain's per-frame face inputs (FaceFrame) — the branch of processFrame
at /root/reference/client/src/core/frameProcessorTest.ts:125-150 plus the main
loop's lastAffine bookkeeping (client/src/core/main.ts:50-94):

    const det = await runFaceDetector(videoElement, opts.faceSession!);        # :133
    ... cropFaceROI / runLandmarks468 / estimateAffineFromLandmarks ...        # :139-150
    lastAffine = lastAffine ? blend(lastAffine, M, WARP_GAIN) : M;             # main.ts:79-89

becomes

    tracker = FaceTracker(detector_session, landmark_session)                  # vsf_create
    faces = tracker.track(frames, mask_wh=(256, 144))                          # -> [FaceFrame]
    post.set_faces(faces); post.process(...)

or, device-resident, tracker.track_device(...) -> post.set_faces_device(...).
Fails loudly without the HIP library: there is no CPU fallback.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import FaceFrame, VssError
from . import lib as _vss_lib

_bound = False
DECODE_FIELDS = ("has_det", "score", "x0", "y0", "x1", "y1", "roi_x0", "roi_y0", "roi_w", "roi_h", "has_m",
                 "a11", "a12", "tx", "a21", "a22", "ty")


class VsfConfig(ctypes.Structure):
    _fields_ = [("interval", ctypes.c_int), ("warp_gain", ctypes.c_double), ("face_score_thresh", ctypes.c_double),
                ("landmark_score_thresh", ctypes.c_double), ("roi_pad", ctypes.c_double)]


def lib():
    global _bound
    L = _vss_lib()
    if not _bound:
        P, I, S = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
        sig = {
            "vsf_config_default": ([ctypes.POINTER(VsfConfig)], None),
            "vsf_create": ([P, P, ctypes.POINTER(VsfConfig), I, ctypes.POINTER(P)], I),
            "vsf_destroy": ([P], None),
            "vsf_last_error": ([P], ctypes.c_char_p),
            "vsf_reset": ([P], I),
            "vsf_track_device": ([P, P, I, I, I, I, S, S, I, I, P, P], I),
            "vsf_track": ([P, P, I, I, I, I, S, I, I, P], I),
            "vsf_inspect": ([P, I, I, P, I, ctypes.POINTER(ctypes.c_longlong)], I),
            "vsf_last_face_count": ([P], I),
        }
        for name, (args, res) in sig.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = res
        _bound = True
    return L


def _check(rc, h=None):
    if rc < 0:
        msg = lib().vsf_last_error(h)
        raise VssError(rc, msg.decode() if msg else "")
    return rc


def default_config() -> VsfConfig:
    c = VsfConfig()
    lib().vsf_config_default(ctypes.byref(c))
    return c


class FaceTracker:
    """One video stream's face stage on one GPU, driving two ONNX sessions
    (ort.InferenceSession) of the reference's MediaPipe models."""

    def __init__(self, detector, landmarks, device_id: int = 0, **cfg):
        c = default_config()
        for k, v in cfg.items():
            if not hasattr(c, k):
                raise TypeError(f"unknown face-stage option {k!r}")
            setattr(c, k, v)
        self.config = c
        self._sessions = (detector, landmarks)  # keep them alive
        h = ctypes.c_void_p()
        _check(lib().vsf_create(detector._h, landmarks._h, ctypes.byref(c), device_id, ctypes.byref(h)))
        self._h = h

    def reset(self):
        _check(lib().vsf_reset(self._h), self._h)

    def track(self, frames: np.ndarray, mask_wh) -> list:
        """frames [n][H][W][C] u8 consecutive frames of the stream -> n FaceFrame."""
        f = np.ascontiguousarray(frames, np.uint8)
        if f.ndim != 4:
            raise ValueError("frames must be [n][H][W][C]")
        n, h, w, c = f.shape
        out = (FaceFrame * max(n, 1))()
        _check(lib().vsf_track(self._h, f.ctypes.data, n, h, w, c, w * c, int(mask_wh[0]), int(mask_wh[1]),
                               ctypes.cast(out, ctypes.c_void_p)), self._h)
        return list(out)[:n]

    def track_device(self, frames_ptr: int, n: int, h: int, w: int, c: int, row_stride: int, frame_stride: int,
                     mask_wh, faces_ptr: int, stream: int = 0):
        """Device pointers: frames (u8) -> faces (n vss_face_frame), on `stream`."""
        _check(lib().vsf_track_device(self._h, frames_ptr, n, h, w, c, row_stride, frame_stride, int(mask_wh[0]),
                                      int(mask_wh[1]), faces_ptr, stream or None), self._h)

    def last_face_count(self) -> int:
        return _check(lib().vsf_last_face_count(self._h), self._h)

    def inspect(self, k: int):
        """The last call's k-th face frame: (stream index, {field: array}) with
        the detector / landmark inputs and outputs and the decode record."""
        idx = ctypes.c_longlong()
        res = {}
        for what, name in enumerate(("det_in", "box_coords", "box_scores", "lmk_in", "lmk_scores", "landmarks",
                                     "decode")):
            cnt = _check(lib().vsf_inspect(self._h, k, what, None, 0, None), self._h)
            a = np.empty(cnt, np.float64 if what == 6 else np.float32)
            _check(lib().vsf_inspect(self._h, k, what, a.ctypes.data, cnt, ctypes.byref(idx)), self._h)
            res[name] = a
        return idx.value, res

    def close(self):
        if getattr(self, "_h", None):
            lib().vsf_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
