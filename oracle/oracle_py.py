"""ctypes bindings for liboracle.so (the C restatement).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg — never by the product path.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P, I, Lg = ctypes.c_void_p, ctypes.c_int, ctypes.c_long
        L.vsso_preprocess.argtypes = [P, I, I, I, I, Lg, Lg, I, I, P]
        L.vsso_preprocess.restype = I
        L.vsso_forward.argtypes = [P, Lg, I, P, I, I, I, I, Lg, Lg, I, I, P, I, P]
        L.vsso_forward.restype = I
        L.vsso_layer_shapes.argtypes = [P, Lg, I, I, P, I]
        L.vsso_layer_shapes.restype = I
        L.vsso_post.argtypes = [P, I, I, I, P, I, I, I, Lg, Lg, P, P, P, P, P]
        L.vsso_post.restype = I
        L.vsso_post_guide.argtypes = [P, I, I, I, I, Lg, Lg, I, I, P]
        L.vsso_post_guide.restype = I
        L.vsso_composite.argtypes = [P, I, I, I, I, Lg, Lg, P, I, I, P]
        L.vsso_composite.restype = I
        L.vsso_post_face.argtypes = [P, I, I, I, P, I, I, I, Lg, Lg, P, P, P, P, P, P]
        L.vsso_post_face.restype = I
        L.vsso_upsample_mask.argtypes = [P, I, I, I, I, I, P]
        L.vsso_upsample_mask.restype = I
        L.vsso_bf16_round.argtypes = [ctypes.c_float]
        L.vsso_bf16_round.restype = ctypes.c_float
        _lib = L
    return _lib


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def preprocess(frames: np.ndarray, hm: int, wm: int) -> np.ndarray:
    """frames [N,H,W,C] uint8 (C = 3 or 4) -> [N,3,hm,wm] f32."""
    frames = np.ascontiguousarray(frames)
    n, h, w, c = frames.shape
    out = np.empty((n, 3, hm, wm), np.float32)
    rc = lib().vsso_preprocess(_ptr(frames), n, h, w, c, w * c, h * w * c, hm, wm, _ptr(out))
    if rc:
        raise ValueError(f"vsso_preprocess rc={rc}")
    return out


def layer_shapes(blob: bytes, hm: int, wm: int):
    buf = np.frombuffer(blob, np.uint8)
    chw = np.zeros(3 * 64, np.int32)
    nl = lib().vsso_layer_shapes(_ptr(buf), len(blob), hm, wm, _ptr(chw), 64)
    if nl < 0:
        raise ValueError("bad blob")
    return [tuple(int(v) for v in chw[3 * i:3 * i + 3]) for i in range(nl)]


def forward(blob: bytes, frames: np.ndarray, hm: int, wm: int, mode: int = 0,
            nthreads: int = 0, want_taps: bool = False):
    """Masks [N,hm,wm] f32 (and, with want_taps, per-frame per-layer planar outputs)."""
    frames = np.ascontiguousarray(frames)
    n, h, w, c = frames.shape
    buf = np.frombuffer(blob, np.uint8)
    masks = np.empty((n, hm, wm), np.float32)
    taps_arr = None
    taps_np = None
    if want_taps:
        shapes = layer_shapes(blob, hm, wm)
        nl = len(shapes)
        taps_np = [[np.empty(s, np.float32) for s in shapes] for _ in range(n)]
        taps_arr = (ctypes.c_void_p * (n * nl))(*[t.ctypes.data for fr in taps_np for t in fr])
    rc = lib().vsso_forward(_ptr(buf), len(blob), mode, _ptr(frames), n, h, w, c, w * c, h * w * c,
                            hm, wm, _ptr(masks), nthreads, taps_arr)
    if rc:
        raise ValueError(f"vsso_forward rc={rc}")
    return (masks, taps_np) if want_taps else masks


def bf16_round(x: float) -> float:
    return lib().vsso_bf16_round(x)


class PostConfig(ctypes.Structure):
    """Mirror of vsso_post_cfg; defaults = frameProcessorTest.ts:12-18."""
    _fields_ = [("ema", ctypes.c_double), ("noise_cutoff", ctypes.c_double), ("high_threshold", ctypes.c_double),
                ("gamma", ctypes.c_double), ("sigma_spatial", ctypes.c_double), ("sigma_range", ctypes.c_double),
                ("use_bilateral", ctypes.c_int)]

    @classmethod
    def default(cls):
        return cls(0.55, 0.06, 0.95, 0.4, 1.0, 12.0, 1)


def post_guide(frames: np.ndarray, h: int, w: int) -> np.ndarray:
    frames = np.ascontiguousarray(frames)
    n, fh, fw, c = frames.shape
    out = np.empty((n, h, w, 3), np.uint8)
    if lib().vsso_post_guide(_ptr(frames), n, fh, fw, c, fw * c, fh * fw * c, h, w, _ptr(out)):
        raise ValueError("vsso_post_guide")
    return out


class PostState:
    """prevAlpha of one video stream (frameProcessorTest.ts:47)."""

    def __init__(self, h: int, w: int):
        self.alpha = np.zeros((h, w), np.float32)
        self.valid = ctypes.c_int(0)


class Face(ctypes.Structure):
    """Mirror of vsso_face / vss_face_frame: one frame's face inputs."""
    _fields_ = [("has_affine", ctypes.c_int), ("affine", ctypes.c_double * 6), ("has_box", ctypes.c_int),
                ("box", ctypes.c_double * 4), ("video_w", ctypes.c_int), ("video_h", ctypes.c_int)]

    @classmethod
    def make(cls, affine=None, box=None, video_wh=(0, 0)):
        f = cls()
        if affine is not None:
            f.has_affine = 1
            f.affine[:] = [float(v) for v in affine]
        if box is not None:
            f.has_box = 1
            f.box[:] = [float(v) for v in box]
        f.video_w, f.video_h = video_wh
        return f


def post(masks: np.ndarray, frames: np.ndarray, state: PostState, cfg: PostConfig | None = None, faces=None):
    """(refined alpha [n][H][W] f32, alpha bytes [n][H][W] u8) for consecutive frames of one stream;
    faces: a list of n Face (the stabiliser's inputs) or None."""
    masks = np.ascontiguousarray(masks, np.float32)
    frames = np.ascontiguousarray(frames)
    n, H, W = masks.shape
    _, fh, fw, c = frames.shape
    cfg = cfg or PostConfig.default()
    a = np.empty((n, H, W), np.float32)
    u = np.empty((n, H, W), np.uint8)
    fa = (Face * n)(*faces) if faces is not None else None
    rc = lib().vsso_post_face(_ptr(masks), n, H, W, _ptr(frames), fh, fw, c, fw * c, fh * fw * c,
                              ctypes.byref(cfg), _ptr(state.alpha), ctypes.byref(state.valid), fa, _ptr(a), _ptr(u))
    if rc:
        raise ValueError(f"vsso_post rc={rc}")
    return a, u


def composite(frames: np.ndarray, alpha_u8: np.ndarray) -> np.ndarray:
    """frames [n,fh,fw,3|4] u8 + mask alpha bytes [n,H,W] u8 -> RGBA [n,fh,fw,4] u8
    (frameProcessorTest.ts:170-178 as defined in vss_oracle.c)."""
    frames = np.ascontiguousarray(frames)
    alpha_u8 = np.ascontiguousarray(alpha_u8, np.uint8)
    n, fh, fw, c = frames.shape
    _, H, W = alpha_u8.shape
    out = np.empty((n, fh, fw, 4), np.uint8)
    if lib().vsso_composite(_ptr(frames), n, fh, fw, c, fw * c, fh * fw * c, _ptr(alpha_u8), H, W, _ptr(out)):
        raise ValueError("vsso_composite")
    return out


def upsample_mask(masks: np.ndarray, fh: int, fw: int) -> np.ndarray:
    """VSS_OUT_FRAME's masks: [n][H][W] f32 -> [n][fh][fw] (vsso_upsample_mask)."""
    m = np.ascontiguousarray(masks, np.float32)
    n, H, W = m.shape
    out = np.empty((n, fh, fw), np.float32)
    if lib().vsso_upsample_mask(_ptr(m), n, H, W, fh, fw, _ptr(out)):
        raise ValueError("vsso_upsample_mask")
    return out
