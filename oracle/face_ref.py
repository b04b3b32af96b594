"""CPU restatement of the face stage (include/vsf.h).

TEST INFRASTRUCTURE ONLY: imported by tests/ — never by the product path.

Follows /root/reference/client/src/core/frameProcessorTest.ts and main.ts:
  letterbox_geometry   toSquareLetterbox :613-619 (+ mapFromSquareToSrc :638-641)
  detector_input       toSquareLetterbox's canvas draw (:621-636) + the /255 NCHW
                       packing of preprocessToNCHW (:373-391); the canvas resample
                       is defined as the seam's tfjs-legacy bilinear (vsf.h)
  decode               runFaceDetector :408-452 (with the letterboxMap fix)
                       and cropFaceROI :451-460
  roi_input            cropFaceROI's crop (:462-466) + preprocessToNCHW (:357-391)
  estimate_affine      runLandmarks468's scaling :491-500, transformToFull :471,
                       estimateAffineFromLandmarks :505-563, avg/sum :565-572
  track                processFrame's face branch :125-150 on every
                       `interval`-th frame, main.ts:76-94's WARP_GAIN blend
JS numbers are Python floats (IEEE doubles, no fused multiply-add); model
outputs are float32 widened exactly.  The pure geometry is pinned against the
reference's own functions run under Node (tests/golden/face_geom.npz); the
canvas resample and the letterboxMap fix are this build's spec (vsf.h).
"""
from __future__ import annotations

import math

import numpy as np

import oracle_py

D_COUNT = 17
IDXS = (33, 263, 1, 13, 14)
REF_NORM = ((0.35, 0.4), (0.65, 0.4), (0.50, 0.55), (0.58, 0.70), (0.42, 0.70))


def js_round(x: float) -> float:
    f = math.floor(x)
    return f + 1.0 if x - f >= 0.5 else float(f)


def letterbox_geometry(S: int, w: int, h: int):
    """(scale, draw_w, draw_h, off_x, off_y) of toSquareLetterbox (:614-619)."""
    scale = min(S / w, S / h)
    dw = int(max(1.0, js_round(w * scale)))
    dh = int(max(1.0, js_round(h * scale)))
    return scale, dw, dh, math.floor((S - dw) / 2), math.floor((S - dh) / 2)


def map_from_square(geom, x: float, y: float):
    scale, _, _, ox, oy = geom
    return (x - ox) / scale, (y - oy) / scale


def detector_input(frame: np.ndarray, S: int) -> np.ndarray:
    """frame [H][W][C] u8 -> [1][3][S][S] f32."""
    h, w = frame.shape[:2]
    _, dw, dh, ox, oy = letterbox_geometry(S, w, h)
    out = np.zeros((1, 3, S, S), np.float32)
    out[0, :, oy:oy + dh, ox:ox + dw] = oracle_py.preprocess(frame[None], dh, dw)[0]
    return out


def _js_min(a, b):
    return math.nan if (a != a or b != b) else min(a, b)


def _js_max(a, b):
    return math.nan if (a != a or b != b) else max(a, b)


def crop_roi(x0, y0, x1, y1, w: int, h: int, pad=0.25):
    """cropFaceROI's rectangle (:452-460): (x0, y0, rw, rh)."""
    bw, bh = x1 - x0, y1 - y0
    padX, padY = bw * pad, bh * pad
    rx0 = max(0, math.floor(x0 - padX))
    ry0 = max(0, math.floor(y0 - padY))
    rx1 = min(w, math.ceil(x1 + padX))
    ry1 = min(h, math.ceil(y1 + padY))
    return rx0, ry0, max(1, rx1 - rx0), max(1, ry1 - ry0)


def decode(coords: np.ndarray, scores: np.ndarray, S: int, w: int, h: int, thresh=0.6, pad=0.25) -> np.ndarray:
    """box_coords [A][>=4], box_scores [A] -> the 17-double record of vsf_inspect(what=6)."""
    d = np.zeros(D_COUNT)
    coords = np.asarray(coords, np.float32).reshape(len(np.ravel(scores)), -1)
    scores = np.asarray(scores, np.float32).ravel()
    best, bi = -math.inf, -1
    for i in range(len(scores)):  # :416-423
        s = float(scores[i])
        if s > best:
            best, bi = s, i
    if bi < 0:
        return d
    geom = letterbox_geometry(S, w, h)
    c = [float(v) for v in coords[bi, :4]]
    p0 = map_from_square(geom, c[0] * S, c[1] * S)
    p1 = map_from_square(geom, c[2] * S, c[3] * S)
    x0 = _js_max(0.0, _js_min(float(w), p0[0]))
    y0 = _js_max(0.0, _js_min(float(h), p0[1]))
    x1 = _js_max(0.0, _js_min(float(w), p1[0]))
    y1 = _js_max(0.0, _js_min(float(h), p1[1]))
    if not (x1 > x0) or not (y1 > y0):
        return d
    d[0], d[1], d[2:6] = 1.0, best, (x0, y0, x1, y1)
    if not (best >= thresh):
        return d
    d[6:10] = crop_roi(x0, y0, x1, y1, w, h, pad)
    return d


def roi_input(frame: np.ndarray, d: np.ndarray, LH: int, LW: int) -> np.ndarray:
    """The landmark input [1][3][LH][LW] (zeros when the record has no ROI)."""
    if not d[8] > 0:
        return np.zeros((1, 3, LH, LW), np.float32)
    x0, y0, rw, rh = (int(v) for v in d[6:10])
    return oracle_py.preprocess(np.ascontiguousarray(frame[None, y0:y0 + rh, x0:x0 + rw]), LH, LW)


def procrustes(dst, w: int, h: int, mask_w: int, mask_h: int):
    """estimateAffineFromLandmarks (:526-563) on the 5 anchor points in video
    pixels -> (a11, a12, tx, a21, a22, ty) or None."""
    ref = [(rx * w, ry * h) for rx, ry in REF_NORM]

    def avg(v):
        s = 0.0
        for x in v:
            s += x
        return s / len(v)

    def sm(v):
        s = 0.0
        for x in v:
            s += x
        return s

    cxRef, cyRef = avg([p[0] for p in ref]), avg([p[1] for p in ref])
    cxDst, cyDst = avg([p[0] for p in dst]), avg([p[1] for p in dst])
    refC = [(p[0] - cxRef, p[1] - cyRef) for p in ref]
    dstC = [(p[0] - cxDst, p[1] - cyDst) for p in dst]
    refNormSum = sm([p[0] * p[0] + p[1] * p[1] for p in refC])
    dstNormSum = sm([p[0] * p[0] + p[1] * p[1] for p in dstC])
    if refNormSum < 1e-6 or dstNormSum < 1e-6:
        return None
    Sxx = sm([r[0] * q[0] + r[1] * q[1] for r, q in zip(refC, dstC)])
    Sxy = sm([-r[1] * q[0] + r[0] * q[1] for r, q in zip(refC, dstC)])
    theta = math.atan2(Sxy, Sxx)
    cosT, sinT = math.cos(theta), math.sin(theta)
    s = math.sqrt(dstNormSum / refNormSum)
    tx = cxDst - (s * (cosT * cxRef - sinT * cyRef))
    ty = cyDst - (s * (sinT * cxRef + cosT * cyRef))
    sx, sy = mask_w / w, mask_h / h
    return (s * cosT, -s * sinT, tx * sx, s * sinT, s * cosT, ty * sy)


def estimate_affine(d: np.ndarray, lm_score: float, lm: np.ndarray, w: int, h: int, mask_w: int, mask_h: int,
                    lthresh=0.3) -> np.ndarray:
    """Fills has_m and the matrix of a decode record from the landmark outputs."""
    d = d.copy()
    if not d[8] > 0 or not (float(lm_score) >= lthresh):
        return d
    lm = np.asarray(lm, np.float32).reshape(-1, np.asarray(lm).shape[-1])
    if len(lm) < 300:
        return d
    rx0, ry0, rw, rh = (float(v) for v in d[6:10])
    dst = [(float(lm[i, 0]) * rw + rx0, float(lm[i, 1]) * rh + ry0) for i in IDXS]
    m = procrustes(dst, w, h, mask_w, mask_h)
    if m is not None:
        d[10] = 1.0
        d[11:17] = m
    return d


def blend(last, m, gain=0.7):
    """main.ts:77-89."""
    if last is None:
        return tuple(float(v) for v in m)
    return tuple(float(a) * (1 - gain) + float(b) * gain for a, b in zip(last, m))


class State:
    def __init__(self):
        self.frame_idx = 0
        self.last = None


def scan(dets: dict, n: int, state: State, w: int, h: int, interval=6, gain=0.7):
    """Per-frame (affine or None, box or None) for n frames from the decode
    records of the face frames (dets: stream index -> record)."""
    out = []
    for t in range(n):
        g = state.frame_idx + t
        aff, box = state.last, None
        if g % interval == 0:
            d = dets[g]
            if d[8] > 0:
                box = tuple(float(v) for v in d[2:6])
            if d[10]:
                state.last = blend(state.last, d[11:17], gain)
        out.append((aff, box))
    state.frame_idx += n
    return out


def track(frames: np.ndarray, run_det, run_lmk, S: int, LH: int, LW: int, mask_w: int, mask_h: int, state: State,
          interval=6, gain=0.7, thresh=0.6, lthresh=0.3, pad=0.25):
    """The whole stage for n consecutive frames [n][H][W][C]; run_det(x) ->
    (coords [A][cd], scores [A]); run_lmk(x) -> (score, landmarks [N][D])."""
    n, h, w = frames.shape[:3]
    dets = {}
    for t in range(n):
        g = state.frame_idx + t
        if g % interval:
            continue
        coords, scores = run_det(detector_input(frames[t], S))
        d = decode(coords, scores, S, w, h, thresh, pad)
        if d[8] > 0:
            score, lm = run_lmk(roi_input(frames[t], d, LH, LW))
            d = estimate_affine(d, score, lm, w, h, mask_w, mask_h, lthresh)
        dets[g] = d
    return scan(dets, n, state, w, h, interval, gain), dets
