"""Synthetic webcam frames (SURVEY.md §8(d) "Synthetic inputs").

Frame i of a run is uint8 RGB HWC, packed (row stride = 3*W), drawn from numpy
PCG64 with seed 20251024 + i: uniform noise blended 50/50 with a horizontal
gradient as background, and a fixed-colour ellipse "head" over a rounded
rectangle "torso" as foreground so the mask has structure.  Stands in for
`tf.browser.fromPixels(videoElement)` (frameProcessorTest.ts:79) since there is
no camera on the GPU box.
"""
from __future__ import annotations

import numpy as np

BASE_SEED = 20251024


def make_frame(i: int, h: int = 480, w: int = 640, channels: int = 3) -> np.ndarray:
    rng = np.random.Generator(np.random.PCG64(BASE_SEED + i))
    noise = rng.integers(0, 256, size=(h, w, 3), dtype=np.uint16)
    grad = np.linspace(0.0, 255.0, w, dtype=np.float64)[None, :, None]
    img = 0.5 * noise + 0.5 * np.broadcast_to(grad, (h, w, 3))
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float64)
    # person placement jitters per frame so frames differ in structure too
    cx = w * (0.5 + 0.08 * (rng.random() - 0.5))
    hy = h * 0.33
    head = ((xx - cx) / (0.11 * w)) ** 2 + ((yy - hy) / (0.16 * h)) ** 2 <= 1.0
    tx0, tx1, ty0 = cx - 0.22 * w, cx + 0.22 * w, h * 0.52
    r = 0.06 * w
    qx = np.maximum(np.maximum(tx0 + r - xx, xx - (tx1 - r)), 0.0)
    qy = np.maximum(ty0 + r - yy, 0.0)
    torso = (qx ** 2 + qy ** 2 <= r * r) & (xx >= tx0) & (xx <= tx1) & (yy >= ty0)
    img[head] = (214.0, 160.0, 130.0)
    img[torso] = (40.0, 60.0, 150.0)
    out = np.clip(np.rint(img), 0, 255).astype(np.uint8)
    if channels == 4:
        out = np.concatenate([out, np.full((h, w, 1), 255, np.uint8)], axis=2)
    return np.ascontiguousarray(out)


def make_batch(n: int, h: int = 480, w: int = 640, channels: int = 3, start: int = 0) -> np.ndarray:
    return np.stack([make_frame(start + i, h, w, channels) for i in range(n)])
