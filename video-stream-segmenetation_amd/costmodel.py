"""Algorithmic bytes and FLOPs of each kernel of the forward.

Per launch = per-frame compulsory bytes x frames + the layer's weights once.
Compulsory bytes are the kernel's HBM-side inputs and outputs only: the fused
kernels never write the expanded (hidden) tensor, the resized model input x0
or the upsampled concat tile, so those are not counted (SURVEY §8(d) notes
fusion can push the naive unfused B_alg fraction past 1; this count is the
fused one, which is the stricter roofline).

Frame bytes: the tfjs-legacy resize touches only rows floor/ceil(y*inH/outH)
of the frame; the stem reads whole rows of those, so its compulsory frame
traffic is (distinct rows touched) x row bytes — at 480->144 that is 288 of
480 rows.  `frame_bytes_full` (H*W*C, the survey's count) is reported too.
"""
from __future__ import annotations

import math

import numpy as np

K_STEM, K_IR, K_DEC, K_HEAD = 1, 2, 3, 4
F_EXPAND, F_RESIDUAL = 1, 2
NAMES = {K_STEM: "stem", K_IR: "ir", K_DEC: "dec", K_HEAD: "head"}


def rows_touched(in_len: int, out_len: int) -> int:
    ratio = np.float32(in_len / out_len)
    f = np.arange(out_len, dtype=np.float32) * ratio
    lo = np.floor(np.maximum(f, 0)).astype(np.int64)
    hi = np.minimum(in_len - 1, np.ceil(f)).astype(np.int64)
    return int(np.unique(np.concatenate([lo, hi])).size)


def layer_costs(recs, hm: int, wm: int, fh: int, fw: int, fc: int = 3, pw_weight_bytes: int = 2):
    """List of dicts per layer: name, shape, bytes_per_frame, weight_bytes, flops_per_frame."""
    shapes = []
    out = []
    for i, r in enumerate(recs):
        kind, cin, chid, cout, stride, flags, src, skip = r[:8]
        d = {"layer": i, "kind": NAMES[kind]}
        if kind == K_STEM:
            H, W = hm // 2, wm // 2
            rows = rows_touched(fh, hm)
            d["frame_bytes"] = rows * fw * fc
            d["frame_bytes_full"] = fh * fw * fc
            d["bytes_per_frame"] = d["frame_bytes"] + H * W * cout * 4
            d["weight_bytes"] = (cout * 27 + cout) * 4
            d["flops_per_frame"] = 2 * H * W * cout * 27
        elif kind == K_IR:
            _, Hi, Wi = shapes[src]
            H, W = (Hi + 1) // 2, (Wi + 1) // 2 if stride == 2 else Wi
            if stride == 2:
                H, W = (Hi + 1) // 2, (Wi + 1) // 2
            else:
                H, W = Hi, Wi
            ch = chid if flags & F_EXPAND else cin
            d["bytes_per_frame"] = cin * Hi * Wi * 4 + cout * H * W * 4
            wb = (ch * 9 + ch + cout) * 4 + cout * ch * pw_weight_bytes
            fl = 2 * H * W * ch * 9 + 2 * H * W * ch * cout
            if flags & F_EXPAND:
                wb += ch * cin * pw_weight_bytes + ch * 4
                fl += 2 * Hi * Wi * cin * ch
            d["weight_bytes"] = wb
            d["flops_per_frame"] = fl
        elif kind == K_DEC:
            cl, Hi, Wi = shapes[src]
            cs, H, W = shapes[skip]
            cc = cl + cs
            d["bytes_per_frame"] = cl * Hi * Wi * 4 + cs * H * W * 4 + cout * H * W * 4
            d["weight_bytes"] = (cc * 10 + cout * 3) * 4 + cout * cc * pw_weight_bytes
            d["flops_per_frame"] = 2 * H * W * cc * 9 + 2 * H * W * cc * cout
        elif kind == K_HEAD:
            c, Hi, Wi = shapes[src]
            H, W, cout = hm, wm, 1
            d["bytes_per_frame"] = c * Hi * Wi * 4 + H * W * 4
            d["weight_bytes"] = (c + 1) * 4
            d["flops_per_frame"] = 2 * Hi * Wi * c * 2 + 8 * H * W
        shapes.append((cout, H, W))
        d["out_shape"] = (cout, H, W)
        out.append(d)
    return out


def launch_bytes(cost: dict, n: int) -> int:
    return n * cost["bytes_per_frame"] + cost["weight_bytes"]


def summary(recs, hm, wm, fh, fw, fc=3):
    c = layer_costs(recs, hm, wm, fh, fw, fc)
    return {
        "bytes_per_frame": sum(x["bytes_per_frame"] for x in c),
        "weight_bytes": sum(x["weight_bytes"] for x in c),
        "flops_per_frame": sum(x["flops_per_frame"] for x in c),
        "io_bytes_per_frame": c[0]["frame_bytes"] + hm * wm * 4,
    }


if __name__ == "__main__":
    import os
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(here, "model"))
    import make_weights as mw
    recs, _, _ = mw.parse_blob(open(mw.DEFAULT_BLOB, "rb").read())
    for x in layer_costs(recs, 144, 256, 480, 640):
        print(x)
    print(summary(recs, 144, 256, 480, 640))
    _ = math


def post_bytes(hm: int, wm: int, fh: int, fw: int, fc: int = 3, n: int = 8) -> dict:
    """Compulsory HBM bytes per frame of the post-processing chain (csrc/vss_post.hip)
    for n consecutive frames per call:
      k_post_ema    : seam mask read + EMA write (4+4 B/px) + the stream state
                      read and written once per call (8 B/px / n);
      k_post_filter : EMA read (4 B/px), the guide's frame rows (rows touched x
                      row bytes, as the stem), refinedAlpha f32 write + alpha u8
                      write (5 B/px)."""
    p = hm * wm
    frame = rows_touched(fh, hm) * fw * fc
    ema = 8 * p + 8 * p / n
    filt = 4 * p + frame + 5 * p
    return {"ema": ema, "filter": filt, "total": ema + filt, "frame": frame}
