"""Independent PyTorch-CPU functional restatement of the hot path.

TEST INFRASTRUCTURE ONLY (imported by tests/ and tests/golden/make_golden.py,
never by the product).  It cross-checks the C oracle (oracle/vss_oracle.c) with
library ops (F.conv2d with groups, F.interpolate align_corners=False,
instance-norm statistics from torch.var_mean) and generates the committed
golden vectors under tests/golden/.

Reference anchors (/root/reference):
  frameProcessorTest.ts:79-85  fromPixels -> resizeBilinear -> /255 -> NCHW
  frameProcessorTest.ts:91-97  session.run -> [1,1,H,W] -> squeeze -> (alphaRaw, maskW, maskH)
The network is the build-defined layer table (spec.json); see vss_oracle.c's
header for why its parity against the reference is unpinned.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

K_STEM, K_IR, K_DEC, K_HEAD = 1, 2, 3, 4
F_EXPAND, F_RESIDUAL = 1, 2
NONE = 0xFFFFFFFF


def resize_legacy_f64(img: np.ndarray, out_h: int, out_w: int) -> np.ndarray:
    """tfjs 4.22 CPU-backend resizeBilinear (alignCorners=false,
    halfPixelCenters=false) in float64, as its JS implementation computes it:
    srcFrac = r * (inH/outH); floor = max(0, floor(srcFrac));
    ceil = min(inH-1, ceil(srcFrac)); top/bottom lerp on columns, then rows.
    img: [H, W, C] uint8 -> [out_h, out_w, C] float64 (not yet /255)."""
    h, w, c = img.shape
    x = img.astype(np.float64)
    ry, rx = h / out_h, w / out_w
    fy = np.arange(out_h, dtype=np.float64) * ry
    fx = np.arange(out_w, dtype=np.float64) * rx
    y0 = np.maximum(0, np.floor(fy)).astype(np.int64)
    x0 = np.maximum(0, np.floor(fx)).astype(np.int64)
    y1 = np.minimum(h - 1, np.ceil(fy)).astype(np.int64)
    x1 = np.minimum(w - 1, np.ceil(fx)).astype(np.int64)
    dy = (fy - y0)[:, None, None]
    dx = (fx - x0)[None, :, None]
    tl, tr = x[y0][:, x0], x[y0][:, x1]
    bl, br = x[y1][:, x0], x[y1][:, x1]
    top = tl + (tr - tl) * dx
    bot = bl + (br - bl) * dx
    return top + (bot - top) * dy


def preprocess(frames: np.ndarray, hm: int, wm: int) -> torch.Tensor:
    """frames [N,H,W,C] uint8 -> [N,3,hm,wm] f32, WebGL-shader form (f32,
    ratio = float32(inH/outH)), i.e. the same formula the C oracle restates."""
    n, h, w, _ = frames.shape
    ry = np.float32(h / hm)
    rx = np.float32(w / wm)
    fy = torch.arange(hm, dtype=torch.float32) * float(ry)
    fx = torch.arange(wm, dtype=torch.float32) * float(rx)
    y0 = torch.floor(fy.clamp(min=0)).long()
    x0 = torch.floor(fx.clamp(min=0)).long()
    y1 = torch.ceil(fy).long().clamp(max=h - 1)
    x1 = torch.ceil(fx).long().clamp(max=w - 1)
    dy = (fy - y0.float()).view(1, hm, 1, 1)
    dx = (fx - x0.float()).view(1, 1, wm, 1)
    img = torch.from_numpy(np.ascontiguousarray(frames[..., :3])).float()
    tl = img[:, y0][:, :, x0]
    tr = img[:, y0][:, :, x1]
    bl = img[:, y1][:, :, x0]
    br = img[:, y1][:, :, x1]
    top = tl + (tr - tl) * dx
    bot = bl + (br - bl) * dx
    v = top + (bot - top) * dy
    return (v / 255.0).permute(0, 3, 1, 2).contiguous()


def parse_blob(blob: bytes):
    import struct
    magic, ver, nl, nf, eps_bits = struct.unpack_from("<5I", blob, 0)
    assert magic == 0x57535356 and ver == 1
    eps = struct.unpack("<f", struct.pack("<I", eps_bits))[0]
    recs = [list(struct.unpack_from("<16I", blob, 32 + 64 * i)) for i in range(nl)]
    data = torch.from_numpy(np.frombuffer(blob, dtype="<f4", count=nf, offset=32 + 64 * nl).copy())
    return recs, data, eps


def _r(x: torch.Tensor, mode: int) -> torch.Tensor:
    return x.to(torch.bfloat16).float() if mode else x


def forward(blob: bytes, frames: np.ndarray, hm: int, wm: int, mode: int = 0, taps: list | None = None):
    """Return masks [N, hm, wm] f32.  mode 1 mirrors spec.json's bf16 rounding points."""
    recs, data, eps = parse_blob(blob)

    def t(off, shape):
        n = int(np.prod(shape))
        return data[off:off + n].view(*shape)

    x0 = preprocess(frames, hm, wm)
    outs: list = [None] * len(recs)
    normed = [False] * len(recs)
    with torch.no_grad():
        for li, r in enumerate(recs):
            kind, cin, chid, cout, stride, flags, src, skip = r[:8]
            o = r[8:]
            if kind == K_STEM:
                y = F.conv2d(x0, t(o[0], (cout, 3, 3, 3)), t(o[1], (cout,)), stride=2, padding=1)
                y = _r(y.clamp(0, 6), mode)
            elif kind == K_IR:
                x = outs[src]
                h = x
                ch = cin
                if flags & F_EXPAND:
                    ch = chid
                    w1 = _r(t(o[0], (chid, cin, 1, 1)), mode)
                    h = _r(F.conv2d(x, w1, t(o[1], (chid,))).clamp(0, 6), mode)
                d = F.conv2d(h, t(o[2], (ch, 1, 3, 3)), t(o[3], (ch,)), stride=stride, padding=1, groups=ch)
                d = _r(d.clamp(0, 6), mode)
                w2 = _r(t(o[4], (cout, ch, 1, 1)), mode)
                y = F.conv2d(d, w2, t(o[5], (cout,)))
                if flags & F_RESIDUAL:
                    y = y + x
                y = _r(y, mode)
            elif kind == K_DEC:
                a = outs[src]
                if normed[src]:
                    a = _norm_relu(a, recs[src], t, eps)
                u = _r(F.interpolate(a, scale_factor=2, mode="bilinear", align_corners=False), mode)
                c = torch.cat([u, outs[skip]], dim=1)
                cc = cin + chid
                d = _r(F.conv2d(c, t(o[2], (cc, 1, 3, 3)), t(o[3], (cc,)), padding=1, groups=cc), mode)
                w2 = _r(t(o[4], (cout, cc, 1, 1)), mode)
                y = _r(F.conv2d(d, w2, t(o[5], (cout,))), mode)
                normed[li] = True
            elif kind == K_HEAD:
                a = outs[src]
                if normed[src]:
                    a = _norm_relu(a, recs[src], t, eps)
                z = F.conv2d(a, t(o[4], (1, cin, 1, 1)), t(o[5], (1,)))
                u = F.interpolate(z, scale_factor=2, mode="bilinear", align_corners=False)
                y = torch.sigmoid(u)
            else:
                raise ValueError(kind)
            outs[li] = y
            if taps is not None:
                taps.append(y.clone())
    return outs[-1][:, 0].contiguous()


def _norm_relu(a: torch.Tensor, rec, t, eps: float) -> torch.Tensor:
    cout = rec[3]
    g = t(rec[8 + 6], (cout,)).double().view(1, -1, 1, 1)
    b = t(rec[8 + 7], (cout,)).double().view(1, -1, 1, 1)
    ad = a.double()
    var, mean = torch.var_mean(ad, dim=(2, 3), keepdim=True, unbiased=False)
    y = (ad - mean) / torch.sqrt(var + eps) * g + b
    return y.clamp(min=0).float()
