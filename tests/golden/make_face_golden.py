"""Golden vectors for the face stage's geometry (§8(f) row 4), produced by THE
REFERENCE'S OWN CODE run under Node in this container.

Run from the repo root (needs /root/reference and node):
    python tests/golden/make_face_golden.py        (tests/golden/face_geom.npz)

Cut out of /root/reference/client/src/core/frameProcessorTest.ts as text at
generation time, their type annotations dropped (extract_fn / strip_body below:
signatures, `as` casts, typed declarations and arrow parameters, postfix `!`,
`??` for Node 12) and executed by Node:
    cropFaceROI :451-473, runLandmarks468 :475-503 (with preprocessToNCHW
    :357-391 feeding a stub session that returns the case's outputs),
    estimateAffineFromLandmarks :505-563, avg/sum :565-572 — chained as
    processFrame chains them (:139-150);
    toSquareLetterbox :613-642 (its mapFromSquareToSrc);
and from client/src/core/main.ts: WARP_GAIN :12 and the lastAffine update
:79-89.  The DOM they touch (canvas, 2-D context, ImageData) is stubbed with
objects that only carry sizes: the pixels never reach the numbers recorded.
No reference source is stored in this repository: only the vectors.
"""
from __future__ import annotations

import json
import os
import re
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/client/src/core/frameProcessorTest.ts"
MAIN = "/root/reference/client/src/core/main.ts"

OPEN, CLOSE = "({[<", ")}]>"


def _skip_type(t: str, i: int, stops: str) -> int:
    """Index of the first character at depth 0 in `stops` from i (a TS type
    expression: balanced (){}[]<>, `=>` arrows)."""
    depth = 0
    while i < len(t):
        ch = t[i]
        if ch == "=" and t[i + 1:i + 2] == ">":
            i += 2
            continue
        if depth == 0 and ch in stops:
            return i
        if ch in OPEN:
            depth += 1
        elif ch in CLOSE:
            depth -= 1
        i += 1
    return i


def _split_top(t: str):
    parts, depth, cur = [], 0, ""
    for k, ch in enumerate(t):
        if ch == "=" and t[k + 1:k + 2] == ">":
            cur += ch
            continue
        if ch in OPEN and not (ch == "<" and depth == 0 and "=" in cur):
            depth += 1
        elif ch in CLOSE and not (ch == ">" and t[k - 1:k] == "="):
            depth -= 1
        if ch == "," and depth == 0:
            parts.append(cur)
            cur = ""
        else:
            cur += ch
    if cur.strip():
        parts.append(cur)
    return parts


def extract_fn(src: str, name: str) -> str:
    """`[async] function name(...)[: ReturnType] {body}` of a TS source as
    plain JS: parameter and return annotations dropped, the body as written
    (see strip_body)."""
    i = src.index(f"function {name}(")
    is_async = src[max(0, i - 6):i] == "async "
    k = src.index("(", i)
    depth, j = 0, k
    while True:
        depth += {"(": 1, ")": -1}.get(src[j], 0)
        if depth == 0:
            break
        j += 1
    params = []
    for p in _split_top(src[k + 1:j]):
        p = p.strip()
        if not p:
            continue
        m = re.match(r"(\w+)\??", p)
        rest = p[m.end():].lstrip()
        if rest.startswith(":"):
            e = _skip_type(rest, 1, "=")
            rest = rest[e:]
        params.append(m.group(1) + (" " + rest.strip() if rest.strip() else ""))
    b = re.compile(r"\{[ \t]*\n").search(src, j)   # the body's brace ends its line
    depth = 0
    for e in range(b.start(), len(src)):
        depth += {"{": 1, "}": -1}.get(src[e], 0)
        if depth == 0:
            break
    body = src[b.start():e + 1]
    return ("async " if is_async else "") + f"function {name}({', '.join(params)}) " + strip_body(body)


def strip_body(t: str) -> str:
    """The TS-only syntax the face functions use: `x as T` casts, `decl: T =`
    annotations, typed arrow parameters, postfix `!`, and `a ?? b` (Node 12)."""
    t = re.sub(r"\s+as\s+[A-Za-z_][\w.]*(?:<[^>;]*>)?(?:\[\])*", "", t)
    t = re.sub(r"\)!(?=[\s;.,)])", ")", t)
    t = re.sub(r"(\([^()]*\)\[\d+\])\s*\?\?\s*([\w.]+)", r"__nc(\1, \2)", t)
    out, i = "", 0
    decl = re.compile(r"\b(const|let|var)\s+(\w+)\s*:")
    arrow = re.compile(r"\((\w+)\s*:")
    while True:
        m1, m2 = decl.search(t, i), arrow.search(t, i)
        ms = [m for m in (m1, m2) if m]
        if not ms:
            break
        m = min(ms, key=lambda m: m.start())
        if m is m1:
            e = _skip_type(t, m.end(), "=")
            out += t[i:m.start()] + f"{m.group(1)} {m.group(2)} "
        else:
            e = _skip_type(t, m.end(), ")")
            out += t[i:m.start()] + f"({m.group(1)}"
        i = e
    return out + t[i:]


FUNCS = ["preprocessToNCHW", "cropFaceROI", "runLandmarks468", "estimateAffineFromLandmarks", "avg", "sum",
         "toSquareLetterbox"]

STUBS = r"""
class ImageData { constructor(w, h) { this.width = w; this.height = h; this.data = new Uint8ClampedArray(w * h * 4); } }
const ctxStub = {
  createImageData: (w, h) => new ImageData(w, h),
  putImageData() {}, drawImage() {}, clearRect() {},
  getImageData: (x, y, w, h) => new ImageData(w, h),
};
const document = { createElement: () => ({ width: 0, height: 0, getContext: () => ctxStub }) };
const ort = { Tensor: class { constructor(t, d, dims) { this.type = t; this.data = d; this.dims = dims; } } };
const LMK_INPUT = [192, 192];
function __nc(a, b) { return a === undefined || a === null ? b : a; }
const faceCanvas = document.createElement('canvas');
const faceCtx = faceCanvas.getContext('2d', { willReadFrequently: true });
"""

DRIVER = r"""
const fs = require('fs');
const cases = JSON.parse(fs.readFileSync(process.argv[2], 'utf8'));
const lmBuf = fs.readFileSync(process.argv[3]);
(async () => {
  const out = { roi: [], affine: [], score: [], points: [], letterbox: [], blend: [] };
  for (const c of cases.affine) {
    const video = { videoWidth: c.video[0], videoHeight: c.video[1] };
    const box = { x0: c.box[0], y0: c.box[1], x1: c.box[2], y1: c.box[3] };
    const roi = cropFaceROI(video, box, 0.25);
    const o = roi.transformToFull({ x: 0, y: 0 });
    out.roi.push([o.x, o.y, roi.imageData.width, roi.imageData.height]);
    const lm = new Float32Array(lmBuf.buffer.slice(lmBuf.byteOffset + c.lm_off * 4,
                                                   lmBuf.byteOffset + (c.lm_off + c.num * 3) * 4));
    const session = { run: async () => ({ scores: { data: new Float32Array([c.score]), dims: [1] },
                                          landmarks: { data: lm, dims: [1, c.num, 3] } }) };
    const res = await runLandmarks468(roi.imageData, session);
    out.score.push(res.score);
    out.points.push([33, 263, 1, 13, 14].map(i => [res.points[i].x, res.points[i].y]));
    const M = res.score >= 0.3
      ? estimateAffineFromLandmarks(res.points, roi.transformToFull, c.mask[0], c.mask[1], c.video[0], c.video[1])
      : null;
    out.affine.push(M ? [M.a11, M.a12, M.tx, M.a21, M.a22, M.ty] : null);
  }
  for (const c of cases.letterbox) {
    const r = toSquareLetterbox(new ImageData(c.src[0], c.src[1]), c.target);
    out.letterbox.push(c.pts.map(p => { const q = r.mapFromSquareToSrc({ x: p[0], y: p[1] }); return [q.x, q.y]; }));
  }
  for (const c of cases.blend) {
    let lastAffine = c.last ? { a11: c.last[0], a12: c.last[1], tx: c.last[2], a21: c.last[3], a22: c.last[4],
                                ty: c.last[5] } : null;
    const timings = { updatedAffine: { a11: c.m[0], a12: c.m[1], tx: c.m[2], a21: c.m[3], a22: c.m[4], ty: c.m[5] } };
    __BLEND__
    out.blend.push([lastAffine.a11, lastAffine.a12, lastAffine.tx, lastAffine.a21, lastAffine.a22, lastAffine.ty]);
  }
  console.log(JSON.stringify(out));
})();
"""


def cases(seed=11):
    rng = np.random.default_rng(seed)
    aff, lms, off = [], [], 0
    videos = [(640, 480), (1280, 720), (160, 120), (480, 640)]
    masks = [(256, 144), (64, 48), (512, 288)]
    for k in range(24):
        vw, vh = videos[k % len(videos)]
        mw, mh = masks[k % len(masks)]
        x0 = float(rng.uniform(-20, vw * 0.7))
        y0 = float(rng.uniform(-20, vh * 0.7))
        bw, bh = float(rng.uniform(2, vw * 0.4)), float(rng.uniform(2, vh * 0.4))
        box = [max(0.0, x0), max(0.0, y0), min(float(vw), x0 + bw), min(float(vh), y0 + bh)]
        num = 468 if k != 5 else 299          # < 300 points -> null (:513)
        pts = rng.uniform(0, 1, (num, 3)).astype(np.float32)
        if k == 7:                            # all anchors on one point -> null (:546)
            for i in (33, 263, 1, 13, 14):
                pts[i] = pts[1]
        score = float(np.float32(rng.uniform(0.1, 1.0))) if k % 6 else 0.2   # below 0.3 -> no landmarks pass
        aff.append({"video": [vw, vh], "mask": [mw, mh], "box": box, "num": num, "score": score, "lm_off": off})
        lms.append(pts.ravel())
        off += pts.size
    lb = []
    for (w, h) in [(640, 480), (1280, 720), (480, 640), (160, 120), (257, 100), (1, 1), (100, 1000), (1920, 1080)]:
        p = (rng.uniform(0, 1, (6, 2)) * 256).astype(np.float32).astype(np.float64)
        lb.append({"src": [w, h], "target": 256, "pts": p.tolist()})
    bl = []
    for k in range(6):
        m = rng.standard_normal(6).tolist()
        bl.append({"last": None if k == 0 else rng.standard_normal(6).tolist(), "m": m})
    return {"affine": aff, "letterbox": lb, "blend": bl}, np.concatenate(lms).astype(np.float32)


def main():
    src = open(REF).read()
    funcs = "\n\n".join(extract_fn(src, f) for f in FUNCS)
    msrc = open(MAIN).read()
    gain = next(l for l in msrc.split("\n") if l.startswith("const WARP_GAIN"))
    i = msrc.index("lastAffine = lastAffine")
    j = msrc.index(": M;", i) + len(": M;")
    body = gain + "\n" + funcs
    blend = "const M = timings.updatedAffine;\n" + msrc[i:j]
    harness = STUBS + body + DRIVER.replace("__BLEND__", blend)
    cs, lm = cases()
    with tempfile.TemporaryDirectory() as td:
        js = os.path.join(td, "face.js")
        open(js, "w").write(harness)
        open(os.path.join(td, "c.json"), "w").write(json.dumps(cs))
        lm.tofile(os.path.join(td, "lm.bin"))
        out = subprocess.run(["node", js, os.path.join(td, "c.json"), os.path.join(td, "lm.bin")],
                             capture_output=True, text=True, check=True)
    res = json.loads(out.stdout.strip().splitlines()[-1])
    path = os.path.join(HERE, "face_geom.npz")
    has = np.array([a is not None for a in res["affine"]])
    np.savez_compressed(
        path, cases=np.array(json.dumps(cs)), landmarks=lm,
        roi=np.array(res["roi"], np.float64), score=np.array(res["score"], np.float64),
        points=np.array(res["points"], np.float64), has_affine=has,
        affine=np.array([a if a is not None else [0.0] * 6 for a in res["affine"]], np.float64),
        letterbox=np.array(res["letterbox"], np.float64), blend=np.array(res["blend"], np.float64))
    print(path, os.path.getsize(path), "bytes;", int(has.sum()), "of", len(has), "affines")


if __name__ == "__main__":
    main()
