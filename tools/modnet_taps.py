"""Per-stage parity of the MODNet topology (tests/onnx_models.py modnet) on the
GPU session against the oracle with the same operand rounding: every stage
output (enc2x .. fu, the matte) made a graph output, the session run once in
the given precision, each stage's max / mean abs error printed against
onnx_ref.run(conv_operands=precision) and against the f32 oracle — where the
16-bit error first grows past the same-rounding bar names the kernel whose
rounding points differ from the oracle's.  Diagnostic only (a GPU run).

    python tools/modnet_taps.py [--precision bf16|f16] [--size 288x512]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--precision", default="bf16")
    ap.add_argument("--size", default="288x512")
    args = ap.parse_args()
    import bench
    bench._load_pkg()
    import vss_amd.ort as ort
    import onnx_models as M
    import onnx_ref as R

    h, w = (int(v) for v in args.size.split("x"))
    q4f16 = args.precision == "f16"
    taps = {}
    base = M.modnet(h, w, q4f16=q4f16, taps=taps)
    x = np.random.default_rng(21).random((1, 3, h, w), dtype=np.float32)
    names = list(taps)
    m0 = R.load(base)
    want32 = R.run(m0, {"input": x}, want=[taps[k] for k in names])
    elem = R.DT_FLOAT16 if q4f16 else R.DT_FLOAT
    export = [(taps[k], list(want32[taps[k]].shape), elem) for k in names]
    data = M.modnet(h, w, q4f16=q4f16, export=export)
    m = R.load(data)
    want16 = R.run(m, {"input": x}, want=[taps[k] for k in names], conv_operands=args.precision)
    fin32 = R.run(m, {"input": x})
    fin16 = R.run(m, {"input": x}, conv_operands=args.precision)
    with ort.InferenceSession(data, precision=args.precision) as s:
        got = s.run({"input": x})
        launches = s.launches()
    rows = []
    for k in names:
        v = taps[k]
        g = np.asarray(got[v], np.float32)
        a, b = np.asarray(want16[v], np.float32), np.asarray(want32[v], np.float32)
        rows.append({"stage": k, "shape": list(g.shape), "scale": round(float(np.abs(b).max()), 4),
                     "vs_same_rounding_max": float(np.abs(g - a).max()), "vs_same_rounding_mean": float(np.abs(g - a).mean()),
                     "vs_f32_max": float(np.abs(g - b).max()), "oracle_rounding_cost_max": float(np.abs(a - b).max())})
    for k in fin32:
        if k in got and k not in [taps[t] for t in names]:
            g = np.asarray(got[k], np.float32)
            rows.append({"stage": "matte", "vs_same_rounding_max": float(np.abs(g - fin16[k]).max()),
                         "vs_f32_max": float(np.abs(g - fin32[k]).max()),
                         "oracle_rounding_cost_max": float(np.abs(fin16[k] - fin32[k]).max())})
    for r in rows:
        print(json.dumps(r))
    print(json.dumps({"launches": len(launches)}))


if __name__ == "__main__":
    main()
