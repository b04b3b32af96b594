"""Time the GPU ONNX sessions (include/vso.h) on the reference's two real
MediaPipe models (tests/golden/*.npz) and the MODNet-shaped synthetic net:
inputs and outputs resident in HBM, one vso_run_device (hipGraph replay) per
iteration, HIP events on the session's stream.  Prints one JSON line per model.

    python tools/bench_onnx.py [--iters 200] [--modnet 256x256]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--modnet", default="256x256")
    args = ap.parse_args()
    import torch
    import bench
    bench._load_pkg()
    import vss_amd.ort as ort
    import onnx_models as M

    mh, mw = (int(v) for v in args.modnet.split("x"))
    cases = []
    for key in ("mediapipe_face_detector", "mediapipe_face_landmarks"):
        model, feeds, _, _ = M.load_golden(os.path.join(ROOT, "tests", "golden", key + ".npz"))
        cases.append((key, model, None))
    cases.append((f"modnet_like_{mh}x{mw}", M.modnet_like(), (1, 3, mh, mw)))
    for name, model, shape in cases:
        with ort.InferenceSession(model, input_shape=shape) as s:
            din = [torch.rand(sh, dtype=torch.float32, device="cuda") for sh in s.input_shapes]
            dout = [torch.empty(sh, dtype=torch.float32, device="cuda") for sh in s.output_shapes]
            st = torch.cuda.Stream()
            ip, op = [t.data_ptr() for t in din], [t.data_ptr() for t in dout]
            for _ in range(args.warmup):
                s.run_device(ip, op, st.cuda_stream)
            st.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(args.iters):
                s.run_device(ip, op, st.cuda_stream)
            e1.record(st)
            st.synchronize()
            ms = e0.elapsed_time(e1) / args.iters
            print(json.dumps({"model": name, "input": [list(x) for x in s.input_shapes], "ms_per_run": round(ms, 4),
                              "runs_per_s": round(1000.0 / ms, 1), "launches": len(s.launches())}), flush=True)


if __name__ == "__main__":
    main()
