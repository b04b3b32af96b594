"""Time the GPU ONNX sessions (include/vso.h) on the reference's two real
MediaPipe models (tests/golden/*.npz) and the MODNet-shaped synthetic net:
inputs and outputs resident in HBM, one vso_run_device (hipGraph replay) per
iteration, HIP events on the session's stream.  Prints one JSON line per model,
then one for the whole face stage (include/vsf.h: letterbox -> detector ->
decode -> ROI -> landmarks -> affine -> scan) on 640x480 frames in HBM, every
frame a face frame (interval 1), and its cost amortised over the reference's
LANDMARK_INTERVAL of 6.

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
    ap.add_argument("--full", default="288x512", help="the MODNet topology (onnx_models.modnet) at this size")
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--only-modnet", action="store_true")
    ap.add_argument("--cases", default="", help="comma-separated substrings: run only the cases whose name has one")
    args = ap.parse_args()
    import torch
    import bench
    bench._load_pkg()
    import vss_amd.ort as ort
    import onnx_models as M

    mh, mw = (int(v) for v in args.modnet.split("x"))
    fh, fw = (int(v) for v in args.full.split("x"))
    cases = []
    if not args.only_modnet:
        for key in ("mediapipe_face_detector", "mediapipe_face_landmarks"):
            model, feeds, _, _ = M.load_golden(os.path.join(ROOT, "tests", "golden", key + ".npz"))
            cases.append((key, model, None))
        cases.append((f"modnet_like_{mh}x{mw}", M.modnet_like(), (1, 3, mh, mw)))
    for q in (False, True):
        for prec in ("f32", "f16" if q else "bf16"):
            cases.append((f"modnet{'_q4f16' if q else ''}_{fh}x{fw}_b{args.batch}_{prec}", M.modnet(fh, fw, q4f16=q),
                          (args.batch, 3, fh, fw), prec))
    cases = [c if len(c) == 4 else c + ("f32",) for c in cases]
    if args.cases:
        keys = args.cases.split(",")
        cases = [c for c in cases if any(k in c[0] for k in keys)]
    for name, model, shape, prec in cases:
        with ort.InferenceSession(model, input_shape=shape, precision=prec) as s:
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
            frames = s.input_shapes[0][0]
            print(json.dumps({"model": name, "input": [list(x) for x in s.input_shapes], "ms_per_run": round(ms, 4),
                              "runs_per_s": round(1000.0 / ms, 1), "ms_per_frame": round(ms / frames, 4),
                              "launches": len(s.launches()),
                              "tile_convs": s.tile_convs()}), flush=True)
    if not args.only_modnet:
        face_stage(args, torch, ort, M)


def face_stage(args, torch, ort, M):
    import ctypes
    import vss_amd as pkg
    import vss_amd.face as face
    import vss_amd.synthetic as syn
    import numpy as np
    det = M.load_golden(os.path.join(ROOT, "tests", "golden", "mediapipe_face_detector.npz"))[0]
    lmk = M.load_golden(os.path.join(ROOT, "tests", "golden", "mediapipe_face_landmarks.npz"))[0]
    n, fh, fw = 8, 480, 640
    frames = np.stack([syn.make_frame(900 + t, fh, fw, 3) for t in range(n)])
    with ort.InferenceSession(det) as ds, ort.InferenceSession(lmk) as ls:
        tr = face.FaceTracker(ds, ls, interval=1)
        dfr = torch.from_numpy(frames).cuda()
        dfaces = torch.zeros(n * ctypes.sizeof(pkg.FaceFrame), dtype=torch.uint8, device="cuda")
        st = torch.cuda.Stream()

        def call():
            tr.track_device(dfr.data_ptr(), n, fh, fw, 3, fw * 3, fh * fw * 3, (256, 144), dfaces.data_ptr(),
                            st.cuda_stream)

        for _ in range(max(2, args.warmup // 4)):
            call()
        st.synchronize()
        iters = max(5, args.iters // 8)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(iters):
            call()
        e1.record(st)
        st.synchronize()
        ms = e0.elapsed_time(e1) / (iters * n)
        print(json.dumps({"model": "face_stage_mediapipe", "frame": [fh, fw], "ms_per_face_frame": round(ms, 4),
                          "face_frames_per_s": round(1000.0 / ms, 1),
                          "amortised_ms_per_frame_interval6": round(ms / 6, 4)}), flush=True)
        tr.close()


if __name__ == "__main__":
    main()
