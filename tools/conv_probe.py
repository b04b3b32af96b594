"""One dense convolution (Conv k x k + Relu, f32 NCHW in HBM) on the GPU ONNX
session (include/vso.h) at a given shape and operand precision: its run time
(HIP events on the session's stream, ITERS back-to-back runs), the planner's
tile, and the algorithmic rates — the probe behind MODNet's k_conv_tile work
(the 3x3 64-channel layers at 72x128, batch 8).

    python tools/conv_probe.py [--shape N,C,M,H,W] [--k 3] [--prec f16] [--iters 200]

Under `rocprofv3 --kernel-trace` or one `--pmc` pass the same command gives
the kernel's own numbers (every launch is the one convolution)."""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def model(N, C, M, H, W, k, s, up=0):
    """Conv + Relu on x; up > 0: the conv's first `up` channels are the 2x
    linear upsample (pytorch_half_pixel, MODNet's Resize) of lo [N, up, H/2,
    W/2], concatenated with x's C - up (the fusion branch's 35 -> 16 at
    288x512: --up 32 --shape 8,35,16,288,512)."""
    import numpy as np
    import onnx_models as OM
    b = OM.Builder(3)
    Ho, Wo = (H + s - 1) // s, (W + s - 1) // s
    if up:
        r = b.op("Resize", ["lo", "", b.const(np.array([1, 1, 2, 2], np.float32))], mode="linear",
                 coordinate_transformation_mode="pytorch_half_pixel")
        cat = b.op("Concat", [r, "x"], axis=1)
        y = b.op("Relu", [b.conv(cat, C, M, k, stride=s)])
        return b.model([("lo", [N, up, H // 2, W // 2]), ("x", [N, C - up, H, W])], [(y, [N, M, Ho, Wo])]), (Ho, Wo)
    y = b.op("Relu", [b.conv("x", C, M, k, stride=s)])
    return b.model([("x", [N, C, H, W])], [(y, [N, M, Ho, Wo])]), (Ho, Wo)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="8,64,64,72,128")
    ap.add_argument("--k", type=int, default=3)
    ap.add_argument("--s", type=int, default=1)
    ap.add_argument("--prec", default="f16")
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--up", type=int, default=0, help="channels upsampled 2x inside the conv (k_conv_tile_up)")
    a = ap.parse_args()
    N, C, M, H, W = (int(v) for v in a.shape.split(","))
    import torch
    import bench
    bench._load_pkg()
    import vss_amd.ort as ort
    mdl, (Ho, Wo) = model(N, C, M, H, W, a.k, a.s, a.up)
    with ort.InferenceSession(mdl, precision=a.prec) as s:
        din = [torch.rand(sh, dtype=torch.float32, device="cuda") for sh in s.input_shapes]
        dout = [torch.empty(sh, dtype=torch.float32, device="cuda") for sh in s.output_shapes]
        st = torch.cuda.Stream()
        ip, op = [t.data_ptr() for t in din], [t.data_ptr() for t in dout]
        for _ in range(a.warmup):
            s.run_device(ip, op, st.cuda_stream)
        st.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(a.iters):
            s.run_device(ip, op, st.cuda_stream)
        e1.record(st)
        st.synchronize()
        us = e0.elapsed_time(e1) / a.iters * 1e3
        flops = 2.0 * N * M * Ho * Wo * C * a.k * a.k
        byts = 4.0 * N * ((C - a.up) * H * W + a.up * (H // 2) * (W // 2) + M * Ho * Wo)
        print(json.dumps({"shape": [N, C, M, H, W], "k": a.k, "s": a.s, "prec": a.prec, "us_per_run": round(us, 2),
                          "TFLOPs": round(flops / us / 1e6, 1), "TBps": round(byts / us / 1e6, 3),
                          "alg_MB": round(byts / 1e6, 2), "launches": s.launches(), "tile_convs": s.tile_convs()}),
              flush=True)


if __name__ == "__main__":
    main()
