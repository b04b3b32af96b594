"""Experiment: throughput with S batches in flight (S independent handles, one
stream each, steps dealt round-robin) and a per-GPU batch sweep.

    python tools/exp_inflight.py [--steps 200]
"""
from __future__ import annotations

import argparse
import importlib.util
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "video-stream-segmenetation_amd")


def _load_pkg():
    spec = importlib.util.spec_from_file_location("vss_amd", os.path.join(PKG_DIR, "__init__.py"),
                                                  submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["vss_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


def run(pkg, torch, B, S, steps, warmup, fh=480, fw=640):
    import vss_amd.synthetic as syn
    dev = torch.device("cuda", 0)
    frames = syn.make_batch(B, fh, fw, 3)
    d_frames = torch.from_numpy(frames).to(dev)
    sess = [pkg.Session(max_batch=B, max_frame_h=fh, max_frame_w=fw) for _ in range(S)]
    masks = [torch.empty((B, 144 * 256), dtype=torch.float32, device=dev) for _ in range(S)]
    streams = [torch.cuda.Stream(device=dev) for _ in range(S)]
    rs, fs = fw * 3, fh * fw * 3

    def go(k):
        j = k % S
        sess[j].segment_device(d_frames.data_ptr(), B, fh, fw, 3, rs, fs, masks[j].data_ptr(), streams[j].cuda_stream)

    for k in range(warmup):
        go(k)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        go(k)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    ref = masks[0].cpu()
    same = all(torch.equal(m.cpu(), ref) for m in masks)
    for s in sess:
        s.close()
    return {"batch": B, "inflight": S, "fps": round(B * steps / el, 1), "us_per_step": round(el * 1e6 / steps, 2),
            "masks_equal": same}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--warmup", type=int, default=40)
    args = ap.parse_args()
    import torch
    pkg = _load_pkg()
    for B, S in [(8, 1), (8, 2), (8, 3), (8, 4), (16, 1), (16, 2), (32, 1), (32, 2), (64, 1)]:
        print(json.dumps(run(pkg, torch, B, S, args.steps, args.warmup)), flush=True)


if __name__ == "__main__":
    main()
