"""Tile choice under the headline's concurrency (4 batches in flight).

vss_create's autotuner times each layer's compiled tiles alone (8 launches of
one layer back to back).  With four batches in flight, kernels of different
layers share the CUs, and a tile's LDS / wave footprint decides how well it
co-resides.  This tool starts from the autotuner's choice and runs one pass of
coordinate descent over the layers, timing the whole queued forward (frames
already in HBM, `inflight` streams) for every compiled tile of each layer in
turn (pinned with VSS_TILE); a tile is kept when it beats the current choice
by more than `--min-gain`.  Tile choice never changes results (the kernels are
tile-invariant, tests/test_gpu_parity.py), only speed.

  python tools/tune_inflight.py [--batch 8] [--inflight 4] [--steps 400]
prints one JSON line: the autotuned and the tuned VSS_TILE specs and frames/s.
"""
from __future__ import annotations

import argparse
import importlib.util
import json
import os
import re
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "video-stream-segmenetation_amd")


def load_pkg():
    spec = importlib.util.spec_from_file_location("vss_amd", os.path.join(PKG_DIR, "__init__.py"),
                                                  submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["vss_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


def chosen_tiles(sess):
    """layer -> (TH, TW) of the kernel the handle launches (k_block<M, S, TH, TW, ...>)."""
    out = {}
    for i in range(sess.n_layers):
        m = re.search(r"k_block<\s*\d+,\s*\d+,\s*(\d+),\s*(\d+),", sess.layer_kernel(i))
        if m:
            out[i] = (int(m.group(1)), int(m.group(2)))
    return out


def spec_of(tiles):
    return ",".join(f"{l}:{th}x{tw}" for l, (th, tw) in sorted(tiles.items()))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--inflight", type=int, default=4)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--min-gain", type=float, default=0.01)
    args = ap.parse_args()
    import torch

    pkg = load_pkg()
    import vss_amd.synthetic as syn

    dev = torch.device("cuda", 0)
    B, S, fh, fw = args.batch, args.inflight, 480, 640
    d = torch.from_numpy(syn.make_batch(B, fh, fw, 3)).to(dev)

    def measure(spec, autotune=False):
        if spec:
            os.environ["VSS_TILE"] = spec
        else:
            os.environ.pop("VSS_TILE", None)
        with pkg.Session(max_batch=B, max_frame_h=fh, max_frame_w=fw, queue_depth=S, autotune=autotune) as s:
            masks = [torch.empty((B, s.mask_h * s.mask_w), dtype=torch.float32, device=dev) for _ in range(S)]
            streams = [torch.cuda.Stream(device=dev) for _ in range(S)]

            def run(n):
                for i in range(n):
                    s.segment_device(d.data_ptr(), B, fh, fw, 3, fw * 3, fh * fw * 3, masks[i % S].data_ptr(),
                                     streams[i % S].cuda_stream)

            run(40)
            torch.cuda.synchronize(dev)
            best = 0.0
            for _ in range(args.reps):
                t0 = time.perf_counter()
                run(args.steps)
                torch.cuda.synchronize(dev)
                best = max(best, B * args.steps / (time.perf_counter() - t0))
            tiles = chosen_tiles(s)
            cands = {l: s.layer_tiles(l) for l in tiles}
        return best, tiles, cands

    base, tiles, cands = measure(None, autotune=True)
    auto_spec = spec_of(tiles)
    base, _, _ = measure(auto_spec)  # the same tiles, timed the way the trials are
    cur = base
    trials = []
    for layer in sorted(tiles):
        for t in cands[layer]:
            if t == tiles[layer]:
                continue
            trial = dict(tiles)
            trial[layer] = t
            v, _, _ = measure(spec_of(trial))
            trials.append({"layer": layer, "tile": f"{t[0]}x{t[1]}", "value": round(v, 1)})
            print(f"layer {layer} {t}: {v:.0f} (current {cur:.0f})", file=sys.stderr, flush=True)
            if v > cur * (1 + args.min_gain):
                tiles, cur = trial, v
    final, _, _ = measure(spec_of(tiles))
    again, _, _ = measure(auto_spec)
    print(json.dumps({"batch": B, "inflight": S, "autotuned": auto_spec, "autotuned_value": round(base, 1),
                      "autotuned_value_again": round(again, 1), "tuned": spec_of(tiles),
                      "tuned_value": round(final, 1), "trials": trials}))


if __name__ == "__main__":
    main()
