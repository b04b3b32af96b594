"""Workgroup timeline of the bench's steady state (several batches in flight)
from the trace build (lib/libvss_trace.so: every workgroup stamps
s_memrealtime at its start and end, and its HW_ID / XCC_ID).

    make -C video-stream-segmenetation_amd/csrc trace
    python tools/trace_inflight.py [--inflight 4] [--batch 8] [--steps 40]

Runs `steps` batches round-robin on the handle's slot streams (as bench.py),
then one more per slot, and reads every slot's stamps of that last forward.
Prints, per slot, each layer's span and the gap before it; per layer the mean
workgroup lifetime; over the window where all the final forwards overlap, the
resident workgroups per CU (time-averaged) and the fraction of CU-time with
no workgroup; and the hardware queue each slot's work came from."""
import argparse
import collections
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--inflight", type=int, default=4)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    os.environ.setdefault("VSS_LIBRARY", os.path.join(ROOT, "video-stream-segmenetation_amd", "lib",
                                                      "libvss_trace.so"))
    import torch
    from conftest import load_pkg
    pkg = load_pkg()
    import vss_amd.synthetic as syn
    L = pkg.lib()
    L.vss_trace_read_slot.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
    L.vss_trace_read_slot.restype = ctypes.c_int
    B, S = a.batch, a.inflight
    s = pkg.Session(max_batch=B, queue_depth=S, max_frame_h=480, max_frame_w=640)
    frames = syn.make_batch(B, 480, 640, 3)
    df = torch.from_numpy(frames).cuda()
    outs = [torch.empty((B, s.mask_h * s.mask_w), device="cuda") for _ in range(S)]
    streams = [torch.cuda.ExternalStream(s.slot_stream(k)) for k in range(S)]
    names = [s.layer_kernel(i) for i in range(s.n_layers)]
    s.prepare_device(B, 480, 640, 3, 640 * 3, 480 * 640 * 3)
    for i in range(a.steps + S):
        s.segment_device(df.data_ptr(), B, 480, 640, 3, 640 * 3, 480 * 640 * 3, outs[i % S].data_ptr(),
                         streams[i % S].cuda_stream)
    torch.cuda.synchronize()
    recs = []  # slot, layer, start, end, cu key, queue
    for k in range(S):
        for li in range(s.n_layers):
            buf = np.zeros((200000, 16), np.uint64)
            n = L.vss_trace_read_slot(s._h, k, li, buf.ctypes.data, buf.shape[0])
            for row in buf[:max(n, 0)].astype(np.int64):
                hw, xcc = int(row[7]), int(row[15])
                cu = (xcc & 15, (hw >> 13) & 7, (hw >> 12) & 1, (hw >> 8) & 15)
                recs.append((k, li, int(row[0]), int(row[3]), cu, (hw >> 24) & 7))
    t0 = min(r[2] for r in recs)
    tick = 0.01  # us per s_memrealtime tick (100 MHz)
    out = {"per_slot": {}, "per_layer": {}}
    print(f"batch {B}, {S} in flight; {len(recs)} workgroup records; times in us")
    win_lo, win_hi = 0, 1 << 62
    for k in range(S):
        rs = [r for r in recs if r[0] == k]
        lo, hi = min(r[2] for r in rs), max(r[3] for r in rs)
        win_lo, win_hi = max(win_lo, lo), min(win_hi, hi)
        qs = collections.Counter(r[5] for r in rs)
        line, prev = [], None
        for li in range(s.n_layers):
            lr = [r for r in rs if r[1] == li]
            if not lr:
                continue
            a0, a1 = min(r[2] for r in lr), max(r[3] for r in lr)
            gap = (a0 - prev) * tick if prev is not None else 0.0
            line.append((li, round((a0 - t0) * tick, 2), round((a1 - a0) * tick, 2), round(gap, 2)))
            prev = a1
        print(f"slot {k}: forward {((hi - lo) * tick):.1f} us, hw queues {dict(qs)}; (layer, start, span, gap): {line}")
        out["per_slot"][k] = {"forward_us": (hi - lo) * tick, "layers": line, "queues": dict(qs)}
    for li in range(s.n_layers):
        lr = [r for r in recs if r[1] == li]
        if lr:
            life = np.array([(r[3] - r[2]) * tick for r in lr])
            print(f"layer {li:2d}: {len(lr) // S:5d} wgs/forward, lifetime mean {life.mean():.2f} max {life.max():.2f} us  {names[li][:70]}")
            out["per_layer"][li] = {"wgs": len(lr) // S, "life_mean": life.mean(), "life_max": life.max()}
    # CU occupancy over the overlap window of the final forwards
    cus = sorted({r[4] for r in recs})
    if win_hi > win_lo:
        step = 10  # ticks (0.1 us)
        ts = np.arange(win_lo, win_hi, step)
        occ = np.zeros((len(cus), len(ts)), np.int32)
        idx = {c: i for i, c in enumerate(cus)}
        for r in recs:
            m = (ts >= r[2]) & (ts < r[3])
            occ[idx[r[4]]] += m
        print(f"overlap window {(win_hi - win_lo) * tick:.1f} us over {len(cus)} CUs seen: resident workgroups per CU "
              f"mean {occ.mean():.2f}, CU-time idle {float((occ == 0).mean()):.3f}; histogram "
              f"{dict(enumerate(np.bincount(occ.ravel(), minlength=6)[:8] / occ.size))}")
        out["window_us"] = (win_hi - win_lo) * tick
        out["occ_mean"] = float(occ.mean())
        out["idle_frac"] = float((occ == 0).mean())
    if a.json:
        json.dump(out, open(a.json, "w"), default=float)


if __name__ == "__main__":
    main()
