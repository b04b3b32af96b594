"""Per-workgroup phase timeline of one forward (trace build, lib/libvss_trace.so).

    make -C video-stream-segmenetation_amd/csrc trace
    VSS_LIBRARY=video-stream-segmenetation_amd/lib/libvss_trace.so python tools/trace_phases.py [--batch 8]

Thread 0 of every workgroup stamps s_memrealtime (100 MHz) at: 0 start,
1 prologue committed (weights + input tile in LDS), 2 main loop done, 3 end,
4 every prologue load landed, 5 decoder src norm ready, 6 every load issued.
For each layer prints: kernel span (first start -> last end), start skew,
mean/max prologue, main and epilogue, mean workgroup duration, and the gap
to the previous layer's last end.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, nargs="+", default=[1, 8, 32])
    ap.add_argument("--dtype", default="bf16x2")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    os.environ.setdefault("VSS_LIBRARY", os.path.join(ROOT, "video-stream-segmenetation_amd", "lib",
                                                      "libvss_trace.so"))
    import torch
    from conftest import load_pkg
    pkg = load_pkg()
    import vss_amd.synthetic as syn
    L = pkg.lib()
    L.vss_trace_read.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
    L.vss_trace_read.restype = ctypes.c_int
    out = {}
    s = pkg.Session(dtype=a.dtype, max_batch=max(a.batch))
    names = [s.layer_kernel(i) for i in range(s.n_layers)]
    for n in a.batch:
        frames = np.stack([syn.make_frame(i, 480, 640, 3) for i in range(n)])
        df = torch.from_numpy(frames).cuda()
        dm = torch.empty((n, s.mask_h, s.mask_w), dtype=torch.float32, device="cuda")
        st = torch.cuda.current_stream().cuda_stream
        rows = []
        for rep in range(a.reps):
            s.segment_device(df.data_ptr(), n, 480, 640, 3, 640 * 3, 480 * 640 * 3, dm.data_ptr(), st)
        torch.cuda.synchronize()
        stamps = []
        for i in range(s.n_layers):
            buf = np.zeros((200000, 16), np.uint64)
            k = L.vss_trace_read(s._h, i, buf.ctypes.data, buf.shape[0])
            stamps.append(buf[:k].astype(np.int64))
        t0 = min(int(x[:, 0].min()) for x in stamps if len(x))
        prev_end = None
        print(f"\n== batch {n} ({a.dtype}); times in us (s_memrealtime 10 ns ticks)")
        print(f"{'layer':>5} {'wgs':>5} {'span':>6} {'gap':>5} {'skew':>5} {'pro':>5} {'proMx':>5} {'main':>5} "
              f"{'mainMx':>6} {'epi':>5} {'wg':>5} {'iss':>5} {'land':>5} {'norm':>5} {'MHz':>5}  kernel")
        for i, x in enumerate(stamps):
            if not len(x):  # fused into its consumer (the stem with VSS_FUSE_STEM)
                print(f"{i:>5}     - (fused into layer {i + 1})")
                continue
            us = (x - t0) / 100.0
            span = us[:, 3].max() - us[:, 0].min()
            gap = (us[:, 0].min() - prev_end) if prev_end is not None else 0.0
            prev_end = us[:, 3].max()
            pro, main, epi = us[:, 1] - us[:, 0], us[:, 2] - us[:, 1], us[:, 3] - us[:, 2]
            has = lambda k: bool((x[:, k] > 0).all())
            iss = (us[:, 6] - us[:, 0]).mean() if has(6) else float("nan")
            land = (us[:, 4] - us[:, 0]).mean() if has(4) else float("nan")
            nrm = (us[:, 5] - us[:, 4]).mean() if has(5) and has(4) else float("nan")
            # core clock: shader cycles / 10-ns ticks between start and end
            mhz = float(np.median((x[:, 11] - x[:, 8]) / np.maximum(x[:, 3] - x[:, 0], 1))) * 100.0
            row = dict(layer=i, wgs=len(x), span=span, gap=gap, skew=us[:, 0].max() - us[:, 0].min(),
                       issue=iss, landed=land, norm=nrm, mhz=mhz,
                       pro=pro.mean(), pro_max=pro.max(), main=main.mean(), main_max=main.max(), epi=epi.mean(),
                       wg=(us[:, 3] - us[:, 0]).mean(), kernel=names[i])
            rows.append(row)
            print(f"{i:>5} {len(x):>5} {span:6.2f} {gap:5.2f} {row['skew']:5.2f} {row['pro']:5.2f} "
                  f"{row['pro_max']:5.2f} {row['main']:5.2f} {row['main_max']:6.2f} {row['epi']:5.2f} "
                  f"{row['wg']:5.2f} {iss:5.2f} {land:5.2f} {nrm:5.2f} {mhz:5.0f}  {names[i][:60]}")
        total = prev_end - 0.0
        print(f"first start -> last end: {total:.2f} us")
        out[n] = dict(rows=rows, total_us=total)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1, default=float)


if __name__ == "__main__":
    main()
