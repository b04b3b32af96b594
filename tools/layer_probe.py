"""Time every compiled kernel of one layer (pinned with VSS_TILE="layer:#k"):
its isolated duration (launch events, one batch at a time) and the 4-in-flight
headline rate with it.  python tools/layer_probe.py LAYER [--batch 8] [--reps 200]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("layer", type=int)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--only", default="", help="comma-separated candidate indices")
    a = ap.parse_args()
    import torch
    from conftest import load_pkg
    pkg = load_pkg()
    import vss_amd.synthetic as syn
    B, fh, fw = a.batch, 480, 640
    frames = syn.make_batch(B, fh, fw, 3)
    d = torch.from_numpy(frames).cuda()
    with pkg.Session(max_batch=B, autotune=False) as s:
        n = len(s.layer_tiles(a.layer))
        names = [s.layer_tile_kernel(a.layer, k) for k in range(n)]
    ks = [int(x) for x in a.only.split(",")] if a.only else range(n)
    out = []
    for k in ks:
        os.environ["VSS_TILE"] = f"{a.layer}:#{k}"
        with pkg.Session(max_batch=B, queue_depth=4) as s:
            occ = s.layer_occupancy(a.layer)
            outs = [torch.empty((B, s.mask_h * s.mask_w), device="cuda") for _ in range(4)]
            sts = [torch.cuda.Stream() for _ in range(4)]
            s.prepare_device(B, fh, fw, 3, fw * 3, fh * fw * 3)
            s.set_option(pkg.VSS_OPT_PROFILE, 1)
            for i in range(a.reps):
                s.segment_device(d.data_ptr(), B, fh, fw, 3, fw * 3, fh * fw * 3, outs[0].data_ptr(), sts[0].cuda_stream)
            torch.cuda.synchronize()
            s.set_option(pkg.VSS_OPT_PROFILE, 0)
            ms, _ = s.profile_read()
            rates = []
            for rep in range(3):
                for i in range(40):
                    s.segment_device(d.data_ptr(), B, fh, fw, 3, fw * 3, fh * fw * 3, outs[i % 4].data_ptr(),
                                     sts[i % 4].cuda_stream)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for i in range(400):
                    s.segment_device(d.data_ptr(), B, fh, fw, 3, fw * 3, fh * fw * 3, outs[i % 4].data_ptr(),
                                     sts[i % 4].cuda_stream)
                torch.cuda.synchronize()
                rates.append(B * 400 / (time.perf_counter() - t0))
        del os.environ["VSS_TILE"]
        r = {"k": k, "kernel": names[k], "layer_us": round(ms[a.layer] * 1e3, 2), "wg_per_cu": occ[0],
             "lds": occ[1], "fps_4inflight": [round(x) for x in rates], "forward_us": round(sum(ms) * 1e3, 1)}
        print(json.dumps(r), flush=True)
        out.append(r)


if __name__ == "__main__":
    main()
