"""Where a short headline window goes: host time of each step call and the
window, after W warm-up steps (python tools/window_probe.py --warmup 1000)."""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--warmup", type=int, default=1000)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--settle", type=float, default=0.0, help="seconds of sleep after prepare_device")
    ap.add_argument("--spin", type=float, default=0.0, help="seconds of host busy-wait after prepare_device")
    ap.add_argument("--pre", default="none", choices=["none", "query", "sleep", "calls"])
    a = ap.parse_args()
    import torch
    from conftest import load_pkg
    pkg = load_pkg()
    import vss_amd.synthetic as syn
    B, fh, fw, S = 8, 480, 640, 4
    d = torch.from_numpy(syn.make_batch(B, fh, fw, 3)).cuda()
    with pkg.Session(max_batch=B, queue_depth=S) as s:
        outs = [torch.empty((B, s.mask_h * s.mask_w), device="cuda") for _ in range(S)]
        sts = [torch.cuda.Stream() for _ in range(S)]
        s.prepare_device(B, fh, fw, 3, fw * 3, fh * fw * 3)
        time.sleep(a.settle)
        t_end = time.perf_counter() + a.spin
        while time.perf_counter() < t_end:
            pass

        def step(i):
            s.segment_device(d.data_ptr(), B, fh, fw, 3, fw * 3, fh * fw * 3, outs[i % S].data_ptr(),
                             sts[i % S].cuda_stream)
        k = 0
        for rep in range(a.reps):
            t = time.perf_counter()
            for _ in range(a.warmup):
                step(k)
                k += 1
            t_issue = time.perf_counter() - t
            torch.cuda.synchronize()
            t_sync = time.perf_counter() - t
            if a.pre == "query":
                for st in sts:
                    st.query()
            elif a.pre == "sleep":
                time.sleep(0.01)
            elif a.pre == "calls":  # which runtime call absorbs the deferred cost
                import ctypes
                hip = ctypes.CDLL("libamdhip64.so")
                tq = []
                for name, fn in (("hipGetLastError", lambda: hip.hipGetLastError()),
                                 ("hipStreamQuery", lambda: hip.hipStreamQuery(ctypes.c_void_p(sts[0].cuda_stream))),
                                 ("eventRecord", lambda: torch.cuda.Event().record(sts[1])),
                                 ("hipStreamQuery2", lambda: hip.hipStreamQuery(ctypes.c_void_p(sts[2].cuda_stream))),
                                 ("torch empty", lambda: torch.empty(16, device="cuda").fill_(1.0))):
                    c = time.perf_counter()
                    fn()
                    tq.append((name, round((time.perf_counter() - c) * 1e6)))
                torch.cuda.synchronize()
                print("pre-calls us", tq, flush=True)
            calls = []
            t0 = time.perf_counter()
            for _ in range(a.steps):
                c = time.perf_counter()
                step(k)
                k += 1
                calls.append(time.perf_counter() - c)
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            calls = np.array(calls) * 1e6
            print(f"rep {rep} warmup {a.warmup} (issue {t_issue*1e3:.1f} ms, +sync {t_sync*1e3:.1f} ms) "
                  f"steps {a.steps}: window {el*1e6:.0f} us = {B*a.steps/el:.0f} fps; issue {(t1-t0)*1e6:.0f} us; "
                  f"calls us first5 {np.round(calls[:5]).tolist()} median {np.median(calls):.1f} max {calls.max():.0f}",
                  flush=True)


if __name__ == "__main__":
    main()
