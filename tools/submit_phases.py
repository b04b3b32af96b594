"""Host time per phase of the queued submit (VSS_TIME_SUBMIT=1), Python zero-copy
loop at 640x480 batch 8, 4 in flight: python tools/submit_phases.py [iters]"""
import collections
import importlib.util
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["VSS_TIME_SUBMIT"] = "1"
spec = importlib.util.spec_from_file_location("vss_amd", os.path.join(ROOT, "video-stream-segmenetation_amd", "__init__.py"),
                                              submodule_search_locations=[os.path.join(ROOT, "video-stream-segmenetation_amd")])
pkg = importlib.util.module_from_spec(spec)
sys.modules["vss_amd"] = pkg
spec.loader.exec_module(pkg)
import vss_amd.synthetic as syn

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
B, fh, fw, S = 8, 480, 640, 4
frames = syn.make_batch(B, fh, fw, 3)
with pkg.Session(max_batch=B, max_frame_h=fh, max_frame_w=fw, queue_depth=S) as s:
    outs = [pkg.host_empty((B, s.mask_h * s.mask_w)) for _ in range(S + 1)]
    flat = frames.reshape(-1)
    tick = collections.deque()
    t0 = time.perf_counter()
    api = 0.0
    for it in range(iters):
        if len(tick) == S:
            s.wait(tick.popleft())
        slot, buf = s.staging_acquire()
        if it < S:
            buf[:flat.size] = flat
        a = time.perf_counter()
        tick.append(s.submit_staged(slot, B, fh, fw, 3, outs[it % len(outs)]))
        api += time.perf_counter() - a
    while tick:
        s.wait(tick.popleft())
    el = time.perf_counter() - t0
    print(f"zero-copy pinned out: {B * iters / el:.0f} frames/s, {el * 1e3 / iters:.4f} ms/batch, "
          f"submit_staged {api * 1e6 / iters:.1f} us/call", flush=True)
