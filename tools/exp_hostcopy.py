"""Experiment: where the queued host path's time goes when the masks go to
pageable caller memory (bench host_path 'copy') vs vss_host_alloc blocks
('copy_pinned_out').  Prints, per form, frames/s and the mean time the caller
spends inside submit and inside wait.  Run with VSS_TIME_SUBMIT=1 for the
submit phases (printed at handle destruction)."""
import collections
import os
import sys
import time

import numpy as np

ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import load_pkg  # noqa: E402

pkg = load_pkg()
import vss_amd.synthetic as syn  # noqa: E402

B, fh, fw, S = 8, 480, 640, 4
iters = int(os.environ.get("ITERS", "200"))
frames = syn.make_batch(B, fh, fw, 3)
with pkg.Session(max_batch=B, max_frame_h=fh, max_frame_w=fw, queue_depth=S) as s:
    P = s.mask_h * s.mask_w
    for _ in range(3):
        s.segment_frames(frames)
    forms = {"copy": [np.ones((B, P), np.float32) for _ in range(S + 1)],
             "pinned_out": [pkg.host_empty((B, P)) for _ in range(S + 1)]}
    for rep in range(2):
        for name, outs in forms.items():
            q = collections.deque()
            ts = tw = 0.0
            t0 = time.perf_counter()
            for i in range(iters):
                if len(q) == S:
                    a = time.perf_counter()
                    s.wait(q.popleft())
                    tw += time.perf_counter() - a
                a = time.perf_counter()
                q.append(s.submit(frames, out=outs[i % len(outs)]))
                ts += time.perf_counter() - a
            while q:
                s.wait(q.popleft())
            el = time.perf_counter() - t0
            print(f"{name:11s} rep {rep}: {B * iters / el:8.0f} frames/s  {el / iters * 1e6:7.1f} us/batch  "
                  f"submit {ts / iters * 1e6:7.1f} us  wait {tw / iters * 1e6:7.1f} us", flush=True)
