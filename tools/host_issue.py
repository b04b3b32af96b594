"""Is the headline step host-bound?  Times the host side of vss_segment_device
(Python + ctypes + HIP enqueue) per step against the wall time per step, 640x480
batch 8, 4 streams in flight: python tools/host_issue.py [steps]"""
import importlib.util
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("vss_amd", os.path.join(ROOT, "video-stream-segmenetation_amd", "__init__.py"),
                                              submodule_search_locations=[os.path.join(ROOT, "video-stream-segmenetation_amd")])
pkg = importlib.util.module_from_spec(spec)
sys.modules["vss_amd"] = pkg
spec.loader.exec_module(pkg)
import torch
import vss_amd.synthetic as syn

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
B, fh, fw, S = 8, 480, 640, 4
dev = torch.device("cuda", 0)
d = torch.from_numpy(syn.make_batch(B, fh, fw, 3)).to(dev)
with pkg.Session(max_batch=B, max_frame_h=fh, max_frame_w=fw, queue_depth=S) as s:
    masks = [torch.empty((B, s.mask_h * s.mask_w), dtype=torch.float32, device=dev) for _ in range(S)]
    streams = [torch.cuda.Stream(device=dev) for _ in range(S)]
    L = pkg.lib()
    args = [(s._h, d.data_ptr(), B, fh, fw, 3, fw * 3, fh * fw * 3, masks[k].data_ptr(), streams[k].cuda_stream)
            for k in range(S)]
    for i in range(100):
        L.vss_segment_device(*args[i % S])
    torch.cuda.synchronize(dev)
    for rep in range(3):
        host = 0.0
        t0 = time.perf_counter()
        for i in range(steps):
            a = time.perf_counter()
            L.vss_segment_device(*args[i % S])
            host += time.perf_counter() - a
        t1 = time.perf_counter()
        torch.cuda.synchronize(dev)
        el = time.perf_counter() - t0
        print(f"{B * steps / el:.0f} frames/s: wall {el * 1e6 / steps:.1f} us/step, issue loop {(t1 - t0) * 1e6 / steps:.1f}, "
              f"in the call {host * 1e6 / steps:.1f} us/step", flush=True)
