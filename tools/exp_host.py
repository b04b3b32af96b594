"""Experiment: host enqueue cost per bench step vs elapsed (is the 4-in-flight loop host-bound?)."""
import os, sys, time, importlib.util
ROOT = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
sys.path.insert(0, ROOT)
import bench
import torch
pkg = bench._load_pkg()
import vss_amd.synthetic as syn
dev = torch.device("cuda", 0)
B, fh, fw, S = 8, 480, 640, 4
frames = syn.make_batch(B, fh, fw, 3, start=0)
sess = pkg.Session(model_h=144, model_w=256, dtype="bf16x2", device_id=0, max_batch=B, max_frame_h=fh, max_frame_w=fw, queue_depth=S)
d = torch.from_numpy(frames).to(dev)
outs = [torch.empty((B, 144 * 256), dtype=torch.float32, device=dev) for _ in range(S)]
streams = [torch.cuda.Stream(device=dev) for _ in range(S)]
rs, fs = fw * 3, fh * fw * 3
def step(i):
    sess.segment_device(d.data_ptr(), B, fh, fw, 3, rs, fs, outs[i % S].data_ptr(), streams[i % S].cuda_stream)
for i in range(50): step(i)
torch.cuda.synchronize()
for n in (200, 1000):
    t0 = time.perf_counter(); enq = 0.0
    for i in range(n):
        a = time.perf_counter(); step(i); enq += time.perf_counter() - a
    torch.cuda.synchronize(); el = time.perf_counter() - t0
    print(f"steps {n}: elapsed {el/n*1e6:.1f} us/step, host enqueue {enq/n*1e6:.1f} us/step, {B*n/el:.0f} frames/s")
# raw ctypes call cost without the GPU work: query of a done ticket
t0 = time.perf_counter()
for i in range(2000): sess.layer_kernel(1)
print(f"ctypes round trip ~{(time.perf_counter()-t0)/2000*1e6:.1f} us")
