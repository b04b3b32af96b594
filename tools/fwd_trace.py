"""Where the persistent forward's time goes: per-task s_memrealtime stamps
(VSS_FWD_TRACE) of one k_forward launch over a batch -> per layer: tasks,
mean wait for dependencies, mean body time, the layer's window in the launch.
GPU box only.   python tools/fwd_trace.py [batch] [order: layer|diag]"""
import ctypes
import os
import sys

os.environ["VSS_FWD_TRACE"] = "1"
if len(sys.argv) > 2:
    os.environ["VSS_FWD_ORDER"] = sys.argv[2]
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import __graft_entry__ as ge  # noqa: E402

pkg = ge._load_pkg()
import torch  # noqa: E402
import vss_amd.synthetic as syn  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
s = pkg.Session(dtype="bf16x2", max_batch=8)
assert s.persistent
s.set_option(pkg.VSS_OPT_USE_GRAPH, 0)
f = np.stack([syn.make_frame(i) for i in range(n)])
d = torch.from_numpy(f).cuda()
out = torch.empty((n, 144 * 256), dtype=torch.float32, device="cuda")
L = pkg.lib()
L.vss_fwd_trace_read.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
for _ in range(20):  # warm
    s.segment_device(d.data_ptr(), n, 480, 640, 3, 640 * 3, 480 * 640 * 3, out.data_ptr(), 0)
s.synchronize()
buf = (ctypes.c_ulonglong * (4 * 20000))()
k = L.vss_fwd_trace_read(s._h, buf, 20000)
a = np.frombuffer(buf, dtype=np.uint64)[:4 * k].reshape(k, 4).astype(np.int64)
t0 = a[:, 0].min()
a[:, :3] -= t0
us = lambda x: x / 100.0  # 100 MHz ticks -> us
layer_of = (a[:, 3] >> 16) & 0xFF
frame_of = (a[:, 3] >> 24) & 0xFF
a[:, 3] &= 0xFFFF
print(f"tasks {k}, launch span {us(a[:, 2].max()):.1f} us, workgroups {len(np.unique(a[:, 3]))}")
# task -> layer from the task order (layer-major or diagonal): recompute from counts
import vss_amd  # noqa: E402,F401
tiles = []
for li in range(s.n_layers):
    c, h, w = s.layer_shape(li)
tasks_layer = np.full(k, -1)
# read the task table order from the library is not exported: infer from stamps per layer via a second
# launch with profile of layer windows is overkill; the tool prints the time profile by ticket instead.
order = np.argsort(a[:, 0])
wait = a[:, 1] - a[:, 0]
body = a[:, 2] - a[:, 1]
print(f"mean wait {us(wait.mean()):.2f} us, mean body {us(body.mean()):.2f} us, "
      f"sum body / wgs {us(body.sum()) / len(np.unique(a[:, 3])):.1f} us per workgroup")
# per ticket bucket (tickets are in layer-major order by default)
edges = np.linspace(0, k, 25).astype(int)
for lo, hi in zip(edges[:-1], edges[1:]):
    sl = slice(lo, hi)
    print(f"tickets {lo:5d}-{hi:5d}: taken {us(a[sl, 0].min()):7.1f}-{us(a[sl, 0].max()):7.1f} us "
          f"wait {us(wait[sl].mean()):6.2f} body {us(body[sl].mean()):6.2f} (max {us(body[sl].max()):6.2f})")
# per workgroup: busy fraction
wg = a[:, 3]
busy = np.bincount(wg, weights=body) / 100.0
waitw = np.bincount(wg, weights=wait) / 100.0
cnt = np.bincount(wg)
print(f"per workgroup: tasks {cnt[cnt>0].mean():.1f}, body {busy[cnt>0].mean():.1f} us, wait {waitw[cnt>0].mean():.1f} us")
if os.environ.get("VSS_FWD_ONLY"):
    print(f"layer {os.environ['VSS_FWD_ONLY']} alone: body mean {us(body.mean()):.2f} us "
          f"median {us(np.median(body)):.2f} us, span {us(a[:, 2].max()):.1f} us")

print("per layer: tasks, window [first start, last end] us, mean wait, mean body, body sum / 512")
for li in range(s.n_layers):
    m = layer_of == li
    if not m.any():
        continue
    print(f"  layer {li:2d}: {m.sum():5d} tasks  window {us(a[m, 0].min()):6.1f}-{us(a[m, 2].max()):6.1f}  "
          f"wait {us(wait[m].mean()):5.2f}  body {us(body[m].mean()):5.2f} (min {us(body[m].min()):5.2f})  "
          f"occupancy-us {us(body[m].sum()) / 512:5.2f}")
for fr in range(n):
    m = frame_of == fr
    print(f"  frame {fr}: {us(a[m, 0].min()):6.1f}-{us(a[m, 2].max()):6.1f}")
