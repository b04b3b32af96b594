"""Headline benchmark: frames/s of the segmentation seam at 640x480, batch 8 per
GPU (BASELINE.json metric, config 3: bf16 pointwise convs on MFMA), on 1..8
MI355X, one process per GPU.

A step = one pass of the hot path over one batch: 8 synthetic 640x480 RGB
frames already resident in HBM -> fused preprocess + network -> 8 float masks
(144x256), then (N > 1) an RCCL all-gather of every rank's masks so each rank
holds the whole 8N-frame batch in order.  Weak scaling:
per-GPU work is fixed, global batch = 8N.

Also measured in the same run:
  * roofline: the dominant kernel's algorithmic bytes per launch / its mean
    duration from HIP events recorded by the kernel launches themselves
    (hipExtLaunchKernelGGL on the stream the kernels run on) over a second pass
    of K steps, against 8 TB/s;
  * mask max-abs error vs the CPU oracle on this run's frames;
  * cpu_baseline: the oracle (C restatement, f32) on a bounded sample of the
    same frames on this host's cores (rank 0, N=1 only);
  * post: the GPU post-processing chain (EMA ->
    opening -> joint bilateral -> refine -> u8 alpha) over the same batch as
    consecutive frames of one stream: frames/s, its HBM roofline and parity
    with the oracle (rank 0, outside the headline's timed region);
  * host_path: the PCIe-inclusive rate of the host-buffer entry point
    (vss_segment: host frames -> pinned staging -> H2D -> forward -> D2H),
    never `value` (rank 0, outside the timed region).
"""
from __future__ import annotations

import argparse
import importlib.util
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "video-stream-segmenetation_amd")
METRIC = "frames/sec (640×480, batch=8) at 1/2/4/8 MI355X + mask max-abs-err vs ref"
HBM_PEAK = 8.0e12


def _load_pkg():
    if "vss_amd" in sys.modules:
        return sys.modules["vss_amd"]
    spec = importlib.util.spec_from_file_location("vss_amd", os.path.join(PKG_DIR, "__init__.py"),
                                                  submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["vss_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


def cpu_baseline(blob, frames, hm, wm, budget_s):
    """Oracle (C, f32, OpenMP) on a bounded sample of the same frames."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_py  # the checker / CPU baseline only
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(os.cpu_count() or 1, 16)
    res = {}
    for label, nt, budget in (("all", threads, budget_s), ("4", 4, budget_s / 2)):
        oracle_py.forward(blob, frames[:1], hm, wm, mode=0, nthreads=nt)  # warm
        done, t0 = 0, time.perf_counter()
        while True:
            oracle_py.forward(blob, frames, hm, wm, mode=0, nthreads=nt)
            done += len(frames)
            el = time.perf_counter() - t0
            if el >= budget:
                break
        res[label] = (done / el, done, el)
    v, done, el = res["all"]
    return {"value": round(v, 2), "unit": "frames/s", "cores": threads, "kind": "port",
            "value_4_threads": round(res["4"][0], 2),
            "sample": f"{done} frames of the timed batch (640x480 -> 144x256, f32) in {el:.1f} s on "
                      f"{threads} threads; 4 threads: {res['4'][1]} frames in {res['4'][2]:.1f} s"}


def host_leg(sess, frames, d_masks, B, steps):
    """PCIe-inclusive rate of the host-buffer entry point (vss_segment, what the
    N-API addon calls): host u8 frames -> pinned staging -> H2D -> forward ->
    D2H into the caller's f32 masks, synchronous per call.  Never `value`."""
    import numpy as np
    n_iter = max(10, min(steps, 100))
    for _ in range(3):
        masks, _, _ = sess.segment_frames(frames)
    t0 = time.perf_counter()
    for _ in range(n_iter):
        masks, _, _ = sess.segment_frames(frames)
    el = time.perf_counter() - t0
    same = bool(np.array_equal(masks, d_masks.cpu().numpy()))
    return {"value": round(B * n_iter / el, 1), "unit": "frames/s", "ms_per_batch": round(el * 1e3 / n_iter, 4),
            "iters": n_iter, "h2d_bytes_per_batch": int(frames.nbytes), "d2h_bytes_per_batch": int(masks.nbytes),
            "masks_equal_device_path": same,
            "entry": "vss_segment (host frames -> host masks, synchronous, PCIe-inclusive)"}


def post_leg(pkg, sess, d_frames, d_masks, frames, B, fh, fw, hm, wm, stream, steps, warmup, cpu_s):
    """Time the post chain on the seam's masks; check it against the oracle."""
    import torch
    import vss_amd.costmodel as cm
    P = hm * wm
    chain = pkg.PostChain(sess)
    d_alpha = torch.empty((B, P), dtype=torch.float32, device=d_masks.device)
    d_u8 = torch.empty((B, P), dtype=torch.uint8, device=d_masks.device)
    rs, fs = fw * 3, fh * fw * 3

    def run():
        chain.process_device(d_frames.data_ptr(), B, fh, fw, 3, rs, fs, d_masks.data_ptr(), d_alpha.data_ptr(),
                             d_u8.data_ptr(), stream.cuda_stream)

    with torch.cuda.stream(stream):
        for _ in range(warmup):
            run()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(steps):
            run()
        e1.record(stream)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    # parity: a fresh stream state over this batch vs the oracle on the same masks
    chain.reset()
    with torch.cuda.stream(stream):
        run()
    torch.cuda.synchronize()
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_py
    masks = d_masks.cpu().numpy().reshape(B, hm, wm)
    want_a, want_u = oracle_py.post(masks, frames, oracle_py.PostState(hm, wm))
    got_a = d_alpha.cpu().numpy().reshape(B, hm, wm)
    got_u = d_u8.cpu().numpy().reshape(B, hm, wm)
    cpu = None
    if cpu_s > 0:
        done, t0 = 0, time.perf_counter()
        st = oracle_py.PostState(hm, wm)
        while time.perf_counter() - t0 < cpu_s:
            oracle_py.post(masks, frames, st)
            done += B
        cpu = round(done / (time.perf_counter() - t0), 1)
    # compositing (§8(f) row 3) of the same batch: frames + alpha bytes -> RGBA canvas
    d_rgba = torch.empty((B, fh, fw, 4), dtype=torch.uint8, device=d_masks.device)

    def comp():
        pkg.composite_device(sess, d_frames.data_ptr(), B, fh, fw, 3, rs, fs, d_u8.data_ptr(), d_rgba.data_ptr(),
                             stream=stream.cuda_stream)

    with torch.cuda.stream(stream):
        for _ in range(warmup):
            comp()
        c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        c0.record(stream)
        for _ in range(steps):
            comp()
        c1.record(stream)
    torch.cuda.synchronize()
    cms = c0.elapsed_time(c1) / steps
    comp_ok = bool(np.array_equal(d_rgba.cpu().numpy(), oracle_py.composite(frames, got_u)))
    cbytes = fh * fw * 3 + hm * wm + fh * fw * 4
    composite = {"value": round(B / (cms * 1e-3), 1), "unit": "frames/s", "ms_per_batch": round(cms, 5),
                 "alg_bytes_per_frame": cbytes, "GBps": round(cbytes * B / (cms * 1e-3) / 1e9, 1),
                 "frac": round(cbytes * B / (cms * 1e-3) / HBM_PEAK, 4), "bitexact_vs_oracle": comp_ok,
                 "kernel": "k_composite (frame u8 RGB + mask alpha u8 -> RGBA u8 at frame resolution)"}
    chain.close()
    b = cm.post_bytes(hm, wm, fh, fw, 3, B)
    achieved = b["total"] * B / (ms * 1e-3)
    return {"value": round(B / (ms * 1e-3), 1), "unit": "frames/s", "ms_per_batch": round(ms, 5),
            "alg_bytes_per_frame": round(b["total"]), "GBps": round(achieved / 1e9, 1),
            "frac": round(achieved / HBM_PEAK, 4), "alpha_max_abs_err": float(np.abs(got_a - want_a).max()),
            "u8_mismatches": int((got_u != want_u).sum()), "cpu_baseline_fps_1thread": cpu,
            "kernels": "k_post_ema + k_post_filter (timed together with torch events on the launch stream)",
            "composite": composite}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=8, help="frames per GPU per step")
    ap.add_argument("--frame", default="480x640")
    ap.add_argument("--model", default="144x256")
    ap.add_argument("--dtype", default="bf16x2", choices=["bf16x2", "f32"])
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--branches", type=int, default=1, help="concurrent sub-batch chains inside the graph")
    ap.add_argument("--cpu-budget-s", type=float, default=8.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-post", action="store_true", help="skip the post-processing leg")
    ap.add_argument("--no-host", action="store_true", help="skip the PCIe-inclusive host-buffer leg")
    ap.add_argument("--persistent", action="store_true",
                    help="run the forward as ONE persistent k_forward launch (VSS_FORWARD=1) instead of "
                         "one launch per layer")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "latest_traffic.json"),
                    help="per-kernel HBM traffic from tools/prof_summary.py (PMC passes)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # VSS_BENCH_BACKEND=gloo: rehearse the N > 1 code path with ranks sharing
    # fewer GPUs than ranks (plumbing check only; RCCL is the measured backend)
    backend = os.environ.get("VSS_BENCH_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    gpu = local % ndev if backend != "nccl" else local
    if world > 1:
        torch.cuda.set_device(gpu)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", gpu if world > 1 else 0)

    pkg = _load_pkg()
    import vss_amd.synthetic as syn
    import vss_amd.costmodel as cm

    fh, fw = (int(v) for v in args.frame.split("x"))
    hm, wm = (int(v) for v in args.model.split("x"))
    B = args.batch
    frames = syn.make_batch(B, fh, fw, 3, start=rank * B)
    if args.persistent:
        os.environ["VSS_FORWARD"] = "1"  # read by vss_create
    sess = pkg.Session(model_h=hm, model_w=wm, dtype=args.dtype, device_id=dev.index, max_batch=B,
                       max_frame_h=fh, max_frame_w=fw)
    if args.no_graph:
        sess.set_option(pkg.VSS_OPT_USE_GRAPH, 0)
    sess.set_option(pkg.VSS_OPT_BRANCHES, args.branches)
    d_frames = torch.from_numpy(frames).to(dev)
    # two mask buffers: the all-gather of step i (RCCL's own stream) overlaps the
    # forward of step i+1; step i+2 waits for gather i before it rewrites buffer i%2
    d_masks2 = [torch.empty((B, hm * wm), dtype=torch.float32, device=dev) for _ in range(2)]
    d_masks = d_masks2[0]
    gathered2 = [torch.empty((world * B, hm * wm), dtype=torch.float32, device=dev) for _ in range(2)] \
        if world > 1 else None
    pending = [None, None]
    stream = torch.cuda.Stream(device=dev)
    rs, fs = fw * 3, fh * fw * 3
    it = [0]

    def step():
        k = it[0] & 1
        it[0] += 1
        if pending[k] is not None:
            pending[k].wait()  # the forward's stream waits for gather i-2 (reads this buffer)
            pending[k] = None
        sess.segment_device(d_frames.data_ptr(), B, fh, fw, 3, rs, fs, d_masks2[k].data_ptr(), stream.cuda_stream)
        if gathered2 is not None:
            pending[k] = dist.all_gather_into_tensor(gathered2[k], d_masks2[k], async_op=True)

    def drain():
        for k in range(2):
            if pending[k] is not None:
                pending[k].wait()
                pending[k] = None

    with torch.cuda.stream(stream):
        for _ in range(args.warmup):
            step()
        drain()
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        drain()
        torch.cuda.synchronize(dev)
        el = time.perf_counter() - t0
        if world > 1:
            dist.barrier()
    if world > 1:  # the gathered batch holds every rank's masks in frame order
        last = (it[0] - 1) & 1
        assert torch.equal(gathered2[last][rank * B:(rank + 1) * B], d_masks2[last])
    d_masks = d_masks2[(it[0] - 1) & 1]
    t = torch.tensor([el], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el_max = float(t.item())
    value = world * B * args.steps / el_max

    # ---- kernel timing pass (events recorded by the launches themselves) ----
    persistent = sess.persistent

    def profiled_pass():
        sess.set_option(pkg.VSS_OPT_PROFILE, 1)
        with torch.cuda.stream(stream):
            for _ in range(args.steps):
                sess.segment_device(d_frames.data_ptr(), B, fh, fw, 3, rs, fs, d_masks.data_ptr(),
                                    stream.cuda_stream)
        torch.cuda.synchronize(dev)
        sess.set_option(pkg.VSS_OPT_PROFILE, 0)

    fwd_ms = fwd_cnt = None
    if persistent:
        profiled_pass()
        fwd_ms, fwd_cnt = sess.profile_read_forward()
        faults = sess.forward_faults()
        if faults:
            raise RuntimeError(f"k_forward: {faults} dependency waits gave up")
        sess.set_option(pkg.VSS_OPT_FORWARD, 0)  # per-layer breakdown from layer launches
    profiled_pass()
    ms, cnt = sess.profile_read()
    if persistent:
        sess.set_option(pkg.VSS_OPT_FORWARD, 1)

    blob = open(sess.weights_path, "rb").read()
    sys.path.insert(0, os.path.join(PKG_DIR, "model"))
    import make_weights as mw
    recs, _, _ = mw.parse_blob(blob)
    costs = cm.layer_costs(recs, hm, wm, fh, fw, 3, pw_weight_bytes=2 if args.dtype == "bf16x2" else 4)
    names = [sess.layer_kernel(i) for i in range(len(ms))]
    per_layer = [{"layer": i, "kind": costs[i]["kind"], "kernel": names[i], "ms": round(m, 5),
                  "GBps": round(cm.launch_bytes(costs[i], B) / (m * 1e-3) / 1e9, 1) if m > 0 else None}
                 for i, m in enumerate(ms)]
    if persistent:
        # the dominant (only) kernel is the whole forward: every layer's
        # compulsory HBM bytes (each activation written once, read once)
        dom_name = sess.forward_kernel()
        dom_label = f"persistent forward: {dom_name}"
        dom_bytes = sum(cm.launch_bytes(c, B) for c in costs)
        dom_ms, dom_cnt = fwd_ms, fwd_cnt
    else:
        dom = int(np.argmax(ms))
        dom_name = names[dom]
        dom_label = f"layer {dom} ({costs[dom]['kind']}): {dom_name}"
        dom_bytes = cm.launch_bytes(costs[dom], B)
        dom_ms, dom_cnt = ms[dom], cnt
    achieved = dom_bytes / (dom_ms * 1e-3)
    traffic = None
    if args.traffic_json and os.path.exists(args.traffic_json):
        t = json.load(open(args.traffic_json)).get(dom_name)
        if t and t.get("traffic_bytes"):
            traffic = round(t["traffic_bytes"] / 1e6, 3)

    post = None
    if rank == 0 and not args.no_post:
        post = post_leg(pkg, sess, d_frames, d_masks, frames, B, fh, fw, hm, wm, stream, args.steps,
                        args.warmup, 0.0 if args.no_cpu else 2.0)

    host = None
    if rank == 0 and not args.no_host:
        host = host_leg(sess, frames, d_masks, B, args.steps)

    out = None
    if rank == 0:
        masks = d_masks.cpu().numpy()
        err = None
        cpu = None
        if not args.no_cpu:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import oracle_py
            ref = oracle_py.forward(blob, frames, hm, wm, mode=0).reshape(B, -1)
            err = float(np.abs(masks - ref).max())
            if world == 1:
                cpu = cpu_baseline(blob, frames, hm, wm, args.cpu_budget_s)
        out = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(el_max * 1e3 / args.steps, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16" if args.dtype == "bf16x2" else "f32",
            "data": "synthetic",
            "config": {
                "workload": f"{B} synthetic {fw}x{fh} RGB u8 frames per GPU per step (resident in HBM) -> "
                            f"{wm}x{hm} f32 masks" + (", RCCL all-gather of masks (overlapped with the next step's forward)" if world > 1 else ""),
                "global_batch": world * B,
                "frame": f"{fw}x{fh}x3",
                "model_res": f"{wm}x{hm}",
                "pw_gemm": "v_mfma_f32_16x16x32_bf16, f32 activations split hi+lo" if args.dtype == "bf16x2"
                           else "v_mfma_f32_16x16x4_f32",
                "graph": not args.no_graph,
                "persistent_forward": persistent,
                "branches": args.branches,
                "parallelism": f"dp{world}",
            },
            "mask_max_abs_err": err,
            "roofline": {
                "bound": "hbm",
                "kernel": dom_label,
                "achieved": round(achieved / 1e9, 1),
                "peak": HBM_PEAK / 1e9,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK, 4),
                "traffic": traffic,
                "traffic_unit": "MB/launch (rocprofv3 PMC: 2*FETCH_SIZE + WRITE_SIZE, gfx950-corrected)",
                "alg_bytes_per_launch": dom_bytes,
                "mean_kernel_ms": round(dom_ms, 5),
                "events_count": dom_cnt,
            },
            "kernels": per_layer,
            "kernels_note": ("per-layer breakdown from the same plan run as one launch per layer "
                             "(VSS_OPT_FORWARD=0); the headline runs the persistent forward")
                            if persistent else "one launch per layer",
            "layer_launches_sum_ms": round(float(sum(ms)), 5),
            "cpu_baseline": cpu,
            "post": post,
            "host_path": host,
        }
        print(json.dumps(out), flush=True)
    sess.close()
    if world > 1:
        dist.destroy_process_group()
    return out


if __name__ == "__main__":
    main()
