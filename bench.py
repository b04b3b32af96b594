"""Headline benchmark: frames/s of the segmentation seam at 640x480, batch 8 per
GPU (BASELINE.json metric, config 3: bf16 pointwise convs on MFMA), on 1..8
MI355X, one process per GPU.

A step = one pass of the hot path over one batch: 8 synthetic 640x480 RGB
frames already resident in HBM -> fused preprocess + network -> 8 float masks
(144x256), and (N > 1) the RCCL all-gather of every rank's masks inside the C
ABI (vss_segment_gather_device: each rank's handle joined one clique with
vss_comm_init_rank), so each rank holds the whole 8N-frame batch in order
(SURVEY.md §8(e)).  Weak scaling: per-GPU work is fixed, global batch = 8N.
Steps are issued round-robin on `--inflight` streams (default: the handle's
queue depth, 4): consecutive batches take consecutive slots of the handle (own
activations) and run concurrently — the serving engine's steady state, where
the next batch's kernels fill the gaps of this one's launch chain.  K steps
are timed between barriers + device synchronisation; value = frames / time.

Also measured in the same run (rank 0):
  * roofline: the dominant kernel's algorithmic bytes per launch / its mean
    duration from HIP events recorded by the kernel launches themselves
    (hipExtLaunchKernelGGL on the stream the kernels run on, one batch at a
    time) against 8 TB/s; plus the whole step's algorithmic bytes at `value`;
  * batch_sweep: 8 / 32 / 64 frames per step, one and `inflight` in flight;
  * mask max-abs error vs the CPU oracle on this run's frames;
  * cpu_baseline: the oracle (C restatement, f32, frames x channels OpenMP) on
    a bounded sample of the same frames on this host's cores (N = 1 only);
  * post: the GPU post-processing chain over the same batch (outside the
    headline's timed region);
  * host_path: the PCIe-inclusive queued host entry point (vss_submit: host
    frames -> pinned staging -> H2D -> forward -> D2H, `inflight` batches in
    flight), from caller memory and zero-copy from the pinned staging, at
    640x480 and 1920x1080 (never `value`);
  * ts_path: the TypeScript host (Segmenter.segmentFrames, Node child
    process) end to end — throughput and one-call latency.
"""
from __future__ import annotations

import argparse
import collections
import importlib.util
import json
import os
import subprocess
import shutil
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


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(blob, frames, hm, wm, budget_s):
    """Oracle (C, f32; frames x channels in nested OpenMP teams) on a bounded
    sample of the same frames: every usable core of this process's share, and
    4 threads (ORT-web's default intra-op cap)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_py  # the checker / CPU baseline only
    usable = len(os.sched_getaffinity(0))
    env_threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    # the GPU box sets OMP_NUM_THREADS to its CPU share (the affinity mask shows
    # the whole machine there); without it, every core in the affinity mask
    threads = min(usable, env_threads) if env_threads else usable
    res = {}
    for label, nt, budget in (("all", threads, budget_s), ("4", 4, budget_s / 2)):
        oracle_py.forward(blob, frames, hm, wm, mode=0, nthreads=nt)  # warm
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
            "value_4_threads": round(res["4"][0], 2), "scaling_4_to_all": round(v / res["4"][0], 2),
            "nproc": usable, "omp_num_threads_env": env_threads or None, "cpu_model": cpu_model(),
            "sample": f"{done} frames of the timed batch (640x480 -> 144x256, f32, the build's C restatement; the "
                      f"reference's ORT-web path cannot run here) in {el:.1f} s on {threads} threads; 4 threads: "
                      f"{res['4'][1]} frames in {res['4'][2]:.1f} s"}


def host_leg(pkg, frames, B, fh, fw, inflight, iters, d_ref=None):
    """PCIe-inclusive rate of the queued host entry point (vss_submit, what the
    N-API addon calls): host u8 frames -> pinned staging -> H2D -> forward ->
    D2H into the caller's masks, `inflight` batches in flight.  Two forms:
    'copy' (frames in the caller's memory, staged by the copy pool) and
    'zero_copy' (the frames are already in the pinned staging buffer, as a
    decoder writing there would leave them).  Never `value`."""
    out = {}
    warm = max(20, iters // 2)
    with pkg.Session(max_batch=B, max_frame_h=fh, max_frame_w=fw, queue_depth=inflight) as s:
        masks = np.empty((B, s.mask_h * s.mask_w), np.float32)
        for _ in range(3):
            s.segment_frames(frames)
        flat = frames.reshape(-1)
        filled = set()

        def queued(outs, staged, n):
            """n batches, `inflight` in flight; staged: frames decoded into a
            leased slot's pinned staging (the synthetic "decoder" fills each
            slot's buffer once, every later lease of that slot finds them
            there), else copied from the caller's frames.  -> (seconds, last masks)"""
            q = collections.deque()
            last = None
            t0 = time.perf_counter()
            for i in range(n):
                if len(q) == inflight:
                    last = s.wait(q.popleft())[0]
                o = outs[i % len(outs)]
                if staged:
                    slot, buf = s.staging_acquire()
                    if slot not in filled:
                        buf[:flat.size] = flat
                        filled.add(slot)
                    q.append(s.submit_staged(slot, B, fh, fw, 3, o))
                else:
                    q.append(s.submit(frames, out=o))
            while q:
                last = s.wait(q.popleft())[0]
            return time.perf_counter() - t0, last

        # each form runs an untimed pass of its own loop first (the copy pool's
        # threads, the caller's result pages and the DMA queues warm up: the
        # first ~100 batches of a cold loop run up to 1.6x slower)
        forms = {
            # frames and masks in the caller's ordinary (pageable) memory; the
            # caller reuses its result buffers (a fresh np.empty per batch would
            # time numpy's page faults on 1.2 MB of new pages, not the library)
            "copy": ([np.ones((B, s.mask_h * s.mask_w), np.float32) for _ in range(inflight + 1)], False),
            # masks into pinned blocks (host_empty / vss_host_alloc, what the
            # N-API addon hands out): the D2H fills them, no completion copy
            "copy_pinned_out": ([pkg.host_empty((B, s.mask_h * s.mask_w)) for _ in range(inflight + 1)], False),
            # zero-copy: frames already in the leased staging
            "zero_copy": ([masks], True),
            # zero-copy both ways
            "zero_copy_pinned_out": ([pkg.host_empty((B, s.mask_h * s.mask_w)) for _ in range(inflight + 1)], True),
        }
        for name, (outs, staged) in forms.items():
            queued(outs, staged, warm)
            el, last = queued(outs, staged, iters)
            same = bool(np.array_equal(last, d_ref)) if d_ref is not None else None
            out[name] = {"value": round(B * iters / el, 1), "ms_per_batch": round(el * 1e3 / iters, 4),
                         "masks_equal_device_path": same}
    out.update({"unit": "frames/s", "frame": f"{fw}x{fh}x3", "batch": B, "inflight": inflight, "iters": iters,
                "warmup_iters": warm, "h2d_bytes_per_batch": int(frames.nbytes), "d2h_bytes_per_batch": int(B * 144 * 256 * 4),
                "entry": "vss_submit / vss_wait (host frames -> host masks, queued, PCIe-inclusive)"})
    return out


def ts_leg(B, fh, fw, iters, inflight):
    """The TypeScript host end to end in a Node child process (tools/bench_ts.js)."""
    node = shutil.which("node")
    if not node:
        return None
    try:
        r = subprocess.run([node, os.path.join(ROOT, "tools", "bench_ts.js"), str(fh), str(fw), str(B), str(iters),
                            str(inflight)], capture_output=True, text=True, timeout=240)
    except subprocess.TimeoutExpired:
        return {"error": "timeout"}
    if r.returncode != 0:
        return {"error": r.stderr.strip()[-400:]}
    return json.loads(r.stdout.strip().splitlines()[-1])


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


class Watchdog:
    """No progress for `limit_s` seconds -> one JSON line (stdout and stderr)
    naming the rank, the stage, the last step issued, the handle's gather
    counter and each slot communicator's ncclCommGetAsyncError, then
    os._exit(3) (never a re-exec).  The main thread beats at every step it
    issues and after every synchronize, so a collective that never completes
    (a rank that died, a deadlock between the per-slot communicators) ends
    the run with a record instead of at the driver's timeout.  Armed only
    around GPU phases; `status` is a lock-free callable (Session.comm_status)."""

    def __init__(self, limit_s, rank, world):
        import threading
        self.limit, self.rank, self.world = limit_s, rank, world
        self.stage, self.step, self.t = "start", -1, time.monotonic()
        self.armed, self.status = False, None
        self.gather_form = None  # the all-gather form the ranks run (VSS_OPT_GATHER_FORM)
        self._lock = threading.Lock()
        if limit_s > 0:
            threading.Thread(target=self._run, daemon=True).start()

    def beat(self, stage=None, step=None):
        with self._lock:
            if stage is not None:
                self.stage = stage
            if step is not None:
                self.step = step
            self.t = time.monotonic()

    def arm(self, stage):
        self.beat(stage)
        self.armed = True

    def disarm(self):
        self.armed = False

    def _run(self):
        while True:
            time.sleep(min(1.0, self.limit / 4))
            with self._lock:
                idle = time.monotonic() - self.t
                stage, step = self.stage, self.step
            if not self.armed or idle < self.limit:
                continue
            rec = {"watchdog": "no progress", "rank": self.rank, "world": self.world, "stage": stage,
                   "last_step_issued": step, "seconds_without_progress": round(idle, 1),
                   "gather_form": self.gather_form}
            try:
                if self.status is not None:
                    rec.update(self.status())
            except Exception as e:  # the record must still go out
                rec["status_error"] = repr(e)
            line = json.dumps(rec) + "\n"
            for fd in (sys.stderr.fileno(), sys.stdout.fileno()):
                try:
                    os.write(fd, line.encode())
                except OSError:
                    pass
            os._exit(3)


def latency_leg(sess, torch, dev, d_frames, fh, fw, iters):
    """One call at a time, the way the reference runs its model
    (runModnetExclusive serialises every processFrame, main.ts:18-22, 66-74;
    its overlay's `Latency` is session.run's wall time, frameProcessorTest.ts:
    90-92): the host wall time of vss_segment_device + stream synchronize for
    1 frame and for a batch of 8, frames already in HBM.  p50 / p99 / min in
    ms and the serial frames/s (never `value`)."""
    out = {}
    st = torch.cuda.Stream(device=dev)
    P = sess.mask_h * sess.mask_w
    masks = torch.empty((8, P), dtype=torch.float32, device=dev)
    for n in (1, 8):
        sess.prepare_device(n, fh, fw, 3, fw * 3, fh * fw * 3)
        for _ in range(50):
            sess.segment_device(d_frames.data_ptr(), n, fh, fw, 3, fw * 3, fh * fw * 3, masks.data_ptr(), st.cuda_stream)
        st.synchronize()
        lat = []
        t1 = time.perf_counter()
        for _ in range(iters):
            t0 = time.perf_counter()
            sess.segment_device(d_frames.data_ptr(), n, fh, fw, 3, fw * 3, fh * fw * 3, masks.data_ptr(), st.cuda_stream)
            st.synchronize()
            lat.append((time.perf_counter() - t0) * 1e3)
        el = time.perf_counter() - t1
        lat = np.sort(np.array(lat))
        out[f"batch{n}"] = {"latency_ms_p50": round(float(lat[len(lat) // 2]), 4),
                            "latency_ms_p99": round(float(lat[min(len(lat) - 1, int(0.99 * len(lat)))]), 4),
                            "latency_ms_min": round(float(lat[0]), 4), "calls": iters,
                            "frames_per_s_serial": round(n * iters / el, 1)}
    out["entry"] = "vss_segment_device + hipStreamSynchronize, one call at a time (frames resident in HBM)"
    return out


def run_steps(sess, streams, n_steps, launch, start=0, wd=None):
    """Issue n_steps round-robin over the streams (launch(k, stream) per step).
    `start` continues the global step count: step k uses stream, output buffer
    and (the handle's round-robin over device calls) slot k % S, so a slot
    always meets the same buffers and its graph is never patched."""
    for i in range(start, start + n_steps):
        launch(i, streams[i % len(streams)])
        if wd is not None:
            wd.beat(step=i)
    return start + n_steps


def _free_port() -> int:
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_ranks(n: int, check_gpus: bool = True) -> int:
    """--gpus N without a torch.distributed launcher: start N rank processes
    (torch.distributed.run, one per GPU) from this process, which has not
    touched the GPU (device_count() does not initialise HIP on this image),
    and return their exit code.  Fewer than N visible GPUs is an error (except
    for --dry-run-dist, which never reaches a GPU call)."""
    import torch
    ndev = torch.cuda.device_count()
    if check_gpus and ndev < n:
        print(f"bench.py: --gpus {n} needs {n} GPUs, {ndev} visible", file=sys.stderr, flush=True)
        return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    return subprocess.run(cmd, env=env).returncode


def sweep(pkg, torch, dev, fh, fw, dtype, inflight, steps):
    """Frames/s at 8 / 32 / 64 frames per step, one batch and `inflight` batches in flight."""
    import vss_amd.synthetic as syn
    out = []
    for B in (8, 32, 64):
        frames = syn.make_batch(B, fh, fw, 3)
        d = torch.from_numpy(frames).to(dev)
        with pkg.Session(dtype=dtype, max_batch=B, max_frame_h=fh, max_frame_w=fw, queue_depth=inflight) as s:
            masks = [torch.empty((B, s.mask_h * s.mask_w), dtype=torch.float32, device=dev) for _ in range(inflight)]
            for S in sorted({1, inflight}):
                streams = [torch.cuda.Stream(device=dev) for _ in range(S)]

                def go(i, st):
                    s.segment_device(d.data_ptr(), B, fh, fw, 3, fw * 3, fh * fw * 3, masks[i % S].data_ptr(),
                                     st.cuda_stream)

                s.prepare_device(B, fh, fw, 3, fw * 3, fh * fw * 3)

                k = run_steps(s, streams, 10, go)
                torch.cuda.synchronize(dev)
                n = max(20, steps * 8 // B)
                t0 = time.perf_counter()
                run_steps(s, streams, n, go, start=k)
                torch.cuda.synchronize(dev)
                el = time.perf_counter() - t0
                out.append({"batch": B, "inflight": S, "value": round(B * n / el, 1),
                            "ms_per_step": round(el * 1e3 / n, 5)})
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # (2000 steps: a ~75 ms window; 200-step windows (~8.5 ms) read 187-191k
    # against 213-215k on the same box, the pipeline's fill / drain and the
    # first calls' host costs spread over too few steps — profiles/NOTES.md "Short
    # windows"; the per-step work is the same)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=8, help="frames per GPU per step")
    ap.add_argument("--frame", default="480x640")
    ap.add_argument("--model", default="144x256")
    ap.add_argument("--dtype", default="bf16x2", choices=["bf16x2", "f32"])
    ap.add_argument("--inflight", type=int, default=4, help="batches in flight (streams = the handle's queue depth)")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--streams", default="torch", choices=["slot", "torch"],
                    help="step streams: new torch streams (default; measured 184-187k vs 142-147k on plain slot "
                         "streams, which share the runtime's pooled queues — see profiles/NOTES.md) or the handle's slot "
                         "streams (run with VSS_SLOT_QUEUES=cumask for dedicated queues)")
    ap.add_argument("--cpu-budget-s", type=float, default=8.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-post", action="store_true", help="skip the post-processing leg")
    ap.add_argument("--no-host", action="store_true", help="skip the PCIe-inclusive host-buffer legs")
    ap.add_argument("--no-ts", action="store_true", help="skip the TypeScript (Node) leg")
    ap.add_argument("--no-sweep", action="store_true", help="skip the batch sweep")
    ap.add_argument("--no-latency", action="store_true", help="skip the one-call-at-a-time latency leg")
    ap.add_argument("--gather", action="store_true",
                    help="run the multi-GPU step (RCCL clique all-gather) even at one rank (a rehearsal of N > 1)")
    ap.add_argument("--gather-form", default="ordered", choices=["ordered", "concurrent"],
                    help="how the N > 1 all-gathers are issued (VSS_OPT_GATHER_FORM, DESIGN.md §6): 'ordered' "
                         "(default: one communicator per rank, its collectives one at a time in call order by an "
                         "event chain) or 'concurrent' (one communicator per slot; opt-in until an 8-GPU "
                         "record exists)")
    ap.add_argument("--dry-run-dist", action="store_true",
                    help="rehearse the multi-rank plumbing only (launch_ranks -> torch.distributed.run -> gloo "
                         "-> the clique-id broadcast, with placeholder id bytes) and stop before the first GPU "
                         "call: each rank prints one JSON line; runs on a machine without GPUs")
    # (the HIP runtime retires the warm-up's commands on its own threads for a
    # few hundred us after a synchronize; step calls made meanwhile took 25-70
    # us instead of 12-16 and the GPU started the window with 1-2 batches in
    # flight: the driver's 20-step window read 129-193k (mean 162.5k) with no
    # pause against 167-184k (mean 174.4k) after 5 ms, median steps alike —
    # profiles/NOTES.md "The short window's first calls", profiles/r06j.  The
    # first step call after the pause still paid 36-190 us unless the slots
    # had each run a step since: the warm-up's last S steps therefore run after
    # the pause — W warm-up steps in all — profiles/r06z)
    ap.add_argument("--settle-ms", type=float, default=5.0,
                    help="untimed pause inside the warm-up: after its first W - S steps and their synchronize, "
                         "before its last S steps (one per slot) and the timed window's barrier + synchronize")
    ap.add_argument("--watchdog-s", type=float, default=60.0,
                    help="no step issued or completed for this long during a GPU phase: print a JSON record "
                         "(rank, stage, gather counter, communicators' async errors) and exit 3; 0 = off")
    ap.add_argument("--test-stall-rank", type=int, default=-1, help=argparse.SUPPRESS)  # tests: a rank that hangs
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "latest_traffic.json"),
                    help="per-kernel HBM traffic from tools/prof_summary.py (PMC passes)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, check_gpus=not args.dry_run_dist))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} ranks", file=sys.stderr, flush=True)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    fh, fw = (int(v) for v in args.frame.split("x"))
    hm, wm = (int(v) for v in args.model.split("x"))
    B = args.batch

    ts = None
    if rank == 0 and world == 1 and not args.no_ts and not args.dry_run_dist:
        # (a fixed 600 batches per timed loop, whatever --steps: at the driver's
        # --steps 20 the legs ran 100 batches, ~15 ms windows that read 36-57k
        # on one box, profiles/r06c)
        ts = ts_leg(B, fh, fw, 600, args.inflight)  # before this process touches the GPU
        # the Node process's GPU context is torn down after it exits; one full
        # bench (r03i) timed its headline 9 % under its own median step right
        # after this leg, so the headline starts on a settled device
        time.sleep(2.0)

    import torch
    import torch.distributed as dist

    if world > 1:
        # the process group carries only the clique id, barriers and the max-time
        # reduction (CPU tensors); the masks go over the handle's own RCCL clique
        dist.init_process_group("gloo")
    wd = Watchdog(args.watchdog_s, rank, world)
    gather = world > 1 or args.gather
    wd.gather_form = args.gather_form if gather else None
    if args.dry_run_dist:
        # the same broadcast the GPU run makes (rank 0's clique ids -> every
        # rank), with placeholder bytes of the real size: RCCL's ncclGetUniqueId
        # needs a GPU.  4 slots x sizeof(ncclUniqueId) = 128 B each.
        import hashlib
        ids = [os.urandom(args.inflight * 128) if rank == 0 else None]
        wd.arm("dry-run: clique-id broadcast")
        if world > 1:
            dist.broadcast_object_list(ids, src=0)
            if rank == args.test_stall_rank:  # (tests: this rank never reaches the barrier)
                wd.beat("dry-run: stalled rank")
                time.sleep(3600)
            wd.beat("dry-run: barrier")
            dist.barrier()
        wd.disarm()
        # one write per line: the ranks share the launcher's stdout pipe, and
        # print()'s separate newline write let two ranks' lines interleave
        line = json.dumps({"dry_run": True, "rank": rank, "world": world, "local_rank": local,
                           "env_world_size": os.environ.get("WORLD_SIZE"), "ids_len": len(ids[0]),
                           "ids_sha256": hashlib.sha256(ids[0]).hexdigest(),
                           "gather_form": wd.gather_form})
        os.write(sys.stdout.fileno(), (line + "\n").encode())
        if world > 1:
            dist.destroy_process_group()
        return
    ndev = torch.cuda.device_count()
    if ndev < 1 or (world > 1 and local >= ndev):
        print(f"bench.py: rank {rank} (local {local}) has no GPU ({ndev} visible)", file=sys.stderr, flush=True)
        sys.exit(2)
    gpu = local
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)

    pkg = _load_pkg()
    import vss_amd.synthetic as syn
    import vss_amd.costmodel as cm

    frames = syn.make_batch(B, fh, fw, 3, start=rank * B)
    S = args.inflight
    sess = pkg.Session(model_h=hm, model_w=wm, dtype=args.dtype, device_id=dev.index, max_batch=B,
                       max_frame_h=fh, max_frame_w=fw, queue_depth=S)
    if args.no_graph:
        sess.set_option(pkg.VSS_OPT_USE_GRAPH, 0)
    if gather:
        sess.gather_form = args.gather_form  # (fixed by comm_init_rank)
    wd.arm("clique init")
    if world > 1:
        ids = [sess.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(ids, src=0)
        sess.comm_init_rank(world, rank, ids[0])
    elif gather:
        sess.comm_init_rank(1, 0, sess.comm_unique_id())
    # the communicators' health only once they exist (the record names the stage before)
    wd.status = sess.comm_status
    if gather:
        wd.gather_form = sess.gather_form
    d_frames = torch.from_numpy(frames).to(dev)
    P = hm * wm
    # one output buffer per stream: step i writes buffer i % S on stream i % S
    outs = [torch.empty((world * B, P), dtype=torch.float32, device=dev) for _ in range(S)]
    if args.streams == "slot":
        streams = [torch.cuda.ExternalStream(sess.slot_stream(k), device=dev) for k in range(S)]
    else:
        streams = [torch.cuda.Stream(device=dev) for _ in range(S)]
    rs, fs = fw * 3, fh * fw * 3

    def step(i, st):
        if gather:
            sess.segment_gather_device(d_frames.data_ptr(), B, fh, fw, 3, rs, fs, outs[i % S].data_ptr(),
                                       st.cuda_stream)
        else:
            sess.segment_device(d_frames.data_ptr(), B, fh, fw, 3, rs, fs, outs[i % S].data_ptr(), st.cuda_stream)

    # every slot's graph for this shape is built before the first step, so no
    # build (and, with the buffer pairing of run_steps, no patch) happens in
    # the timed region at any --warmup
    wd.beat("prepare")
    sess.prepare_device(B, fh, fw, 3, rs, fs)
    wd.beat("warmup")
    # W warm-up steps: W - S of them, a synchronize and the settle pause, then
    # the last S (one per slot, the window's first S slots warm again)
    tail = min(args.warmup, S) if args.settle_ms > 0 else 0
    k = run_steps(sess, streams, args.warmup - tail, step, wd=wd)
    torch.cuda.synchronize(dev)
    if args.settle_ms > 0:
        time.sleep(args.settle_ms / 1e3)
        k = run_steps(sess, streams, tail, step, start=k, wd=wd)
    wd.beat("barrier before the timed steps")
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    builds0, patches0 = sess.graph_builds, sess.graph_patches
    wd.beat("timed steps")
    t0 = time.perf_counter()
    k = run_steps(sess, streams, args.steps, step, start=k, wd=wd)
    wd.beat("timed steps: synchronize")
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    wd.beat("barrier after the timed steps")
    if world > 1:
        dist.barrier()
    wd.beat("event pass")
    timed_builds, timed_patches = sess.graph_builds - builds0, sess.graph_patches - patches0
    last = (k - 1) % S
    # per-step completion times (a second pass of the same K steps, events on
    # each step's stream; kept out of the headline window): the median interval
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    k_ev = k

    def step_ev(i, st):
        step(i, st)
        ends[i - k_ev].record(st)

    e0 = torch.cuda.Event(enable_timing=True)
    e0.record(streams[k % S])
    k = run_steps(sess, streams, args.steps, step_ev, start=k, wd=wd)
    torch.cuda.synchronize(dev)
    wd.beat("profile pass")
    # completions arrive in bursts (the batches in flight finish close
    # together), so the step interval is taken over S consecutive completions
    done_ms = np.sort(np.array([e0.elapsed_time(e) for e in ends]))
    iv = (done_ms[S:] - done_ms[:-S]) / S if len(done_ms) > S else np.diff(done_ms)
    median_step_ms = float(np.median(iv)) if len(iv) else None
    n_ranks = sess.comm_ranks if gather else world
    d_masks = outs[last][rank * B:(rank + 1) * B] if world > 1 else outs[last][:B]
    if gather:  # the gathered batch holds every rank's masks in frame order
        assert all(torch.equal(outs[last], o) for o in outs), "every step gathers the same masks"
    t = torch.tensor([el], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el_max = float(t.item())
    wd.beat("profile pass")
    value = world * B * args.steps / el_max

    # ---- kernel timing pass (events recorded by the launches, one batch at a time) ----
    sess.set_option(pkg.VSS_OPT_PROFILE, 1)
    prof_masks = torch.empty((B, P), dtype=torch.float32, device=dev)
    for _ in range(args.steps):
        sess.segment_device(d_frames.data_ptr(), B, fh, fw, 3, rs, fs, prof_masks.data_ptr(), streams[0].cuda_stream)
    torch.cuda.synchronize(dev)
    sess.set_option(pkg.VSS_OPT_PROFILE, 0)
    ms, cnt = sess.profile_read()
    wd.disarm()  # (the legs below synchronise per call and run no collective)

    blob = open(sess.weights_path, "rb").read()
    sys.path.insert(0, os.path.join(PKG_DIR, "model"))
    import make_weights as mw
    recs, _, _ = mw.parse_blob(blob)
    costs = cm.layer_costs(recs, hm, wm, fh, fw, 3, pw_weight_bytes=2 if args.dtype == "bf16x2" else 4)
    names = [sess.layer_kernel(i) for i in range(len(ms))]
    tile_spec = sess.tile_spec()  # VSS_TILE pinning these kernels (tools/tiles_of.py, rocprof passes)
    occ = [sess.layer_occupancy(i) for i in range(len(ms))]
    per_layer = [{"layer": i, "kind": costs[i]["kind"], "kernel": names[i], "ms": round(m, 5),
                  "GBps": round(cm.launch_bytes(costs[i], B) / (m * 1e-3) / 1e9, 1) if m > 0 else None,
                  "wg_per_cu": occ[i][0] or None, "lds_bytes": occ[i][1] or None}
                 for i, m in enumerate(ms)]
    dom = int(np.argmax(ms))
    dom_name = names[dom]
    dom_bytes = cm.launch_bytes(costs[dom], B)
    achieved = dom_bytes / (ms[dom] * 1e-3)
    step_bytes = sum(cm.launch_bytes(c, B) for c in costs)  # every launch's algorithmic bytes, one batch
    traffic = None
    if args.traffic_json and os.path.exists(args.traffic_json):
        tj = json.load(open(args.traffic_json)).get(dom_name)
        if tj and tj.get("traffic_bytes"):
            traffic = round(tj["traffic_bytes"] / 1e6, 3)

    post = host = batch_sweep = latency = None
    if rank == 0 and world == 1 and not args.no_latency:
        latency = latency_leg(sess, torch, dev, d_frames, fh, fw, max(200, min(args.steps, 1000)))
    if rank == 0 and not args.no_post:
        post = post_leg(pkg, sess, d_frames, d_masks, frames, B, fh, fw, hm, wm, streams[0], args.steps,
                        args.warmup, 0.0 if args.no_cpu else 2.0)
    if rank == 0 and world == 1 and not args.no_host:
        ref = d_masks.cpu().numpy()
        host = {"vga": host_leg(pkg, frames, B, fh, fw, S, 600, ref)}
        big = syn.make_batch(B, 1080, 1920, 3)
        host["1080p"] = host_leg(pkg, big, B, 1080, 1920, S, 200)
    if rank == 0 and world == 1 and not args.no_sweep:
        batch_sweep = sweep(pkg, torch, dev, fh, fw, args.dtype, S, args.steps)

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
            "n_gpus": n_ranks,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(el_max * 1e3 / args.steps, 5),
            "median_step_ms": round(median_step_ms, 5) if median_step_ms else None,
            "value_at_median_step": round(world * B / (median_step_ms * 1e-3), 1) if median_step_ms else None,
            "graph_builds_in_timed_region": timed_builds,
            "settle_ms_before_window": args.settle_ms,
            "warmup_steps_after_settle": tail,
            "graph_patches_in_timed_region": timed_patches,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16" if args.dtype == "bf16x2" else "f32",
            "data": "synthetic",
            "config": {
                "workload": f"{B} synthetic {fw}x{fh} RGB u8 frames per GPU per step (resident in HBM) -> "
                            f"{wm}x{hm} f32 masks, {S} steps in flight (one handle, {S} slots, {S} streams)"
                            + (", RCCL all-gather of masks in the C ABI (vss_segment_gather_device)"
                               if world > 1 else ""),
                "global_batch": world * B,
                "frame": f"{fw}x{fh}x3",
                "model_res": f"{wm}x{hm}",
                "pw_gemm": "v_mfma_f32_16x16x32_bf16, f32 activations split hi+lo" if args.dtype == "bf16x2"
                           else "v_mfma_f32_16x16x4_f32",
                "graph": not args.no_graph,
                "inflight": S,
                "parallelism": f"dp{world}",
                "gather_form": sess.gather_form if gather else None,
            },
            "mask_max_abs_err": err,
            "roofline": {
                "bound": "hbm",
                "kernel": f"layer {dom} ({costs[dom]['kind']}): {dom_name}",
                "achieved": round(achieved / 1e9, 1),
                "peak": HBM_PEAK / 1e9,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK, 4),
                "traffic": traffic,
                "traffic_unit": "MB/launch (rocprofv3 PMC: 2*FETCH_SIZE + WRITE_SIZE, gfx950-corrected)",
                "alg_bytes_per_launch": dom_bytes,
                "mean_kernel_ms": round(ms[dom], 5),
                "events_count": cnt,
                "step_alg_bytes": step_bytes,
                "step_frac_at_value": round(step_bytes / B * value / world / HBM_PEAK, 4),
            },
            "kernels": per_layer,
            "tile_spec": tile_spec,
            "layer_launches_sum_ms": round(float(sum(ms)), 5),
            "launches_per_forward": sum(1 for n in names if not n.startswith("(fused")),
            "batch_sweep": batch_sweep,
            "latency": latency,
            "cpu_baseline": cpu,
            "post": post,
            "host_path": host,
            "ts_path": ts,
        }
        print(json.dumps(out), flush=True)
    sess.close()
    if world > 1:
        dist.destroy_process_group()
    return out


if __name__ == "__main__":
    main()
