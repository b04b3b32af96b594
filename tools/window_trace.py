"""The driver's short headline window on the GPU's own clock: W warm-up steps,
a pause, then K timed steps exactly as bench.py issues them (4 slots, torch
streams, graph replays, synchronize on both sides).  Run it under
`rocprofv3 --kernel-trace` and give the trace to `report`:

  rocprofv3 --kernel-trace --output-format csv -d OUT -o run -- python3 tools/window_trace.py run
  python3 tools/window_trace.py report OUT/run_kernel_trace.csv

`run` prints the host's view (each step call's duration, the window);
`report` splits the GPU's view of the timed window: host issue -> first kernel,
the first step's completion, the steady completion interval, the tail."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def run(K=20, W=5, pre="sleep"):
    import numpy as np
    import torch
    from conftest import load_pkg
    pkg = load_pkg()
    import vss_amd.synthetic as syn
    B, fh, fw, S = 8, 480, 640, 4
    d = torch.from_numpy(syn.make_batch(B, fh, fw, 3)).cuda()
    with pkg.Session(max_batch=B, queue_depth=S, max_frame_h=fh, max_frame_w=fw) as s:
        outs = [torch.empty((B, s.mask_h * s.mask_w), device="cuda") for _ in range(S)]
        sts = [torch.cuda.Stream() for _ in range(S)]
        s.prepare_device(B, fh, fw, 3, fw * 3, fh * fw * 3)

        def step(i):
            s.segment_device(d.data_ptr(), B, fh, fw, 3, fw * 3, fh * fw * 3, outs[i % S].data_ptr(),
                             sts[i % S].cuda_stream)

        extra = []
        if pre == "sleep_xs":  # 24 more streams, each used once: does the post-sync cost grow with them?
            extra = [torch.cuda.Stream() for _ in range(24)]
            for st in extra:
                torch.cuda.Event().record(st)
        for i in range(W):
            step(i)
        torch.cuda.synchronize()
        if pre == "sleep_ss":  # the pause, then each step stream synchronized (no device-wide synchronize)
            time.sleep(0.05)
            for st in sts:
                st.synchronize()
        elif pre in ("sleep", "sleep_event", "sleep_xs"):
            time.sleep(0.05)  # a gap that marks the timed window in the trace
        if pre in ("event", "sleep_event"):  # one event record on every step stream (no kernel)
            for st in sts:
                torch.cuda.Event().record(st)
        if pre in ("sleep_busy", "sleep_busy_step"):  # the pause, then the device busy ~50 us right up to the sync
            time.sleep(0.05)
            if pre == "sleep_busy":
                torch.cuda._sleep(120000)
            else:  # or one untimed step on every slot
                for i in range(S):
                    step(i)
        if pre != "sleep_ss":
            torch.cuda.synchronize()
        if pre == "q_event":  # one host-side HIP query after the sync (no GPU work)
            torch.cuda.Event().query()
        elif pre == "q_stream":
            sts[0].query()
        elif pre == "sync2":
            torch.cuda.synchronize()
        elif pre == "sleep1ms":
            time.sleep(0.001)
        elif pre in ("spin1ms", "sleep_spin"):  # the host thread busy right up to the window
            if pre == "sleep_spin":
                time.sleep(0.05)
            t_end = time.perf_counter() + (0.001 if pre == "spin1ms" else 0.0003)
            while time.perf_counter() < t_end:
                pass
        import resource
        calls, durs, faults, csw = [], [], [], []
        t0 = time.perf_counter()
        for i in range(W, W + K):
            r0 = resource.getrusage(resource.RUSAGE_THREAD) if i < W + 4 else None
            c0 = time.perf_counter()
            step(i)
            calls.append((c0 - t0) * 1e6)
            durs.append((time.perf_counter() - c0) * 1e6)
            if r0 is not None:  # minor faults and context switches of this thread during the call
                r1 = resource.getrusage(resource.RUSAGE_THREAD)
                faults.append(r1.ru_minflt - r0.ru_minflt)
                csw.append((r1.ru_nvcsw - r0.ru_nvcsw, r1.ru_nivcsw - r0.ru_nivcsw))
        t_issued = (time.perf_counter() - t0) * 1e6
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) * 1e6
    print(json.dumps({"pre": pre, "window_us": round(el, 1), "issued_us": round(t_issued, 1),
                      "call_us": [round(c, 1) for c in durs], "minor_faults": faults, "ctx_switches": csw,
                      "call_start_us": [round(c, 1) for c in calls], "frames_per_s": round(B * K / el * 1e6, 1)}))


def report(path, K=20):
    import csv
    rows = []
    for r in csv.DictReader(open(path)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    # the timed window: the kernels after the largest start gap
    gaps = [(rows[i + 1][0] - rows[i][1], i + 1) for i in range(len(rows) - 1)]
    _, cut = max(gaps)
    win = rows[cut:]
    heads = sorted(e for s, e, n in win if "k_head" in n)
    first = win[0][0]
    last = max(e for _, e, _ in win)
    done = [(h - first) / 1e3 for h in heads]
    iv = [done[i + 1] - done[i] for i in range(len(done) - 1)]
    iv4 = [(done[i + 4] - done[i]) / 4 for i in range(len(done) - 4)]
    busy = 0
    cur_s, cur_e = None, None
    for s, e, _ in win:  # union of kernel intervals
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    print(json.dumps({"kernels": len(win), "steps": len(heads), "gpu_window_us": round((last - first) / 1e3, 1),
                      "first_step_done_us": round(done[0], 1) if done else None,
                      "step_done_us": [round(x, 1) for x in done],
                      "median_interval_4_us": round(sorted(iv4)[len(iv4) // 2], 2) if iv4 else None,
                      "gpu_busy_frac": round(busy / (last - first), 3)}))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(pre=sys.argv[2] if len(sys.argv) > 2 else "sleep")
    else:
        report(sys.argv[2])
