"""Per-launch timing of one GPU ONNX session (include/vso.h) from a rocprofv3
kernel trace: which layers of a model the run time goes to.

On the GPU box (from the repo root):
    cd /tmp && rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/ol -o run -- \
        python3 $R/tools/onnx_layers.py run mediapipe_face_detector $R/gpurun_out/ol/launches.json
then anywhere:
    python tools/onnx_layers.py report gpurun_out/ol/launches.json gpurun_out/ol/<...>/run_kernel_trace.csv

`run` replays the session ITERS times (inputs / outputs in HBM) and writes the
launch list (vso_launch_name order); `report` matches the trace's vso::
dispatches to it position by position and prints the average duration and grid
of each launch, sorted by total time.
"""
from __future__ import annotations

import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ITERS = 30


def run(key, out):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch
    import bench
    bench._load_pkg()
    import vss_amd.ort as ort
    import onnx_models as M
    if key.startswith("modnet"):  # modnet[_q4f16]:B:PREC — the full topology at 288x512
        name, b, prec = (key.split(":") + ["1", "bf16"])[:3]
        model = M.modnet(288, 512, q4f16=name.endswith("q4f16"))
        kw = {"input_shape": (int(b), 3, 288, 512), "precision": prec}
    else:
        model = M.load_golden(os.path.join(ROOT, "tests", "golden", key + ".npz"))[0]
        kw = {}
    with ort.InferenceSession(model, **kw) as s:
        din = [torch.rand(sh, dtype=torch.float32, device="cuda") for sh in s.input_shapes]
        dout = [torch.empty(sh, dtype=torch.float32, device="cuda") for sh in s.output_shapes]
        st = torch.cuda.Stream()
        for _ in range(5 + ITERS):
            s.run_device([t.data_ptr() for t in din], [t.data_ptr() for t in dout], st.cuda_stream)
        st.synchronize()
        os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
        json.dump({"key": key, "iters": ITERS, "launches": s.launches()}, open(out, "w"))


def report(launches_path, trace_path):
    meta = json.load(open(launches_path))
    names = meta["launches"]
    L = len(names)
    rows = sorted((r for r in csv.DictReader(open(trace_path)) if "vso::" in r["Kernel_Name"]),
                  key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[-meta["iters"] * L:]
    assert len(rows) == meta["iters"] * L, (len(rows), L)
    dur = [[] for _ in range(L)]
    grid = [None] * L
    base = lambda n: n.split("(")[0].replace("void ", "")
    # per iteration, each dispatch (in start order) goes to the first launch of
    # its name not yet matched: with two capture lanes (vso_lane_count) the
    # lanes' dispatches interleave, each lane in launch order
    for it in range(meta["iters"]):
        free = list(range(L))
        for r in rows[it * L:(it + 1) * L]:
            k = next((j for j in free if base(names[j]) == base(r["Kernel_Name"])), None)
            assert k is not None, (it, r["Kernel_Name"])
            free.remove(k)
            dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
            grid[k] = (r.get("Grid_Size_X") or r.get("Grid_X"), r.get("Grid_Size_Y") or r.get("Grid_Y"),
                       r.get("Grid_Size_Z") or r.get("Grid_Z"))
    starts = [int(r["Start_Timestamp"]) for r in rows]
    ends = [int(r["End_Timestamp"]) for r in rows]
    span = [(ends[(i + 1) * L - 1] - starts[i * L]) / 1000.0 for i in range(meta["iters"])]
    avg = [sum(d) / len(d) for d in dur]
    busy = sum(avg)
    wall = sum(span) / len(span)
    print(f"{meta['key']}: {L} launches, kernel time {busy:.1f} us, first-to-last {wall:.1f} us "
          f"(gaps {wall - busy:.1f} us; negative: launches overlapping on the capture lanes)")
    order = sorted(range(L), key=lambda k: -avg[k])
    for k in order[:25]:
        print(f"  #{k:3d} {avg[k]:7.2f} us  grid {grid[k]}  {names[k].split('(')[0]}")
    by = {}
    for k in range(L):
        n = names[k].split("(")[0].replace("void ", "")
        by.setdefault(n, [0, 0.0])
        by[n][0] += 1
        by[n][1] += avg[k]
    for n, (c, t) in sorted(by.items(), key=lambda x: -x[1][1]):
        print(f"  {n:28s} x{c:3d} {t:8.1f} us")


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2], sys.argv[3])
    else:
        report(sys.argv[2], sys.argv[3])
