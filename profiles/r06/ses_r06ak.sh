#!/bin/bash
# Round-6 session ak: the ordered all-gather at one rank under a kernel +
# memory-copy trace: what the gather stream runs per step and for how long.
TAG=${1:-r06ak}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
cd /tmp && export TMPDIR=/tmp
for form in ordered concurrent; do
  timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$R/gpurun_out/prof_${TAG}_$form" -o run -- \
    python3 "$R/bench.py" --steps 200 --warmup 5 --gather --gather-form $form --no-cpu --no-host --no-ts --no-post --no-sweep --no-latency > "$R/gpurun_out/${TAG}_$form.log" 2>&1; rc=$?; fatal $rc
done
cd "$R"
python3 - gpurun_out/prof_${TAG}_ordered gpurun_out/prof_${TAG}_concurrent <<'PY'
import csv, glob, sys
from collections import defaultdict
for root in sys.argv[1:]:
    rows = []
    for f in glob.glob(root + "/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][:60], r.get("Queue_Id", ""), r.get("Stream_Id", "")))
    mc = []
    for f in glob.glob(root + "/**/*memory_copy_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            mc.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Direction", r.get("Kind", "")), r.get("Size", r.get("Bytes", ""))))
    d = defaultdict(list)
    for s, e, k, q, st in rows:
        d[k].append((e - s) / 1e3)
    print(root)
    for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1]))[:16]:
        v.sort()
        print(f"   {k:60s} n {len(v):5d} p50 {v[len(v)//2]:8.2f} us  max {v[-1]:8.2f}")
    if mc:
        v = sorted((e - s) / 1e3 for s, e, _, _ in mc)
        print(f"   memory copies n {len(mc)} p50 {v[len(v)//2]:.2f} us, kinds {set(x[2] for x in mc)}, sizes {sorted(set(x[3] for x in mc))[:5]}")
    # the non-forward kernels: their start relative to the previous k_head end
    heads = sorted(e for s, e, k, q, st in rows if "k_head" in k)
    others = sorted((s, e, k) for s, e, k, q, st in rows if "vss::" not in k and "vso::" not in k)
    import bisect
    lag = []
    for s, e, k in others[-300:]:
        i = bisect.bisect_left(heads, s)
        if i > 0:
            lag.append((s - heads[i - 1]) / 1e3)
    if lag:
        lag.sort()
        print(f"   non-vss kernels start after the latest k_head end: p50 {lag[len(lag)//2]:.1f} us")
PY
