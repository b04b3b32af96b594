#!/bin/bash
# Round-6 session bc: SQ wave states of the 320 -> 1280 1x1 on k_conv_pw alone
# (tools/conv_probe.py), and of the 16 -> 32 at 72x128 — where their time goes.
TAG=${1:-r06bc}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for sh in 8,320,1280,9,16 8,16,32,72,128; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
    SQ_ACTIVE_INST_LDS SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d "$R/gpurun_out/prof_${TAG}_$sh" -o run -- \
    python3 "$R/tools/conv_probe.py" --k 1 --shape $sh --prec f16 --iters 50 > "$R/gpurun_out/${TAG}_$sh.log" 2>&1 || { tail -5 "$R/gpurun_out/${TAG}_$sh.log"; exit 1; }
  python3 - "$R/gpurun_out/prof_${TAG}_$sh" <<'PY'
import csv, sys, glob
from collections import defaultdict
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
d = defaultdict(lambda: defaultdict(list))
for r in csv.DictReader(open(f)):
    d[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in d.items():
    if "k_conv_pw" not in k: continue
    m = {n: sum(v) / len(v) for n, v in c.items()}
    wc = m.get("SQ_WAVE_CYCLES", 0) or 1
    print(f"wait {m.get('SQ_WAIT_ANY', 0) / wc:5.2f} issue-stall {m.get('SQ_WAIT_INST_ANY', 0) / wc:5.2f} active "
          f"{m.get('SQ_ACTIVE_INST_ANY', 0) / wc:5.2f} (valu {m.get('SQ_ACTIVE_INST_VALU', 0) / wc:5.2f} lds "
          f"{m.get('SQ_ACTIVE_INST_LDS', 0) / wc:5.2f})  waves {m.get('SQ_WAVES', 0):.0f} wave-cyc/wave {wc / max(m.get('SQ_WAVES', 1), 1):8.0f} busy {m.get('SQ_BUSY_CYCLES', 0):.0f}  {k[:50]}")
PY
done
