#!/bin/bash
# SQ wave-state pass over the headline bench (4 batches in flight): per kernel,
# wave cycles split into waiting (s_waitcnt / barrier), issue-stalled and
# active, and the VALU / LDS share of the active cycles (MI355X_MICROARCH.md:
# WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~ WAVE_CYCLES).
#   bash tools/prof_stall.sh TAG
set -euo pipefail
TAG=${1:-stall}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
  SQ_ACTIVE_INST_LDS SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d "$OUT/stall" -o run -- \
  python3 "$R/bench.py" --no-cpu --no-host --no-ts --no-sweep --no-post --steps 20 --warmup 5 > "$OUT/stall.log" 2>&1
cd "$R"
python3 - "$OUT/stall/run_counter_collection.csv" <<'PY'
import csv, sys
from collections import defaultdict
d = defaultdict(lambda: defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    d[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
hot = max(len(c.get("SQ_WAVES", [])) for c in d.values())
for k, c in sorted(d.items(), key=lambda kv: -len(kv[1].get("SQ_WAVES", []))):
    m = {n: sum(v) / len(v) for n, v in c.items()}
    wc = m.get("SQ_WAVE_CYCLES", 0) or 1
    if len(c.get("SQ_WAVES", [])) < 0.8 * hot:  # the timed forwards' kernels only
        continue
    print(f"wait {m.get('SQ_WAIT_ANY', 0) / wc:5.2f} issue-stall {m.get('SQ_WAIT_INST_ANY', 0) / wc:5.2f} active "
          f"{m.get('SQ_ACTIVE_INST_ANY', 0) / wc:5.2f} (valu {m.get('SQ_ACTIVE_INST_VALU', 0) / wc:5.2f} lds "
          f"{m.get('SQ_ACTIVE_INST_LDS', 0) / wc:5.2f})  wave-cyc/wave {wc / max(m.get('SQ_WAVES', 1), 1):8.0f}  {k[:80]}")
PY
