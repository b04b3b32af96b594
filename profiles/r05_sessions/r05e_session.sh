#!/bin/bash
# k_ir_b16 time attribution on MODNet b8 bf16: the per-launch table under each
# VSO_IR_PROBE value (vso_kernels.h IrParams::probe: phases skipped, results
# invalid), then one SQ wave-state PMC pass (probe 0).
#   PROBES="0 1 2 4 8 16 31" bash tools/r05e_session.sh TAG
TAG=${1:-e}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
export TMPDIR=/tmp
for pr in ${PROBES:-0 1 2 4 8 16 31}; do
  cd /tmp
  VSO_IR_PROBE=$pr timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/${TAG}_p$pr" -o run -- \
    python3 "$R/tools/onnx_layers.py" run modnet:8:bf16 "$R/gpurun_out/${TAG}_p$pr/launches.json" > "$R/gpurun_out/${TAG}_p$pr.log" 2>&1
  rc=$?; cd "$R"; fatal $rc
  python3 tools/onnx_layers.py report gpurun_out/${TAG}_p$pr/launches.json gpurun_out/${TAG}_p$pr/run_kernel_trace.csv \
    > gpurun_out/${TAG}_p${pr}_report.txt 2>&1
  echo "== probe $pr: $(head -1 gpurun_out/${TAG}_p${pr}_report.txt)"
  grep "k_ir" gpurun_out/${TAG}_p${pr}_report.txt | grep " x " || true
done
echo "== wave state (probe 0)"
cd /tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
  SQ_ACTIVE_INST_LDS SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d "$R/gpurun_out/${TAG}_ws" -o run -- \
  python3 "$R/tools/bench_onnx.py" --only-modnet --batch 8 --iters 10 --warmup 3 --cases b8_bf16 > "$R/gpurun_out/${TAG}_ws.log" 2>&1
rc=$?; cd "$R"; fatal $rc
python3 - "gpurun_out/${TAG}_ws/run_counter_collection.csv" <<'PY'
import csv, sys
from collections import defaultdict
d = defaultdict(lambda: defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    d[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in sorted(d.items()):
    m = {n: sum(v) / len(v) for n, v in c.items()}
    wc = m.get("SQ_WAVE_CYCLES", 0) or 1
    w = m.get("SQ_WAVES", 1) or 1
    print(f"wait {m.get('SQ_WAIT_ANY', 0) / wc:5.2f} issue-stall {m.get('SQ_WAIT_INST_ANY', 0) / wc:5.2f} active "
          f"{m.get('SQ_ACTIVE_INST_ANY', 0) / wc:5.2f} (valu {m.get('SQ_ACTIVE_INST_VALU', 0) / wc:5.2f} lds "
          f"{m.get('SQ_ACTIVE_INST_LDS', 0) / wc:5.2f})  wave-cyc/wave {4 * wc / w:8.0f}  waves {w:6.0f}  {k}")
PY
