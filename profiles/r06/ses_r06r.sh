#!/bin/bash
# Round-6 session r: MODNet's 3x3 64 -> 64 layer at 72x128, batch 8, f16 (and
# its neighbours) alone (tools/conv_probe.py): time, kernel trace, wave states,
# HBM bytes.
TAG=${1:-r06r}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
for sh in 8,64,64,72,128 8,99,64,72,128 8,64,32,72,128 8,64,64,144,256 1,64,64,72,128; do
  timeout -k 10 120 python3 tools/conv_probe.py --shape $sh > gpurun_out/${TAG}_t.log 2>&1; rc=$?; fatal $rc
  grep -h '^{' gpurun_out/${TAG}_t.log | cut -c1-400
done
for e in VSO_CONV_MAX_TH=4 VSO_CONV_MAX_TH=0 VSO_CONV_BM_MAX=32 VSO_CONV_WANT=4096; do
  env $e timeout -k 10 120 python3 tools/conv_probe.py > gpurun_out/${TAG}_t.log 2>&1; rc=$?; fatal $rc
  grep -h '^{' gpurun_out/${TAG}_t.log | cut -c1-300 | sed "s|^|[$e] |"
done
cd /tmp && export TMPDIR=/tmp
P="python3 $R/tools/conv_probe.py --iters 50 --warmup 5"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_${TAG}/trace" -o run -- $P > "$R/gpurun_out/${TAG}_trace.log" 2>&1; rc=$?; fatal $rc
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES SQ_BUSY_CYCLES \
  --output-format csv -d "$R/gpurun_out/prof_${TAG}/stall" -o run -- $P > "$R/gpurun_out/${TAG}_stall.log" 2>&1; rc=$?; fatal $rc
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/prof_${TAG}/fetch" -o run -- $P > /dev/null 2>&1; rc=$?; fatal $rc
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/prof_${TAG}/write" -o run -- $P > /dev/null 2>&1; rc=$?; fatal $rc
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE \
  --output-format csv -d "$R/gpurun_out/prof_${TAG}/insts" -o run -- $P > /dev/null 2>&1; rc=$?; fatal $rc
cd "$R"
python3 - gpurun_out/prof_${TAG} <<'PY'
import csv, glob, sys
from collections import defaultdict
root = sys.argv[1]
d = defaultdict(lambda: defaultdict(list))
for f in glob.glob(root + "/*/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        d[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for f in glob.glob(root + "/trace/**/run_kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        d[r["Kernel_Name"].split("(")[0]]["dur_us"].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        d[r["Kernel_Name"].split("(")[0]]["grid"].append(float(r["Grid_Size_X"]))
for k, c in d.items():
    m = {n: sum(v) / len(v) for n, v in c.items()}
    print(k, {n: round(v, 3) for n, v in sorted(m.items())})
PY
