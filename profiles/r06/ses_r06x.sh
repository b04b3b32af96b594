#!/bin/bash
# Round-6 session x: wave states and instruction counts of the fused-upsample
# fusion layer (35 -> 16 at 288x512) and the 3x3 64 -> 64 at 72x128 alone;
# the tile knobs on the latter after the XCD order.
TAG=${1:-r06x}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
for e in - VSO_CONV_BM_MAX=32 VSO_CONV_WANT=2048 VSO_CONV_WANT=512 VSO_CONV_MAX_TH=4; do
  env $( [ "$e" = "-" ] || echo $e ) timeout -k 10 120 python3 tools/conv_probe.py > gpurun_out/${TAG}_t.log 2>&1; rc=$?; fatal $rc
  grep -h '^{' gpurun_out/${TAG}_t.log | cut -c1-300 | sed "s|^|[$e] |"
done
cd /tmp && export TMPDIR=/tmp
for arg in "--up 32 --shape 8,35,16,288,512" "--shape 8,64,64,72,128"; do
  D="$R/gpurun_out/prof_${TAG}/$(echo $arg | tr -d ' -' | tr ',' '_')"
  P="python3 $R/tools/conv_probe.py $arg --iters 30 --warmup 3"
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES SQ_BUSY_CYCLES \
    --output-format csv -d "$D/stall" -o run -- $P > /dev/null 2>&1; rc=$?; fatal $rc
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE \
    --output-format csv -d "$D/insts" -o run -- $P > /dev/null 2>&1; rc=$?; fatal $rc
  timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_EXP SQ_INSTS_SMEM SQ_VALU_MFMA_BUSY_CYCLES \
    --output-format csv -d "$D/misc" -o run -- $P > /dev/null 2>&1; rc=$?; echo "misc rc=$rc"; fatal $rc
  python3 - "$D" "$arg" <<'PY'
import csv, glob, sys
from collections import defaultdict
d = defaultdict(list)
for f in glob.glob(sys.argv[1] + "/*/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_conv_tile" in r["Kernel_Name"]:
            d[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {k: sum(v) / len(v) for k, v in d.items()}
w = m.get("SQ_WAVES", 1)
print(sys.argv[2], "waves", w)
for k in sorted(m):
    print(f"   {k:28s} {m[k]:14.0f}  per wave {m[k] / w:10.1f}")
PY
done
