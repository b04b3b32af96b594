#!/bin/bash
# Round-6 session av: MODNet's 1x1 convolutions on k_conv_pw alone (tools/conv_probe.py --k 1),
# to separate their own time from the two-lane overlap in the model's trace.
TAG=${1:-r06av}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
for sh in 8,320,1280,9,16 8,16,32,144,256 8,16,32,72,128 8,96,576,18,32 8,32,192,72,128; do
  timeout -k 10 120 python tools/conv_probe.py --k 1 --shape $sh --prec f16 --iters 200 > gpurun_out/${TAG}_$sh.log 2>&1; rc=$?; fatal $rc
  [ $rc -ne 0 ] && { tail -5 gpurun_out/${TAG}_$sh.log; exit $rc; }
  grep -h '^{' gpurun_out/${TAG}_$sh.log
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_${TAG}" -o run -- \
  python3 "$R/tools/conv_probe.py" --k 1 --shape 8,320,1280,9,16 --prec f16 --iters 100 > "$R/gpurun_out/${TAG}_prof.log" 2>&1; rc=$?
cd "$R"; fatal $rc
python3 - <<PY
import csv,glob
f=glob.glob('gpurun_out/prof_${TAG}/**/*kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)): print(r['Name'][:60], r['Calls'], r['AverageNs'])
PY
