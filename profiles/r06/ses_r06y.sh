#!/bin/bash
# Round-6 session y: one small batch's staging copy and DMA in two halves
# (VSS_COPY_SPLIT) — the engine / parity / TS GPU tests, the TS phase table
# and the bench's host legs interleaved against VSS_COPY_SPLIT=0; the
# upsample tiles' height knob (VSO_UP_MAX_TH) on the fusion layer and MODNet.
TAG=${1:-r06y}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_engine.py tests/test_ts.py tests/test_gpu_parity.py tests/test_gpu_configs.py > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_tests.log; fatal $rc; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for sp in 1 0; do
    export VSS_COPY_SPLIT=$sp
    timeout -k 10 300 node tools/ts_prof.js 400 > gpurun_out/${TAG}_tsprof_${sp}_$i.json 2>&1; rc=$?; fatal $rc
    python3 -c "
import json;d=json.load(open('gpurun_out/${TAG}_tsprof_${sp}_$i.json'))
for m,v in d.items():
  if m.startswith('segmentFrame'): print('split $sp',$i,m,{k:v[k]['p50'] for k in v if k.endswith('_us')})"
  done
done
unset VSS_COPY_SPLIT
cd /tmp && export TMPDIR=/tmp
for e in - VSO_UP_MAX_TH=4 VSO_UP_MAX_TH=2; do
  D="$R/gpurun_out/prof_${TAG}/fu_${e//=/_}"
  env $( [ "$e" = "-" ] || echo $e ) timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$D" -o run -- python3 $R/tools/conv_probe.py --up 32 --shape 8,35,16,288,512 --iters 50 --warmup 5 > /dev/null 2>&1; rc=$?; fatal $rc
  python3 - "$D" "$e" <<'PY'
import csv, glob, sys
dur = {}
for f in glob.glob(sys.argv[1] + "/**/run_kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if "vso::" in k:
            dur.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in dur.items():
    v.sort()
    print(f"{sys.argv[2]:18s} {k:44s} n {len(v):3d} p50 {v[len(v)//2]:7.2f} us")
PY
done
cd "$R"
for r in 1 2; do
  for e in - VSO_UP_MAX_TH=4; do
    env $( [ "$e" = "-" ] || echo $e ) timeout -k 10 300 python tools/bench_onnx.py --only-modnet --batch 8 --iters 50 --cases b8_bf16,b8_f16 > gpurun_out/${TAG}_onnx.log 2>&1; rc=$?; fatal $rc
    grep -h '^{' gpurun_out/${TAG}_onnx.log | cut -c1-100 | sed "s|^|[$e] |"
  done
done
