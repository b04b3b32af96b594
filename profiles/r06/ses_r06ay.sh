#!/bin/bash
# Round-6 session ay: the large InstanceNorm planes (36864 elements) on 1024
# (default), 512 and 256-thread workgroups (VSO_NORM_BIG): ONNX norm / MODNet
# tests under each, MODNet b8 interleaved, the kernels' times under the trace.
TAG=${1:-r06ay}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
for nb in 256 512; do
  VSO_NORM_BIG=$nb timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_onnx.py -k "norm or modnet_topology" > gpurun_out/${TAG}_tests_$nb.log 2>&1; rc=$?
  tail -2 gpurun_out/${TAG}_tests_$nb.log | sed "s|^|[$nb] |"; fatal $rc; [ $rc -ne 0 ] && exit $rc
done
for r in 1 2; do
  for nb in 1024 256 512; do
    VSO_NORM_BIG=$nb timeout -k 10 300 python tools/bench_onnx.py --only-modnet --batch 8 --iters 50 --cases b8_bf16,b8_f16 > gpurun_out/${TAG}_onnx.log 2>&1; rc=$?; fatal $rc
    [ $rc -ne 0 ] && { tail -5 gpurun_out/${TAG}_onnx.log; exit $rc; }
    grep -h '^{' gpurun_out/${TAG}_onnx.log | cut -c1-100 | sed "s|^|[$nb] |"
  done
done
cd /tmp && export TMPDIR=/tmp
for nb in 1024 256 512; do
  VSO_NORM_BIG=$nb timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_${TAG}_$nb" -o run -- \
    python3 "$R/tools/bench_onnx.py" --only-modnet --batch 8 --iters 30 --cases q4f16_288x512_b8_f16 > "$R/gpurun_out/${TAG}_prof_$nb.log" 2>&1; rc=$?
  fatal $rc; [ $rc -ne 0 ] && exit $rc
  python3 - <<PY
import csv,glob
f=glob.glob('$R/gpurun_out/prof_${TAG}_$nb/**/*kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'norm_plane' in r['Name']: print('[$nb]', r['Name'][:50], r['Calls'], round(float(r['AverageNs'])/1e3,2), 'us')
PY
done
