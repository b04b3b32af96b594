#!/bin/bash
# Round-6 session az: k_conv_pw over a split K (pw_split_plan; VSO_PW_SPLIT=0
# off): the ONNX GPU tests, the deep 1x1 probes alone, MODNet b8 interleaved.
TAG=${1:-r06az}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_onnx.py > gpurun_out/${TAG}_onnx_tests.log 2>&1; rc=$?
tail -3 gpurun_out/${TAG}_onnx_tests.log; fatal $rc; [ $rc -ne 0 ] && exit $rc
for sh in 8,320,1280,9,16 8,96,576,18,32 1,320,1280,9,16; do
  for sp in 1 0; do
    VSO_PW_SPLIT=$sp timeout -k 10 120 python tools/conv_probe.py --k 1 --shape $sh --prec f16 --iters 200 > gpurun_out/${TAG}_$sh.log 2>&1; rc=$?; fatal $rc
    [ $rc -ne 0 ] && { tail -5 gpurun_out/${TAG}_$sh.log; exit $rc; }
    grep -h '^{' gpurun_out/${TAG}_$sh.log | cut -c1-130 | sed "s|^|[split=$sp] |"
  done
done
for r in 1 2; do
  for sp in 1 0; do
    VSO_PW_SPLIT=$sp timeout -k 10 300 python tools/bench_onnx.py --only-modnet --batch 8 --iters 50 --cases b8_bf16,b8_f16 > gpurun_out/${TAG}_onnx.log 2>&1; rc=$?; fatal $rc
    [ $rc -ne 0 ] && { tail -5 gpurun_out/${TAG}_onnx.log; exit $rc; }
    grep -h '^{' gpurun_out/${TAG}_onnx.log | cut -c1-100 | sed "s|^|[split=$sp] |"
  done
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
