#!/bin/bash
# Two capture lanes: ONNX + face GPU tests, then MODNet / face timings with
# VSO_LANES=2 (default) and 1, interleaved.
TAG=${1:-u}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
timeout -k 10 480 python -u -m pytest tests/test_gpu_onnx.py tests/test_gpu_face.py -m gpu -q -s --timeout 250 \
  --timeout-method thread > gpurun_out/${TAG}_onnx.log 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_onnx.log; grep -E "^(FAILED|ERROR)|lanes|operand oracle" gpurun_out/${TAG}_onnx.log | cut -c1-200 | head; fatal $rc
[ $rc -ne 0 ] && exit $rc
for k in 1 2; do
  for l in 2 1; do
    VSO_LANES=$l timeout -k 10 300 python tools/bench_onnx.py --batch 8 --iters 50 > gpurun_out/${TAG}_b8.log 2>&1; rc=$?
    grep -h '^{' gpurun_out/${TAG}_b8.log | cut -c1-140 | sed "s/^/lanes $l b8 /"; fatal $rc
    VSO_LANES=$l timeout -k 10 300 python tools/bench_onnx.py --only-modnet --batch 1 --iters 100 --cases b1_bf16,b1_f16 \
      > gpurun_out/${TAG}_b1.log 2>&1; rc=$?
    grep -h '^{' gpurun_out/${TAG}_b1.log | cut -c1-140 | sed "s/^/lanes $l b1 /"; fatal $rc
  done
done
