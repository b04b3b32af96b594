#!/bin/bash
# Size-based lane policy: the full GPU suite, then MODNet b8 / b1 and face
# timings under the default policy and VSO_LANES=1.
TAG=${1:-v}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread \
  > gpurun_out/${TAG}_gpu.log 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_gpu.log; grep -E "^(FAILED|ERROR)" gpurun_out/${TAG}_gpu.log | cut -c1-200 | head; fatal $rc
[ $rc -ne 0 ] && exit $rc
for l in default 1; do
  e=""; [ $l != default ] && e="VSO_LANES=$l"
  env $e timeout -k 10 300 python tools/bench_onnx.py --batch 8 --iters 50 > gpurun_out/${TAG}_b8.log 2>&1; rc=$?
  grep -h '^{' gpurun_out/${TAG}_b8.log | cut -c1-140 | sed "s/^/lanes $l b8 /"; fatal $rc
  env $e timeout -k 10 300 python tools/bench_onnx.py --only-modnet --batch 1 --iters 100 --cases b1_bf16,b1_f16 \
    > gpurun_out/${TAG}_b1.log 2>&1; rc=$?
  grep -h '^{' gpurun_out/${TAG}_b1.log | cut -c1-140 | sed "s/^/lanes $l b1 /"; fatal $rc
done
