#!/bin/bash
# Validation of the tree: GPU tests, smoke, MODNet batch-8 f32 / bf16 / q4f16-f16
# timings with the fused blocks on and off, the default bench and the driver's
# short window.  Each GPU step has its own limit; a crash / time-out ends it.
#   bash tools/r05j_session.sh TAG
TAG=${1:-j}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
echo "== tests"
timeout -k 10 480 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread \
  > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_tests.log; grep -E "^(FAILED|ERROR)" gpurun_out/${TAG}_tests.log | head -20; fatal $rc
echo "== smoke"
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1; rc=$?
tail -1 gpurun_out/${TAG}_smoke.log; fatal $rc
echo "== MODNet batch 8"
for ir in 1 0; do
  VSO_IR=$ir timeout -k 10 300 python tools/bench_onnx.py --only-modnet --batch 8 --iters 50 \
    > gpurun_out/${TAG}_modnet_ir$ir.log 2>&1; rc=$?
  grep -h '^{' gpurun_out/${TAG}_modnet_ir$ir.log | cut -c1-150 | sed "s/^/VSO_IR=$ir /"; fatal $rc
done
timeout -k 10 300 python tools/bench_onnx.py --only-modnet --batch 1 --iters 100 --cases b1_bf16,b1_f16 \
  > gpurun_out/${TAG}_modnet_b1.log 2>&1; rc=$?
grep -h '^{' gpurun_out/${TAG}_modnet_b1.log | cut -c1-150; fatal $rc
[ "${NOBENCH:-0}" = 1 ] && exit 0
echo "== bench (default)"
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.log 2>&1; rc=$?; fatal $rc
tail -1 gpurun_out/${TAG}_bench.log > gpurun_out/${TAG}_bench.json
python3 tools/bench_brief.py gpurun_out/${TAG}_bench.json
for k in 1 2 3; do
  echo "== bench --steps 20 --warmup 5 ($k)"
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --no-host --no-ts --no-post \
    > gpurun_out/${TAG}_short$k.log 2>&1; rc=$?; fatal $rc
  tail -1 gpurun_out/${TAG}_short$k.log > gpurun_out/${TAG}_short$k.json
  python3 tools/bench_brief.py gpurun_out/${TAG}_short$k.json
done
