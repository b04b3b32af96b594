#!/bin/bash
# Round-5 GPU session: GPU tests, smoke, the default bench line and the
# driver's short window (--steps 20 --warmup 5) three times; then, unless
# NOPROF=1, the rocprof passes (trace + FETCH / WRITE / SQ, SQ, wave state)
# with the bench's tiles pinned.  Every step has its own time limit; a
# time-out, abort or crash stops the script (a failing test only reports).
#   bash tools/r05_session.sh TAG
TAG=${1:-s}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
if [ "${NOTESTS:-0}" != 1 ]; then
echo "== tests"
timeout -k 10 420 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread \
  > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_tests.log; grep -E "^(FAILED|ERROR)" gpurun_out/${TAG}_tests.log | head -20; fatal $rc
echo "== smoke"
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1; rc=$?
tail -1 gpurun_out/${TAG}_smoke.log; fatal $rc
fi
if [ "${ONNX:-0}" = 1 ]; then
  echo "== ONNX: fused inverted residuals, MODNet parity prints"
  timeout -k 10 400 python -u -m pytest tests/test_gpu_onnx.py -m gpu -s -q --timeout 200 --timeout-method thread \
    -k "modnet_topology or inverted or conv_up or synthetic" > gpurun_out/${TAG}_onnx.log 2>&1; rc=$?
  tail -2 gpurun_out/${TAG}_onnx.log; grep -E "^(FAILED|ERROR)|max abs err|oracle" gpurun_out/${TAG}_onnx.log | cut -c1-200 | head -40; fatal $rc
  for k in 1 2; do
    for arm in "1 1" "1 0" "0 1"; do
      set -- $arm
      VSO_IR=$1 VSO_IR_B16=$2 timeout -k 10 200 python tools/bench_onnx.py --only-modnet --batch 8 --iters 50 \
        > gpurun_out/${TAG}_modnet_ir$1$2.log 2>&1; rc=$?
      echo "VSO_IR=$1 VSO_IR_B16=$2: $(grep -h '^{' gpurun_out/${TAG}_modnet_ir$1$2.log | grep b8_bf16 | cut -c1-160)"; fatal $rc
    done
  done
fi
if [ -n "${AB_LIBS:-}" ]; then
  echo "== A/B vs $AB_LIBS"
  timeout -k 10 600 bash tools/ab_quick.sh ${AB_ROUNDS:-3} $AB_LIBS; fatal $?
fi
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
[ "${NOPROF:-0}" = 1 ] && exit 0
export VSS_TILE=$(python3 tools/tiles_of.py gpurun_out/${TAG}_bench.json)
echo "VSS_TILE=$VSS_TILE"
echo "== rocprof passes"
timeout -k 10 500 bash tools/prof_run.sh "$TAG" > gpurun_out/${TAG}_prof.log 2>&1; fatal $?
echo "== SQ pass"
timeout -k 10 200 bash tools/prof_sq.sh "$TAG"; fatal $?
echo "== wave-state pass"
timeout -k 10 200 bash tools/prof_stall.sh "$TAG"; fatal $?
