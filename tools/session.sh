#!/bin/bash
# One GPU box, several measurements (boxes are scarce; each step has its own
# time limit, and a GPU fault / abort / kill / time-out stops the script):
#   1 the GPU test suite          2 interleaved A/B vs the base library
#   3 an SQ PMC pass (VALU / LDS / MFMA per kernel)
#   4 a wave-state pass   5 a MODNet b8 kernel trace and its per-launch table
# Usage: bash tools/session.sh TAG [LIB ...]   (default: every ablib/libvss_*.so)
TAG=${1:-s}
shift || true
LIBS="$*"
[ -z "$LIBS" ] && LIBS=$(ls ablib/libvss_*.so 2>/dev/null | tr '\n' ' ')
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
echo "== tests"
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread \
  > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
tail -3 gpurun_out/${TAG}_tests.log; grep -E "^(FAILED|ERROR)" gpurun_out/${TAG}_tests.log | head -20; fatal $rc
echo "== A/B vs $LIBS"
if [ -n "$LIBS" ]; then timeout -k 10 700 bash tools/ab_quick.sh 2 $LIBS; fatal $?; fi
echo "== SQ pass"
timeout -k 10 200 bash tools/prof_sq.sh ${TAG}; fatal $?
echo "== stall pass"
timeout -k 10 200 bash tools/prof_stall.sh ${TAG}; fatal $?
echo "== MODNet b8 trace"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${TAG}_modnet" -o run -- \
  python3 "$R/tools/bench_onnx.py" --only-modnet --batch 8 --iters 50 --cases b8_bf16 > "$R/gpurun_out/${TAG}_modnet.log" 2>&1
rc=$?; cd "$R"; tail -2 gpurun_out/${TAG}_modnet.log; fatal $rc
python3 tools/trace_top.py gpurun_out/${TAG}_modnet/run_kernel_stats.csv 25
echo "== MODNet b8 bf16 per launch"
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/${TAG}_ml" -o run -- \
  python3 "$R/tools/onnx_layers.py" run modnet:8:bf16 "$R/gpurun_out/${TAG}_ml/launches.json" > "$R/gpurun_out/${TAG}_ml.log" 2>&1
rc=$?; cd "$R"; fatal $rc
python3 tools/onnx_layers.py report gpurun_out/${TAG}_ml/launches.json gpurun_out/${TAG}_ml/run_kernel_trace.csv 2>&1 | head -60
