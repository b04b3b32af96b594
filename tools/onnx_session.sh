#!/bin/bash
# One GPU box for the ONNX sessions: the ONNX GPU tests on build A, an
# interleaved MODNet 288x512 batch-8 bf16 A/B over the given builds, and the
# per-launch MODNet table of build A (rocprofv3 kernel trace).
#   bash tools/onnx_session.sh TAG LIB_A [LIB_B ...]
TAG=$1; A=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
echo "== ONNX tests on $A"
VSS_LIBRARY=$A timeout -k 10 400 python -u -m pytest tests/test_gpu_onnx.py tests/test_gpu_face.py -m gpu -q --timeout 150 \
  --timeout-method thread > gpurun_out/${TAG}_onnx_tests.log 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_onnx_tests.log; grep -E "^(FAILED|ERROR)" gpurun_out/${TAG}_onnx_tests.log | head -20; fatal $rc
echo "== MODNet b8 bf16 A/B"
for r in 1 2; do
  for lib in "$A" "$@"; do
    VSS_LIBRARY=$lib timeout -k 10 200 python tools/bench_onnx.py --only-modnet --batch 8 --iters 50 --cases b8_bf16 \
      > gpurun_out/${TAG}_abo.log 2>&1; rc=$?
    [ $rc -ne 0 ] && { tail -5 gpurun_out/${TAG}_abo.log; fatal $rc; exit 1; }
    grep -h '^{' gpurun_out/${TAG}_abo.log | cut -c1-200 | sed "s|^|$(basename $lib) |"
  done
done
echo "== MODNet b8 bf16 per launch ($A)"
cd /tmp && export TMPDIR=/tmp
VSS_LIBRARY=$R/$A timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/${TAG}_ml" -o run -- \
  python3 "$R/tools/onnx_layers.py" run modnet:8:bf16 "$R/gpurun_out/${TAG}_ml/launches.json" > "$R/gpurun_out/${TAG}_ml.log" 2>&1
rc=$?; cd "$R"; fatal $rc
python3 tools/onnx_layers.py report gpurun_out/${TAG}_ml/launches.json gpurun_out/${TAG}_ml/run_kernel_trace.csv 2>&1 | head -70
