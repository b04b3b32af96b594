#!/bin/bash
# The ONNX GPU tests on build A, then MODNet 288x512 batch 8 bf16 interleaved
# over builds A B ... and A's per-launch table: bash tools/onnx_ab_quick.sh TAG A [B ...]
TAG=$1; A=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
VSS_LIBRARY=$A timeout -k 10 300 python -u -m pytest tests/test_gpu_onnx.py tests/test_gpu_face.py -m gpu -q --timeout 150 \
  --timeout-method thread > gpurun_out/${TAG}_onnx_tests.log 2>&1; rc=$?
tail -1 gpurun_out/${TAG}_onnx_tests.log; grep -E "^(FAILED|ERROR)" gpurun_out/${TAG}_onnx_tests.log | head; fatal $rc
for r in 1 2; do
  for lib in "$A" "$@"; do
    VSS_LIBRARY=$lib timeout -k 10 200 python tools/bench_onnx.py --only-modnet --batch 8 --iters 50 --cases b8_bf16 \
      > gpurun_out/${TAG}_abo.log 2>&1; rc=$?
    [ $rc -ne 0 ] && { tail -5 gpurun_out/${TAG}_abo.log; fatal $rc; exit 1; }
    grep -h '^{' gpurun_out/${TAG}_abo.log | cut -c1-110 | sed "s|^|$(basename $lib) |"
  done
done
cd /tmp && export TMPDIR=/tmp
VSS_LIBRARY=$R/$A timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/${TAG}_ml" -o run -- \
  python3 "$R/tools/onnx_layers.py" run modnet:8:bf16 "$R/gpurun_out/${TAG}_ml/launches.json" > "$R/gpurun_out/${TAG}_ml.log" 2>&1
rc=$?; cd "$R"; fatal $rc
python3 tools/onnx_layers.py report gpurun_out/${TAG}_ml/launches.json gpurun_out/${TAG}_ml/run_kernel_trace.csv 2>&1 | tail -26
