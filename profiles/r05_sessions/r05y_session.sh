#!/bin/bash
# UP staging reads unconditional: ONNX GPU tests, interleaved MODNet A/B
# against the old staging build, and per-launch tables of both.
TAG=${1:-y}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 480 python -u -m pytest tests/test_gpu_onnx.py -m gpu -x -q --timeout 250 \
  --timeout-method thread > gpurun_out/${TAG}_onnx.log 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_onnx.log; grep -E "^(FAILED|ERROR)" gpurun_out/${TAG}_onnx.log | cut -c1-200 | head
[ $rc -ne 0 ] && exit $rc
timeout -k 10 500 bash tools/ab_libs_onnx.sh 3 b8_bf16,b8_f16 abvar/libvss_upold.so || exit 1
ARMS="VSS_LIBRARY=video-stream-segmenetation_amd/lib/libvss.so;VSS_LIBRARY=abvar/libvss_upold.so" GREP="k_conv_tile_up" \
  timeout -k 10 500 bash tools/arms_layers.sh r05y modnet:8:bf16
