#!/bin/bash
# Persistent k_conv_tile: ONNX GPU tests, interleaved A/B (persist on / off /
# the pre-persistent build / the old UP staging), per-launch tables.
TAG=${1:-z}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 480 python -u -m pytest tests/test_gpu_onnx.py -m gpu -x -q --timeout 250 \
  --timeout-method thread > gpurun_out/${TAG}_onnx.log 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_onnx.log; grep -E "^(FAILED|ERROR)" gpurun_out/${TAG}_onnx.log | cut -c1-200 | head
[ $rc -ne 0 ] && exit $rc
ARMS="VSO_CONV_PERSIST=1;VSO_CONV_PERSIST=0;VSS_LIBRARY=abvar/libvss_prepersist.so;VSS_LIBRARY=abvar/libvss_upold.so" \
  timeout -k 10 600 bash tools/ab_arms_onnx.sh 2 b8_bf16,b8_f32 || exit 1
ARMS="VSO_CONV_PERSIST=1;VSO_CONV_PERSIST=0" GREP="k_conv_tile" timeout -k 10 400 bash tools/arms_layers.sh r05z modnet:8:bf16
