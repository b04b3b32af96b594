#!/bin/bash
# ONNX GPU tests on the tree's library, then per-launch MODNet tables of the
# tree's library and of abvar/libvss_irold.so (the previous k_ir_b16).
TAG=${1:-t}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_onnx.py -m gpu -q -s --timeout 200 --timeout-method thread \
  -k "inverted or modnet_topology" > gpurun_out/${TAG}_onnx.log 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_onnx.log; grep -E "^(FAILED|ERROR)|ir_chain|operand oracle" gpurun_out/${TAG}_onnx.log | cut -c1-200; fatal $rc
[ $rc -ne 0 ] && exit $rc
ARMS="VSS_LIBRARY=video-stream-segmenetation_amd/lib/libvss.so;VSS_LIBRARY=abvar/libvss_irold.so;VSS_LIBRARY=video-stream-segmenetation_amd/lib/libvss.so;VSS_LIBRARY=abvar/libvss_irold.so" \
  bash tools/arms_layers.sh ${TAG}
