#!/bin/bash
# k_conv_tile conflict-free layouts: ONNX + face GPU tests, then an
# interleaved MODNet A/B against the VSO_CONV_SWZ=0 build.
TAG=${1:-w}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 480 python -u -m pytest tests/test_gpu_onnx.py tests/test_gpu_face.py -m gpu -x -q --timeout 250 \
  --timeout-method thread > gpurun_out/${TAG}_onnx.log 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_onnx.log; grep -E "^(FAILED|ERROR)" gpurun_out/${TAG}_onnx.log | cut -c1-200 | head
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 bash tools/ab_onnx.sh abvar/libvss_convswz0.so 2
