#!/bin/bash
# SE chain: Gemm activation epilogue, per-plane binary, wave-per-plane GAP:
# ONNX + face GPU tests, interleaved MODNet A/B against all three off,
# per-launch tables.
TAG=${1:-ah}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 480 python -u -m pytest tests/test_gpu_onnx.py tests/test_gpu_face.py -m gpu -x -q --timeout 250 \
  --timeout-method thread > gpurun_out/${TAG}_onnx.log 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_onnx.log; grep -E "^(FAILED|ERROR)" gpurun_out/${TAG}_onnx.log | cut -c1-200 | head
[ $rc -ne 0 ] && exit $rc
OFF="VSO_GEMM_ACT=0 VSO_BIN_PLANES=0 VSO_GAP_WAVE=0"
ARMS="VSO_X=0;$OFF" timeout -k 10 500 bash tools/ab_arms_onnx.sh 3 b8_bf16,b8_f32 || exit 1
ARMS="VSO_X=0;$OFF" BATCH=1 timeout -k 10 300 bash tools/ab_arms_onnx.sh 2 b1_bf16 || exit 1
ARMS="VSO_X=0;$OFF" GREP="k_gap|k_gemm|k_binary|k_unary" timeout -k 10 400 bash tools/arms_layers.sh r05ah modnet:8:bf16
