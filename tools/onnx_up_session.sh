#!/bin/bash
# ONNX / face GPU tests on the in-tree build, then MODNet b8 bf16 with and
# without the Resize-in-convolution fusion, then the per-launch table.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
TAG=${1:-up}
timeout -k 10 300 python -u -m pytest tests/test_gpu_onnx.py tests/test_gpu_face.py -m gpu -q -x --timeout 150 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
tail -3 gpurun_out/${TAG}_tests.log; grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/${TAG}_tests.log | head -20
[ $rc -ne 0 ] && exit $rc
bash tools/onnx_env_ab.sh "-" "VSO_UP_FUSE=0" 2>&1 | grep -v "^[0-9]* passed" || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/${TAG}_ml" -o run -- \
  python3 "$R/tools/onnx_layers.py" run modnet:8:bf16 "$R/gpurun_out/${TAG}_ml/launches.json" > "$R/gpurun_out/${TAG}_ml.log" 2>&1 || exit $?
cd "$R"; python3 tools/onnx_layers.py report gpurun_out/${TAG}_ml/launches.json gpurun_out/${TAG}_ml/run_kernel_trace.csv 2>&1 | tail -40
