#!/bin/bash
# Partial-chunk quad skip in k_conv_tile: ONNX + face GPU tests, interleaved
# A/B against VSO_CONV_QSKIP=0 (every bench_onnx case at batch 8), per-launch
# tables of the conv tiles.
TAG=${1:-aj}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 480 python -u -m pytest tests/test_gpu_onnx.py tests/test_gpu_face.py -m gpu -x -q --timeout 250 \
  --timeout-method thread > gpurun_out/${TAG}_onnx.log 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_onnx.log; grep -E "^(FAILED|ERROR)" gpurun_out/${TAG}_onnx.log | cut -c1-200 | head
[ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for a in "VSO_X=0" "VSO_CONV_QSKIP=0"; do
    env $a timeout -k 10 300 python tools/bench_onnx.py --batch 8 --iters 50 > gpurun_out/${TAG}_b8.log 2>&1 || exit 1
    grep -h '^{' gpurun_out/${TAG}_b8.log | python3 -c '
import json, sys
for l in sys.stdin:
    d = json.loads(l); print(sys.argv[1], d["model"], d.get("ms_per_run", d.get("ms_per_face_frame")))' "$a"
  done
done
ARMS="VSO_X=0;VSO_CONV_QSKIP=0" GREP="k_conv_tile" timeout -k 10 400 bash tools/arms_layers.sh r05aj modnet:8:bf16
