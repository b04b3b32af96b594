#!/bin/bash
# Concat tails read by their k_conv_tile consumer (ConvTileParams::x2) and the
# 256-VGPR cap on the upsample tiles: ONNX + face GPU tests, interleaved A/B
# against VSO_CAT_TAIL=0 (every bench_onnx case at batch 8, MODNet batch 1),
# per-launch tables.
TAG=${1:-al}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 480 python -u -m pytest tests/test_gpu_onnx.py tests/test_gpu_face.py -m gpu -x -q --timeout 250 \
  --timeout-method thread > gpurun_out/${TAG}_onnx.log 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_onnx.log; grep -E "^(FAILED|ERROR)" gpurun_out/${TAG}_onnx.log | cut -c1-200 | head
[ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for a in "VSO_X=0" "VSO_CAT_TAIL=0"; do
    env $a timeout -k 10 300 python tools/bench_onnx.py --batch 8 --iters 50 > gpurun_out/${TAG}_b8.log 2>&1 || exit 1
    grep -h '^{' gpurun_out/${TAG}_b8.log | python3 -c '
import json, sys
for l in sys.stdin:
    d = json.loads(l); print(sys.argv[1], d["model"], d.get("ms_per_run", d.get("ms_per_face_frame")), d.get("launches"))' "$a"
  done
done
ARMS="VSO_X=0;VSO_CAT_TAIL=0" BATCH=1 timeout -k 10 300 bash tools/ab_arms_onnx.sh 2 b1_bf16,b1_f32 || exit 1
ARMS="VSO_X=0;VSO_CAT_TAIL=0" GREP="k_conv_tile|k_copy" timeout -k 10 400 bash tools/arms_layers.sh r05al modnet:8:bf16
