#!/bin/bash
# Persistent k_conv_tile for f32 operands only: ONNX + face GPU tests, then
# in-tree vs the pre-persistent build (all bench_onnx cases, batch 8 and 1).
TAG=${1:-aa}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 480 python -u -m pytest tests/test_gpu_onnx.py tests/test_gpu_face.py -m gpu -x -q --timeout 250 \
  --timeout-method thread > gpurun_out/${TAG}_onnx.log 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_onnx.log; grep -E "^(FAILED|ERROR)" gpurun_out/${TAG}_onnx.log | cut -c1-200 | head
[ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for lib in video-stream-segmenetation_amd/lib/libvss.so abvar/libvss_upold.so; do
    VSS_LIBRARY=$lib timeout -k 10 300 python tools/bench_onnx.py --batch 8 --iters 50 > gpurun_out/${TAG}_b8.log 2>&1 || exit 1
    grep -h '^{' gpurun_out/${TAG}_b8.log | python3 -c '
import json, sys
for l in sys.stdin:
    d = json.loads(l); print(sys.argv[1], "b8", d["model"], d.get("ms_per_run", d.get("ms_per_face_frame")))' $(basename $lib)
    VSS_LIBRARY=$lib timeout -k 10 300 python tools/bench_onnx.py --only-modnet --batch 1 --iters 100 --cases b1_f32,b1_bf16 > gpurun_out/${TAG}_b1.log 2>&1 || exit 1
    grep -h '^{' gpurun_out/${TAG}_b1.log | python3 -c '
import json, sys
for l in sys.stdin:
    d = json.loads(l); print(sys.argv[1], "b1", d["model"], d["ms_per_run"])' $(basename $lib)
  done
done
