#!/bin/bash
# Seam weight DMA ordering / coverage A/B: parity tests on the all-layers
# build, then interleaved 400-step runs of the in-tree build, DMA-first and
# DMA-first-all-layers (per-kernel times from the event pass).
TAG=${1:-an}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
for v in wfirst wall; do
  VSS_LIBRARY=$R/abvar/libvss_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 \
    --timeout-method thread > gpurun_out/${TAG}_$v.log 2>&1 || { tail -20 gpurun_out/${TAG}_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/${TAG}_$v.log)"
done
for r in 1 2 3; do
  for lib in video-stream-segmenetation_amd/lib/libvss.so abvar/libvss_wfirst.so abvar/libvss_wall.so; do
    VSS_LIBRARY=$R/$lib timeout -k 10 120 python bench.py --no-cpu --no-host --no-ts --no-post --steps 400 > gpurun_out/${TAG}_b.log 2>&1 || exit 1
    tail -1 gpurun_out/${TAG}_b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], d["value"], [k["ms"] for k in d["kernels"]])' $(basename $lib)
  done
done
