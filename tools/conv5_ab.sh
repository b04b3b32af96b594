#!/bin/bash
# A/B of the deep 16-bit 5x5 tile rule (VSO_CONV_DEEP_TILE) on MODNet 288x512
# batch 8: kernel-trace passes of tools/bench_onnx.py, per-launch durations of
# the 5x5 convolutions; then one SQ pass (MFMA busy) with the rule on.
# Usage (repo root on the box): bash tools/conv5_ab.sh TAG
set -euo pipefail
TAG=${1:-c5}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
for v in 0 1 2 0 1 2; do
  VSO_CONV_DEEP_TILE=$v timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/t$v" -o run -- \
    python3 "$R/tools/bench_onnx.py" --only-modnet --batch 8 --cases modnet_288x512_b8_bf16 --iters 20 --warmup 5 \
    > "$OUT/t$v.log" 2>&1
  grep modnet "$OUT/t$v.log" | cut -c1-160
  python3 "$R/tools/conv5_ab.py" "$OUT/t$v"
done
VSO_CONV_DEEP_TILE=1 timeout -k 10 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE SQ_BUSY_CYCLES \
  --output-format csv -d "$OUT/sq" -o run -- \
  python3 "$R/tools/bench_onnx.py" --only-modnet --batch 8 --cases modnet_288x512_b8_bf16 --iters 2 --warmup 1 \
  > "$OUT/sq.log" 2>&1
echo "done $OUT"
