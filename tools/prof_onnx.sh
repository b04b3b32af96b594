#!/bin/bash
# Profile tools/bench_onnx.py on the GPU box, as tools/prof_run.sh does bench.py:
# one kernel-trace/stats pass and three PMC passes (FETCH_SIZE, WRITE_SIZE,
# MFMA/VALU/LDS activity), each in a run of its own.
# Usage (from the repo root on the box): bash tools/prof_onnx.sh TAG [bench_onnx args...]
set -euo pipefail
TAG=${1:-onnx}
shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
  python3 "$R/tools/bench_onnx.py" "$@" > "$OUT/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- \
  python3 "$R/tools/bench_onnx.py" "$@" > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- \
  python3 "$R/tools/bench_onnx.py" "$@" > "$OUT/write.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F32 \
  SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d "$OUT/mfma" -o run -- \
  python3 "$R/tools/bench_onnx.py" "$@" > "$OUT/mfma.log" 2>&1
echo "profiles in $OUT"
