#!/bin/bash
# Profile bench.py on the GPU box: one kernel-trace/stats pass and two PMC
# passes (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950: TCC slots).
# Usage (from the repo root on the box): bash tools/prof_run.sh TAG [bench args...]
set -euo pipefail
TAG=${1:-r01}
shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
  python3 "$R/bench.py" --no-cpu --no-host --no-ts --no-sweep --no-post "$@" > "$OUT/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- \
  python3 "$R/bench.py" --no-cpu --no-host --no-ts --no-sweep --no-post --steps 20 --warmup 5 "$@" > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- \
  python3 "$R/bench.py" --no-cpu --no-host --no-ts --no-sweep --no-post --steps 20 --warmup 5 "$@" > "$OUT/write.log" 2>&1
# MFMA / VALU / LDS activity (SQ slots: 7 of 8; GRBM 1 of 2)
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F32 \
  SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d "$OUT/mfma" -o run -- \
  python3 "$R/bench.py" --no-cpu --no-host --no-ts --no-sweep --no-post --steps 20 --warmup 5 "$@" > "$OUT/mfma.log" 2>&1
echo "profiles in $OUT"
