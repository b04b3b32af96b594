#!/bin/bash
# One SQ PMC pass over the headline bench (the bench's tiles pinned from a
# previous bench line if VSS_TILE is set): per-kernel SQ_INSTS_VALU / LDS / MFMA
# means, printed as a table (tools/sq_table.py).  Usage: bash tools/prof_sq.sh TAG
set -euo pipefail
TAG=${1:-sq}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_WAVES GRBM_GUI_ACTIVE \
  --output-format csv -d "$OUT/mfma" -o run -- \
  python3 "$R/bench.py" --no-cpu --no-host --no-ts --no-sweep --no-post --steps 20 --warmup 5 > "$OUT/mfma.log" 2>&1
cd "$R"
python3 tools/sq_table.py "$OUT/mfma/run_counter_collection.csv"
