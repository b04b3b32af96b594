#!/bin/bash
# Seam weight image by LDS-DMA: full GPU tests, smoke, then interleaved short
# bench runs against the VSS_WDMA=0 build (per-kernel times in each line).
TAG=${1:-ac}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -5 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
STEPS=400 timeout -k 10 900 bash tools/ab_lib.sh abvar/libvss_wdma0.so 3
