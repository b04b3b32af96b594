#!/bin/bash
# Per-layer weight DMA: A/B against the VSS_WDMA=0 build (GPU tests first),
# then the full validation (r05j_session: tests, smoke, MODNet, default bench,
# the driver's short window x3).
TAG=${1:-ad}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
STEPS=400 timeout -k 10 600 bash tools/ab_lib.sh abvar/libvss_wdma0.so 3 || exit $?
timeout -k 10 900 bash tools/r05j_session.sh ${TAG}
