#!/bin/bash
# Full check of the current tree on the GPU box: GPU tests, smoke(), the default
# bench line (with the CPU baseline and mask parity), then the rocprof passes.
# Usage (from the repo root on the box): bash tools/round_check.sh TAG
set -euo pipefail
TAG=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/gpu_tests_$TAG.log 2>&1 || { tail -40 gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -3 gpurun_out/gpu_tests_$TAG.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 \
  || { tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
echo smoke ok
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log > gpurun_out/bench_$TAG.json
cut -c1-300 gpurun_out/bench_$TAG.json
# the profiled runs replay the tiles the bench's autotuner chose: autotuning
# under the profiler's per-dispatch overhead picks differently, and the
# summary's durations must describe the kernels the bench line timed
export VSS_TILE=$(python3 tools/tiles_of.py gpurun_out/bench_$TAG.json)
echo "VSS_TILE=$VSS_TILE"
bash tools/prof_run.sh "$TAG"
