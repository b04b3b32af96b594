#!/bin/bash
# End-of-session check of the tree as committed: every GPU test, smoke(), the
# default bench line.  Stops at the first failing step.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-final}
mkdir -p "$R/gpurun_out"
cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
  > "gpurun_out/gpu_tests_$TAG.log" 2>&1 || { tail -30 "gpurun_out/gpu_tests_$TAG.log"; exit 1; }
tail -2 "gpurun_out/gpu_tests_$TAG.log"
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "gpurun_out/smoke_$TAG.log" 2>&1 \
  || { tail -20 "gpurun_out/smoke_$TAG.log"; exit 1; }
tail -1 "gpurun_out/smoke_$TAG.log"
timeout -k 10 300 python bench.py > "gpurun_out/bench_$TAG.log" 2>&1 || { tail -20 "gpurun_out/bench_$TAG.log"; exit 1; }
tail -1 "gpurun_out/bench_$TAG.log" > "gpurun_out/bench_$TAG.json"
cut -c1-400 "gpurun_out/bench_$TAG.json"
