#!/bin/bash
# GPU tests, then N short bench runs (headline config, no CPU / post legs)
# printing frames/s and the per-layer kernel times.  Usage: bash tools/quick_ab.sh [N]
set -e
N=${1:-3}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/qab_tests.log 2>&1 || { tail -30 gpurun_out/qab_tests.log; exit 1; }
tail -1 gpurun_out/qab_tests.log
for r in $(seq 1 $N); do
  timeout -k 10 120 python bench.py --no-cpu --no-post --steps 400 > gpurun_out/qab_$r.log 2>&1
  tail -1 gpurun_out/qab_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["mask_max_abs_err"], [k["ms"] for k in d["kernels"]])'
done
