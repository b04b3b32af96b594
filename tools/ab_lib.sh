#!/bin/bash
# A/B of the in-tree libvss.so (A) against another build of the same ABI (B,
# given as a path): GPU tests on A, then N interleaved short bench runs of each
# (headline config and the post / compositing legs; no CPU or host legs).
# Usage: bash tools/ab_lib.sh LIB_B [N]
set -e
B=$1
N=${2:-3}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
for r in $(seq 1 $N); do
  timeout -k 10 120 python bench.py --no-cpu --no-host --steps ${STEPS:-400} ${BENCH_ARGS} > gpurun_out/ab_a$r.log 2>&1
  tail -1 gpurun_out/ab_a$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("A", d["value"], d["post"]["value"], d["post"]["composite"]["value"], [k["ms"] for k in d["kernels"]])'
  VSS_LIBRARY=$B timeout -k 10 120 python bench.py --no-cpu --no-host --steps ${STEPS:-400} ${BENCH_ARGS} > gpurun_out/ab_b$r.log 2>&1
  tail -1 gpurun_out/ab_b$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("B", d["value"], d["post"]["value"], d["post"]["composite"]["value"], [k["ms"] for k in d["kernels"]])'
done
