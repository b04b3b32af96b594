#!/bin/bash
# Interleaved MODNet batch-8 timings under environment arms ("A;B;..." — each
# an env assignment list, VSS_LIBRARY=relative paths allowed):
#   ARMS="VSO_X=0;VSO_X=1" bash tools/ab_arms_onnx.sh ROUNDS CASES
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
N=$1; CASES=$2
mkdir -p gpurun_out
IFS=';' read -ra arms <<< "$ARMS"
for r in $(seq 1 $N); do
  for a in "${arms[@]}"; do
    env $a timeout -k 10 200 python tools/bench_onnx.py --only-modnet --batch ${BATCH:-8} --iters 60 --cases "$CASES" \
      > gpurun_out/aba.log 2>&1 || { tail -5 gpurun_out/aba.log; exit 1; }
    grep -h '^{' gpurun_out/aba.log | python3 -c '
import json, sys
for l in sys.stdin:
    d = json.loads(l); print(sys.argv[1], d["model"], d["ms_per_run"])' "$a"
  done
done
