#!/bin/bash
# Interleaved MODNet batch-8 A/B over several builds (the in-tree libvss.so
# first): bash tools/ab_libs_onnx.sh ROUNDS CASES LIB_B [LIB_C ...]
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
N=$1; CASES=$2; shift 2
mkdir -p gpurun_out
for r in $(seq 1 $N); do
  for lib in video-stream-segmenetation_amd/lib/libvss.so "$@"; do
    VSS_LIBRARY=$lib timeout -k 10 200 python tools/bench_onnx.py --only-modnet --batch 8 --iters 60 --cases "$CASES" \
      > gpurun_out/abl.log 2>&1 || { tail -5 gpurun_out/abl.log; exit 1; }
    grep -h '^{' gpurun_out/abl.log | python3 -c '
import json, sys
for l in sys.stdin:
    d = json.loads(l); print(sys.argv[1], d["model"], d["ms_per_run"])' "$(basename $lib)"
  done
done
