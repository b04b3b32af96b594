#!/bin/bash
# The TS path at several queue depths (tools/bench_ts.js, 640x480 batch 8).
set -e
mkdir -p gpurun_out
for d in 4 6 8; do
  timeout -k 10 120 node tools/bench_ts.js 480 640 8 400 $d > gpurun_out/tsd_$d.json
  echo "depth $d $(cut -c1-420 gpurun_out/tsd_$d.json)"
done
