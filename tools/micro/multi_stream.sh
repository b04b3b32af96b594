#!/bin/bash
# tools/micro/multi_stream under several hardware-queue settings (run on the GPU box)
set -e
cd "$(dirname "$0")"
for q in 4 2 8 16; do
  for mode in "graph" "stream" "graph prio"; do
    echo "== GPU_MAX_HW_QUEUES=$q $mode"
    GPU_MAX_HW_QUEUES=$q timeout -k 5 60 ./multi_stream $mode
  done
done
