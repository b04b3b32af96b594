#!/bin/bash
# tools/micro/queue_map, one process per case (run on the GPU box)
cd "$(dirname "$0")"
for touch in 0 1; do
  for extra in 0 1 2 3 5; do
    for mode in normal high cumask; do
      timeout -k 5 30 ./queue_map $extra $mode $touch || echo "case $extra $mode $touch failed"
    done
  done
done
