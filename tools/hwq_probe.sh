#!/bin/bash
# headline at several in-flight depths, default and 8 hardware queues
mkdir -p gpurun_out
for q in 4 8; do
  for inf in 4 6 8; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 150 python bench.py --no-cpu --no-host --no-ts --no-post --no-sweep --steps 400 --inflight $inf > gpurun_out/hwq.log 2>&1 || { tail -5 gpurun_out/hwq.log; exit 1; }
    tail -1 gpurun_out/hwq.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('hwq $q inflight $inf', d['value'], d.get('median_value', d.get('value_median')), d['ms_per_step'])"
  done
done
