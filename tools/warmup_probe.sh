#!/bin/bash
# headline window vs median step by --warmup (and --steps): bash tools/warmup_probe.sh
mkdir -p gpurun_out
for r in 1 2; do
  for w in 5 20 200 1000; do
    for k in 20 200; do
      timeout -k 10 150 python bench.py --no-cpu --no-host --no-ts --no-post --no-sweep --steps $k --warmup $w \
        > gpurun_out/wup.log 2>&1 || { tail -5 gpurun_out/wup.log; exit 1; }
      tail -1 gpurun_out/wup.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('warmup $w steps $k', d['value'], d['value_at_median_step'])"
    done
  done
done
