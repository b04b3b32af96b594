#!/bin/bash
# Interleaved A/B of one environment setting on the headline and the sweep:
#   bash tools/ab_env.sh N "VAR=a" "VAR=b"
N=$1; A=$2; B=$3
mkdir -p gpurun_out
for r in $(seq 1 $N); do
  for e in "$A" "$B"; do
    env $e timeout -k 10 150 python bench.py --no-cpu --no-host --no-ts --no-post --steps 400 > gpurun_out/abe.log 2>&1 \
      || { tail -5 gpurun_out/abe.log; exit 1; }
    tail -1 gpurun_out/abe.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$e', d['value'], d['value_at_median_step'], [(s['batch'], s['inflight'], s['value']) for s in d['batch_sweep']])"
  done
done
