#!/bin/bash
# Interleaved A/B of environment settings under the driver's short window
# (--steps 20 --warmup 5): headline, median step, the batch-8 sweep (1 / 4 in
# flight) and the one-call-at-a-time latency leg, per setting and round.
#   bash tools/ab_short.sh N "VAR=a" "VAR=b" ...   ("-" = no setting)
N=$1; shift
mkdir -p gpurun_out
for r in $(seq 1 $N); do
  for e in "$@"; do
    ev=$e; [ "$e" = "-" ] && ev="VSS_AB_NONE=1"
    env $ev timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --no-host --no-ts --no-post \
      > gpurun_out/abs.log 2>&1 || { tail -5 gpurun_out/abs.log; exit 1; }
    tail -1 gpurun_out/abs.log | python -c "
import json, sys
d = json.loads(sys.stdin.read())
sw = {(s['batch'], s['inflight']): s['value'] for s in d['batch_sweep']}
lt = d.get('latency') or {}
print('$e', d['value'], d['value_at_median_step'], 'b8/1', sw.get((8, 1)), 'b8/4', sw.get((8, 4)),
      'lat1', lt.get('batch1', {}).get('latency_ms_p50'), 'lat8', lt.get('batch8', {}).get('latency_ms_p50'),
      [round(k['ms'] * 1000, 2) for k in d['kernels']])"
  done
done
