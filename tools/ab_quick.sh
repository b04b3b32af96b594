#!/bin/bash
# Interleaved A/B of the in-tree libvss.so (A) against other builds of the same
# ABI (no tests): headline value, the batch sweep, per-layer event times.
#   bash tools/ab_quick.sh N LIB_B [LIB_C ...]
set -e
N=$1; shift
mkdir -p gpurun_out
for r in $(seq 1 $N); do
  for lib in video-stream-segmenetation_amd/lib/libvss.so "$@"; do
    VSS_LIBRARY=$lib timeout -k 10 150 python bench.py --no-cpu --no-host --no-ts --no-post --steps 400 \
      > gpurun_out/abq.log 2>&1 || { tail -5 gpurun_out/abq.log; exit 1; }
    tail -1 gpurun_out/abq.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib'.split('/')[-1], d['value'], [(s['batch'], s['inflight'], s['value']) for s in d['batch_sweep']], [round(k['ms']*1000,2) for k in d['kernels']])"
  done
done
