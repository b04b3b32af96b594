#!/bin/bash
# Headline value against the number of batches in flight (--inflight), short
# (the driver's --steps 20 --warmup 5) and long (2000-step) windows, twice.
#   IF="2 3 4 5 6" bash tools/inflight_scan.sh TAG
TAG=${1:-ifs}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
for rep in 1 2; do
  for n in ${IF:-2 3 4 5 6}; do
    for st in "20 5" "2000 50"; do
      set -- $st
      timeout -k 10 120 python bench.py --inflight $n --steps $1 --warmup $2 --no-cpu --no-host --no-ts --no-post \
        --no-sweep --no-latency > gpurun_out/${TAG}.log 2>&1; rc=$?; fatal $rc
      tail -1 gpurun_out/${TAG}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('inflight $n steps $1: value', d['value'], 'median-step value', d.get('value_at_median_step'))"
    done
  done
done
