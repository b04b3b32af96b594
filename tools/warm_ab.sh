#!/bin/bash
# The driver's short window (--steps 20) after 5 vs 500 untimed warmup steps,
# interleaved: does the window carry a device ramp beyond the pipeline's fill?
#   bash tools/warm_ab.sh TAG
TAG=${1:-warm}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
for rep in 1 2 3; do
  for w in 5 500; do
    timeout -k 10 120 python bench.py --steps 20 --warmup $w --no-cpu --no-host --no-ts --no-post --no-sweep --no-latency \
      > gpurun_out/${TAG}.log 2>&1; rc=$?; fatal $rc
    tail -1 gpurun_out/${TAG}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('warmup $w: value', d['value'], 'median-step value', d.get('value_at_median_step'))"
  done
done
for rep in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --no-host --no-post > gpurun_out/${TAG}.log 2>&1; rc=$?; fatal $rc
  tail -1 gpurun_out/${TAG}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('full legs, warmup 5: value', d['value'], 'median-step value', d.get('value_at_median_step'))"
done
