#!/bin/bash
# Round-6 session j: the driver's command with an untimed settle before the
# timed window (bench.py --settle-ms 0 / 5 / 20), interleaved x6.
TAG=${1:-r06j}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
B="--no-ts --no-host --no-post --no-cpu --no-sweep --no-latency"
for i in 1 2 3 4 5 6; do
  for st in 0 5 20; do
    timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --settle-ms $st $B > gpurun_out/${TAG}_s${st}_$i.log 2>&1; rc=$?; fatal $rc
    python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_s${st}_$i.log').read().splitlines()[-1]);print('settle',$st,$i,d['value'],d['value_at_median_step'])"
  done
done
