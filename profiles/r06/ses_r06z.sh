#!/bin/bash
# Round-6 session z: the window's first call after bench's settle form
# (synchronize, pause, synchronize) against the device kept busy up to the
# last synchronize (a ~50 us spin kernel, or one untimed step per slot).
TAG=${1:-r06z}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
for i in 1 2 3 4; do
  for pre in sleep sleep_busy sleep_busy_step; do
    VSS_TIME_DEVICE=1 timeout -k 10 120 python3 tools/window_trace.py run $pre > gpurun_out/${TAG}_${pre}_$i.json 2> gpurun_out/${TAG}_${pre}_$i.err; rc=$?; fatal $rc
    python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_${pre}_$i.json').read().splitlines()[-1]);print(d['pre'],$i,'window',d['window_us'],'calls',d['call_us'][:4])"
  done
done
