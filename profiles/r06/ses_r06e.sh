#!/bin/bash
# Round-6 session e: the short window's first step call (tools/window_trace.py
# host view with VSS_TIME_DEVICE=1 phase stamps) for four pre-window states.
TAG=${1:-r06e}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
for i in 1 2; do
  for pre in none sleep event sleep_event; do
    VSS_TIME_DEVICE=1 timeout -k 10 120 python3 tools/window_trace.py run $pre > gpurun_out/${TAG}_${pre}_$i.json 2> gpurun_out/${TAG}_${pre}_$i.err; rc=$?; fatal $rc
    python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_${pre}_$i.json').read().splitlines()[-1]);print(d['pre'],$i,'window',d['window_us'],'fps',d['frames_per_s'],'calls',d['call_us'][:6])"
    grep "call " gpurun_out/${TAG}_${pre}_$i.err | tail -21 | head -4
  done
done
