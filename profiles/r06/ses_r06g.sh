#!/bin/bash
# Round-6 session g: which host call pays the first-call penalty after a
# device synchronize (tools/window_trace.py variants, VSS_TIME_DEVICE=1), x2.
TAG=${1:-r06g}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
for i in 1 2; do
  for pre in none q_event q_stream sync2 sleep1ms; do
    VSS_TIME_DEVICE=1 timeout -k 10 120 python3 tools/window_trace.py run $pre > gpurun_out/${TAG}_${pre}_$i.json 2> gpurun_out/${TAG}_${pre}_$i.err; rc=$?; fatal $rc
    python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_${pre}_$i.json').read().splitlines()[-1]);print(d['pre'],$i,'window',d['window_us'],'fps',d['frames_per_s'],'calls',d['call_us'][:6])"
    grep "call " gpurun_out/${TAG}_${pre}_$i.err | tail -20 | head -2
  done
done
