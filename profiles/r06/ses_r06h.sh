#!/bin/bash
# Round-6 session h: where the short window's early-call penalty goes
# (tools/window_trace.py none / sleep1ms, VSS_TIME_DEVICE=1) under runtime and
# library variants: default, no slot wait (diagnostic), HSA_ENABLE_INTERRUPT=0.
TAG=${1:-r06h}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
for i in 1 2; do
  for v in default noclaim nointr; do
    for pre in none sleep1ms; do
      case $v in
        default) E="";;
        noclaim) E="VSS_TEST_NO_CLAIM=1";;
        nointr) E="HSA_ENABLE_INTERRUPT=0";;
      esac
      env $E VSS_TIME_DEVICE=1 timeout -k 10 120 python3 tools/window_trace.py run $pre > gpurun_out/${TAG}_${v}_${pre}_$i.json 2> gpurun_out/${TAG}_${v}_${pre}_$i.err; rc=$?; fatal $rc
      python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_${v}_${pre}_$i.json').read().splitlines()[-1]);print('$v',d['pre'],$i,'window',d['window_us'],'fps',d['frames_per_s'],'calls',d['call_us'][:5])"
      grep "call " gpurun_out/${TAG}_${v}_${pre}_$i.err | tail -20 | head -2
    done
  done
done
