#!/bin/bash
# Round-6 session i: the host thread's state before the short window (none /
# sleep1ms / spin1ms / sleep + spin), tools/window_trace.py x3 each, and the
# process's CPU affinity and quota.
TAG=${1:-r06i}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
python3 -c "import os;print('affinity',len(os.sched_getaffinity(0)))"; cat /sys/fs/cgroup/cpu.max 2>/dev/null; cat /sys/fs/cgroup/cpu.stat 2>/dev/null | head -6
for i in 1 2 3; do
  for pre in none sleep1ms spin1ms sleep_spin; do
    VSS_TIME_DEVICE=1 timeout -k 10 120 python3 tools/window_trace.py run $pre > gpurun_out/${TAG}_${pre}_$i.json 2> gpurun_out/${TAG}_${pre}_$i.err; rc=$?; fatal $rc
    python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_${pre}_$i.json').read().splitlines()[-1]);print(d['pre'],$i,'window',d['window_us'],'fps',d['frames_per_s'],'calls',d['call_us'][:5])"
    grep "call " gpurun_out/${TAG}_${pre}_$i.err | tail -20 | head -1
  done
done
cat /sys/fs/cgroup/cpu.stat 2>/dev/null | head -6
