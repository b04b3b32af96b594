#!/bin/bash
# Round-6 session n/o/p: the first call after the window's synchronize —
# page faults, context switches, streams, the device-wide synchronize, and the
# runtime's knobs (tools/window_trace.py, bench's settle form "sleep").
TAG=${1:-r06p}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
one() {  # name env...
  local name=$1; shift
  env "$@" VSS_TIME_DEVICE=1 timeout -k 10 120 python3 tools/window_trace.py run sleep > gpurun_out/${TAG}_${name}_$i.json 2> gpurun_out/${TAG}_${name}_$i.err; rc=$?; fatal $rc
  python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_${name}_$i.json').read().splitlines()[-1]);print('$name',$i,'window',d['window_us'],'calls',d['call_us'][:4])"
}
for i in 1 2 3; do
  one base A=1
  one devkarg HIP_FORCE_DEV_KERNARG=1
  one nowait ROC_ACTIVE_WAIT_TIMEOUT=0
  one noreclaim HSA_NO_SCRATCH_RECLAIM=1
  one nomarker HIP_FORCE_QUEUE_PROFILING=0 ROC_SKIP_KERNEL_ARG_COPY=1
done
