#!/bin/bash
# Round-6 session d: the driver's short window on the GPU clock
# (tools/window_trace.py under a kernel trace, x2, and its host view x3), then
# the TS bench (tools/bench_ts.js, 600 batches per loop) for the copy pool's
# two protocols, interleaved x3.
TAG=${1:-r06d}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
for i in 1 2 3; do
  timeout -k 10 120 python3 tools/window_trace.py run > gpurun_out/${TAG}_win_host_$i.json 2>&1; rc=$?; fatal $rc
  cut -c1-400 gpurun_out/${TAG}_win_host_$i.json
done
for i in 1 2; do
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/${TAG}_win_$i" -o run -- \
    python3 "$R/tools/window_trace.py" run > "$R/gpurun_out/${TAG}_win_trace_$i.log" 2>&1; rc=$?
  cd "$R"; fatal $rc
  python3 tools/window_trace.py report gpurun_out/${TAG}_win_$i/run_kernel_trace.csv
done
for i in 1 2 3; do
  for arm in new waitall; do
    if [ $arm = waitall ]; then export VSS_COPY_WAIT_ALL=1; else unset VSS_COPY_WAIT_ALL; fi
    timeout -k 10 200 node tools/bench_ts.js 480 640 8 600 4 > gpurun_out/${TAG}_ts_${arm}_$i.json 2>&1; rc=$?; fatal $rc
    python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_ts_${arm}_$i.json').read().splitlines()[-1]);print('$arm',$i,'TS',d['value'],'zc',d['zero_copy']['value'],'batch p50',d['latency_ms_p50'],'frame p50',d['single_frame']['latency_ms_p50'])"
  done
done
unset VSS_COPY_WAIT_ALL
