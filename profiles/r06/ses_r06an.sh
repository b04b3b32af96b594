#!/bin/bash
# Round-6 session an: one-frame calls moving the frame's rows with
# k_fetch_rows (reads of pinned host memory) instead of one DMA of the whole
# frame (VSS_FETCH_SINGLE=1) — the TS phase table and the bench's host / TS
# legs interleaved x3, the engine / TS / parity GPU tests with it on.
TAG=${1:-r06an}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
VSS_FETCH_SINGLE=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_engine.py tests/test_ts.py tests/test_gpu_parity.py > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_tests.log; fatal $rc; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for fs in 1 0; do
    export VSS_FETCH_SINGLE=$fs
    timeout -k 10 300 node tools/ts_prof.js 400 > gpurun_out/${TAG}_tsprof_${fs}_$i.json 2>&1; rc=$?; fatal $rc
    python3 -c "
import json;d=json.load(open('gpurun_out/${TAG}_tsprof_${fs}_$i.json'))
v=d['segmentFrame'];print('fetch $fs',$i,'segmentFrame',{k:v[k]['p50'] for k in v if k in ('total_us','submit_us','device_us','deliver_hop_us')})"
    timeout -k 10 300 python bench.py --steps 200 --no-cpu --no-post --no-sweep > gpurun_out/${TAG}_b_${fs}_$i.log 2>&1; rc=$?; fatal $rc
    python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_b_${fs}_$i.log').read().splitlines()[-1]);h=d['host_path']['vga'];t=d['ts_path'];print('fetch $fs',$i,'C pinned',h['copy_pinned_out']['value'],'TS',t['value'],'frame p50',t['single_frame']['latency_ms_p50'],'p99',t['single_frame'].get('latency_ms_p99'))"
  done
done
