#!/bin/bash
# Round-6 session ae: the completion thread polling its batch's event for up to
# VSS_COMPLETION_SPIN_US before the blocking wait — the TS phase table and
# the bench's TS / host legs, interleaved x3.
TAG=${1:-r06ae}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
for i in 1 2 3; do
  for sp in 0 300; do
    export VSS_COMPLETION_SPIN_US=$sp
    timeout -k 10 300 node tools/ts_prof.js 400 > gpurun_out/${TAG}_tsprof_${sp}_$i.json 2>&1; rc=$?; fatal $rc
    python3 -c "
import json;d=json.load(open('gpurun_out/${TAG}_tsprof_${sp}_$i.json'))
for m,v in d.items():
  if m.startswith('segmentFrame'): print('spin $sp',$i,m,{k:v[k]['p50'] for k in v if k in ('total_us','submit_us','device_us','deliver_hop_us')}, v.get('frames_per_s',''))"
    timeout -k 10 300 python bench.py --steps 200 --no-cpu --no-post --no-sweep --no-latency > gpurun_out/${TAG}_b_${sp}_$i.log 2>&1; rc=$?; fatal $rc
    python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_b_${sp}_$i.log').read().splitlines()[-1]);h=d['host_path']['vga'];t=d['ts_path'];print('spin $sp',$i,'C copy',h['copy']['value'],'pinned',h['copy_pinned_out']['value'],'zc',h['zero_copy']['value'],'TS',t['value'],'frame p50',t['single_frame']['latency_ms_p50'])"
  done
done
