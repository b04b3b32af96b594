#!/bin/bash
# Round-6 session ao: one frame's staging copy on the copy pool
# (VSS_COPY_INLINE_BYTES=262144: 0.55 MB in 256 KB pieces) against the
# calling thread alone (default 1 MiB) — TS phase table and the bench's TS /
# host legs, interleaved x3 (k_fetch_rows for one frame on in both).
TAG=${1:-r06ao}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
for i in 1 2 3; do
  for ib in 262144 1048576; do
    export VSS_COPY_INLINE_BYTES=$ib
    timeout -k 10 300 node tools/ts_prof.js 400 > gpurun_out/${TAG}_tsprof_${ib}_$i.json 2>&1; rc=$?; fatal $rc
    python3 -c "
import json;d=json.load(open('gpurun_out/${TAG}_tsprof_${ib}_$i.json'))
v=d['segmentFrame'];print('inline $ib',$i,'segmentFrame',{k:v[k]['p50'] for k in v if k in ('total_us','submit_us','device_us','deliver_hop_us')})"
    timeout -k 10 300 python bench.py --steps 200 --no-cpu --no-post --no-sweep > gpurun_out/${TAG}_b_${ib}_$i.log 2>&1; rc=$?; fatal $rc
    python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_b_${ib}_$i.log').read().splitlines()[-1]);h=d['host_path']['vga'];t=d['ts_path'];print('inline $ib',$i,'C copy',h['copy']['value'],'pinned',h['copy_pinned_out']['value'],'TS',t['value'],'frame p50',t['single_frame']['latency_ms_p50'])"
  done
done
