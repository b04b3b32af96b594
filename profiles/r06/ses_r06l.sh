#!/bin/bash
# Round-6 session l: one frame per call (the reference's serial usage) under
# runtime variants — default, HSA_ENABLE_SDMA=0 (blit kernels for H2D / D2H),
# AMD_DIRECT_DISPATCH=0 — with the submit's phases (VSS_TIME_SUBMIT=1): the TS
# phase table and the bench's latency leg, x2.
TAG=${1:-r06l}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
for i in 1 2; do
  for v in default nosdma nodirect; do
    case $v in
      default) E="";;
      nosdma) E="HSA_ENABLE_SDMA=0";;
      nodirect) E="AMD_DIRECT_DISPATCH=0";;
    esac
    env $E VSS_TIME_SUBMIT=1 timeout -k 10 300 node tools/ts_prof.js 300 > gpurun_out/${TAG}_${v}_$i.json 2> gpurun_out/${TAG}_${v}_$i.err; rc=$?; fatal $rc
    python3 -c "
import json;d=json.load(open('gpurun_out/${TAG}_${v}_$i.json'))
for m,x in d.items(): print('$v',$i,m,{k:x[k]['p50'] for k in x if k.endswith('_us')}, x.get('frames_per_s',''))"
    grep "submit phases" gpurun_out/${TAG}_${v}_$i.err | head -4
    env $E timeout -k 10 200 python bench.py --steps 400 --no-ts --no-host --no-post --no-cpu --no-sweep > gpurun_out/${TAG}_${v}_bench_$i.log 2>&1; rc=$?; fatal $rc
    python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_${v}_bench_$i.log').read().splitlines()[-1]);l=d['latency'];print('$v',$i,'value',d['value'],'b1 p50',l['batch1']['latency_ms_p50'],'b8 p50',l['batch8']['latency_ms_p50'])"
  done
done
