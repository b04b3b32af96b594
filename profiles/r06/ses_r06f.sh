#!/bin/bash
# Round-6 session f: GPU tests; then A/B of the claim query (VSS_CLAIM_QUERY=0
# vs default) on the driver's 20-step window x4 interleaved; the window's
# first calls again (tools/window_trace.py none / sleep); and the batch-1
# tiles (VSS_SMALL_TILES=0 vs default) on the latency leg x2.
TAG=${1:-r06f}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_tests.log; grep -E "^(FAILED|ERROR)" gpurun_out/${TAG}_tests.log | head; fatal $rc; [ $rc -ne 0 ] && exit 1
B="--no-ts --no-host --no-post --no-cpu --no-sweep"
for i in 1 2 3 4; do
  for arm in wait query; do
    if [ $arm = wait ]; then export VSS_CLAIM_QUERY=0; else unset VSS_CLAIM_QUERY; fi
    timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 $B --no-latency > gpurun_out/${TAG}_${arm}_$i.log 2>&1; rc=$?; fatal $rc
    python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_${arm}_$i.log').read().splitlines()[-1]);print('$arm',$i,d['value'],d['value_at_median_step'])"
  done
done
unset VSS_CLAIM_QUERY
for pre in none sleep; do
  VSS_TIME_DEVICE=1 timeout -k 10 120 python3 tools/window_trace.py run $pre > gpurun_out/${TAG}_win_$pre.json 2> gpurun_out/${TAG}_win_$pre.err; rc=$?; fatal $rc
  python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_win_$pre.json').read().splitlines()[-1]);print(d['pre'],'window',d['window_us'],'fps',d['frames_per_s'],'calls',d['call_us'][:8])"
  grep "call " gpurun_out/${TAG}_win_$pre.err | tail -20 | head -5
done
for i in 1 2; do
  for arm in b8tiles small; do
    if [ $arm = b8tiles ]; then export VSS_SMALL_TILES=0; else unset VSS_SMALL_TILES; fi
    timeout -k 10 200 python bench.py --steps 400 $B > gpurun_out/${TAG}_lat_${arm}_$i.log 2>&1; rc=$?; fatal $rc
    python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_lat_${arm}_$i.log').read().splitlines()[-1]);l=d['latency'];print('$arm',$i,'value',d['value'],'b1 p50',l['batch1']['latency_ms_p50'],'b8 p50',l['batch8']['latency_ms_p50'])"
  done
done
unset VSS_SMALL_TILES
