#!/bin/bash
# Round-6 session m: GPU tests on the lean LDS layouts, then an interleaved
# A/B against a -DVSS_LEAN=0 build (abvar/libvss_nolean.so): 400-step windows
# with the batch sweep and per-layer event times x3, the driver's command x3.
TAG=${1:-r06m}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_tests.log; grep -E "^(FAILED|ERROR)" gpurun_out/${TAG}_tests.log | head; fatal $rc; [ $rc -ne 0 ] && exit 1
timeout -k 10 900 bash tools/ab_quick.sh 3 abvar/libvss_nolean.so; fatal $?
for i in 1 2 3; do
  for lib in video-stream-segmenetation_amd/lib/libvss.so abvar/libvss_nolean.so; do
    VSS_LIBRARY=$lib timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-ts --no-host --no-post --no-cpu --no-sweep --no-latency > gpurun_out/${TAG}_drv.log 2>&1; rc=$?; fatal $rc
    python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_drv.log').read().splitlines()[-1]);print('drv','$lib'.split('/')[-1],$i,d['value'],d['value_at_median_step'],[(k['layer'],k['wg_per_cu']) for k in d['kernels'] if k['layer'] in (2,10)])"
  done
done
