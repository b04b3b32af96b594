#!/bin/bash
# Round-6 session al: the ordered all-gather on the caller's stream behind its
# forward, chained to the previous call's gather by an event, at one rank:
# RCCL GPU tests, then ordered (new) / ordered (HEAD's gather stream) /
# concurrent / none, 400- and 20-step windows, interleaved x2.
TAG=${1:-r06al}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_rccl.py tests/test_gpu_engine.py > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_tests.log; fatal $rc; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for arm in ord orduhead conc none; do
    unset VSS_LIBRARY
    case $arm in
      ord) A="--gather --gather-form ordered";;
      orduhead) A="--gather --gather-form ordered"; export VSS_LIBRARY=$R/abvar/libvss_head.so;;
      conc) A="--gather --gather-form concurrent";;
      none) A="";;
    esac
    for st in 400 20; do
      timeout -k 10 200 python bench.py --steps $st --warmup 5 $A --no-cpu --no-host --no-ts --no-post --no-sweep --no-latency > gpurun_out/${TAG}_${arm}_${st}_$i.log 2>&1; rc=$?; fatal $rc
      python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_${arm}_${st}_$i.log').read().splitlines()[-1]);print('$arm',$st,$i,'value',d['value'],'median',d['value_at_median_step'],'err',d['mask_max_abs_err'])"
    done
  done
done
