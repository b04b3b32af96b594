#!/bin/bash
# Round-6 session ai: the ordered form's gather stream at the highest stream
# priority (VSS_GATHER_PRIORITY) at one rank, against default priority, the
# concurrent form and no gather; RCCL GPU tests.
TAG=${1:-r06ai}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_rccl.py > gpurun_out/${TAG}_rccl.log 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_rccl.log; fatal $rc; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for arm in ordhi ordlo conc; do
    case $arm in
      ordhi) export VSS_GATHER_PRIORITY=1; A="--gather --gather-form ordered";;
      ordlo) export VSS_GATHER_PRIORITY=0; A="--gather --gather-form ordered";;
      conc) export VSS_GATHER_PRIORITY=1; A="--gather --gather-form concurrent";;
    esac
    for st in 400 20; do
      timeout -k 10 200 python bench.py --steps $st --warmup 5 $A --no-cpu --no-host --no-ts --no-post --no-sweep --no-latency > gpurun_out/${TAG}_${arm}_${st}_$i.log 2>&1; rc=$?; fatal $rc
      python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_${arm}_${st}_$i.log').read().splitlines()[-1]);print('$arm',$st,$i,'value',d['value'],'median',d['value_at_median_step'])"
    done
  done
done
