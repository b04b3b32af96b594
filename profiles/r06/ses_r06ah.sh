#!/bin/bash
# Round-6 session ah: the all-gather forms at one rank (a one-rank clique,
# bench.py --gather): ordered (the N > 1 default) against concurrent, and no
# gather, 400-step and 20-step windows, interleaved x2.
TAG=${1:-r06ah}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
for i in 1 2; do
  for form in none ordered concurrent; do
    for st in 400 20; do
      if [ $form = none ]; then A=""; else A="--gather --gather-form $form"; fi
      timeout -k 10 200 python bench.py --steps $st --warmup 5 $A --no-cpu --no-host --no-ts --no-post --no-sweep --no-latency > gpurun_out/${TAG}_${form}_${st}_$i.log 2>&1; rc=$?; fatal $rc
      python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_${form}_${st}_$i.log').read().splitlines()[-1]);print('$form',$st,$i,'value',d['value'],'median',d['value_at_median_step'],'form',d['config'].get('gather_form'))"
    done
  done
done
