#!/bin/bash
# Round-6 session aj: the ordered all-gather at one rank with more batches in
# flight (--inflight 6 / 8: each slot's forward -> gather -> next-forward chain
# gets more slack), against 4 and the concurrent form; plain N=1 at 6 / 8 too.
TAG=${1:-r06aj}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
for i in 1 2; do
  for arm in ord4 ord6 ord8 conc4 none6 none8; do
    case $arm in
      ord*) A="--gather --gather-form ordered --inflight ${arm#ord}";;
      conc*) A="--gather --gather-form concurrent --inflight ${arm#conc}";;
      none*) A="--inflight ${arm#none}";;
    esac
    for st in 400 20; do
      timeout -k 10 200 python bench.py --steps $st --warmup 8 $A --no-cpu --no-host --no-ts --no-post --no-sweep --no-latency > gpurun_out/${TAG}_${arm}_${st}_$i.log 2>&1; rc=$?; fatal $rc
      python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_${arm}_${st}_$i.log').read().splitlines()[-1]);print('$arm',$st,$i,'value',d['value'],'median',d['value_at_median_step'])"
    done
  done
done
