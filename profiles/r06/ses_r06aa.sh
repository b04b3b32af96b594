#!/bin/bash
# Round-6 session aa: the driver's command with the warm-up's last S steps
# after the settle pause (bench.py) against the pause after all W warm-up
# steps (the previous bench.py), interleaved x4.
TAG=${1:-r06aa}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
for i in 1 2 3 4; do
  for b in bench bench_prev; do
    timeout -k 10 300 python $b.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_${b}_$i.log 2>&1; rc=$?; fatal $rc
    python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_${b}_$i.log').read().splitlines()[-1]);print('$b',$i,'value',d['value'],'median',d['value_at_median_step'],'ms/step',d['ms_per_step'],'b1',d['roofline']['mean_kernel_ms'])"
  done
done
