#!/bin/bash
# Interleaved A/B of environment arms (ARMS="A=1;A=0"), headline legs only,
# in the driver's short window (--steps 20 --warmup 5) and a 2000-step one.
#   ARMS="X=1;X=0" ROUNDS=3 bash tools/ab_env_win.sh TAG
TAG=${1:-abw}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
IFS=';' read -ra arms <<< "${ARMS}"
for rep in $(seq 1 ${ROUNDS:-3}); do
  for a in "${arms[@]}"; do
    for st in "20 5" "2000 50"; do
      set -- $st
      env $a timeout -k 10 120 python bench.py --steps $1 --warmup $2 --no-cpu --no-host --no-ts --no-post --no-sweep \
        --no-latency > gpurun_out/${TAG}.log 2>&1; rc=$?; fatal $rc
      tail -1 gpurun_out/${TAG}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$a steps $1: value', d['value'], 'median-step value', d.get('value_at_median_step'))"
    done
  done
done
