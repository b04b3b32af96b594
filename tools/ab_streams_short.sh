#!/bin/bash
# The driver's short window only (--steps 20 --warmup 5, full default legs off
# except the headline), torch streams vs CU-masked slot streams, interleaved.
#   ROUNDS=8 bash tools/ab_streams_short.sh TAG
TAG=${1:-abss}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
run() {
  env $2 timeout -k 10 120 python bench.py --streams $3 --steps 20 --warmup 5 --no-cpu --no-host --no-ts --no-post \
    --no-sweep --no-latency > gpurun_out/${TAG}.log 2>&1; rc=$?; fatal $rc
  tail -1 gpurun_out/${TAG}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1: value', d['value'], 'median-step value', d.get('value_at_median_step'))"
}
for rep in $(seq 1 ${ROUNDS:-8}); do
  run torch VSS_NONE=1 torch
  run slot-cumask VSS_SLOT_QUEUES=cumask slot
done
