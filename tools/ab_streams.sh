#!/bin/bash
# The headline's step streams: new torch streams (default) against the handle's
# slot streams (bench --streams slot), plain or on dedicated CU-masked hardware
# queues (VSS_SLOT_QUEUES=cumask); interleaved, short and long windows.
#   ROUNDS=4 bash tools/ab_streams.sh TAG
TAG=${1:-abs}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
run() {  # label env streams steps warmup
  env $2 timeout -k 10 120 python bench.py --streams $3 --steps $4 --warmup $5 --no-cpu --no-host --no-ts --no-post \
    --no-sweep --no-latency > gpurun_out/${TAG}.log 2>&1; rc=$?; fatal $rc
  tail -1 gpurun_out/${TAG}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1 steps $4: value', d['value'], 'median-step value', d.get('value_at_median_step'))"
}
for rep in $(seq 1 ${ROUNDS:-4}); do
  for st in "20 5" "2000 50"; do
    set -- $st
    run torch VSS_NONE=1 torch $1 $2
    run slot-cumask VSS_SLOT_QUEUES=cumask slot $1 $2
    run slot-plain VSS_NONE=1 slot $1 $2
  done
done
