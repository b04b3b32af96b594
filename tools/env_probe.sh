#!/bin/bash
# headline (400 steps, 4 in flight) under HIP runtime knobs, one run each:
#   bash tools/env_probe.sh
mkdir -p gpurun_out
run() {
  env "$@" timeout -k 10 150 python bench.py --no-cpu --no-host --no-ts --no-post --no-sweep --steps 400 \
    > gpurun_out/envp.log 2>&1 || { tail -5 gpurun_out/envp.log; exit 1; }
  tail -1 gpurun_out/envp.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$*', d['value'], d['value_at_median_step'])"
}
run X=0
run DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
run DEBUG_CLR_GRAPH_PACKET_CAPTURE=1
run HIP_FORCE_DEV_KERNARG=0
run HIP_FORCE_DEV_KERNARG=1
run GPU_MAX_HW_QUEUES=2
run GPU_MAX_HW_QUEUES=3
run X=0
