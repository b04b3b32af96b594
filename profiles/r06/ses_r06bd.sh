#!/bin/bash
# Round-6 session bd: the final library, the driver's command x5 (the spread
# of the headline window on one box) and the default bench line.
TAG=${1:-r06bd}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
for i in 1 2 3 4 5; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_drv$i.log 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_drv$i.log').read().splitlines()[-1]);print('drv',d['value'],d['value_at_median_step'],'frac',d['roofline']['frac'],'ts',d['ts_path']['value'],d['ts_path']['single_frame']['latency_ms_p50'],'C pinned',d['host_path']['vga']['copy_pinned_out']['value'])"
done
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.log 2>&1 || exit 1
python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_bench.log').read().splitlines()[-1]);print('default',d['value'],d['value_at_median_step'],'frac',d['roofline']['frac'],'sweep',[(s['batch'],s['inflight'],s['value']) for s in d['batch_sweep']])"
