#!/bin/bash
# Round-6 session aq: the driver's command with the one-frame row fetch on
# and off (VSS_FETCH_SINGLE=1 / 0), interleaved x3 on one box.
TAG=${1:-r06aq}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
for i in 1 2 3; do
  for fs in 1 0; do
    VSS_FETCH_SINGLE=$fs timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > gpurun_out/${TAG}_${fs}_$i.log 2>&1 || exit 1
    python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_${fs}_$i.log').read().splitlines()[-1]);t=d['ts_path']['single_frame'];print('fetch $fs',$i,'drv',d['value'],'ts',d['ts_path']['value'],'frame p50',t['latency_ms_p50'],'p99',t.get('latency_ms_p99'),'C pinned',d['host_path']['vga']['copy_pinned_out']['value'])"
  done
done
