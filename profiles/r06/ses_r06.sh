#!/bin/bash
# Round-6 GPU session: GPU tests + smoke + default bench (tools/final_tests.sh),
# the TS phase table (tools/ts_prof.js), then the driver's 20-step bench x3.
# Usage (repo root on the box): bash tools/ses_r06.sh TAG
TAG=${1:-r06}
bash tools/final_tests.sh $TAG || exit 1
timeout -k 10 300 node tools/ts_prof.js 400 > gpurun_out/${TAG}_tsprof.json 2> gpurun_out/${TAG}_tsprof.err || { tail -5 gpurun_out/${TAG}_tsprof.err; exit 1; }
cut -c1-600 gpurun_out/${TAG}_tsprof.json
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-ts --no-host --no-post --no-cpu > gpurun_out/${TAG}_drv$i.log 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_drv$i.log').read().splitlines()[-1]);print('drv',d['value'],d['value_at_median_step'],[(s['batch'],s['inflight'],s['value']) for s in d['batch_sweep']][:2])"
done
