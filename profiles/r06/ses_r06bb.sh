#!/bin/bash
# Round-6 session bb: the library rebuilt from HEAD after the reverted A/B
# builds — every GPU test and smoke().
TAG=${1:-r06bb}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_gpu_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_gpu_tests.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_drv.log 2>&1 || exit 1
python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_drv.log').read().splitlines()[-1]);print('drv',d['value'],d['value_at_median_step'],'frac',d['roofline']['frac'])"
