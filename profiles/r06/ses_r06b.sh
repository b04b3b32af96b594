#!/bin/bash
# Round-6 session b: GPU tests, the TS phase table, the autotune table, then an
# interleaved A/B of the tile objective (latency vs VSS_AUTOTUNE=lds) on the
# driver's 20-step window and a 400-step window.
TAG=${1:-r06b}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_tests.log; grep -E "^(FAILED|ERROR)" gpurun_out/${TAG}_tests.log | head; fatal $rc; [ $rc -ne 0 ] && exit 1
timeout -k 10 300 node tools/ts_prof.js 400 > gpurun_out/${TAG}_tsprof.json 2> gpurun_out/${TAG}_tsprof.err; rc=$?
cut -c1-3000 gpurun_out/${TAG}_tsprof.json; fatal $rc
VSS_AUTOTUNE_DUMP=1 timeout -k 10 200 python bench.py --steps 400 --no-ts --no-host --no-post --no-cpu --no-sweep --no-latency > gpurun_out/${TAG}_dump.log 2>&1; rc=$?; fatal $rc
grep autotune gpurun_out/${TAG}_dump.log | head -80
for i in 1 2 3; do
  for arm in latency lds; do
    if [ $arm = lds ]; then export VSS_AUTOTUNE=lds; else unset VSS_AUTOTUNE; fi
    for w in 20 400; do
      timeout -k 10 200 python bench.py --steps $w --warmup 5 --no-ts --no-host --no-post --no-cpu --no-sweep --no-latency > gpurun_out/${TAG}_${arm}_${w}_$i.log 2>&1; rc=$?; fatal $rc
      python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_${arm}_${w}_$i.log').read().splitlines()[-1]);print('$arm', $w, $i, d['value'], d['value_at_median_step'], d['tile_spec'], round(d['layer_launches_sum_ms']*1e3,1))"
    done
  done
done
unset VSS_AUTOTUNE
