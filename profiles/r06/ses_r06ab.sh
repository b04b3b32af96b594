#!/bin/bash
# Round-6 session ab: the tree's full check (tools/round_check.sh: GPU tests,
# smoke, default bench, the rocprof passes), the driver's command x3, the TS
# phase table, MODNet batch 8 (f32 / bf16 / f16) and batch 1.
TAG=${1:-r06ab}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
bash tools/round_check.sh $TAG > gpurun_out/${TAG}_rc.log 2>&1; rc=$?
tail -8 gpurun_out/${TAG}_rc.log | cut -c1-400
[ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_drv$i.log 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_drv$i.log').read().splitlines()[-1]);print('drv',d['value'],d['value_at_median_step'],'ts',d['ts_path']['value'],d['ts_path']['single_frame']['latency_ms_p50'],'C pinned',d['host_path']['vga']['copy_pinned_out']['value'],'b1',d['latency']['batch1']['latency_ms_p50'],'frac',d['roofline']['frac'],'cpu',d['cpu_baseline']['value'])"
done
timeout -k 10 300 node tools/ts_prof.js 400 > gpurun_out/${TAG}_tsprof.json 2>&1 || exit 1
python3 -c "
import json;d=json.load(open('gpurun_out/${TAG}_tsprof.json'))
for m,v in d.items(): print('  ',m,{k:v[k]['p50'] for k in v if k.endswith('_us')}, v.get('frames_per_s',''))"
timeout -k 10 300 python tools/bench_onnx.py --only-modnet --batch 8 --iters 50 > gpurun_out/${TAG}_onnx8.log 2>&1 || exit 1
grep -h '^{' gpurun_out/${TAG}_onnx8.log | cut -c1-110
timeout -k 10 300 python tools/bench_onnx.py --only-modnet --batch 1 --iters 100 > gpurun_out/${TAG}_onnx1.log 2>&1 || exit 1
grep -h '^{' gpurun_out/${TAG}_onnx1.log | cut -c1-110
