#!/bin/bash
# Round-6 session ax: the final tree (after the VSO_PW knob) — every GPU test, smoke(), the default
# bench line, the driver's command x3, MODNet batch 8 and 1.
TAG=${1:-r06ax}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_gpu_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_gpu_tests.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_bench.log').read().splitlines()[-1]);print('default',d['value'],d['value_at_median_step'],'frac',d['roofline']['frac'],'err',d['mask_max_abs_err'],'cpu',d['cpu_baseline']['value'])"
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_drv$i.log 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_drv$i.log').read().splitlines()[-1]);print('drv',d['value'],d['value_at_median_step'],'ts',d['ts_path']['value'],d['ts_path']['single_frame']['latency_ms_p50'],'C pinned',d['host_path']['vga']['copy_pinned_out']['value'],'b1',d['latency']['batch1']['latency_ms_p50'],'frac',d['roofline']['frac'],'cpu',d['cpu_baseline']['value'],d['cpu_baseline'].get('value_4_threads'))"
done
timeout -k 10 300 python tools/bench_onnx.py --only-modnet --batch 8 --iters 50 > gpurun_out/${TAG}_onnx8.log 2>&1 || exit 1
grep -h '^{' gpurun_out/${TAG}_onnx8.log | cut -c1-110
timeout -k 10 300 python tools/bench_onnx.py --only-modnet --batch 1 --iters 100 > gpurun_out/${TAG}_onnx1.log 2>&1 || exit 1
grep -h '^{' gpurun_out/${TAG}_onnx1.log | cut -c1-110
