# GPU tests + one bench line + batch-8 phase trace (for iterating on kernels).
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 120 python bench.py --steps 300 --warmup 30 --no-cpu > gpurun_out/quick_bench.log 2>&1
tail -1 gpurun_out/quick_bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("fps", d["value"], "ms", d["ms_per_step"])'
timeout -k 10 120 python tools/trace_phases.py --batch 8 > gpurun_out/quick_trace.log 2>&1
cut -c1-100 gpurun_out/quick_trace.log | tail -16
