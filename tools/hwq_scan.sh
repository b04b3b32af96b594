set -e
mkdir -p gpurun_out
for q in 4 5 6 4; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 150 python bench.py --no-cpu --no-host --no-ts --no-post --steps 400 > gpurun_out/hwq.log 2>&1
  tail -1 gpurun_out/hwq.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('q=$q', d['value'], [(s['batch'], s['inflight'], s['value']) for s in d['batch_sweep']])"
done
