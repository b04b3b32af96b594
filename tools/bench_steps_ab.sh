mkdir -p gpurun_out
for r in 1 2; do
for st in 200 2000; do
  timeout -k 10 200 python bench.py --steps $st --no-cpu --no-post --no-host --no-ts --no-sweep > gpurun_out/bs.log 2>&1 || { tail -5 gpurun_out/bs.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/bs.log').read().strip().splitlines()[-1]); print('steps', $st, d['value'], d['ms_per_step'], d.get('median_step_ms'), d.get('value_at_median_step'))"
done
done
timeout -k 10 200 python bench.py --steps 2000 --inflight 8 --no-cpu --no-post --no-host --no-ts --no-sweep > gpurun_out/bs.log 2>&1 || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/bs.log').read().strip().splitlines()[-1]); print('inflight8 steps 2000', d['value'], d['ms_per_step'], d.get('median_step_ms'))"
