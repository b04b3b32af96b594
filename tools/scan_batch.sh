set -e
for b in 1 8 32; do timeout -k 10 120 python bench.py --steps 50 --warmup 10 --batch $b --no-cpu > gpurun_out/scan_b$b.log 2>&1; done
python -c '
import json
for b in (1,8,32):
    d=json.loads(open(f"gpurun_out/scan_b{b}.log").read().strip().splitlines()[-1])
    print(b, d["value"], d["ms_per_step"], [k["ms"] for k in d["kernels"]])
'
