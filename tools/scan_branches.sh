set -e
for br in 1 2 4 8; do timeout -k 10 120 python bench.py --steps 100 --warmup 20 --no-cpu --branches $br > gpurun_out/br_$br.log 2>&1; done
python -c '
import json
for b in (1,2,4,8):
    d=json.loads(open(f"gpurun_out/br_{b}.log").read().strip().splitlines()[-1])
    print("branches", b, d["value"], d["ms_per_step"], "err", d["mask_max_abs_err"])
'
