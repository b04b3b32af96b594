# Hidden-split threshold scan (VSS_KSPLIT_PIXELS): bench + phase trace per value.
set -e
mkdir -p gpurun_out
for px in 0 144 576 2304; do
  VSS_KSPLIT_PIXELS=$px timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no-cpu > gpurun_out/ks_$px.log 2>&1
  VSS_KSPLIT_PIXELS=$px timeout -k 10 120 python tools/trace_phases.py --batch 8 > gpurun_out/ks_trace_$px.log 2>&1
done
python -c '
import json
for px in (0, 144, 576, 2304):
    d=json.loads(open(f"gpurun_out/ks_{px}.log").read().strip().splitlines()[-1])
    print("ksplit_pixels", px, d["value"], d["ms_per_step"], "err", d["mask_max_abs_err"])
'
