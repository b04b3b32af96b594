set -e
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 120 node tools/bench_ts.js 480 640 8 400 4 > gpurun_out/tsab_p$r.json
  echo "pinned $(cat gpurun_out/tsab_p$r.json | cut -c1-400)"
  VSS_NAPI_PINNED=0 timeout -k 10 120 node tools/bench_ts.js 480 640 8 400 4 > gpurun_out/tsab_m$r.json
  echo "malloc $(cat gpurun_out/tsab_m$r.json | cut -c1-400)"
done
