#!/bin/bash
# Round-6 session q: kernel arguments in device memory (HIP_FORCE_DEV_KERNARG=1)
# against the default, the driver's bench command, interleaved x3; then the
# MODNet b8 f16 tile knobs of vso_conv.hip (interleaved x2).
TAG=${1:-r06q}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
for i in 1 2 3; do
  for arm in base devkarg; do
    if [ $arm = devkarg ]; then export HIP_FORCE_DEV_KERNARG=1; else unset HIP_FORCE_DEV_KERNARG; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_${arm}_$i.log 2>&1; rc=$?; fatal $rc
    python3 - gpurun_out/${TAG}_${arm}_$i.log $arm $i <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[1]).read().splitlines() if x.startswith("{")][-1])
b81 = next((r["value"] for r in d.get("batch_sweep") or [] if r["batch"] == 8 and r["inflight"] == 1), None)
b84 = next((r["value"] for r in d.get("batch_sweep") or [] if r["batch"] == 8 and r["inflight"] == 4), None)
lat = d.get("latency", {})
print(sys.argv[2], sys.argv[3], "value", d["value"], "median", d.get("value_at_median_step"),
      "b1 ms", d["roofline"].get("mean_kernel_ms"), "frac", d["roofline"]["frac"], "b8/1", b81, "b8/4", b84,
      "lat1", lat.get("batch1", {}).get("latency_ms_p50"), "lat8", lat.get("batch8", {}).get("latency_ms_p50"),
      "ts", d.get("ts_path", {}).get("value"), "frame", d.get("ts_path", {}).get("single_frame", {}).get("latency_ms_p50"))
PY
  done
done
unset HIP_FORCE_DEV_KERNARG
for r in 1 2; do
  for e in - VSO_CONV_MAX_TH=4 VSO_CONV_MAX_TH=0 VSO_CONV_WANT=2048 VSO_CONV_WANT=512 VSO_CONV_BM_MAX=32 HIP_FORCE_DEV_KERNARG=1; do
    env $( [ "$e" = "-" ] || echo $e ) timeout -k 10 200 python tools/bench_onnx.py --only-modnet --batch 8 --iters 50 \
      --cases q4f16_288x512_b8_f16 > gpurun_out/${TAG}_onnx.log 2>&1; rc=$?; fatal $rc
    grep -h '^{' gpurun_out/${TAG}_onnx.log | cut -c1-120 | sed "s|^|[$e] |"
  done
done
