#!/bin/bash
# Round-6 session s: k_conv_tile's XCD-contiguous item order (VSO_CONV_XCD)
# — the single layers' kernel time and fetched bytes, MODNet b8 f16 / bf16
# interleaved, and the ONNX GPU tests.
TAG=${1:-r06s}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_onnx.py > gpurun_out/${TAG}_onnx_tests.log 2>&1; rc=$?
tail -3 gpurun_out/${TAG}_onnx_tests.log; fatal $rc; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
for sh in 8,64,64,72,128 8,99,64,72,128 8,64,32,72,128 8,64,64,144,256 8,32,32,144,256; do
  for x in 0 1; do
    D="$R/gpurun_out/prof_${TAG}/${sh//,/_}_x$x"
    VSO_CONV_XCD=$x timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$D/trace" -o run -- python3 $R/tools/conv_probe.py --shape $sh --iters 50 --warmup 5 > /dev/null 2>&1; rc=$?; fatal $rc
    VSO_CONV_XCD=$x timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$D/fetch" -o run -- python3 $R/tools/conv_probe.py --shape $sh --iters 50 --warmup 5 > /dev/null 2>&1; rc=$?; fatal $rc
    python3 - "$D" $sh $x <<'PY'
import csv, glob, sys
D = sys.argv[1]
dur, fetch = [], []
for f in glob.glob(D + "/trace/**/run_kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_conv_tile" in r["Kernel_Name"]:
            dur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for f in glob.glob(D + "/fetch/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_conv_tile" in r["Kernel_Name"]:
            fetch.append(float(r["Counter_Value"]))
dur.sort()
print(f"shape {sys.argv[2]} xcd {sys.argv[3]}: kernel p50 {dur[len(dur)//2]:.2f} us min {dur[0]:.2f}, FETCH_SIZE {sum(fetch)/max(len(fetch),1)/1024:.2f} MiB (x2 = {2*sum(fetch)/max(len(fetch),1)/1024:.1f})")
PY
  done
done
cd "$R"
for r in 1 2; do
  for x in 1 0; do
    VSO_CONV_XCD=$x timeout -k 10 200 python tools/bench_onnx.py --only-modnet --batch 8 --iters 50 \
      --cases q4f16_288x512_b8_f16,modnet_288x512_b8_bf16 > gpurun_out/${TAG}_onnx.log 2>&1; rc=$?; fatal $rc
    grep -h '^{' gpurun_out/${TAG}_onnx.log | cut -c1-110 | sed "s|^|[xcd $x] |"
  done
done
