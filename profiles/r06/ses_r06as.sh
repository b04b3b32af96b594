#!/bin/bash
# Round-6 session as: k_conv_tile_up computing its plain chunk's item offsets
# lazily, against HEAD's build: ONNX GPU tests, the
# two fused-upsample layers alone, MODNet b8 interleaved.
TAG=${1:-r06as}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_onnx.py > gpurun_out/${TAG}_onnx_tests.log 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_onnx_tests.log; fatal $rc; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
for arg in "--up 32 --shape 8,35,16,288,512" "--up 32 --shape 8,64,32,144,256" "--shape 8,1280,96,18,32 --k 5"; do
  for L in new head; do
    if [ $L = new ]; then unset VSS_LIBRARY; else export VSS_LIBRARY=$R/abvar/libvss_$L.so; fi
    D="$R/gpurun_out/prof_${TAG}/$(echo $arg | tr -d ' -' | tr ',' '_')_$L"
    timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$D" -o run -- python3 $R/tools/conv_probe.py $arg --iters 50 --warmup 5 > /dev/null 2>&1; rc=$?; fatal $rc
    python3 - "$D" "$arg" $L <<'PY'
import csv, glob, sys
dur = {}
for f in glob.glob(sys.argv[1] + "/**/run_kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if "vso::" in k:
            dur.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in dur.items():
    v.sort()
    print(f"{sys.argv[2]:34s} {sys.argv[3]:5s} {k:44s} n {len(v):3d} p50 {v[len(v)//2]:7.2f} us")
PY
  done
done
unset VSS_LIBRARY
cd "$R"
for r in 1 2 3; do
  for L in new head; do
    if [ $L = new ]; then unset VSS_LIBRARY; else export VSS_LIBRARY=$R/abvar/libvss_$L.so; fi
    timeout -k 10 300 python tools/bench_onnx.py --only-modnet --batch 8 --iters 50 --cases b8_bf16,b8_f16 > gpurun_out/${TAG}_onnx.log 2>&1; rc=$?; fatal $rc
    grep -h '^{' gpurun_out/${TAG}_onnx.log | cut -c1-100 | sed "s|^|[$L] |"
  done
done
