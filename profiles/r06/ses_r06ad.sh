#!/bin/bash
# Round-6 session ad: k_conv_pw (plain 1x1) with two chunks of B staging in
# flight, against HEAD's build: ONNX GPU tests (with the XCD-order bitwise
# test), MODNet b8 interleaved, the per-kernel table.
TAG=${1:-r06ad}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_onnx.py tests/test_gpu_face.py > gpurun_out/${TAG}_onnx_tests.log 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_onnx_tests.log; fatal $rc; [ $rc -ne 0 ] && exit $rc
for r in 1 2 3; do
  for L in new head; do
    if [ $L = head ]; then export VSS_LIBRARY=$R/abvar/libvss_$L.so; else unset VSS_LIBRARY; fi
    if [ $L = wave ]; then export VSO_IR_WAVE=1; else unset VSO_IR_WAVE; fi
    timeout -k 10 300 python tools/bench_onnx.py --only-modnet --batch 8 --iters 50 --cases b8_bf16,b8_f16 > gpurun_out/${TAG}_onnx.log 2>&1; rc=$?; fatal $rc
    grep -h '^{' gpurun_out/${TAG}_onnx.log | cut -c1-100 | sed "s|^|[$L] |"
  done
done
unset VSS_LIBRARY VSO_IR_WAVE
bash tools/prof_onnx.sh ${TAG}_f16 --only-modnet --batch 8 --iters 50 --cases q4f16_288x512_b8_f16 > gpurun_out/${TAG}_prof.log 2>&1; rc=$?; fatal $rc
python3 tools/onnx_prof_table.py gpurun_out/prof_${TAG}_f16 70 40 | grep -E "kernel time|k_conv_pw|kernel  "
