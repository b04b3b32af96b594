#!/bin/bash
# Round-6 session v: k_conv_tile_up's interpolation with unconditional reads
# (no branch per channel) against the base build: ONNX GPU tests, MODNet b8
# interleaved, the per-kernel table.
TAG=${1:-r06v}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
timeout -k 10 400 python -u -m pytest -x -q -s --timeout 120 --timeout-method thread tests/test_gpu_onnx.py > gpurun_out/${TAG}_onnx_tests.log 2>&1; rc=$?
tail -3 gpurun_out/${TAG}_onnx_tests.log; fatal $rc; [ $rc -ne 0 ] && exit $rc
grep -h "conv_up" gpurun_out/${TAG}_onnx_tests.log | head -8
for r in 1 2; do
  for L in new region interp base; do
    if [ $L = new ]; then unset VSS_LIBRARY; else export VSS_LIBRARY=$R/abvar/libvss_$L.so; fi
    timeout -k 10 300 python tools/bench_onnx.py --only-modnet --batch 8 --iters 50 --cases b8_bf16,b8_f16 > gpurun_out/${TAG}_onnx.log 2>&1; rc=$?; fatal $rc
    grep -h '^{' gpurun_out/${TAG}_onnx.log | cut -c1-100 | sed "s|^|[$L] |"
  done
done
unset VSS_LIBRARY
bash tools/prof_onnx.sh ${TAG}_f16 --only-modnet --batch 8 --iters 50 --cases q4f16_288x512_b8_f16 > gpurun_out/${TAG}_prof.log 2>&1; rc=$?; fatal $rc
python3 tools/onnx_prof_table.py gpurun_out/prof_${TAG}_f16 70 16
