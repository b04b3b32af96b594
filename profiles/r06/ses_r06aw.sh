#!/bin/bash
# Round-6 session aw: plain 1x1 convolutions on k_conv_pw (default) against
# k_conv_small / k_conv_gemm (VSO_PW=0): the probes alone, then MODNet b8.
TAG=${1:-r06aw}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
for sh in 8,320,1280,9,16 8,16,32,144,256 8,16,32,72,128 8,96,576,18,32 8,32,192,72,128; do
  for pw in 1 0; do
    VSO_PW=$pw timeout -k 10 120 python tools/conv_probe.py --k 1 --shape $sh --prec f16 --iters 200 > gpurun_out/${TAG}_$sh.log 2>&1; rc=$?; fatal $rc
    [ $rc -ne 0 ] && { tail -5 gpurun_out/${TAG}_$sh.log; exit $rc; }
    grep -h '^{' gpurun_out/${TAG}_$sh.log | cut -c1-200 | sed "s|^|[pw=$pw] |"
  done
done
for r in 1 2; do
  for pw in 1 0; do
    VSO_PW=$pw timeout -k 10 300 python tools/bench_onnx.py --only-modnet --batch 8 --iters 50 --cases b8_bf16,b8_f16 > gpurun_out/${TAG}_onnx.log 2>&1; rc=$?; fatal $rc
    [ $rc -ne 0 ] && { tail -5 gpurun_out/${TAG}_onnx.log; exit $rc; }
    grep -h '^{' gpurun_out/${TAG}_onnx.log | cut -c1-100 | sed "s|^|[pw=$pw] |"
  done
done
