#!/bin/bash
# Round-6 session af: the inverted residuals' slice knobs (VSO_IR_KS1,
# VSO_IR_CPS, VSO_IR_WGS) on MODNet b8 f16 / bf16, interleaved x2.
TAG=${1:-r06af}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
for r in 1 2; do
  for e in - VSO_IR_KS1=4096 VSO_IR_KS1=100000 VSO_IR_CPS=4 VSO_IR_CPS=8 VSO_IR_CPS=12; do
    env $( [ "$e" = "-" ] || echo $e ) timeout -k 10 300 python tools/bench_onnx.py --only-modnet --batch 8 --iters 50 --cases b8_bf16,b8_f16 > gpurun_out/${TAG}_onnx.log 2>&1; rc=$?; fatal $rc
    grep -h '^{' gpurun_out/${TAG}_onnx.log | cut -c1-100 | sed "s|^|[$e] |"
  done
done
