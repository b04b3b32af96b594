#!/bin/bash
# A/B of k_conv_dwpw's channel groups per workgroup (VSO_DWPW_SPLIT=1: one 64-channel
# group each, the round-2 form) on MODNet 288x512 batch 8 bf16 and batch 1,
# after the ONNX GPU tests.  Usage (repo root on the box): bash tools/dwpw_ab.sh
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_onnx.py tests/test_gpu_face.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/dw_tests.log 2>&1; rc=$?; tail -2 gpurun_out/dw_tests.log; [ $rc -ne 0 ] && exit $rc
for v in 1 0 1 0; do
  for b in 8 1; do
    VSO_DWPW_SPLIT=$v timeout -k 10 120 python tools/bench_onnx.py --only-modnet --batch $b --cases modnet_288x512_b${b}_bf16 \
      --iters 50 --warmup 10 2>/dev/null | grep modnet | sed "s/^/split=$v /" | cut -c1-170
  done
done
timeout -k 10 200 python tools/bench_onnx.py --iters 100 > gpurun_out/dw_onnx_all.log 2>&1; grep -v "^W20" gpurun_out/dw_onnx_all.log | cut -c1-170
