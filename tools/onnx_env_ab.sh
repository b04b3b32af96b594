#!/bin/bash
# MODNet 288x512 batch 8 bf16, interleaved over environment settings of the
# in-tree build: bash tools/onnx_env_ab.sh "A=1" "A=2 B=3" ...  ("-" = none)
mkdir -p gpurun_out
for r in 1 2; do
  for e in "$@"; do
    env $( [ "$e" = "-" ] || echo $e ) timeout -k 10 200 python tools/bench_onnx.py --only-modnet --batch 8 --iters 50 \
      --cases b8_bf16 > gpurun_out/abe.log 2>&1 || { tail -5 gpurun_out/abe.log; exit 1; }
    grep -h '^{' gpurun_out/abe.log | cut -c1-160 | sed "s|^|[$e] |"
  done
done
