#!/bin/bash
# Interleaved A/B of MODNet 288x512 (bench_onnx --only-modnet) between the
# in-tree libvss.so and another build: bash tools/ab_onnx.sh LIB_B [N]
set -e
B=$1; N=${2:-2}
mkdir -p gpurun_out
for r in $(seq 1 $N); do
  for lib in video-stream-segmenetation_amd/lib/libvss.so $B; do
    for bt in 1 8; do
      VSS_LIBRARY=$lib timeout -k 10 200 python tools/bench_onnx.py --only-modnet --batch $bt --iters 50 > gpurun_out/abo.log 2>&1 || { tail -5 gpurun_out/abo.log; exit 1; }
      grep -h '^{' gpurun_out/abo.log | cut -c1-260 | sed "s|^|$(basename $lib) b$bt |"
    done
  done
done
