#!/bin/bash
# Round-6 session t: MODNet q4f16 288x512 batch 8 f16 per kernel — trace,
# FETCH_SIZE, WRITE_SIZE (tools/prof_onnx.sh, tools/onnx_prof_table.py).
TAG=${1:-r06t}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
bash tools/prof_onnx.sh ${TAG}_f16 --only-modnet --batch 8 --iters 50 --cases q4f16_288x512_b8_f16 > gpurun_out/${TAG}_prof.log 2>&1; rc=$?; fatal $rc
python3 tools/onnx_prof_table.py gpurun_out/prof_${TAG}_f16 70 45
