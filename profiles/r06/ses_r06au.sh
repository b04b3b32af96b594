#!/bin/bash
# Round-6 session au: the rocprof passes of the final tree — the seam (trace,
# FETCH_SIZE, WRITE_SIZE, MFMA/VALU/LDS; the tiles the default bench line's
# autotuner chose) and MODNet 288x512 batch 8 at f16 and bf16 (the same four
# passes, per-kernel tables).
TAG=${1:-r06au}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.log 2>&1; rc=$?; fatal $rc; [ $rc -ne 0 ] && exit $rc
tail -1 gpurun_out/${TAG}_bench.log > gpurun_out/bench_${TAG}.json
cut -c1-200 gpurun_out/bench_${TAG}.json
export VSS_TILE=$(python3 tools/tiles_of.py gpurun_out/bench_${TAG}.json)
echo "VSS_TILE=$VSS_TILE"
bash tools/prof_run.sh "$TAG" > gpurun_out/${TAG}_prof.log 2>&1; rc=$?; fatal $rc; [ $rc -ne 0 ] && exit $rc
unset VSS_TILE
echo "== seam"; python3 tools/pmc_table.py gpurun_out/prof_${TAG}/mfma/run_counter_collection.csv 14
for c in b8_f16 b8_bf16; do
  bash tools/prof_onnx.sh ${TAG}_modnet_$c --only-modnet --batch 8 --iters 50 --cases $c > gpurun_out/${TAG}_modnet_$c.log 2>&1; rc=$?; fatal $rc
  [ $rc -ne 0 ] && exit $rc
  echo "== MODNet $c"
  python3 tools/onnx_prof_table.py gpurun_out/prof_${TAG}_modnet_$c 50 40
  python3 tools/pmc_table.py gpurun_out/prof_${TAG}_modnet_$c/mfma/run_counter_collection.csv 24
done
