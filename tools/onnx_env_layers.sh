#!/bin/bash
# Per-launch tables of MODNet 288x512 b8 bf16 under environment settings of
# the in-tree build: bash tools/onnx_env_layers.sh TAG "A=1" "A=2 B=3" ...
# (-> gpurun_out/TAG_<k>_ml for the k-th setting, "-" = none)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
TAG=$1; shift
k=0
for e in "$@"; do
  (
    [ "$e" = "-" ] || export $e
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/${TAG}_${k}_ml" -o run -- \
      python3 "$R/tools/onnx_layers.py" run modnet:8:bf16 "$R/gpurun_out/${TAG}_${k}_ml/launches.json" > "$R/gpurun_out/${TAG}_${k}_ml.log" 2>&1
  ) || exit $?
  echo "[$k: $e] $(python3 tools/onnx_layers.py report gpurun_out/${TAG}_${k}_ml/launches.json gpurun_out/${TAG}_${k}_ml/run_kernel_trace.csv 2>&1 | head -1)"
  k=$((k+1))
done
