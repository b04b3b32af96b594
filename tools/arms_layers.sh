#!/bin/bash
# Per-launch MODNet b8 bf16 tables under several environment arms (one
# rocprofv3 kernel trace each), printing the rows matching GREP (default
# k_ir) and each arm's total.
#   ARMS="VSO_IR_WAVE=0;VSO_IR_WAVE=1 VSO_IR_WGS=256" GREP=k_ir bash tools/arms_layers.sh TAG [model key]
TAG=${1:-arms}
KEY=${2:-modnet:8:bf16}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
export TMPDIR=/tmp
IFS=';' read -ra arms <<< "${ARMS:-VSO_IR_WAVE=1}"
k=0
for a in "${arms[@]}"; do
  k=$((k + 1))
  a=${a//VSS_LIBRARY=/VSS_LIBRARY=$R/}  # (the profiled run starts in /tmp)
  cd /tmp
  env $a timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/${TAG}_a$k" -o run -- \
    python3 "$R/tools/onnx_layers.py" run "$KEY" "$R/gpurun_out/${TAG}_a$k/launches.json" > "$R/gpurun_out/${TAG}_a$k.log" 2>&1
  rc=$?; cd "$R"; fatal $rc
  python3 tools/onnx_layers.py report gpurun_out/${TAG}_a$k/launches.json gpurun_out/${TAG}_a$k/run_kernel_trace.csv \
    > gpurun_out/${TAG}_a${k}_report.txt 2>&1
  echo "== $a: $(head -1 gpurun_out/${TAG}_a${k}_report.txt)"
  grep -E "${GREP:-k_ir}" gpurun_out/${TAG}_a${k}_report.txt | grep " x " || true
done
