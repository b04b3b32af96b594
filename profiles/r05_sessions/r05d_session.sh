#!/bin/bash
# Round-5 MODNet iteration: the ONNX GPU tests (prints), a MODNet b8 bf16 A/B
# over environment arms (ARMS, each "VAR=v VAR2=w"), and the per-launch table.
#   ARMS="VSO_IR_B16=1;VSO_IR_B16=0" bash tools/r05d_session.sh TAG
TAG=${1:-d}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
if [ "${NOTESTS:-0}" != 1 ]; then
  echo "== ONNX tests"
  timeout -k 10 400 python -u -m pytest tests/test_gpu_onnx.py -m gpu -s -q --timeout 200 --timeout-method thread \
    > gpurun_out/${TAG}_onnx.log 2>&1; rc=$?
  tail -2 gpurun_out/${TAG}_onnx.log; grep -E "^(FAILED|ERROR)|ir_chain|modnet" gpurun_out/${TAG}_onnx.log | cut -c1-200 | head -40
  fatal $rc
  [ $rc -ne 0 ] && [ "${CONTINUE:-0}" != 1 ] && exit $rc
fi
IFS=';' read -ra arms <<< "${ARMS:-VSO_IR_B16=1;VSO_IR_B16=0}"
for k in 1 2; do
  for a in "${arms[@]}"; do
    env $a timeout -k 10 200 python tools/bench_onnx.py --only-modnet --batch 8 --iters 50 --cases b8_bf16 \
      > gpurun_out/${TAG}_arm.log 2>&1; rc=$?
    echo "$a: $(grep -h '^{' gpurun_out/${TAG}_arm.log | cut -c1-170)"; fatal $rc
  done
done
echo "== MODNet b8 bf16 per launch"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/${TAG}_ml" -o run -- \
  python3 "$R/tools/onnx_layers.py" run modnet:8:bf16 "$R/gpurun_out/${TAG}_ml/launches.json" > "$R/gpurun_out/${TAG}_ml.log" 2>&1
rc=$?; cd "$R"; fatal $rc
python3 tools/onnx_layers.py report gpurun_out/${TAG}_ml/launches.json gpurun_out/${TAG}_ml/run_kernel_trace.csv \
  > gpurun_out/${TAG}_ml_report.txt 2>&1
head -70 gpurun_out/${TAG}_ml_report.txt
