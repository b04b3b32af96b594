#!/bin/bash
# Round-5 MODNet session: per-stage parity (tools/modnet_taps.py, bf16 and
# f16), the per-launch MODNet b8 bf16 table (rocprofv3 kernel trace), the
# PMC passes on it (tools/prof_onnx.sh: FETCH / WRITE / MFMA-busy), and the
# seam's LDS-layout A/B (VSS_SWZ=0 build) unless NOAB=1.  Every GPU step has
# its own time limit; a time-out, abort or crash ends the script.
#   bash tools/r05c_session.sh TAG
TAG=${1:-c}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
for prec in bf16 f16; do
  echo "== MODNet stages, $prec"
  timeout -k 10 300 python -u tools/modnet_taps.py --precision $prec > gpurun_out/${TAG}_taps_$prec.log 2>&1; rc=$?
  cut -c1-220 gpurun_out/${TAG}_taps_$prec.log | tail -20; fatal $rc
done
echo "== MODNet b8 bf16 per launch"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/${TAG}_ml" -o run -- \
  python3 "$R/tools/onnx_layers.py" run modnet:8:bf16 "$R/gpurun_out/${TAG}_ml/launches.json" > "$R/gpurun_out/${TAG}_ml.log" 2>&1
rc=$?; cd "$R"; fatal $rc
python3 tools/onnx_layers.py report gpurun_out/${TAG}_ml/launches.json gpurun_out/${TAG}_ml/run_kernel_trace.csv \
  > gpurun_out/${TAG}_ml_report.txt 2>&1
head -60 gpurun_out/${TAG}_ml_report.txt
if [ "${NOPMC:-0}" != 1 ]; then
  echo "== MODNet b8 bf16 PMC passes"
  timeout -k 10 900 bash tools/prof_onnx.sh ${TAG}_onnx --only-modnet --batch 8 --iters 20 --warmup 5 --cases b8_bf16; fatal $?
fi
if [ "${NOAB:-0}" != 1 ]; then
  echo "== A/B vs abvar/libvss_swz0.so"
  timeout -k 10 600 bash tools/ab_quick.sh ${AB_ROUNDS:-3} abvar/libvss_swz0.so; fatal $?
fi
