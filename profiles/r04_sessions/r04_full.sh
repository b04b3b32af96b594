#!/bin/bash
# One GPU box, the whole check of the in-tree build: every GPU test, smoke,
# the default bench line, the rocprof passes (kernel trace + FETCH / WRITE /
# MFMA, SQ, wave state), then MODNet 288x512 batch 8 bf16 against other builds
# and its per-launch table.  Each step has its own time limit; a time-out,
# abort or crash stops the script (a failing test only reports).
#   bash tools/r04_full.sh TAG [LIB ...]
TAG=${1:-full}
shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
A=video-stream-segmenetation_amd/lib/libvss.so
echo "== tests"
timeout -k 10 420 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread \
  > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_tests.log; grep -E "^(FAILED|ERROR)" gpurun_out/${TAG}_tests.log | head -20; fatal $rc
echo "== smoke"
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1; rc=$?
tail -1 gpurun_out/${TAG}_smoke.log; fatal $rc
echo "== MODNet b8 bf16 A/B"
for r in 1 2; do
  for lib in "$A" "$@"; do
    VSS_LIBRARY=$lib timeout -k 10 200 python tools/bench_onnx.py --only-modnet --batch 8 --iters 50 --cases b8_bf16 \
      > gpurun_out/${TAG}_abo.log 2>&1; rc=$?
    [ $rc -ne 0 ] && { tail -5 gpurun_out/${TAG}_abo.log; fatal $rc; break; }
    grep -h '^{' gpurun_out/${TAG}_abo.log | cut -c1-200 | sed "s|^|$(basename $lib) |"
  done
done
echo "== MODNet b1 / b8, every precision"
timeout -k 10 300 python tools/bench_onnx.py --only-modnet --batch 8 --iters 50 > gpurun_out/${TAG}_onnx_b8.log 2>&1; fatal $?
grep -h '^{' gpurun_out/${TAG}_onnx_b8.log | cut -c1-200
timeout -k 10 300 python tools/bench_onnx.py --iters 100 > gpurun_out/${TAG}_onnx_b1.log 2>&1; fatal $?
grep -h '^{' gpurun_out/${TAG}_onnx_b1.log | cut -c1-200
echo "== MODNet b8 bf16 per launch"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/${TAG}_ml" -o run -- \
  python3 "$R/tools/onnx_layers.py" run modnet:8:bf16 "$R/gpurun_out/${TAG}_ml/launches.json" > "$R/gpurun_out/${TAG}_ml.log" 2>&1
rc=$?; cd "$R"; fatal $rc
python3 tools/onnx_layers.py report gpurun_out/${TAG}_ml/launches.json gpurun_out/${TAG}_ml/run_kernel_trace.csv 2>&1 | tail -26
echo "== bench"
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.log 2>&1; rc=$?; fatal $rc
tail -1 gpurun_out/${TAG}_bench.log > gpurun_out/${TAG}_bench.json
python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_bench.json')); print(d['value'], d.get('value_at_median_step'), d['roofline']['frac'], d['roofline']['kernel'][:60], d['cpu_baseline'], [(s['batch'], s['inflight'], s['value']) for s in d['batch_sweep']])" | cut -c1-600
export VSS_TILE=$(python3 tools/tiles_of.py gpurun_out/${TAG}_bench.json)
echo "VSS_TILE=$VSS_TILE"
echo "== rocprof passes"
timeout -k 10 500 bash tools/prof_run.sh "$TAG" > gpurun_out/${TAG}_prof.log 2>&1; fatal $?
echo "== SQ pass"
timeout -k 10 200 bash tools/prof_sq.sh "$TAG" | grep -v '^   30 '; fatal $?
echo "== wave-state pass"
timeout -k 10 200 bash tools/prof_stall.sh "$TAG"; fatal $?
