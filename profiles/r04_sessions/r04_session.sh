#!/bin/bash
# One GPU box: the GPU tests, an interleaved A/B of the in-tree libvss.so
# against other builds, then (unless NOPROF=1) smoke, the default bench line
# and the rocprof passes (kernel trace + FETCH / WRITE / MFMA, SQ, wave state)
# of the in-tree build.  Each step has its own time limit; a time-out, abort or
# crash stops the script (a failing test only reports).
#   bash tools/r04_session.sh TAG [LIB ...]
TAG=${1:-s}
shift || true
LIBS="$*"
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
echo "== tests"
timeout -k 10 420 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread \
  > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_tests.log; grep -E "^(FAILED|ERROR)" gpurun_out/${TAG}_tests.log | head -20; fatal $rc
if [ -n "$LIBS" ]; then
  echo "== A/B vs $LIBS"
  timeout -k 10 400 bash tools/ab_quick.sh 2 $LIBS; fatal $?
fi
[ "${NOPROF:-0}" = 1 ] && exit 0
echo "== smoke"
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1; rc=$?
tail -1 gpurun_out/${TAG}_smoke.log; fatal $rc
echo "== bench"
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.log 2>&1; rc=$?; fatal $rc
tail -1 gpurun_out/${TAG}_bench.log > gpurun_out/${TAG}_bench.json
python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_bench.json')); print(d['value'], d.get('value_at_median_step'), d['roofline'], [(s['batch'], s['inflight'], s['value']) for s in d['batch_sweep']])" | cut -c1-500
export VSS_TILE=$(python3 tools/tiles_of.py gpurun_out/${TAG}_bench.json)
echo "VSS_TILE=$VSS_TILE"
echo "== rocprof passes"
timeout -k 10 500 bash tools/prof_run.sh "$TAG" > gpurun_out/${TAG}_prof.log 2>&1; fatal $?
echo "== SQ pass"
timeout -k 10 200 bash tools/prof_sq.sh "$TAG"; fatal $?
echo "== wave-state pass"
timeout -k 10 200 bash tools/prof_stall.sh "$TAG"; fatal $?
