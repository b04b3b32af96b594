#!/bin/bash
# One GPU call for the end of a session: the 5x5 conv A/B (short), then the
# full round check (GPU tests, smoke, bench, rocprof passes).  Stops after any
# step that times out or crashes (exit >= 124); a failing test still reports.
# Usage (repo root on the box): bash tools/final_check.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-final}
mkdir -p "$R/gpurun_out"
cd "$R"
timeout -k 10 400 bash tools/conv5_ab.sh "c5_$TAG" > "gpurun_out/c5_$TAG.log" 2>&1
rc=$?
tail -14 "gpurun_out/c5_$TAG.log"
if [ $rc -ge 124 ]; then echo "conv A/B ended with $rc: stopping"; exit $rc; fi
bash tools/round_check.sh "$TAG" > "gpurun_out/rc_$TAG.log" 2>&1
rc=$?
tail -6 "gpurun_out/rc_$TAG.log" | cut -c1-400
exit $rc
