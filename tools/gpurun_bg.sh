#!/bin/bash
# Run one gpurun call in the background, retrying only while the pool has no
# free box or slot (exit 3: nothing ran, nothing charged).  Any other exit ends
# it.  Output: gpurun_out/<TAG>_call.txt (+ "exit N").
#   bash tools/gpurun_bg.sh TAG TIMEOUT 'command'
TAG=$1; TO=$2; CMD=$3
OUT=gpurun_out/${TAG}_call.txt
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$OUT" 2>&1
  rc=$?
  echo "exit $rc (try $i)" >> "$OUT"
  [ $rc -ne 3 ] && exit $rc
  sleep 150
done
