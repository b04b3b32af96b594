#!/bin/bash
# Retry gpurun ONLY when the box could not be acquired/prepared (status=transient
# or exit code 3: nothing ran on a GPU, nothing charged). Any other outcome —
# success, test failure, GPU fault, timeout — is returned as is, never retried.
# Usage: tools/gpurun_retry.sh TIMEOUT 'command'
T=$1; shift
for attempt in $(seq 1 ${GPURUN_ATTEMPTS:-12}); do
  out=$(/usr/local/graft/bin/gpurun --timeout "$T" -- "$@" 2>&1); rc=$?
  if [ $rc -eq 3 ] || echo "$out" | grep -q "status=transient"; then
    echo "[retry] attempt $attempt: box not acquired (nothing ran); waiting" >&2
    sleep 60; continue
  fi
  echo "$out"; exit $rc
done
echo "$out"; exit $rc
