#!/bin/bash
# The Node host's exit path and the staging copy: the GPU TS tests, the
# 400-batch TS copy probe twice (VSS_TIME_SUBMIT=1: the run that once
# segfaulted at exit) with a native backtrace on a fatal signal, then the
# bench's host and TS legs.  Stops after the first failing step.
mkdir -p gpurun_out
export VSS_NAPI_SEGV_TRACE=1
timeout -k 10 300 python -u -m pytest tests/test_ts.py -x -q --timeout 200 --timeout-method thread > gpurun_out/tsx_tests.log 2>&1; rc=$?
tail -2 gpurun_out/tsx_tests.log; [ $rc -ne 0 ] && exit $rc
for k in 1 2 3; do
  VSS_TIME_SUBMIT=1 timeout -k 10 150 node tools/ts_copy_probe.js 400 > gpurun_out/tsx_probe$k.log 2>&1; rc=$?
  echo "probe $k rc=$rc"; tail -4 gpurun_out/tsx_probe$k.log | cut -c1-220; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 300 python bench.py --no-cpu --no-sweep --no-post > gpurun_out/tsx_bench.log 2>&1; rc=$?
tail -1 gpurun_out/tsx_bench.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], {k:v["value"] for k,v in d["host_path"]["vga"].items() if isinstance(v,dict)}, d["ts_path"]["value"], d["ts_path"]["zero_copy"]["value"])'
exit $rc
