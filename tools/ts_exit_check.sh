mkdir -p gpurun_out
export VSS_NAPI_SEGV_TRACE=1
timeout -k 10 120 node tools/bench_ts.js 480 640 8 60 4 > gpurun_out/tsx_bench.log 2>&1; rc=$?; echo "bench_ts rc=$rc"; tail -3 gpurun_out/tsx_bench.log | cut -c1-200
if [ $rc -ge 124 ] || [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 node tools/ts_copy_probe.js 60 > gpurun_out/tsx_probe.log 2>&1; rc=$?; echo "probe rc=$rc"; tail -25 gpurun_out/tsx_probe.log | cut -c1-200
if [ $rc -ne 0 ]; then exit $rc; fi
VSS_TIME_SUBMIT=1 timeout -k 10 120 node tools/ts_copy_probe.js 60 > gpurun_out/tsx_probe2.log 2>&1; rc=$?; echo "probe+timing rc=$rc"; tail -25 gpurun_out/tsx_probe2.log | cut -c1-200
exit $rc
