#!/bin/bash
# GPU tests of the in-tree build, then an interleaved A/B of it against other
# builds (tools/ab_quick.sh).  Usage: bash tools/test_ab.sh N LIB_B [LIB_C ...]
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/tab_tests.log 2>&1 || { tail -60 gpurun_out/tab_tests.log; exit 1; }
tail -2 gpurun_out/tab_tests.log
bash tools/ab_quick.sh "$@"
