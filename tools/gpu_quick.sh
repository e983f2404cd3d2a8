#!/bin/bash
# quick GPU pass: selected GPU tests then the default bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $TESTS > gpurun_out/quick_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/quick_tests.log; exit 1; }
tail -3 gpurun_out/quick_tests.log
if [ -n "$BENCH" ]; then
  timeout -k 10 300 python -u bench.py $BENCH > gpurun_out/quick_bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/quick_bench.log; exit 1; }
  tail -1 gpurun_out/quick_bench.log
fi
