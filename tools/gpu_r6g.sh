#!/bin/bash
# round-6 checkpoint: full GPU suite, smoke, B=1 and B=8 bench lines
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r6g_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" gpurun_out/r6g_tests.log | head -20; tail -30 gpurun_out/r6g_tests.log; exit 1; }
tail -2 gpurun_out/r6g_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6g_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r6g_smoke.log; exit 1; }
timeout -k 10 300 python -u bench.py > gpurun_out/r6g_bench_b1.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/r6g_bench_b1.log; exit 1; }
timeout -k 10 300 python -u bench.py --batch 8 --speakers 2 --no-cpu-baseline > gpurun_out/r6g_bench_b8.log 2>&1 || { echo "bench b8 failed"; tail -30 gpurun_out/r6g_bench_b8.log; exit 1; }
tail -1 gpurun_out/r6g_bench_b1.log | cut -c1-300
