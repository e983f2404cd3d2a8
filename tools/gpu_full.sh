#!/bin/bash
# full GPU suite, then the B=1 step profile and bench line (+ optional extra bench args as B8=1)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/full_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" gpurun_out/full_tests.log | head -20; tail -30 gpurun_out/full_tests.log; exit 1; }
tail -2 gpurun_out/full_tests.log
bash tools/prof_step.sh r6_steps_b1 --steps 300 --warmup 20 > /dev/null 2>&1 || { echo "prof failed"; tail -20 gpurun_out/r6_steps_b1.log; exit 1; }
head -40 gpurun_out/r6_steps_b1_steps.txt
timeout -k 10 300 python -u bench.py > gpurun_out/r6_bench_b1.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/r6_bench_b1.log; exit 1; }
tail -1 gpurun_out/r6_bench_b1.log | cut -c1-600
