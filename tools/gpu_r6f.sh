#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_lm.py -k "lm_ffn" > gpurun_out/r6f_tests.log 2>&1 || { echo "lm tests failed"; grep -E "FAILED|Error|error" gpurun_out/r6f_tests.log | head; tail -30 gpurun_out/r6f_tests.log; exit 1; }
grep -E "PASSED|step " gpurun_out/r6f_tests.log | tail -12
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fullsize.py tests/test_gpu_lm.py > gpurun_out/r6f_tests2.log 2>&1 || { echo "tests2 failed"; grep -E "FAILED|Error" gpurun_out/r6f_tests2.log | head; tail -20 gpurun_out/r6f_tests2.log; exit 1; }
tail -1 gpurun_out/r6f_tests2.log
bash tools/prof_step.sh r6_steps_b8 --batch 8 --speakers 2 --steps 200 --warmup 20 > /dev/null 2>&1 || { echo "prof failed"; tail -20 gpurun_out/r6_steps_b8.log; exit 1; }
head -20 gpurun_out/r6_steps_b8_steps.txt
timeout -k 10 300 python -u bench.py --batch 8 --speakers 2 --no-cpu-baseline > gpurun_out/r6_bench_b8.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/r6_bench_b8.log; exit 1; }
tail -1 gpurun_out/r6_bench_b8.log | cut -c1-300
