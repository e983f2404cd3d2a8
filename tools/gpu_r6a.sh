#!/bin/bash
# round 6: codec tile tests, then a B=1 step profile and bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_codec.py tests/test_gpu_tokenizer_api.py tests/test_gpu_fullsize_b1.py > gpurun_out/r6a_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" gpurun_out/r6a_tests.log | head -20; tail -40 gpurun_out/r6a_tests.log; exit 1; }
tail -3 gpurun_out/r6a_tests.log
grep -E "frame .* rel" gpurun_out/r6a_tests.log | tail -30
bash tools/prof_step.sh r6_steps_b1 --steps 300 --warmup 20 > /dev/null 2>&1 || { echo "prof failed"; tail -20 gpurun_out/r6_steps_b1.log; exit 1; }
head -32 gpurun_out/r6_steps_b1_steps.txt
timeout -k 10 300 python -u bench.py --steps 750 --warmup 20 > gpurun_out/r6a_bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/r6a_bench.log; exit 1; }
tail -1 gpurun_out/r6a_bench.log | cut -c1-400
