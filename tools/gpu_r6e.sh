#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_codec.py tests/test_gpu_tokenizer_api.py tests/test_gpu_fullsize.py > gpurun_out/r6e_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" gpurun_out/r6e_tests.log | head; tail -20 gpurun_out/r6e_tests.log; exit 1; }
tail -2 gpurun_out/r6e_tests.log
timeout -k 10 300 python -u tools/codec_tile_stamps.py > gpurun_out/tile_stamps4.txt 2>&1 || { echo "stamps failed"; tail gpurun_out/tile_stamps4.txt; exit 1; }
tail -14 gpurun_out/tile_stamps4.txt
bash tools/prof_step.sh r6_steps_b8 --batch 8 --speakers 2 --steps 200 --warmup 20 > /dev/null 2>&1 || { echo "prof failed"; tail -20 gpurun_out/r6_steps_b8.log; exit 1; }
head -24 gpurun_out/r6_steps_b8_steps.txt
timeout -k 10 300 python -u bench.py --batch 8 --speakers 2 --no-cpu-baseline > gpurun_out/r6_bench_b8.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/r6_bench_b8.log; exit 1; }
tail -1 gpurun_out/r6_bench_b8.log | cut -c1-300
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r6_bench_b1.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/r6_bench_b1.log; exit 1; }
tail -1 gpurun_out/r6_bench_b1.log | cut -c1-300
