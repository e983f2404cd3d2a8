#!/bin/bash
# MFMA PMC passes (N1 evidence in the loop: k_head_m16 at 2 / 16 rows, k_lm_ffn), then B = 8 profile + bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
rm -f gpurun_out/head_mfma.txt
bash tools/run_head_mfma.sh "--n 1" "--n 8" "--lmffn" || { echo "pmc failed"; cat gpurun_out/head_mfma.txt; exit 1; }
cat gpurun_out/head_mfma.txt
bash tools/prof_step.sh r6_steps_b8 --batch 8 --speakers 2 --steps 200 --warmup 20 > /dev/null 2>&1 || { echo "prof failed"; tail -20 gpurun_out/r6_steps_b8.log; exit 1; }
head -30 gpurun_out/r6_steps_b8_steps.txt
timeout -k 10 300 python -u bench.py --batch 8 --speakers 2 --no-cpu-baseline > gpurun_out/r6_bench_b8.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/r6_bench_b8.log; exit 1; }
tail -1 gpurun_out/r6_bench_b8.log | cut -c1-400
