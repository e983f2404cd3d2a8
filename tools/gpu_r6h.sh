#!/bin/bash
# round-6 final checkpoint: full GPU suite, smoke, B=1 / B=8 / Large / 64K-context bench lines
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/gpu_r6g.sh || exit 1
timeout -k 10 300 python -u bench.py --model Large --no-cpu-baseline > gpurun_out/r6h_bench_large.log 2>&1 || { echo "bench large failed"; tail -30 gpurun_out/r6h_bench_large.log; exit 1; }
timeout -k 10 400 python -u bench.py --context 65000 --no-cpu-baseline > gpurun_out/r6h_bench_ctx65k.log 2>&1 || { echo "bench 65k failed"; tail -30 gpurun_out/r6h_bench_ctx65k.log; exit 1; }
tail -1 gpurun_out/r6h_bench_large.log | cut -c1-200
