#!/bin/bash
# Per-step kernel breakdown of a bench.py configuration under rocprofv3:
# tools/prof_step.sh <tag> <bench args...>  ->  gpurun_out/<tag>/ (trace + stats CSV),
# gpurun_out/<tag>_steps.txt (profiles/summarize.py over the last 20 steps)
set -eu
tag=$1; shift
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$tag -o run -- \
  python3 $R/bench.py --no-cpu-baseline "$@" > $R/gpurun_out/$tag.log 2>&1
csv=$(find $R/gpurun_out/$tag -name "*kernel_trace.csv" | head -1)
python3 $R/profiles/summarize.py "$csv" 20 $R/gpurun_out/${tag}_steps.json > $R/gpurun_out/${tag}_steps.txt
find $R/gpurun_out/$tag -name "*kernel_trace.csv" -delete
head -40 $R/gpurun_out/${tag}_steps.txt
