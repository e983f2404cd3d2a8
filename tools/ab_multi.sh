#!/bin/bash
# Interleaved same-box comparison of several configurations:
# tools/ab_multi.sh <rounds> "<cfg>" "<cfg>" ...  (cfg: 'base', a tools/ab_bench.py switch 'name v,..',
# or 'lib tools/lib_x.so'); prints ms_per_step per run; each run under its own time limit
# env: STEPS (timed steps, 200), EXTRA (more bench.py args, e.g. '--batch 8 --speakers 2')
set -u
rounds=$1; shift
run() {
  if [ "$1" = base ]; then timeout -k 10 150 python bench.py --steps ${STEPS:-200} --no-cpu-baseline ${EXTRA:-}
  else timeout -k 10 150 python tools/ab_bench.py $1 --steps ${STEPS:-200} --no-cpu-baseline ${EXTRA:-}; fi
}
for i in $(seq $rounds); do
  for v in "$@"; do
    out=$(run "$v" 2>/dev/null | tail -1) || { echo "run failed: $v"; exit 1; }
    echo "$v | $(echo "$out" | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
  done
done
