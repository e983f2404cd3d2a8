#!/bin/bash
# Interleaved same-box A/B of bench.py: tools/ab_pair.sh <pairs> "<A args to tools/ab_bench.py or 'base'>" "<B ...>"
# prints ms_per_step of each run; every run under its own time limit
set -u
pairs=$1; A=$2; B=$3
run() {
  if [ "$1" = base ]; then timeout -k 10 150 python bench.py --steps ${STEPS:-200} --no-cpu-baseline
  else timeout -k 10 150 python tools/ab_bench.py $1 --steps ${STEPS:-200} --no-cpu-baseline; fi
}
for i in $(seq $pairs); do
  for v in "$A" "$B"; do
    out=$(run "$v" 2>/dev/null | tail -1) || { echo "run failed: $v"; exit 1; }
    echo "$v | $(echo "$out" | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
  done
done
