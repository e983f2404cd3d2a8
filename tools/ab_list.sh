#!/bin/bash
# Interleaved same-box A/B over several variants: tools/ab_list.sh "<bench args>" "<variant>" ...
# variant: "base" or "<switch> <value>" for tools/ab_bench.py; prints ms_per_step per run, each
# run under its own time limit, the list run twice.
set -u
args=$1; shift
for rep in 1 2; do
  for v in "$@"; do
    if [ "$v" = base ]; then out=$(timeout -k 10 200 python bench.py $args --no-cpu-baseline 2>/dev/null | tail -1)
    else out=$(timeout -k 10 200 python tools/ab_bench.py $v $args --no-cpu-baseline 2>/dev/null | tail -1); fi
    rc=$?
    if [ $rc -ne 0 ]; then echo "run failed ($rc): $v"; exit $rc; fi
    echo "$v | $(echo "$out" | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
  done
done
