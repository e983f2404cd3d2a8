#!/bin/bash
# Interleaved same-box A/B of two builds of the library: tools/ab_lib.sh <variant.so> <pairs> [bench args]
# (the snapshot's libvibevoice_hip.so is swapped in place; prints ms_per_step per run)
set -u
var=$1; pairs=$2; shift 2
L=vibevoice_amd/libvibevoice_hip.so
cp $L /tmp/vv_base.so || exit 1
for i in $(seq $pairs); do
  for v in base variant; do
    if [ $v = base ]; then cp /tmp/vv_base.so $L; else cp $var $L; fi || exit 1
    out=$(timeout -k 10 200 python bench.py --no-cpu-baseline "$@" 2>/dev/null | tail -1) || { echo "run failed: $v"; cp /tmp/vv_base.so $L; exit 1; }
    echo "$v $* | $(echo "$out" | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
  done
done
cp /tmp/vv_base.so $L
