#!/bin/bash
# Build a diagnostic variant of the library: tools/build_variant.sh <name> <extra hipcc flags...>
# -> tools/lib_<name>.so (objects in /tmp/vv_<name>/); used with tools/gemm_bench.py --lib etc.
set -e
name=$1; shift
src=$(cd "$(dirname "$0")/../vibevoice_amd/csrc" && pwd)
out=/tmp/vv_$name; mkdir -p $out
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-function -Wno-unused-variable $*"
for f in $src/*.hip; do b=$(basename $f .hip); /opt/rocm/bin/hipcc $F -c $f -o $out/$b.o & done
/opt/rocm/bin/hipcc $F -x hip -c $src/engine.cpp -o $out/engine.o &
wait
/opt/rocm/bin/hipcc $F -shared $out/*.o -o "$(dirname "$0")/lib_$name.so" -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
