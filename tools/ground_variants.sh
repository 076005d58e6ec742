#!/bin/bash
# Builds compile-flag variants of ground.hip into rnnlogic_amd/_build/variants/<name>.so
# (selected at run time with RNNL_LIB=...) for A/B runs.
# Usage: tools/ground_variants.sh name "flags" [name "flags" ...]
set -e
cd "$(dirname "$0")/../rnnlogic_amd/csrc"
OUT=../_build/variants
rm -rf $OUT && mkdir -p $OUT
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
B="--offload-arch=gfx950 -O3 -fPIC -std=c++17"
make -s -C . ../_build/graph.cpp.o ../_build/rotate.hip.o ../_build/encode.hip.o ../_build/batch.hip.o ../_build/mine.hip.o
while [ $# -ge 2 ]; do
  $HIPCC $B $2 -c ground.hip -o $OUT/$1.o &
  shift 2
done
wait
for o in $OUT/*.o; do
  $HIPCC --offload-arch=gfx950 -shared -fPIC ../_build/graph.cpp.o ../_build/rotate.hip.o ../_build/encode.hip.o ../_build/batch.hip.o ../_build/mine.hip.o $o -o ${o%.o}.so
done
rm -f $OUT/*.o
ls $OUT
