#!/bin/bash
# Builds compile-flag variants of one kernel source (ground.hip or rotate.hip)
# into rnnlogic_amd/_build/variants/<name>.so, for A/B runs through
# tools/ab_run.py (python tools/ab_run.py rnnlogic_amd/_build/variants/a.so
# tools/sort_ab.py ...: the same script against each build in one GPU call).
# Usage: tools/build_variants.sh <source>.hip name "flags" [name "flags" ...]
set -e
src=$1
shift
cd "$(dirname "$0")/../rnnlogic_amd/csrc"
OUT=../_build/variants
rm -rf $OUT && mkdir -p $OUT
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
B="--offload-arch=gfx950 -O3 -fPIC -std=c++17"
[ "$src" = rotate.hip ] && B="$B -mllvm -amdgpu-mfma-vgpr-form"
others=""
for f in graph.cpp ground.hip score.hip predictor.hip rotate.hip encode.hip batch.hip mine.hip loss.hip backward.hip wide.hip pna_grad.hip; do
  [ "$f" = "$src" ] || others="$others ../_build/$f.o"
done
make -s -C . $others
while [ $# -ge 2 ]; do
  $HIPCC $B $2 -c $src -o $OUT/$1.o &
  shift 2
done
wait
for o in $OUT/*.o; do
  $HIPCC --offload-arch=gfx950 -shared -fPIC $others $o -o ${o%.o}.so
done
rm -f $OUT/*.o
ls $OUT
