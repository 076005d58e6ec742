#!/bin/bash
# On the GPU box: bench.py (bias feature, 3 steps) once per variant library
# in rnnlogic_amd/_build/variants/ plus the main build; prints kernels_ms.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for lib in "" rnnlogic_amd/_build/variants/*.so; do
  name=${lib:-main}
  RNNL_LIB=${lib:+$PWD/$lib} timeout -k 10 300 python bench.py --steps 3 --warmup 1 --feature ${FEATURE:-bias} \
      --no-cpu-baseline > gpurun_out/v.json 2>/dev/null || { echo "$name FAILED"; continue; }
  echo "$(basename $name) $(grep -o '"kernels_ms": {[^}]*}' gpurun_out/v.json)"
done
