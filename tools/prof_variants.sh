#!/bin/bash
# rocprofv3 kernel averages (us) of the bias bench per variant library
# (rnnlogic_amd/_build/variants/*.so) plus the main build.
set -o pipefail
export TMPDIR=/tmp
for lib in "" rnnlogic_amd/_build/variants/*.so; do
  name=$(basename ${lib:-main} .so)
  RNNL_LIB=${lib:+$PWD/$lib} timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pv_$name -o run -- \
      python3 bench.py --feature bias --steps 3 --warmup 1 --profile-only > /dev/null 2>&1 || { echo "$name FAILED"; exit 1; }
  python3 tools/rocpd_top.py gpurun_out/pv_$name/run_results.db "$name"
done
