#!/bin/bash
# bench.py --profile-only per variant library (tools/*_variants.sh) and feature
# Usage: TAG=name VARS="a b" FEATS="RotatE bias" bash tools/var_bench.sh
set -o pipefail
o=gpurun_out/${TAG:-var}; mkdir -p $o
for v in ${VARS:-gbase}; do
  for f in ${FEATS:-RotatE}; do
    RNNL_LIB=rnnlogic_amd/_build/variants/$v.so timeout -k 10 300 python -u bench.py --profile-only --feature $f --steps 20 --warmup 3 > $o/bench_${v}_$f.json 2> $o/bench_${v}_$f.err || { tail -20 $o/bench_${v}_$f.err; exit 1; }
    python -c "import json; d=json.load(open('$o/bench_${v}_$f.json')); print('$v $f', d['value'], d['ms_per_step'], d['kernels_ms'])"
  done
done
