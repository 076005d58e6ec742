#!/bin/bash
# Bias-feature bench (grounding + scoring alone) per ground.hip variant
# (tools/ground_variants.sh): VARS="a b" bash tools/var_bias.sh
set -o pipefail
o=gpurun_out/${TAG:-varbias}; mkdir -p $o
for rep in 1 2; do
for v in ${VARS:-base}; do
  RNNL_LIB=rnnlogic_amd/_build/variants/$v.so timeout -k 10 300 python -u bench.py --feature bias --profile-only > $o/bias_$v.json 2> $o/bias_$v.err || { tail -20 $o/bias_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$o/bias_$v.json'));print('$v', d['value'], d['ms_per_step'])"
done
done
