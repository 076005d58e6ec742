#!/bin/bash
# Bias step and RotatE step per ground.hip variant (tools/ground_variants.sh):
# VARS="a b" bash tools/var_step.sh
set -o pipefail
o=gpurun_out/${TAG:-varstep}; mkdir -p $o
for rep in 1 2; do
for v in ${VARS:-base}; do
  RNNL_LIB=rnnlogic_amd/_build/variants/$v.so timeout -k 10 300 python -u bench.py --feature bias --profile-only > $o/bias_$v.json 2> $o/bias_$v.err || { tail -20 $o/bias_$v.err; exit 1; }
  RNNL_LIB=rnnlogic_amd/_build/variants/$v.so timeout -k 10 300 python -u bench.py --profile-only > $o/rot_$v.json 2> $o/rot_$v.err || { tail -20 $o/rot_$v.err; exit 1; }
  python -c "import json;b=json.load(open('$o/bias_$v.json'));d=json.load(open('$o/rot_$v.json'));print('$v bias', b['ms_per_step'], 'rotate', d['ms_per_step'], d['kernels_ms']['base_score'])"
done
done
