#!/bin/bash
# WN18RR line per ground.hip variant (tools/ground_variants.sh): VARS="a b" bash tools/var_wn.sh
set -o pipefail
o=gpurun_out/${TAG:-varwn}; mkdir -p $o
for v in ${VARS:-w2}; do
  RNNL_LIB=rnnlogic_amd/_build/variants/$v.so timeout -k 10 300 python -u tools/wn_profile.py > $o/wn_$v.log 2>&1 || { tail -20 $o/wn_$v.log; exit 1; }
  python -c "import ast;d=ast.literal_eval(open('$o/wn_$v.log').read().strip().splitlines()[-1]);print('$v', d['ms_per_step'], d['kernels_ms'])"
done
