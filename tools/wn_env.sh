#!/bin/bash
# WN18RR line under environment settings: bash tools/wn_env.sh "A=1 B=2" "A=0" ...
set -o pipefail
o=gpurun_out/wnenv; mkdir -p $o
i=0
for setting in "$@"; do
  i=$((i+1))
  env $setting timeout -k 10 300 python -u tools/wn_profile.py > $o/wn_$i.log 2>&1 || { tail -20 $o/wn_$i.log; exit 1; }
  python -c "import ast;d=ast.literal_eval(open('$o/wn_$i.log').read().strip().splitlines()[-1]);print('$setting', d['ms_per_step'], d['kernels_ms'])"
done
