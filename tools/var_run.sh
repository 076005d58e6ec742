#!/bin/bash
set -o pipefail
o=gpurun_out/${TAG:-var}; mkdir -p $o
timeout -k 10 300 python -u tools/bench_rotate.py > $o/rot.txt 2>&1 || { tail -20 $o/rot.txt; exit 1; }
cat $o/rot.txt
for v in ${VARS:-base}; do
  RNNL_LIB=rnnlogic_amd/_build/variants/$v.so timeout -k 10 300 python -u bench.py --profile-only --steps 20 --warmup 3 > $o/bench_$v.json 2> $o/bench_$v.err || { tail -20 $o/bench_$v.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$o/bench_$v.json')); print('$v', d['value'], d['ms_per_step'], d['roofline']['ms'])"
done
