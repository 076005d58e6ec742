#!/bin/bash
# PMC FETCH_SIZE / WRITE_SIZE of the bias step per ground.hip variant: VARS="a b" bash tools/var_traffic.sh
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${TAG:-vartraffic}; mkdir -p $o
for v in ${VARS:-base}; do
  for c in FETCH_SIZE WRITE_SIZE; do
    RNNL_LIB=rnnlogic_amd/_build/variants/$v.so timeout -s KILL 200 rocprofv3 --pmc $c --output-format csv -d $o/${v}_$c -o run -- \
      python3 bench.py --feature bias --steps 2 --warmup 1 --profile-only > /dev/null 2> $o/${v}_$c.err || { tail -5 $o/${v}_$c.err; exit 1; }
  done
done
ls $o
