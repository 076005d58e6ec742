#!/bin/bash
# GPU tests, then the WN18RR (config 3) line with the per-query PNA scoring
# kernel (RNNL_PNA_CHUNKED=0) and the chunked one (default), two runs each.
set -o pipefail
o=gpurun_out/${TAG:-pnachunk}; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider ${PYTEST_K:+-k "$PYTEST_K"} > $o/pytest_gpu.log 2>&1 || { tail -40 $o/pytest_gpu.log; exit 1; }
tail -2 $o/pytest_gpu.log
for v in 0 1 0 1; do
  RNNL_PNA_CHUNKED=$v timeout -k 10 300 python -u tools/wn_profile.py > $o/wn_$v.log 2>&1 || { tail -20 $o/wn_$v.log; exit 1; }
  python -c "import ast;d=ast.literal_eval(open('$o/wn_$v.log').read().strip().splitlines()[-1]);print('chunked=$v', d['ms_per_step'], d['kernels_ms'])"
done
