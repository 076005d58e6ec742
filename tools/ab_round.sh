#!/bin/bash
# One GPU-box pass for a round's A/B: parity tests on the in-tree library,
# then bench lines for each variant library (tools/env_ab.sh), VALU counters
# of the in-tree library and the grounding phase profile of each variant.
# Usage (GPU box, repo root): TAG=r04x VALS="a.so b.so" LINES="bias rotate wn" bash tools/ab_round.sh
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${TAG:-ab}; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail 5 --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $o/pytest_gpu.log 2>&1
tail -3 $o/pytest_gpu.log
grep -q " passed" $o/pytest_gpu.log || exit 1
TAG=${TAG:-ab}_ab VAR=RNNL_LIB VALS="$VALS" LINES="${LINES:-bias rotate wn}" bash tools/env_ab.sh || exit 1
for v in $VALS; do
  RNNL_LIB=$v timeout -k 10 300 python -u tools/profile_phases.py > $o/phases_$(basename $v .so).txt 2>&1 || exit 1
done
bash tools/pmc_valu.sh && cp gpurun_out/pmc_valu_fb.txt gpurun_out/pmc_valu_wn.txt $o/
