#!/bin/bash
# A/B of the scoring kernels (RNNL_SCORE_GRP=1 group kernel vs 0 one-lane kernels):
# bias bench + WN18RR line, after the forward/eval parity tests.
set -o pipefail
tag=${1:-ab}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_forward.py tests/test_gpu_eval.py tests/test_gpu_edge_cases.py -x -q -s --timeout 200 --timeout-method thread -p no:cacheprovider > $out/pytest.log 2>&1 || { echo "tests failed"; tail -30 $out/pytest.log; exit 1; }
grep -E "passed|differing" $out/pytest.log | cut -c1-200
for g in 1 0; do
  RNNL_SCORE_GRP=$g timeout -k 10 300 python -u bench.py --feature bias --profile-only > $out/bias$g.json 2> $out/bias$g.err || { tail -20 $out/bias$g.err; exit 1; }
  python -c "import json;d=json.load(open('$out/bias$g.json'));print('grp=$g bias', d['value'], d['ms_per_step'], d['kernels_ms'])"
  RNNL_SCORE_GRP=$g timeout -k 10 300 python -u tools/wn_profile.py > $out/wn$g.log 2>&1 || { tail -20 $out/wn$g.log; exit 1; }
  python -c "import ast;d=ast.literal_eval(open('$out/wn$g.log').read().strip().splitlines()[-1]);print('grp=$g wn', d['ms_per_step'], d['kernels_ms'])"
done
