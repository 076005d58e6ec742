#!/bin/bash
# A/B of an environment switch on the bias and RotatE benches, after the forward parity tests.
# Usage (GPU box): ENVVAR=RNNL_SCORE_MEMO VALUES="1 0" bash tools/ab_env.sh tag
set -o pipefail
tag=${1:-abenv}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_forward.py tests/test_gpu_eval.py tests/test_gpu_edge_cases.py tests/test_gpu_flow.py tests/test_gpu_ranges.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $out/pytest.log 2>&1 || { echo "tests failed"; tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for rep in 1 2; do
for v in ${VALUES:-1 0}; do
  env $ENVVAR=$v timeout -k 10 300 python -u bench.py --feature bias --profile-only > $out/bias$v.json 2> $out/bias$v.err || { tail -20 $out/bias$v.err; exit 1; }
  python -c "import json;d=json.load(open('$out/bias$v.json'));print('$ENVVAR=$v bias', d['value'], d['ms_per_step'])"
  env $ENVVAR=$v timeout -k 10 300 python -u bench.py --profile-only > $out/rot$v.json 2> $out/rot$v.err || { tail -20 $out/rot$v.err; exit 1; }
  python -c "import json;d=json.load(open('$out/rot$v.json'));print('$ENVVAR=$v rotate', d['value'], d['ms_per_step'], d['kernels_ms'])"
done
done
