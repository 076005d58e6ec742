#!/bin/bash
# A/B of one environment variable over the bench lines (GPU box, repo root),
# or, with VAR=LIB, of library builds from tools/build_variants.sh (loaded
# through tools/ab_run.py):
#   VAR=LIB VALS="rnnlogic_amd/_build/variants/a.so rnnlogic_amd/_build/variants/b.so" LINES="bias wn rotate" bash tools/env_ab.sh
# optional GPU tests first (TESTS=1).  Two runs per value, interleaved.
set -o pipefail
o=gpurun_out/${TAG:-envab}; mkdir -p $o
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $o/pytest_gpu.log 2>&1 || { tail -40 $o/pytest_gpu.log; exit 1; }
  tail -1 $o/pytest_gpu.log
fi
for rep in 1 2; do
for v in ${VALS:-0 1}; do
  for l in ${LINES:-bias wn rotate}; do
    f=$o/${l}_$(basename "$v" .so)_$rep.log
    if [ "$VAR" = LIB ]; then run="timeout -k 10 300 python -u tools/ab_run.py $v"; else run="env $VAR=$v timeout -k 10 300 python -u"; fi
    case $l in
      bias) $run bench.py --feature bias --no-cpu-baseline --profile-only > $f 2> $f.err ;;
      rotate) $run bench.py --no-cpu-baseline --profile-only > $f 2> $f.err ;;
      wn) $run tools/wn_profile.py > $f 2> $f.err ;;
      kin) $run tools/kin_profile.py > $f 2> $f.err ;;
    esac || { tail -20 $f.err; exit 1; }
    python - "$f" "$l" "$VAR=$v" <<'PY'
import ast, json, sys
f, l, tag = sys.argv[1:]
txt = open(f).read().strip().splitlines()[-1]
d = json.loads(txt) if txt.startswith("{\"") else ast.literal_eval(txt)
print(tag, l, d["ms_per_step"], d.get("kernels_ms"))
PY
  done
done
done
