#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench, rocprof kernel stats of the bench.
# Usage (from the repo root on the box): bash tools/gpu_check.sh [tag]
set -o pipefail
tag=${1:-run}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $out/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 $out/pytest_gpu.log; exit 1; }
tail -3 $out/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 600 python -u bench.py > $out/bench.json 2> $out/bench.err || { echo "bench failed"; tail -30 $out/bench.err; exit 1; }
cat $out/bench.json
