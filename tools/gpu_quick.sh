#!/bin/bash
# Parity tests + both bench features without the CPU baselines (iteration loop).
# Usage (GPU box, repo root): bash tools/gpu_quick.sh tag [pytest -k expr]
set -o pipefail
tag=${1:-quick}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
if [ -n "$2" ]; then kx=(-k "$2"); else kx=(); fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider "${kx[@]}" > $out/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 $out/pytest_gpu.log; exit 1; }
tail -2 $out/pytest_gpu.log
timeout -k 10 300 python -u bench.py --feature bias --no-cpu-baseline > $out/bias.json 2> $out/bias.err || { echo "bias bench failed"; tail -30 $out/bias.err; exit 1; }
python -c "import json;d=json.load(open('$out/bias.json'));print('bias', d['value'], d['ms_per_step'], d['kernels_ms'], d['roofline_grounding']['frac'])"
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $out/bench.json 2> $out/bench.err || { echo "bench failed"; tail -30 $out/bench.err; exit 1; }
python -c "import json;d=json.load(open('$out/bench.json'));print('rotate', d['value'], d['ms_per_step'], d['kernels_ms'])"
