#!/bin/bash
# bench.py (RotatE, --profile-only) per environment setting (space-separated VAR=val,... lists)
set -o pipefail
for cfg in ${CFGS}; do
  env $(echo $cfg | tr ',' ' ') timeout -k 10 200 python bench.py --steps 8 --warmup 3 --profile-only ${BENCH_ARGS} > gpurun_out/ov.json 2>gpurun_out/ov.err || { echo "$cfg FAILED"; tail -3 gpurun_out/ov.err; exit 1; }
  echo "$cfg $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ov.json) $(grep -o '"kernels_ms": {[^}]*}' gpurun_out/ov.json)"
done
