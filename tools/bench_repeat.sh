#!/bin/bash
# bench.py --profile-only N times in a row (run-to-run spread)
set -o pipefail
for i in $(seq ${N:-4}); do
  timeout -k 10 200 python bench.py --steps 5 --warmup 1 --profile-only ${ARGS} > gpurun_out/rep.json 2>/dev/null || { echo "run $i FAILED"; exit 1; }
  echo "run $i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/rep.json) $(grep -o '"kernels_ms": {[^}]*}' gpurun_out/rep.json)"
done
