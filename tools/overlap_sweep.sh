#!/bin/bash
# bench.py (RotatE, --profile-only) per overlap setting: "off" or the chunk count
set -o pipefail
for k in ${CHUNKS:-off 1 2 3}; do
  if [ "$k" = off ]; then env="RNNL_OVERLAP=0"; else env="RNNL_OVERLAP_CHUNKS=$k"; fi
  env $env timeout -k 10 300 python bench.py --steps 5 --warmup 1 --profile-only > gpurun_out/ov.json 2>/dev/null || { echo "$k FAILED"; exit 1; }
  echo "overlap=$k $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ov.json) $(grep -o '"kernels_ms": {[^}]*}' gpurun_out/ov.json)"
done
