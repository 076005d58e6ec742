#!/bin/bash
# bench.py (RotatE, --profile-only) per side-stream workgroup caps "ground:score"
# (0 = full occupancy) and chunk count
set -o pipefail
for cfg in ${CFGS:-"0:0:2" "256:0:2" "256:512:2" "512:512:2" "256:256:2" "256:512:3"}; do
  IFS=: read g s k <<< "$cfg"
  RNNL_OVERLAP_GROUND_WG=$g RNNL_OVERLAP_SCORE_WG=$s RNNL_OVERLAP_CHUNKS=$k timeout -k 10 200 python bench.py --steps 5 --warmup 1 --profile-only > gpurun_out/ov.json 2>/dev/null || { echo "$cfg FAILED"; exit 1; }
  echo "g:s:k=$cfg $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ov.json) $(grep -o '"kernels_ms": {[^}]*}' gpurun_out/ov.json)"
done
