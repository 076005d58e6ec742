#!/bin/bash
# bench.py (RotatE) per overlap chunking; prints ms_per_step and the kernel split
set -o pipefail
for k in ${CHUNKS:-1 2 4 8}; do
  RNNL_OVERLAP_CHUNKS=$k timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/ov.json 2>/dev/null || { echo "chunks=$k FAILED"; exit 1; }
  echo "chunks=$k $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ov.json) $(grep -o '"kernels_ms": {[^}]*}' gpurun_out/ov.json)"
done
