#!/bin/bash
# rocprofv3 kernel stats of the bias-feature bench (ground + score kernels dominate)
# Usage (GPU box, repo root): bash tools/prof_bias.sh <tag>
set -o pipefail
export TMPDIR=/tmp
tag=${1:-bias}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run -- python3 bench.py --feature bias --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_$tag.json 2> gpurun_out/prof_$tag.err || { tail -20 gpurun_out/prof_$tag.err; exit 1; }
f=$(find gpurun_out/prof_$tag -name "*kernel_stats.csv" | head -1)
cut -d, -f1-4 "$f" | head -14
