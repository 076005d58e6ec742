#!/bin/bash
# Kernel stats + PMC FETCH/WRITE of the bias step (grounding + scoring alone).
# Usage (GPU box, repo root): bash tools/prof_bias.sh tag
set -o pipefail
export TMPDIR=/tmp
tag=${1:-bias}
o=gpurun_out/prof_$tag
mkdir -p $o
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/bias -o run -- \
    python3 bench.py --feature bias --steps 10 --warmup 2 --profile-only > $o/bias.json 2> $o/bias.err || { tail -5 $o/bias.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $o/bfetch -o run -- \
    python3 bench.py --feature bias --steps 3 --warmup 1 --profile-only > /dev/null 2> $o/bfetch.err || { tail -5 $o/bfetch.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $o/bwrite -o run -- \
    python3 bench.py --feature bias --steps 3 --warmup 1 --profile-only > /dev/null 2> $o/bwrite.err || { tail -5 $o/bwrite.err; exit 1; }
find $o -name "*kernel_stats.csv" | head -3 | xargs -I{} head -6 {}
