#!/bin/bash
# Round profile set for profiles/: rocprofv3 kernel stats of the bench and
# two PMC passes (FETCH_SIZE, WRITE_SIZE) -> per-kernel HBM traffic JSON.
# Usage (GPU box, repo root): bash tools/profile_round.sh rNN
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r01}
o=gpurun_out/prof_$tag
mkdir -p $o
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $o/stats -o run -- \
    python3 bench.py --steps 10 --warmup 2 --profile-only > $o/bench.json 2> $o/bench.err || { tail -5 $o/bench.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $o/fetch -o run -- \
    python3 bench.py --steps 3 --warmup 1 --profile-only > /dev/null 2> $o/fetch.err || { tail -5 $o/fetch.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $o/write -o run -- \
    python3 bench.py --steps 3 --warmup 1 --profile-only > /dev/null 2> $o/write.err || { tail -5 $o/write.err; exit 1; }
ls $o/stats $o/fetch $o/write | head -20
cat $o/bench.json
# the grounding kernels alone (bias feature: one ground + one score launch per step)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/bias -o run -- \
    python3 bench.py --feature bias --steps 10 --warmup 2 --profile-only > $o/bias.json 2> $o/bias.err || { tail -5 $o/bias.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $o/bfetch -o run -- \
    python3 bench.py --feature bias --steps 3 --warmup 1 --profile-only > /dev/null 2> $o/bfetch.err || { tail -5 $o/bfetch.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $o/bwrite -o run -- \
    python3 bench.py --feature bias --steps 3 --warmup 1 --profile-only > /dev/null 2> $o/bwrite.err || { tail -5 $o/bwrite.err; exit 1; }
cat $o/bias.json
# per-kernel traffic summaries, stamped with the kernel sources (bench.py checks the stamp)
python3 tools/pmc_traffic.py $o/fetch $o/write $o/traffic_rotate.json "FB15k-237 RotatE bench step (bench.py --profile-only, $tag)" "${COMMIT:-?}" > /dev/null
python3 tools/pmc_traffic.py $o/bfetch $o/bwrite $o/traffic_bias.json "FB15k-237 bias-feature bench step: grounding + scoring in one launch (bench.py --feature bias --profile-only, $tag)" "${COMMIT:-?}" > /dev/null
rm -rf $o/fetch $o/write $o/bfetch $o/bwrite
