#!/bin/bash
# End-of-round GPU pass: parity tests + smoke + the default bench line
# (tools/gpu_check.sh), the rocprofv3 stats / PMC traffic set
# (tools/profile_round.sh) and the per-kernel VALU counts (tools/pmc_valu.sh).
# Usage (GPU box, repo root): COMMIT=<id> bash tools/final_round.sh rNN
set -o pipefail
tag=${1:-r04}
bash tools/gpu_check.sh $tag || exit 1
bash tools/profile_round.sh $tag > gpurun_out/prof_$tag.log 2>&1 || { tail -5 gpurun_out/prof_$tag.log; exit 1; }
tail -2 gpurun_out/prof_$tag.log | cut -c1-200
bash tools/pmc_valu.sh || exit 1
echo final round pass done
