#!/bin/bash
# One rocprofv3 --pmc pass of SQ counters over the bias bench (2 steps);
# prints per-kernel means (tools/pmc_summary.py).
set -o pipefail
export TMPDIR=/tmp
tag=${1:-sq}
C=${COUNTERS:-"SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES"}
timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc_$tag -o run -- \
    python3 bench.py --feature bias --steps 2 --warmup 1 --profile-only > gpurun_out/pmc_$tag.json 2> gpurun_out/pmc_$tag.err \
    || { tail -5 gpurun_out/pmc_$tag.err; exit 1; }
python3 tools/pmc_summary.py gpurun_out/pmc_$tag rnnl:: | grep -E "ground_kernel|score_sum|score_linear|memo_sum|chunk_" | tail -6
