#!/bin/bash
# SQ counter passes (one rocprofv3 --pmc run each, <= 8 SQ counters) over the
# bias bench's side kernels, the RotatE bench step and RotatE alone; per-kernel
# means via tools/pmc_summary.py.  GPU box, repo root: bash tools/pmc_passes.sh
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/pmcp; mkdir -p $o
P1="SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_CVT SQ_INSTS_SALU"
P2="SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_LDS SQ_INSTS_VMEM_RD"
P3="SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES SQ_BUSY_CYCLES"
run() {  # tag counters cmd...
  local tag=$1 c=$2; shift 2
  timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d $o/$tag -o run -- "$@" > $o/$tag.out 2> $o/$tag.err \
    || { tail -5 $o/$tag.err; return 1; }
}
run bias1 "$P1" python3 bench.py --feature bias --steps 2 --warmup 1 --profile-only --no-cpu-baseline &&
run bias2 "$P2" python3 bench.py --feature bias --steps 2 --warmup 1 --profile-only --no-cpu-baseline &&
run rot3 "$P3" python3 bench.py --steps 2 --warmup 1 --profile-only --no-cpu-baseline &&
run alone3 "$P3" python3 tools/rotate_alone.py || exit 1
for t in bias1 bias2; do
  python3 tools/pmc_summary.py $o/$t rnnl:: | grep -E "ground_kernel|score_sum_chunk" | tail -2
done
python3 tools/pmc_summary.py $o/rot3 rnnl:: | grep -E "rotate_direct|ground_kernel|score_sum_chunk" | tail -3
python3 tools/pmc_summary.py $o/alone3 rnnl:: | grep -E "rotate_direct" | tail -1
