#!/bin/bash
# VALU / SALU wave-instruction counts per kernel (one rocprofv3 --pmc pass
# each) for the FB15k-237 RotatE step and the WN18RR step: the side-stream
# kernels' VALU instructions against RotatE's (interference).
set -o pipefail
export TMPDIR=/tmp
C="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES"
timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc_valu_fb -o run -- \
    python3 bench.py --steps 2 --warmup 1 --profile-only --no-cpu-baseline > gpurun_out/pmc_valu_fb.json 2> gpurun_out/pmc_valu_fb.err \
    || { tail -5 gpurun_out/pmc_valu_fb.err; exit 1; }
python3 tools/pmc_summary.py gpurun_out/pmc_valu_fb rnnl:: > gpurun_out/pmc_valu_fb.txt
timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc_valu_wn -o run -- \
    python3 tools/wn_profile.py > gpurun_out/pmc_valu_wn.json 2> gpurun_out/pmc_valu_wn.err \
    || { tail -5 gpurun_out/pmc_valu_wn.err; exit 1; }
python3 tools/pmc_summary.py gpurun_out/pmc_valu_wn rnnl:: > gpurun_out/pmc_valu_wn.txt
rm -rf gpurun_out/pmc_valu_fb gpurun_out/pmc_valu_wn
