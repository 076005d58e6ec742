# config 2 step: grounding phases, then a kernel trace of 50 steps split per step
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/kin
timeout -k 10 200 python -u tools/kinship_profile.py > gpurun_out/kin/phases.txt 2> gpurun_out/kin/phases.err || { tail -20 gpurun_out/kin/phases.err; exit 1; }
cat gpurun_out/kin/phases.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kin/prof -o kin -- python3 tools/kinship_profile.py > gpurun_out/kin/trace_run.txt 2>&1 || { tail -20 gpurun_out/kin/trace_run.txt; exit 1; }
python3 tools/step_trace.py gpurun_out/kin/prof lstm_trie_level_kernel 3 > gpurun_out/kin/steps.txt 2>&1; tail -40 gpurun_out/kin/steps.txt
