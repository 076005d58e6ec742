# WN18RR (config 3) step timeline: rocprofv3 kernel trace of tools/wn_profile.py, split per step
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/wntr
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/wntr/prof -o wn -- python3 tools/wn_profile.py > gpurun_out/wntr/run.txt 2>&1 || { tail -20 gpurun_out/wntr/run.txt; exit 1; }
python3 tools/step_trace.py gpurun_out/wntr/prof > gpurun_out/wntr/steps.txt 2>&1; tail -30 gpurun_out/wntr/steps.txt
