COMMIT=$1 bash tools/final_round.sh r04 || exit 1
mkdir -p gpurun_out/wntr2 && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/wntr2 -o run -- python3 tools/wn_steps.py > /dev/null 2>&1 && python3 tools/step_trace.py gpurun_out/wntr2 > gpurun_out/wntr2/steps.txt; head -30 gpurun_out/wntr2/steps.txt
