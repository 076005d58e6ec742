# N = 8 slowest shard (rank 3): side-stream workgroup caps, then a kernel trace of its step
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/sh
timeout -k 10 300 python -u tools/shard_run.py 8 3 20 128/128 64/64 96/96 256/256 128/64 64/128 128/128 > gpurun_out/sh/caps.txt 2> gpurun_out/sh/caps.err || { tail -20 gpurun_out/sh/caps.err; exit 1; }
cat gpurun_out/sh/caps.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sh/prof -o sh -- python3 tools/shard_run.py 8 3 8 > gpurun_out/sh/trace_run.txt 2>&1 || { tail -20 gpurun_out/sh/trace_run.txt; exit 1; }
python3 tools/step_trace.py gpurun_out/sh/prof > gpurun_out/sh/steps.txt 2>&1; tail -40 gpurun_out/sh/steps.txt
