# The reference call pattern's cost split: host vs the C call, and the per-call GPU chain (rocprofv3 kernel trace)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/pb
timeout -k 10 200 python -u tools/per_batch_host.py > gpurun_out/pb/host.txt 2> gpurun_out/pb/host.err || { tail -20 gpurun_out/pb/host.err; exit 1; }
cat gpurun_out/pb/host.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pb/prof -o pb -- python3 tools/per_batch_forward.py 400 > gpurun_out/pb/trace_run.txt 2>&1 || { tail -20 gpurun_out/pb/trace_run.txt; exit 1; }
python3 tools/per_batch_trace.py gpurun_out/pb/prof > gpurun_out/pb/trace.txt 2>&1; tail -30 gpurun_out/pb/trace.txt
