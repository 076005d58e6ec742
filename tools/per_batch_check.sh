set -o pipefail
mkdir -p gpurun_out/pb
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/per_batch_forward.py > gpurun_out/pb/fwd.txt 2> gpurun_out/pb/fwd.err || { tail -5 gpurun_out/pb/fwd.err; exit 1; }
cat gpurun_out/pb/fwd.txt
timeout -k 10 300 python -u tools/per_batch_host.py 400 > gpurun_out/pb/host.txt 2> gpurun_out/pb/host.err || { tail -5 gpurun_out/pb/host.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pb/tr -- python -u tools/per_batch_forward.py 300 > gpurun_out/pb/tr.log 2>&1 || { tail -5 gpurun_out/pb/tr.log; exit 1; }
python tools/per_batch_trace.py gpurun_out/pb/tr > gpurun_out/pb/trace.txt && cat gpurun_out/pb/trace.txt
rm -rf gpurun_out/pb/tr
timeout -k 10 400 python -u tools/train_timing.py 500 > gpurun_out/pb/timing.txt 2> gpurun_out/pb/timing.err || { tail -5 gpurun_out/pb/timing.err; exit 1; }
cat gpurun_out/pb/timing.txt
