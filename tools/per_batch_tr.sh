set -o pipefail
mkdir -p gpurun_out/pb
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pb/tr -- python -u tools/per_batch_forward.py 300 > gpurun_out/pb/tr.log 2>&1 || { tail -5 gpurun_out/pb/tr.log; exit 1; }
python tools/per_batch_trace.py gpurun_out/pb/tr > gpurun_out/pb/trace.txt && cat gpurun_out/pb/trace.txt
rm -rf gpurun_out/pb/tr
