set -o pipefail
tag=r06f
mkdir -p gpurun_out/$tag
( set -x; rm -rf rnnlogic_amd/_build oracle/_build; hipcc --version | head -2;   timeout -k 10 900 python -u -c "import time, __graft_entry__ as g; t = time.time(); g.build(); print('build() %.1f s' % (time.time() - t))";   ls -la rnnlogic_amd/_build/librnnlogic_hip.so ) > gpurun_out/$tag/build_on_box.log 2>&1 || { tail -20 gpurun_out/$tag/build_on_box.log; exit 1; }
tail -2 gpurun_out/$tag/build_on_box.log
bash tools/gpu_check.sh $tag
