timeout -k 10 500 python -u -m pytest tests/test_0_rccl_bench.py tests/test_0_bench_world3.py -m gpu -x -q --timeout 450 --timeout-method thread -p no:cacheprovider > gpurun_out/rccl.log 2>&1; tail -3 gpurun_out/rccl.log
for rep in 1 2; do for v in g256 g512 g128; do
RNNL_LIB=rnnlogic_amd/_build/variants/$v.so timeout -k 10 300 python3 bench.py --feature bias --steps 10 --warmup 2 --profile-only 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print(\"$v\", d[\"ms_per_step\"], d[\"kernels_ms\"][\"tail_after_base\"])"
done; done
mkdir -p gpurun_out/wntr2 && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/wntr2 -o run -- python3 tools/wn_steps.py > /dev/null 2>&1 && python3 tools/step_trace.py gpurun_out/wntr2 | head -45
