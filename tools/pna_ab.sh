set -o pipefail
mkdir -p gpurun_out/pna
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pna/tests.log 2>&1 || { tail -30 gpurun_out/pna/tests.log; exit 1; }
tail -3 gpurun_out/pna/tests.log
TAG=pna VARS="old w2 w2v4" bash tools/var_wn.sh
for v in old w2 w2v4; do
  RNNL_LIB=rnnlogic_amd/_build/variants/$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pna/prof_$v -o run -- python3 tools/wn_profile.py > /dev/null 2> gpurun_out/pna/prof_$v.err || { tail -5 gpurun_out/pna/prof_$v.err; exit 1; }
done
