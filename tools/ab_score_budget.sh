set -o pipefail
VARIANTS="s0 s1" bash tools/ab_kinship.sh || exit 1
mkdir -p gpurun_out/abs
for v in s1 s3; do
  timeout -k 10 300 python -u tools/ab_run.py rnnlogic_amd/_build/variants/$v.so tools/sort_ab.py -1 > gpurun_out/abs/$v.txt 2> gpurun_out/abs/$v.err || { tail -5 gpurun_out/abs/$v.err; exit 1; }
  echo $v; cat gpurun_out/abs/$v.txt
done
