# Times A/B library builds (tools/build_variants.sh) with tools/sort_ab.py: VARIANTS="a b" bash tools/ab_time.sh
set -o pipefail
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
for v in $VARIANTS; do
  timeout -k 10 300 python -u tools/ab_run.py rnnlogic_amd/_build/variants/$v.so tools/sort_ab.py -1 > gpurun_out/ab/$v.txt 2> gpurun_out/ab/$v.err || { echo "ab $v failed"; tail -20 gpurun_out/ab/$v.err; exit 1; }
  echo $v; cat gpurun_out/ab/$v.txt
done
