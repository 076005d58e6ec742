# A/B of phase A's leaf merge (RNNL_LEAF_MERGE variants from tools/build_variants.sh)
set -o pipefail
mkdir -p gpurun_out/ab1
export TMPDIR=/tmp
for v in ${VARIANTS:-m0 m1 m2}; do
  timeout -k 10 200 python -u tools/ab_run.py rnnlogic_amd/_build/variants/$v.so tools/diag_ground.py > gpurun_out/ab1/diag_$v.txt 2> gpurun_out/ab1/diag_$v.err || { echo "diag $v failed"; tail -20 gpurun_out/ab1/diag_$v.err; exit 1; }
  echo $v; cat gpurun_out/ab1/diag_$v.txt
done
for v in ${VARIANTS:-m0 m1 m2}; do
  timeout -k 10 300 python -u tools/ab_run.py rnnlogic_amd/_build/variants/$v.so tools/sort_ab.py -1 > gpurun_out/ab1/$v.txt 2> gpurun_out/ab1/$v.err || { echo "ab $v failed"; tail -20 gpurun_out/ab1/$v.err; exit 1; }
  echo $v; cat gpurun_out/ab1/$v.txt
done
