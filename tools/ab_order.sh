# A/B of the grounding's dequeue order (RNNL_HEAVY_FIRST variants): tools/sort_ab.py twice per variant, interleaved
set -o pipefail
mkdir -p gpurun_out/abo
for rnd in 1 2; do
for v in ${VARIANTS:-h0 h1 h2}; do
  timeout -k 10 300 python -u tools/ab_run.py rnnlogic_amd/_build/variants/$v.so tools/sort_ab.py -1 > gpurun_out/abo/$v.$rnd.txt 2> gpurun_out/abo/$v.$rnd.err || { tail -5 gpurun_out/abo/$v.$rnd.err; exit 1; }
  echo $v; cat gpurun_out/abo/$v.$rnd.txt
done
done
