# A/B of the grounding's workgroup shape on one-window graphs (kinship): RNNL_SMALL_GRAPH_WG variants
set -o pipefail
mkdir -p gpurun_out/absg
for rnd in 1 2; do
for v in ${VARIANTS:-k0 k3}; do
  timeout -k 10 200 python -u tools/ab_run.py rnnlogic_amd/_build/variants/$v.so tools/kinship_profile.py > gpurun_out/absg/$v.$rnd.txt 2> gpurun_out/absg/$v.$rnd.err || { tail -5 gpurun_out/absg/$v.$rnd.err; exit 1; }
  echo $v; head -4 gpurun_out/absg/$v.$rnd.txt
done
done
