# A/B of the scoring pass's register budgets on small / few-row launches (tools/build_variants.sh score.hip ...):
# kinship (config 2) step, and the reference per-batch call pattern with the RotatE and bias features
set -o pipefail
mkdir -p gpurun_out/abk
for v in ${VARIANTS:-s0 s1}; do
  L=rnnlogic_amd/_build/variants/$v.so
  timeout -k 10 200 python -u tools/ab_run.py $L tools/kinship_profile.py > gpurun_out/abk/$v.txt 2> gpurun_out/abk/$v.err || { tail -5 gpurun_out/abk/$v.err; exit 1; }
  timeout -k 10 200 python -u tools/ab_run.py $L tools/per_batch_forward.py 600 RotatE >> gpurun_out/abk/$v.txt 2>> gpurun_out/abk/$v.err || { tail -5 gpurun_out/abk/$v.err; exit 1; }
  timeout -k 10 200 python -u tools/ab_run.py $L tools/per_batch_forward.py 600 bias >> gpurun_out/abk/$v.txt 2>> gpurun_out/abk/$v.err || { tail -5 gpurun_out/abk/$v.err; exit 1; }
  echo $v; grep -v "^  " gpurun_out/abk/$v.txt | head -8
done
