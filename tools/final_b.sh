# final pass part 2: rocprofv3 stats + PMC traffic (tools/profile_round.sh) and VALU counts (tools/pmc_valu.sh)
set -o pipefail
COMMIT=9804fc7 bash tools/profile_round.sh r06f > gpurun_out/prof_r06f.log 2>&1 || { tail -5 gpurun_out/prof_r06f.log; exit 1; }
tail -2 gpurun_out/prof_r06f.log | cut -c1-300
bash tools/pmc_valu.sh || exit 1
echo profile pass done
