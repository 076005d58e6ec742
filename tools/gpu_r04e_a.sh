# Round-4 GPU pass: parity suite, VALU rates microbenchmark, per-batch forward,
# A/B of the scoring variants (bench lines), VALU counters per kernel.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r04e; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail 5 --timeout 300 --timeout-method thread -p no:cacheprovider > $o/pytest_gpu.log 2>&1
rc=$?
tail -5 $o/pytest_gpu.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 ./tools/micro/valu_rates > $o/valu_rates.txt 2>&1 && tail -8 $o/valu_rates.txt && \
timeout -k 10 300 python -u tools/per_batch_forward.py > $o/per_batch.txt 2>&1 && tail -1 $o/per_batch.txt && \
TAG=r04e_ab VAR=RNNL_LIB VALS="rnnlogic_amd/_build/variants/cur.so rnnlogic_amd/_build/variants/coop.so" LINES="rotate bias" bash tools/env_ab.sh && \
timeout -k 10 300 python -u tools/wn_profile.py > $o/wn.txt 2>&1 && tail -1 $o/wn.txt && \
bash tools/pmc_valu.sh && cp gpurun_out/pmc_valu_fb.txt gpurun_out/pmc_valu_wn.txt $o/ && \
TAG=r04e_k VALS="rnnlogic_amd/_build/variants/cur.so" bash tools/kstats_ab.sh
