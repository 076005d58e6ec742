set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r04e; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail 5 --timeout 300 --timeout-method thread -p no:cacheprovider > $o/pytest_gpu.log 2>&1
rc=$?
tail -5 $o/pytest_gpu.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 ./tools/micro/valu_rates > $o/valu_rates.txt 2>&1 && cat $o/valu_rates.txt | tail -8 && \
timeout -k 10 300 python -u tools/per_batch_forward.py > $o/per_batch.txt 2>&1 && tail -1 $o/per_batch.txt
