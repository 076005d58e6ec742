set -o pipefail
mkdir -p gpurun_out/t1
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_rotate_grad.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t1/pytest.log 2>&1 || { tail -60 gpurun_out/t1/pytest.log; exit 1; }
tail -3 gpurun_out/t1/pytest.log
timeout -k 10 300 python -u tools/train_profile.py > gpurun_out/t1/rotate.txt 2> gpurun_out/t1/rotate.err || { tail -20 gpurun_out/t1/rotate.err; exit 1; }
timeout -k 10 300 python -u tools/train_profile.py emb > gpurun_out/t1/emb.txt 2> gpurun_out/t1/emb.err || { tail -20 gpurun_out/t1/emb.err; exit 1; }
head -1 gpurun_out/t1/rotate.txt; head -1 gpurun_out/t1/emb.txt
timeout -k 10 300 python -u tools/train_timing.py 1000 > gpurun_out/t1/timing.txt 2> gpurun_out/t1/timing.err || { tail -20 gpurun_out/t1/timing.err; exit 1; }
cat gpurun_out/t1/timing.txt
timeout -k 10 300 python -u tools/train_timing.py 300 profile > gpurun_out/t1/loop_prof.txt 2> gpurun_out/t1/loop_prof.err || { tail -20 gpurun_out/t1/loop_prof.err; exit 1; }
