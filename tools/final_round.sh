#!/bin/bash
# End-of-round GPU pass: parity tests + smoke + the default bench line
# (tools/gpu_check.sh), the rocprofv3 stats / PMC traffic set
# (tools/profile_round.sh) and the per-kernel VALU counts (tools/pmc_valu.sh).
# Usage (GPU box, repo root): COMMIT=<id> bash tools/final_round.sh rNN
set -o pipefail
tag=${1:-r06}
mkdir -p gpurun_out/$tag
# the library rebuilt from source on the box (build() as the driver runs it), logged
( set -x; rm -rf rnnlogic_amd/_build oracle/_build; hipcc --version | head -2; \
  timeout -k 10 900 python -u -c "import time, __graft_entry__ as g; t = time.time(); g.build(); print('build() %.1f s' % (time.time() - t))"; \
  ls -la rnnlogic_amd/_build/librnnlogic_hip.so ) > gpurun_out/$tag/build_on_box.log 2>&1 || { tail -20 gpurun_out/$tag/build_on_box.log; exit 1; }
tail -2 gpurun_out/$tag/build_on_box.log
# parity tests + smoke (the bench waits for the traffic stamps below)
NO_BENCH=1 bash tools/gpu_check.sh $tag || exit 1
bash tools/profile_round.sh $tag > gpurun_out/prof_$tag.log 2>&1 || { tail -5 gpurun_out/prof_$tag.log; exit 1; }
tail -2 gpurun_out/prof_$tag.log | cut -c1-200
# the default bench line, reading traffic summaries stamped with these kernel sources
cp gpurun_out/prof_$tag/traffic_rotate.json gpurun_out/prof_$tag/traffic_bias.json profiles/
timeout -k 10 600 python -u bench.py > gpurun_out/$tag/bench.json 2> gpurun_out/$tag/bench.err || { tail -30 gpurun_out/$tag/bench.err; exit 1; }
cut -c1-400 gpurun_out/$tag/bench.json
bash tools/pmc_valu.sh || exit 1
echo final round pass done
