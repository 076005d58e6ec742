#!/bin/bash
# A/B of kernel time and HBM traffic on the bias bench (one-stream grounding +
# scoring) for builds from tools/build_variants.sh: per variant, kernel stats
# and the FETCH_SIZE / WRITE_SIZE passes, summarised by tools/pmc_traffic.py.
# GPU box, repo root: bash tools/traffic_ab.sh base nt ...
set -o pipefail
export TMPDIR=/tmp
for v in "$@"; do
  lib=rnnlogic_amd/_build/variants/$v.so
  o=gpurun_out/tab_$v; rm -rf $o; mkdir -p $o
  B="tools/ab_run.py $lib bench.py --feature bias --profile-only --no-cpu-baseline"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/stats -o run -- \
      python3 $B --steps 10 --warmup 2 > $o/bias.json 2> $o/bias.err || { tail -5 $o/bias.err; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $o/fetch -o run -- \
      python3 $B --steps 3 --warmup 1 > /dev/null 2> $o/fetch.err || { tail -5 $o/fetch.err; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $o/write -o run -- \
      python3 $B --steps 3 --warmup 1 > /dev/null 2> $o/write.err || { tail -5 $o/write.err; exit 1; }
  python3 tools/pmc_traffic.py $o/fetch $o/write $o/traffic.json "$v" "-" > /dev/null
  python3 - "$o" "$v" <<'PY'
import csv, glob, json, sys
o, v = sys.argv[1], sys.argv[2]
t = json.load(open(o + "/traffic.json"))["kernels"]
st = {r["Name"].split("(")[0].replace("void ", ""): float(r["AverageNs"]) / 1e6
      for r in csv.DictReader(open(glob.glob(o + "/stats/**/*kernel_stats.csv", recursive=True)[0]))}
for k in sorted(t):
    if "ground" in k or "score_sum" in k:
        print("%s %-45s %7.3f ms  fetch %6.2f GB  write %6.2f GB" % (v, k, st.get(k, 0), 2 * t[k]["fetch_kib"] * 1024 / 1e9,
                                                                   t[k]["write_kib"] * 1024 / 1e9))
PY
  rm -rf $o/fetch $o/write
done
