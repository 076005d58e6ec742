#!/bin/bash
# Per-kernel device time (rocprofv3 --kernel-trace --stats) of the bias-feature
# bench step (one stream: grounding + scoring) for each variant library.
# Usage (GPU box): TAG=x VALS="a.so b.so" bash tools/kstats_ab.sh
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/${TAG:-kstats}; mkdir -p $o
for v in $VALS; do
  n=$(basename $v .so)
  RNNL_LIB=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/$n -o run -- \
      python3 bench.py --feature bias --steps 10 --warmup 2 --profile-only --no-cpu-baseline > $o/$n.json 2> $o/$n.err \
      || { tail -5 $o/$n.err; exit 1; }
  f=$(find $o/$n -name "*kernel_stats.csv" | head -1)
  cp $f $o/${n}_kernel_stats.csv
  python3 - "$o/${n}_kernel_stats.csv" "$n" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:8]:
    print(sys.argv[2], r["Name"][:60], r["Calls"], "%.3f ms avg" % (float(r["AverageNs"]) / 1e6))
PY
  rm -rf $o/$n
done
