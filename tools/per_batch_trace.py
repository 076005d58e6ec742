"""Per-call GPU timeline of the per-batch PredictorPlus.forward loop from a
rocprofv3 --kernel-trace CSV: per call, the span from its first kernel's start
to its last kernel's end, the busy time (union of kernel intervals) and the
per-kernel mean durations.  Calls are split at the rotate_hr_kernel launches
(one per call; or at MARKER, with BACK kernels before it counted in the
call).  Usage: python tools/per_batch_trace.py DIR [MARKER BACK]"""
import collections
import csv
import glob
import sys

rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]))
rows.sort()
marker = sys.argv[2] if len(sys.argv) > 2 else "rotate_hr_kernel"
back = int(sys.argv[3]) if len(sys.argv) > 3 else 8
starts = [i for i, r in enumerate(rows) if marker in r[2]]
spans, busy, gaps = [], [], []
per = collections.defaultdict(list)
for a, b in zip(starts[5:-2], starts[6:-1]):
    call = rows[a - back:b - back]  # the kernels before rotate_hr belong to the call too
    if not call:
        continue
    s0 = min(c[0] for c in call)
    s1 = max(c[1] for c in call)
    spans.append(s1 - s0)
    iv = sorted((c[0], c[1]) for c in call)
    u, cur = 0, None
    for x, y in iv:
        if cur is None or x > cur[1]:
            if cur:
                u += cur[1] - cur[0]
            cur = [x, y]
        else:
            cur[1] = max(cur[1], y)
    u += cur[1] - cur[0]
    busy.append(u)
    for c in call:
        per[c[2]].append(c[1] - c[0])
n = len(spans)
period = (rows[starts[-2]][0] - rows[starts[5]][0]) / max(len(starts) - 7, 1)
print("calls %d: period %.1f us, kernel span %.1f us, busy %.1f us" % (
    n, period / 1e3, sum(spans) / n / 1e3, sum(busy) / n / 1e3))
for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
    print("  %-45s n/call %.2f  mean %.1f us" % (k[-45:], len(v) / n, sum(v) / len(v) / 1e3))
# two consecutive calls, kernel by kernel (offsets in us from the first's rotate_hr start)
if len(starts) > 12:
    a, b = starts[10], starts[12]
    t0 = rows[a][0]
    print("two calls (offsets in us from the marker start):")
    for r in rows[a - back:b - back]:
        print("  %9.1f %9.1f  %s" % ((r[0] - t0) / 1e3, (r[1] - t0) / 1e3, r[2][-60:]))
