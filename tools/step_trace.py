"""Per-step GPU timeline of `bench.py --profile-only` from a rocprofv3
--kernel-trace CSV: steps are split at the rotate_hr_kernel launches (one per
step); per step the period (rotate_hr start to the next one's), the RotatE
pass, the span from the step's first kernel to its last, the idle time
(period minus the union of kernel intervals) and where the idle sits (before
RotatE starts / after it ends).  Usage: python tools/step_trace.py DIR
[SPLIT_KERNEL [EVERY]] — split at every EVERY-th launch of another kernel
(e.g. lstm_trie_level_kernel 4 for a step without RotatE)."""
import collections
import csv
import glob
import statistics
import sys

rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]))
rows.sort()
split = sys.argv[2] if len(sys.argv) > 2 else "rotate_hr_kernel"
every = int(sys.argv[3]) if len(sys.argv) > 3 else 1
hr = [i for i, r in enumerate(rows) if split in r[2]][::every]
rot = [i for i, r in enumerate(rows) if "rotate_direct_kernel" in r[2] or "rotate_mfma_kernel" in r[2]]


def union(iv):
    u, cur = 0, None
    for x, y in sorted(iv):
        if cur is None or x > cur[1]:
            if cur:
                u += cur[1] - cur[0]
            cur = [x, y]
        else:
            cur[1] = max(cur[1], y)
    return u + (cur[1] - cur[0] if cur else 0)


stat = collections.defaultdict(list)
per = collections.defaultdict(list)
for a, b in zip(hr[:-1], hr[1:]):
    t0, t1 = rows[a][0], rows[b][0]
    ks = [r for r in rows if t0 <= r[0] < t1]
    rk = [r for r in ks if "rotate_direct" in r[2] or "rotate_mfma" in r[2]]
    stat["period_ms"].append((t1 - t0) / 1e6)
    stat["busy_ms"].append(union([(r[0], min(r[1], t1)) for r in ks]) / 1e6)
    if rk:
        stat["rotate_ms"].append(sum(r[1] - r[0] for r in rk) / 1e6)
        stat["hr_to_rotate_start_ms"].append((rk[0][0] - t0) / 1e6)
        last = max(r[1] for r in ks)
        stat["rotate_end_to_last_kernel_ms"].append((last - rk[-1][1]) / 1e6)
        stat["last_kernel_to_next_step_ms"].append((t1 - last) / 1e6)
    for r in ks:
        per[r[2]].append((r[1] - r[0]) / 1e6)
print("steps: %d" % len(stat["period_ms"]))
for k, v in stat.items():
    print("  %-32s mean %.3f  min %.3f  max %.3f" % (k, statistics.mean(v), min(v), max(v)))
print("kernels (mean ms per launch, launches per step):")
ns = max(len(stat["period_ms"]), 1)
for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
    print("  %-60s %9.3f  x%.1f" % (k[-60:], statistics.mean(v), len(v) / ns))
# the head of one step (what runs before RotatE starts), as offsets from rotate_hr
if len(hr) > 3:
    a, b = hr[2], hr[3]
    t0 = rows[a][0]
    prev_end = max(r[1] for r in rows[:a]) if a else t0
    print("one step (offsets in us from rotate_hr start; previous step's last kernel ended at %.1f):"
          % ((prev_end - t0) / 1e3))
    for r in rows:
        if rows[a - 12][0] <= r[0] < rows[b][0] and (r[0] - t0) < 2e6:
            print("  %10.1f %10.1f  %s" % ((r[0] - t0) / 1e3, (r[1] - t0) / 1e3, r[2][-70:]))
