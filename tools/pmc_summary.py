"""Sum rocprofv3 --pmc CSV counters per (dispatch, kernel) for kernels whose
name contains a filter string.  Usage: python tools/pmc_summary.py DIR [filter]"""
import collections
import csv
import glob
import sys

root = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else ""
for f in sorted(glob.glob(root + "/**/*_counter_collection.csv", recursive=True)):
    agg = collections.OrderedDict()
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"]
        if filt not in k:
            continue
        key = (int(row["Dispatch_Id"]), k.split("(")[0])
        agg.setdefault(key, collections.defaultdict(float))[row["Counter_Name"]] += float(row["Counter_Value"])
    for (d, k), c in agg.items():
        print(d, k, " ".join("%s=%.4g" % kv for kv in sorted(c.items())))
