"""HBM traffic per launch from two rocprofv3 --pmc passes (FETCH_SIZE and
WRITE_SIZE, separate runs of the same command), corrected as
MI355X_MICROARCH.md §HBM prescribes (gfx950 FETCH_SIZE counts half of a
coalesced read stream: doubled; WRITE_SIZE exact; both in KiB).  Writes
profiles/<name>.json, which bench.py reads for roofline.traffic.

Usage: python tools/pmc_traffic.py FETCH_DIR WRITE_DIR OUT.json "workload string" [COMMIT]

The summary is stamped with the sha256 of the kernel sources it was captured
with (bench.csrc_fingerprint) and the commit id given (the GPU box has no
git); bench.py reports a summary's traffic only while the stamp matches.
"""
import os
import collections
import csv
import glob
import json
import sys


def per_kernel(root, counter):
    vals = collections.defaultdict(list)
    for f in glob.glob(root + "/**/*_counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if row["Counter_Name"] != counter:
                continue
            name = row["Kernel_Name"].split("(")[0].replace("void ", "")
            vals[(name, row["Dispatch_Id"])].append(float(row["Counter_Value"]))
    out = collections.defaultdict(list)
    for (name, _), v in vals.items():
        out[name].append(sum(v))
    return {k: sum(v) / len(v) for k, v in out.items()}


fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
write = per_kernel(sys.argv[2], "WRITE_SIZE")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import csrc_fingerprint  # noqa: E402

res = {"workload": sys.argv[4], "commit": sys.argv[5] if len(sys.argv) > 5 else "?",
       "csrc_sha256": csrc_fingerprint(),
       "source": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate passes); bytes = 2 x FETCH_SIZE KiB "
                 "(gfx950 counts half of a coalesced read stream) + WRITE_SIZE KiB, per launch (mean over launches)",
       "kernels": {}}
for k in sorted(set(fetch) | set(write)):
    if not k.startswith("rnnl::"):
        continue
    f, w = fetch.get(k, 0.0), write.get(k, 0.0)
    res["kernels"][k] = {"fetch_kib": f, "write_kib": w, "bytes": int(2 * f * 1024 + w * 1024)}
json.dump(res, open(sys.argv[3], "w"), indent=1)
print(json.dumps(res, indent=1))
