"""Print the kernel averages of a rocprofv3 rocpd database (top_kernels view)."""
import sqlite3
import sys

db, tag = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else ""
c = sqlite3.connect(db)
rows = c.execute("select name, total_calls, average from top_kernels").fetchall()
keep = [(n.split("(")[0].replace("void ", "").replace("rnnl::", ""), k, a) for n, k, a in rows
        if "rnnl::" in n and a > 50]
print(tag, "  ".join("%s x%d %.0fus" % r for r in keep[:6]))
