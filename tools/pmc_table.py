"""Per-dispatch PMC table from rocprofv3 --pmc CSV outputs (one dir per pass)."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else ""
rows = defaultdict(dict)  # (kernel, grid, dispatch#) -> counter -> value
names = {}
for f in sorted(glob.glob(os.path.join(root, "p*", "*counter_collection.csv"))):
    seen = defaultdict(int)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if filt not in k:
            continue
        key = (k, r.get("Grid_Size", ""), r["Dispatch_Id"])
        rows[key][r["Counter_Name"]] = float(r["Counter_Value"])
        names[r["Counter_Name"]] = 1
# aggregate per (kernel, grid)
agg = defaultdict(lambda: defaultdict(list))
for (k, g, d), cv in rows.items():
    for c, v in cv.items():
        agg[(k[:60], g)][c].append(v)
for (k, g), cv in agg.items():
    print(f"== {k} grid={g}")
    for c in sorted(cv):
        vals = cv[c]
        print(f"   {c:28s} n={len(vals):3d} mean={sum(vals)/len(vals):.4g}")
