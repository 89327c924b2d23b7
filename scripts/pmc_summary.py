"""Summarise rocprofv3 --pmc csv passes (<dir>/p*/**/counter_collection.csv): per (kernel, grid) the mean
of every counter over its dispatches, all passes joined.  python scripts/pmc_summary.py <dir>"""
import csv
import glob
import re
import sys
from collections import defaultdict

d = sys.argv[1]
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"{d}/p*/**/*counter_collection.csv", recursive=True):
    per = defaultdict(float)
    meta = {}
    for r in csv.DictReader(open(f)):
        key = (r["Dispatch_Id"],)
        per[(key, r["Counter_Name"])] += float(r["Counter_Value"])
        g = f'{int(r["Grid_Size"]) // max(int(r["Workgroup_Size"]), 1)}'
        meta[key] = (re.sub(r"\(anonymous namespace\)::|\(ConvArgs\)|void ", "", r["Kernel_Name"])[:40], g)
    for (key, cn), v in per.items():
        vals[meta[key]][cn].append(v)
names = sorted({c for v in vals.values() for c in v})
for k, v in sorted(vals.items()):
    print(f"{k[0]} WGs={k[1]}")
    print("   " + "  ".join(f"{c}={sum(v[c]) / len(v[c]):.4g}" for c in names if c in v))
