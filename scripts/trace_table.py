"""Per (kernel, grid, block) totals from a rocprofv3 kernel_trace.csv: python scripts/trace_table.py DIR [N] [prefix]"""
import csv
import re
import sys
from collections import defaultdict

d = defaultdict(lambda: [0, 0.0])
import glob
pref = sys.argv[3] if len(sys.argv) > 3 else "bench"
path = sorted(glob.glob(sys.argv[1].rstrip("/") + f"/**/{pref}_kernel_trace.csv", recursive=True) +
              glob.glob(sys.argv[1].rstrip("/") + f"/{pref}_kernel_trace.csv"))[0]
for r in csv.DictReader(open(path)):
    n = r["Kernel_Name"]
    m = re.search(r"::(k_\w+(<[^>]*>)?)", n)
    n = m.group(1) if m else n[:30]
    wg = int(r["Workgroup_Size_X"])
    grid = (int(r["Grid_Size_X"]) // wg, int(r["Grid_Size_Y"]), int(r["Grid_Size_Z"]))
    k = (n, grid, wg)
    d[k][0] += 1
    d[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
tot = sum(v[1] for v in d.values())
print(f"total {tot / 1e3:.1f} ms")
for k, v in sorted(d.items(), key=lambda x: -x[1][1])[:int(sys.argv[2]) if len(sys.argv) > 2 else 40]:
    print(f"{v[1] / 1e3:8.1f}ms {v[0]:6d} {v[1] / v[0]:8.2f}us {k}")
