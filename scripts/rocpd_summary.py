"""Per-kernel summary of a rocprofv3 sqlite trace (rocpd 'kernels' view): calls, average / total device time,
grid, grouped by kernel name and grid.  python scripts/rocpd_summary.py <results.db> [name-regex] [skip-first-N-per-group]"""
import re
import sqlite3
import sys
from collections import defaultdict

db = sys.argv[1]
pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
skip = int(sys.argv[3]) if len(sys.argv) > 3 else 0
c = sqlite3.connect(db)
groups = defaultdict(list)
for name, dur, gx, gy, gz, wx in c.execute(
        "select name, duration, grid_x, grid_y, grid_z, workgroup_x from kernels order by start"):
    if pat and not pat.search(name):
        continue
    groups[(name, gx // max(wx, 1), gy, gz)].append(dur / 1e3)
rows = []
for (name, gx, gy, gz), ds in groups.items():
    ds = ds[skip:] or ds
    rows.append((sum(ds), len(ds), sum(ds) / len(ds), name, f"{gx}x{gy}x{gz}"))
rows.sort(reverse=True)
tot = sum(r[0] for r in rows)
print(f"{'total_us':>10} {'calls':>6} {'avg_us':>8}  grid(WGs)      kernel")
for t, n, a, name, g in rows:
    short = re.sub(r"\(anonymous namespace\)::", "", name)
    short = short[:110]
    print(f"{t:10.1f} {n:6d} {a:8.2f}  {g:14s} {short}")
print(f"{tot:10.1f} total")
