"""Per-kernel PMC summary from a rocprofv3 `--pmc` database (ROCm 7 rocpd): for each kernel name (top N by time),
the dispatch count, average duration and the average of every collected counter per dispatch.
python scripts/rocpd_pmc.py <dir or .db> [N]"""
import glob
import os
import re
import sqlite3
import sys


def summary(path, n=12):
    db = path if path.endswith(".db") else sorted(glob.glob(os.path.join(path, "**", "*.db"), recursive=True))[0]
    c = sqlite3.connect(db)
    names = [r[0] for r in c.execute("select name from sqlite_master where type in ('table', 'view')")]
    view = next((v for v in ("counters_collection", "pmc_events", "counters") if v in names), None)
    if view is None:
        return "no counter view; tables: " + ", ".join(names)
    cols = [r[1] for r in c.execute(f"pragma table_info({view})")]
    kcol = next(k for k in ("kernel_name", "name") if k in cols)
    ccol = next(k for k in ("counter_name", "name") if k in cols and k != kcol)
    vcol = next(k for k in ("value", "counter_value") if k in cols)
    dcol = next((k for k in ("dispatch_id", "id") if k in cols), None)
    top = c.execute("select name, count(*), avg(duration) / 1000.0 from kernels group by name "
                    "order by sum(duration) desc limit ?", (n,)).fetchall()
    out = [f"view {view}: columns {', '.join(cols)}"]
    for name, calls, us in top:
        rows = c.execute(f"select {ccol}, sum({vcol}), count(distinct {dcol}) from {view} where {kcol} = ? "
                         f"group by {ccol}", (name,)).fetchall()
        short = re.sub(r"^void |\(anonymous namespace\)::", "", name).split("(")[0][:56]
        vals = "  ".join(f"{cn}={v / max(d, 1):.4g}" for cn, v, d in rows)
        out.append(f"{short:56s} {calls:5d} x {us:8.2f} us | {vals}")
    return "\n".join(out)


if __name__ == "__main__":
    print(summary(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 12))
