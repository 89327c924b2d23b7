"""Per-kernel table from a rocprofv3 database (ROCm 7 writes `*_results.db` by default, no kernel_stats.csv):
total ms, calls, average us, kernel name, grid, workgroup -- top N by total time.
python scripts/rocpd_table.py <dir or .db> [N]"""
import glob
import os
import re
import sqlite3
import sys


def table(path, n=12):
    db = path if path.endswith(".db") else sorted(glob.glob(os.path.join(path, "**", "*.db"), recursive=True))[0]
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), avg(duration) / 1000.0, sum(duration) / 1e6, grid_x, grid_y, grid_z, "
                     "workgroup_x from kernels group by name, grid_x, grid_y, grid_z "
                     "order by sum(duration) desc limit ?", (n,)).fetchall()
    out = []
    for name, calls, avg_us, tot_ms, gx, gy, gz, wg in rows:
        short = re.sub(r"^void |\(anonymous namespace\)::", "", name).split("(")[0][:60]
        out.append(f"  {tot_ms:8.1f}ms {calls:6d} {avg_us:9.2f}us  {short}  grid ({gx}, {gy}, {gz}) wg {wg}")
    return "\n".join(out)


if __name__ == "__main__":
    print(table(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 12))
