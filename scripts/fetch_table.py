"""Per-(kernel, grid) FETCH_SIZE table of one rocprofv3 --pmc FETCH_SIZE pass: dispatches, mean FETCH_SIZE per
dispatch as reported (KB) and corrected for gfx950 (x2: the counter tallies a wide coalesced streaming read at half
its bytes, MI355X_MICROARCH.md's HBM / rocprofv3 section), in MB (10^6 B).

usage: python scripts/fetch_table.py <pmc dir>"""
import csv
import glob
import re
import sys
from collections import defaultdict


def short(name):
    return re.sub(r"\(anonymous namespace\)::|void ", "", name).split("(")[0]


def main():
    d = sys.argv[1]
    per = defaultdict(float)
    meta = {}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != "FETCH_SIZE":
                continue
            k = (f, r["Dispatch_Id"])
            per[k] += float(r["Counter_Value"])
            meta[k] = (short(r["Kernel_Name"]), int(r["Grid_Size"]), int(r["Workgroup_Size"]))
    rows = defaultdict(list)
    for k, v in per.items():
        rows[meta[k]].append(v)
    print(f"{'kernel':58s} {'grid':>8s} {'wg':>5s} {'n':>6s} {'FETCH KB':>12s} {'x2 MB':>10s}")
    for (name, grid, wg), vals in sorted(rows.items(), key=lambda kv: -sum(kv[1])):
        m = sum(vals) / len(vals)
        print(f"{name[:58]:58s} {grid:8d} {wg:5d} {len(vals):6d} {m:12.1f} {m * 1024 * 2 / 1e6:10.2f}")


if __name__ == "__main__":
    main()
