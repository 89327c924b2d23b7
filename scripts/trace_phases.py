"""GPU busy vs idle over a rocprofv3 kernel trace, split at idle gaps: python scripts/trace_phases.py DIR"""
import csv
import sys

rows = []
for r in csv.DictReader(open(sys.argv[1].rstrip("/") + "/bench_kernel_trace.csv")):
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]))
rows.sort()
t0 = rows[0][0]
busy = 0
gaps = []
end = rows[0][0]
for s, e, n in rows:
    if s > end:
        gaps.append((s - end, end - t0, n))
    busy += e - max(s, end) if e > end else 0
    end = max(end, e)
span = end - t0
print(f"span {span / 1e6:.1f} ms busy {busy / 1e6:.1f} ms idle {(span - busy) / 1e6:.1f} ms")
big = sorted(gaps, reverse=True)[:15]
for g, at, n in big:
    print(f"gap {g / 1e3:9.1f} us at {at / 1e6:9.2f} ms before {n}")
hist = {}
for g, _, _ in gaps:
    k = "<2us" if g < 2e3 else "<5us" if g < 5e3 else "<20us" if g < 2e4 else "<100us" if g < 1e5 else ">=100us"
    hist[k] = hist.get(k, 0) + g
print({k: round(v / 1e6, 1) for k, v in hist.items()}, "ms of idle by gap size")
