"""Per-node timeline of a replayed decode step from a rocprofv3 --kernel-trace csv (AR decode step of
scripts/tts_step_time.py, or any captured step): the kernels of one stream in start order, cut into steps at each
occurrence of the step's first kernel; prints the median over steps of every node's duration and of the gap
from the previous node's end, and the step's span.
    python scripts/step_timeline.py <dir with *_kernel_trace.csv> [first-kernel-regex] [skip-steps]"""
import csv
import glob
import re
import statistics
import sys
from collections import defaultdict

path = sorted(glob.glob(sys.argv[1].rstrip("/") + "/**/*kernel_trace.csv", recursive=True))[0]
first = re.compile(sys.argv[2] if len(sys.argv) > 2 else r"k_gemm<2, 1, true, 16, 4, false>")
skip = int(sys.argv[3]) if len(sys.argv) > 3 else 20
rows = list(csv.DictReader(open(path)))
by_q = defaultdict(list)
for r in rows:
    by_q[(r.get("Queue_Id") or r.get("Stream_Id") or "0")].append(r)
q = max(by_q, key=lambda k: len(by_q[k]))   # the busiest queue: the replayed step
ks = sorted(by_q[q], key=lambda r: int(r["Start_Timestamp"]))


def short(n):
    m = re.search(r"::(k_\w+(<[^>]*>)?)", n)
    return m.group(1) if m else n[:40]


steps, cur = [], []
for r in ks:   # a step starts at `first` right after the previous step's sampler (its last node)
    if first.search(r["Kernel_Name"]) and cur and short(cur[-1]["Kernel_Name"]).startswith("k_sample"):
        steps.append(cur)
        cur = []
    cur.append(r)
steps = [s for s in steps[skip:] if len(s) == len(steps[-1])]
if not steps:
    sys.exit("no complete steps found")
n = len(steps[0])
print(f"{len(steps)} steps of {n} nodes ({path})")
print(f"{'node':>4} {'dur_us':>8} {'gap_us':>8}  kernel")
tot_d = tot_g = 0.0
for i in range(n):
    d = statistics.median((int(s[i]["End_Timestamp"]) - int(s[i]["Start_Timestamp"])) / 1e3 for s in steps)
    g = statistics.median((int(s[i]["Start_Timestamp"]) - int(s[i - 1]["End_Timestamp"])) / 1e3 for s in steps) \
        if i else 0.0
    tot_d += d
    tot_g += g
    print(f"{i:4d} {d:8.2f} {g:8.2f}  {short(steps[0][i]['Kernel_Name'])} grid {steps[0][i].get('Grid_Size_X')}"
          f"/{steps[0][i].get('Workgroup_Size_X')}")
span = statistics.median((int(s[-1]["End_Timestamp"]) - int(s[0]["Start_Timestamp"])) / 1e3 for s in steps)
print(f"sum of node durations {tot_d:.1f} us, sum of gaps {tot_g:.1f} us, step span {span:.1f} us")
