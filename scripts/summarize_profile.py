"""Condense a gpu_profile.sh run (gpurun_out/prof_<R>, gpurun_out/pmc_<R>) into profiles/<R>_*.

profiles/<R>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (verbatim)
profiles/<R>_fetch.json         FETCH_SIZE per dispatch, grouped by kernel + grid, corrected per
                                MI355X_MICROARCH.md: the counter is in KiB and counts half the bytes
                                of 16 B/lane streaming reads on gfx950 -> bytes = value * 1024 * 2
profiles/<R>_summary.md         top kernels + the bench JSON line of the profiled command
usage: python scripts/summarize_profile.py r01
(reads gpurun_out/prof_<R>, pmc_<R>, prof_bench_<R>.log, or scripts/gpu_call.sh's <R>_prof, <R>_pmc, <R>_prof.log)
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(r):
    src = os.path.join(ROOT, "gpurun_out")
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    new = os.path.isdir(os.path.join(src, f"{r}_prof"))   # scripts/gpu_call.sh layout
    prof_dir = os.path.join(src, f"{r}_prof" if new else f"prof_{r}")
    pmc_dir = os.path.join(src, f"{r}_pmc" if new else f"pmc_{r}")
    prof_log = os.path.join(src, f"{r}_prof.log" if new else f"prof_bench_{r}.log")
    shutil.copy(os.path.join(prof_dir, "bench_kernel_stats.csv"), os.path.join(dst, f"{r}_kernel_stats.csv"))
    rows = list(csv.DictReader(open(os.path.join(dst, f"{r}_kernel_stats.csv"))))
    groups = defaultdict(list)
    pmc = os.path.join(pmc_dir, "fetch_counter_collection.csv")
    for row in csv.DictReader(open(pmc)):
        if row["Counter_Name"] != "FETCH_SIZE":
            continue
        groups[(row["Kernel_Name"], int(row["Grid_Size"]))].append(float(row["Counter_Value"]))
    fetch = [{"kernel": k, "grid": g, "dispatches": len(v), "fetch_size_kib_mean": sum(v) / len(v),
              "hbm_bytes_per_launch": sum(v) / len(v) * 1024 * 2} for (k, g), v in sorted(groups.items())]
    json.dump({"round": r, "counter": "FETCH_SIZE", "correction": "KiB * 1024 * 2 (gfx950 streaming-read half count)",
               "groups": fetch}, open(os.path.join(dst, f"{r}_fetch.json"), "w"), indent=1)
    bench_line = None
    for line in open(prof_log):
        if line.startswith("{") and '"metric"' in line:
            bench_line = line.strip()
    total = sum(float(x["TotalDurationNs"]) for x in rows)
    with open(os.path.join(dst, f"{r}_summary.md"), "w") as f:
        f.write(f"# Profile {r}\n\nCommand: `rocprofv3 --kernel-trace --stats -- python3 bench.py --config real "
                f"--steps 2 --warmup 1 --no-cpu-baseline --no-single-user` (scripts/gpu_call.sh prof / gpu_profile.sh)\n\n")
        f.write(f"Total kernel time {total / 1e6:.1f} ms (3 turns + gemm probe + weight fill)\n\n")
        f.write("| % | calls | avg us | kernel |\n|---|---|---|---|\n")
        for x in rows[:30]:
            f.write(f"| {float(x['Percentage']):.2f} | {x['Calls']} | {float(x['AverageNs']) / 1e3:.2f} | "
                    f"`{x['Name'][:100]}` |\n")
        f.write("\n## FETCH_SIZE (separate --pmc pass on the dominant kernel, scripts/gpu_call.sh fetch)\n\n| kernel | grid | n | MB/launch |\n"
                "|---|---|---|---|\n")
        for g in fetch:
            f.write(f"| `{g['kernel'][:70]}` | {g['grid']} | {g['dispatches']} | "
                    f"{g['hbm_bytes_per_launch'] / 1e6:.1f} |\n")
        f.write(f"\n## bench line under the profiler\n\n```\n{bench_line}\n```\n")
    print("wrote", dst, r)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01")
