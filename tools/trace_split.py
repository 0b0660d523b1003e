#!/usr/bin/env python3
"""Per-kernel durations from a rocprofv3 --kernel-trace CSV, with kernels that run at several
grid sizes split by grid size (k_rollout at 65,536 envs: grid 65,536 threads = plain step with
256-thread blocks, 131,072 = the sampler's deferred-emission step with 512-thread blocks; the
trace's Workgroup_Size column reports the kernel's launch-bounds maximum, not the launch). Usage: python tools/trace_split.py <kernel_trace.csv> <out.csv>"""
import csv
import sys
from collections import defaultdict


def main():
    src, out = sys.argv[1], sys.argv[2]
    d = defaultdict(list)
    for r in csv.DictReader(open(src)):
        wg = r.get("Grid_Size") or r.get("Grid_Size_X") or ""
        d[(r["Kernel_Name"], wg)].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    tot = sum(sum(v) for v in d.values())
    rows = sorted(d.items(), key=lambda kv: -sum(kv[1]))
    with open(out, "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["Name", "Grid_Size", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
        for (name, wg), v in rows:
            w.writerow([name, wg, len(v), sum(v), round(sum(v) / len(v), 1), round(100.0 * sum(v) / tot, 2)])
    for (name, wg), v in rows[:12]:
        print(f"{sum(v) / len(v) / 1000:9.2f} us x {len(v):5d}  grid {wg:>7}  {name[:90]}")


if __name__ == "__main__":
    main()
