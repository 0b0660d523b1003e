#!/usr/bin/env python3
"""Summarise an update-phase kernel trace (rocprofv3 --kernel-trace of tools/profile_update.py):
kernels per update and time per kernel family, after the last rollout/emission kernel."""
import collections
import csv
import sys


def main(path, updates=20):
    tr = list(csv.DictReader(open(path)))
    tr.sort(key=lambda r: int(r["Start_Timestamp"]))
    last = max(i for i, r in enumerate(tr) if "k_rollout" in r["Kernel_Name"] or "emit" in r["Kernel_Name"])
    up = tr[last + 1:]
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in up)
    span = int(up[-1]["End_Timestamp"]) - int(up[0]["Start_Timestamp"])
    print(f"kernels/update {len(up) / updates:.1f}  busy {busy / 1e6 / updates:.3f} ms  span {span / 1e6 / updates:.3f} ms")
    agg = collections.defaultdict(lambda: [0, 0])
    for r in up:
        n = r["Kernel_Name"]
        key = (n[:70] + ".." + n[-40:]) if len(n) > 110 else n
        agg[key][0] += 1
        agg[key][1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    for k, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:int(sys.argv[2]) if len(sys.argv) > 2 else 25]:
        print(f"{t / 1e3 / updates:8.1f} us/upd {c / updates:6.1f}/upd {t / c / 1e3:6.2f} us  {k}")


if __name__ == "__main__":
    main(sys.argv[1])
