#!/usr/bin/env python3
"""Per-trainer-step device timeline from a rocprofv3 --kernel-trace CSV of bench.py.

A step starts at the sampler's first kernel (the policy pack k_policy_scales / k_policy_pack_x3
right before the fused horizon kernel, or the fused kernel itself when the graphed step skipped
the pack; without the fused kernel, the pack) and ends at the next one. Prints, for
the timed steps, the step span, the sampler / update split and the number of kernels, then the
kernel-by-kernel timeline (start offset, duration, gap before it) of one even and one odd step.
Usage: python tools/step_timeline.py <kernel_trace.csv> [out.txt]"""
import csv
import sys


def main():
    src = sys.argv[1]
    out = open(sys.argv[2], "w") if len(sys.argv) > 2 else sys.stdout
    rows = list(csv.DictReader(open(src)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    fused = [i for i, r in enumerate(rows) if "k_sample_fused" in r["Kernel_Name"]]
    if fused:
        starts = []
        for j in fused:
            while j > 0 and any(k in rows[j - 1]["Kernel_Name"] for k in ("k_policy_scales", "k_policy_pack_x3")):
                j -= 1
            starts.append(j)
    else:
        starts = [i for i, r in enumerate(rows) if "k_policy_scales" in r["Kernel_Name"]]
    steps = []
    for a, b in zip(starts[:-1], starts[1:]):
        seg = rows[a:b]
        t0 = int(seg[0]["Start_Timestamp"])
        t1 = int(rows[b]["Start_Timestamp"])
        i_emit = max((i for i, r in enumerate(seg) if "k_emit_cells" in r["Kernel_Name"]), default=None)
        samp_end = int(seg[i_emit]["End_Timestamp"]) if i_emit is not None else t0
        busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg)
        if fused and not any("k_gather" in r["Kernel_Name"] for r in seg):
            continue  # a diagnostic fused-kernel launch of bench.py, not a trainer step
        steps.append((t1 - t0, samp_end - t0, t1 - samp_end, len(seg), busy, seg))
    timed = steps[-20:] if len(steps) > 20 else steps
    print(f"{len(steps)} steps; the last {len(timed)}:", file=out)
    for span, samp, upd, nk, busy, _ in timed:
        print(f"  span {span / 1e3:8.1f} us  sample {samp / 1e3:7.1f}  update {upd / 1e3:7.1f}  kernels {nk:4d}"
              f"  busy {busy / 1e3:8.1f}", file=out)
    if timed:
        avg = sum(s[0] for s in timed) / len(timed) / 1e3
        print(f"  mean span {avg:.1f} us", file=out)
    shown = set()
    med = sorted(s[0] for s in timed)[len(timed) // 2] if timed else 0
    for span, samp, upd, nk, busy, seg in reversed(timed):
        if span > 3 * med:  # the last timed step runs into the post-timed diagnostics
            continue
        kind = "long" if nk > sum(s[3] for s in timed) / len(timed) else "short"
        if kind in shown:
            continue
        shown.add(kind)
        print(f"\n== {kind} step: {nk} kernels, span {span / 1e3:.1f} us", file=out)
        t0 = int(seg[0]["Start_Timestamp"])
        prev_end = t0
        for r in seg:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f} gap {(s - prev_end) / 1e3:6.1f}  q{r.get('Queue_Id', '')}"
                  f"  {r['Kernel_Name'][:100]}", file=out)
            prev_end = max(prev_end, e)


if __name__ == "__main__":
    main()
