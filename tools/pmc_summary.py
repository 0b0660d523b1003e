#!/usr/bin/env python3
"""Per-kernel HBM traffic from tools/pmc.sh output -> profiles/<out>.json.

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch. On gfx950 FETCH_SIZE reports half the bytes
of wide coalesced reads (MI355X_MICROARCH.md, HBM section), so reads are doubled; WRITE_SIZE
is taken as is. Bytes per launch = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024 (mean over the
dispatches of that kernel).
Usage: python tools/pmc_summary.py gpurun_out profiles/r01_pmc_traffic.json
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ALIASES = {"rollout_step": "k_rollout<mh::QuadTracking>", "window_emit": "k_emit_fused<12, 4>",
           "replay_gather": "k_gather", "msacl_lyapunov": "k_lyapunov", "msacl_q_target": "k_q_target"}


def load(root, counter):
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(root, f"pmc_{counter}", "**", "*counter_collection*.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            vals[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return vals


def main():
    root, out = sys.argv[1], sys.argv[2]
    fetch, write = load(root, "FETCH_SIZE"), load(root, "WRITE_SIZE")
    res = {"units": "bytes per launch (mean over dispatches); FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE",
           "kernels": {}}
    for name in sorted(set(fetch) | set(write)):
        fk = sum(fetch.get(name, [0])) / max(1, len(fetch.get(name, [])))
        wk = sum(write.get(name, [0])) / max(1, len(write.get(name, [])))
        res["kernels"][name] = {"fetch_kib": fk, "write_kib": wk, "dispatches": len(fetch.get(name, [])),
                                "bytes_per_launch": 2 * fk * 1024 + wk * 1024}
    for alias, pat in ALIASES.items():
        for name, v in res["kernels"].items():
            if pat in name:
                res[alias] = v
                break
    json.dump(res, open(out, "w"), indent=1)
    for a in ALIASES:
        if a in res:
            print(a, res[a])


if __name__ == "__main__":
    main()
