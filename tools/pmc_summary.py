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

# alias -> (kernel-name pattern, grid size in threads or None): at 65,536 envs k_rollout runs a
# 65,536-thread grid for a plain step and 131,072 (4 env + 4 emitter waves per block) for the
# sampler's deferred-emission step (the Workgroup_Size column is the launch-bounds maximum)
ALIASES = {"rollout_emit": ("k_rollout<mh::QuadTracking, true>", 131072),
           "rollout_step": ("k_rollout<mh::QuadTracking, true>", 65536),
           "window_emit": ("k_emit_fused<12, 4>", None), "replay_gather": ("k_gather", None),
           "msacl_lyapunov": ("k_lyapunov", None), "msacl_q_target": ("k_q_target", None),
           "policy_forward": ("k_policy_forward_x3", None),
           "sample_fused": ("k_sample_fused<mh::QuadTracking>", None), "emit_horizon": ("k_emit_cells<12, 4>", None)}


def load(root, counter):
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(root, f"pmc_{counter}", "**", "*counter_collection*.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            g = r.get("Grid_Size") or r.get("Grid_Size_X") or ""
            vals[f'{r["Kernel_Name"]} [grid {g}]'].append(float(r["Counter_Value"]))
    return vals


def main():
    root, out = sys.argv[1], sys.argv[2]
    fetch, write = load(root, "FETCH_SIZE"), load(root, "WRITE_SIZE")
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from tools.kernel_hash import rollout_sources_sha
    res = {"units": "bytes per launch (mean over dispatches); FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE",
           "rollout_sources_sha": rollout_sources_sha(), "kernels": {}}
    for name in sorted(set(fetch) | set(write)):
        fk = sum(fetch.get(name, [0])) / max(1, len(fetch.get(name, [])))
        wk = sum(write.get(name, [0])) / max(1, len(write.get(name, [])))
        res["kernels"][name] = {"fetch_kib": fk, "write_kib": wk, "dispatches": len(fetch.get(name, [])),
                                "bytes_per_launch": 2 * fk * 1024 + wk * 1024}
    for alias, (pat, wg) in ALIASES.items():
        for name, v in res["kernels"].items():
            if pat in name and (wg is None or f"[grid {wg}]" in name):
                res[alias] = dict(v, kernel=name)
                break
    json.dump(res, open(out, "w"), indent=1)
    for a in ALIASES:
        if a in res:
            print(a, res[a])


if __name__ == "__main__":
    main()
