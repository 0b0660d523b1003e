#!/bin/bash
# SQ instruction/stall counters of the fused rollout step (k_rollout<Env>) at E = 65,536
# (separate PMC pass, no trace domains): VALU instructions per wave vs wave cycles vs waits.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/pmc_sq_roll
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES \
  -d gpurun_out/pmc_sq_roll -o sq --output-format csv -- python3 tools/kernel_bench.py --envs ${ENVS:-QuadTracking} \
  --skip env_step,gather,msacl,gae --reps 3 > gpurun_out/pmc_sq_roll.log 2>&1
echo "pmc sq rc=$?"
f=$(find gpurun_out/pmc_sq_roll -name "*counter_collection.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    if "k_rollout" in r["Kernel_Name"]:
        agg[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in agg.items():
    m = {n: sum(v) / len(v) for n, v in c.items()}
    w = m.get("SQ_WAVES", 1)
    print(k, {n: round(v / w, 1) for n, v in m.items()}, "waves", w)
PY
