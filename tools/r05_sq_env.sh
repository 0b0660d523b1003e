#!/bin/bash
# Round 5: the gfx950 counter list (rocprofv3 -L), then SQ instruction / wait counters of the
# env-step kernels (k_rollout<Env, false> via mh_env_step) of TwoLink and SingleTrackCar at
# 4,194,304 envs (separate PMC pass, no trace domains)
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -s KILL 60 rocprofv3 -L > gpurun_out/r05_counters.txt 2>&1
echo "list rc=$?"; grep -o "SQ_INSTS_VALU[A-Z0-9_]*" gpurun_out/r05_counters.txt | sort -u | tr '\n' ' '; echo
rm -rf gpurun_out/pmc_sq_env
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES \
  -d gpurun_out/pmc_sq_env -o sq --output-format csv -- python3 tools/kernel_bench.py --envs TwoLink,SingleTrackCar \
  --sizes 4194304 --skip rollout,gather,msacl,policy,gae --reps 3 > gpurun_out/pmc_sq_env.log 2>&1
echo "pmc sq rc=$?"
f=$(find gpurun_out/pmc_sq_env -name "*counter_collection.csv" | head -1)
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
