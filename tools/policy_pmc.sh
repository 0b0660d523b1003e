#!/bin/bash
# SQ counters of the policy-forward kernels, one PMC pass per kernel variant:
#   x3 (split-f16, default), x6 (split-bf16 layer 2), f32 (all-f32 kernel).
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for K in ${VARIANTS:-x3 x6 f32}; do
  rm -rf gpurun_out/pmc_pol_$K
  export MH_POLICY_KERNEL=$K MH_POLICY_TPW=2
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE \
    -d gpurun_out/pmc_pol_$K -o pol --output-format csv -- python3 tools/policy_bench.py 65536 10 > gpurun_out/pmc_pol_$K.log 2>&1 || { echo "pmc $K failed"; tail -5 gpurun_out/pmc_pol_$K.log; exit 1; }
  python3 - "$K" <<'PY'
import csv, glob, sys
from collections import defaultdict
k = sys.argv[1]
v = defaultdict(list)
for f in glob.glob(f"gpurun_out/pmc_pol_{k}/**/*counter_collection*.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "policy_forward" in r["Kernel_Name"]:
            v[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {c: sum(x) / len(x) for c, x in sorted(v.items())}
w = m["SQ_WAVES"]
print(k, {c: round(x) for c, x in m.items()})
print(k, "per wave (cycles): life", round(4 * m["SQ_WAVE_CYCLES"] / w), "wait_any", round(4 * m["SQ_WAIT_ANY"] / w),
      "wait_inst", round(4 * m["SQ_WAIT_INST_ANY"] / w), "active", round(4 * m["SQ_ACTIVE_INST_ANY"] / w),
      "| mfma busy per SIMD", round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024), "| GRBM_GUI_ACTIVE/8", round(m["GRBM_GUI_ACTIVE"] / 8))
PY
done
