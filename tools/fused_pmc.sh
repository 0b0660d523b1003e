#!/bin/bash
# SQ counters of the fused horizon kernel (k_sample_fused<Env>) at the bench configuration, one
# PMC pass per library (LIBS="name=path ..."; default: the main build), over tools/fused_ab.py.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for spec in ${LIBS:-build=}; do
  name=${spec%%=*}; lib=${spec#*=}
  rm -rf gpurun_out/pmc_fused_$name
  if [ -n "$lib" ]; then export MSACL_HIP_LIB="$lib"; else unset MSACL_HIP_LIB; fi
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE \
    -d gpurun_out/pmc_fused_$name -o fused --output-format csv -- python3 tools/fused_ab.py --reps 3 --rounds 1 \
    > gpurun_out/pmc_fused_$name.log 2>&1 || { echo "pmc $name failed"; tail -5 gpurun_out/pmc_fused_$name.log; exit 1; }
  python3 - "$name" <<'PY'
import csv, glob, sys
from collections import defaultdict
k = sys.argv[1]
v = defaultdict(list)
for f in glob.glob(f"gpurun_out/pmc_fused_{k}/**/*counter_collection*.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_sample_fused" in r["Kernel_Name"]:
            v[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {c: sum(x) / len(x) for c, x in sorted(v.items())}
w = m["SQ_WAVES"]
print(k, {c: round(x) for c, x in m.items()})
print(k, "per wave (cycles): life", round(4 * m["SQ_WAVE_CYCLES"] / w), "wait_any", round(4 * m["SQ_WAIT_ANY"] / w),
      "wait_inst", round(4 * m["SQ_WAIT_INST_ANY"] / w), "active", round(4 * m["SQ_ACTIVE_INST_ANY"] / w),
      "valu/wave", round(m["SQ_INSTS_VALU"] / w),
      "| mfma busy per SIMD", round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024), "| GRBM_GUI_ACTIVE/8", round(m["GRBM_GUI_ACTIVE"] / 8))
PY
done
