#!/bin/bash
# standalone fused-MLP kernel times + one PMC pass over the same command
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/mlp3_bench.py --reps 50 > gpurun_out/mlp3_bench.jsonl 2> gpurun_out/mlp3_bench.err; rc=$?
cat gpurun_out/mlp3_bench.jsonl; [ $rc -eq 0 ] || { tail -20 gpurun_out/mlp3_bench.err; exit $rc; }
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/pmc_mlp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES \
  --kernel-include-regex "mlp3|gemm_deep_multi|gemm_reduce_multi" -d gpurun_out/pmc_mlp -o pmc --output-format csv -- \
  python3 tools/mlp3_bench.py --reps 3 > gpurun_out/pmc_mlp.log 2>&1; echo "pmc rc=$?"
f=$(find gpurun_out/pmc_mlp -name '*counter_collection.csv' | head -1); echo "$f"
[ -n "$f" ] && python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in rows:
    k = (r.get("Kernel_Name", "")[:40], r.get("Grid_Size", ""))
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[(k, r["Counter_Name"])] += 1
for k, d in agg.items():
    print(k, {c: round(v / max(1, n[(k, c)]), 0) for c, v in d.items()})
PY
