#!/bin/bash
# Trainer-level graphed step (sampling + update as one graph) vs the sampler graph + update graph
# pair (MSACL_GRAPH_STEP=0): equivalence tests, a kernel trace of each with the in-step gaps, bench lines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_trainer.py \
  > gpurun_out/gstep_tests.log 2>&1
rc=$?; echo "tests: $(tail -1 gpurun_out/gstep_tests.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/gstep_tests.log; exit $rc; }
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for m in 1 0; do
  rm -rf gpurun_out/gstep_$m
  MSACL_GRAPH_STEP=$m timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/gstep_$m -o bench --output-format csv -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/gstep_$m.log 2>&1 || { tail -5 gpurun_out/gstep_$m.log; exit 1; }
  python3 - "$m" <<'PY'
import csv, glob, sys
m = sys.argv[1]
rows = list(csv.DictReader(open(glob.glob(f'gpurun_out/gstep_{m}/*kernel_trace.csv')[0])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
idx = [i for i, r in enumerate(rows) if 'k_policy_scales' in r['Kernel_Name']]
for a, b in zip(idx[-8:-1], idx[-7:]):
    seg = rows[a:b]
    end_prev = max(int(r['End_Timestamp']) for r in seg)
    g = [i for i in range(a, b) if 'k_gather' in rows[i]['Kernel_Name']][0]
    print('graph_step', m, b - a, 'kernels; gap before gather', round((int(rows[g]['Start_Timestamp']) - int(rows[g - 1]['End_Timestamp'])) / 1e3, 1),
          'us; gap to next step', round((int(rows[b]['Start_Timestamp']) - end_prev) / 1e3, 1), 'us; span',
          round((end_prev - int(rows[a]['Start_Timestamp'])) / 1e3, 1))
PY
done
for r in 1 2; do
for m in 1 0; do
  MSACL_GRAPH_STEP=$m timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/gstep_ab.log 2>&1 || { tail -5 gpurun_out/gstep_ab.log; exit 1; }
  tail -1 gpurun_out/gstep_ab.log | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); print('bench graph_step=$m', d['value'], d['ms_per_step'], d['phases']['host_enqueue_ms_per_step'], d['phases'].get('host_ms_per_step_by_call'))"
done
done
