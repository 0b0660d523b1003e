#!/bin/bash
# Update-graph tail A/B as run for profiles/r05_update_tail_ab.txt (then switched by a temporary
# MSACL_EXP_TAIL=join in algorithm/msacl.py; "join" is now the only layout, so both arms below run
# the same code): kernel traces with the update -> next sampler gap, then alternating bench lines
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for m in base join; do
  rm -rf gpurun_out/tail_$m
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tail_$m -o bench --output-format csv -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/tail_$m.log 2>&1 || { tail -5 gpurun_out/tail_$m.log; exit 1; }
  python3 - "$m" <<'PY'
import csv, glob, sys
m = sys.argv[1]
rows = list(csv.DictReader(open(glob.glob(f'gpurun_out/tail_{m}/*kernel_trace.csv')[0])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
idx = [i for i, r in enumerate(rows) if 'k_policy_scales' in r['Kernel_Name']]
for a, b in zip(idx[-8:-1], idx[-7:]):
    seg = rows[a:b]
    end_prev = max(int(r['End_Timestamp']) for r in seg)
    last = max(seg, key=lambda r: int(r['End_Timestamp']))
    print(m, b - a, 'kernels; gap to next step', round((int(rows[b]['Start_Timestamp']) - end_prev) / 1e3, 1), 'us; span',
          round((end_prev - int(rows[a]['Start_Timestamp'])) / 1e3, 1), 'us; last', last['Kernel_Name'][:28])
PY
done
for r in 1 2; do
for m in base join; do
  timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/tail_ab.log 2>&1 || { tail -5 gpurun_out/tail_ab.log; exit 1; }
  tail -1 gpurun_out/tail_ab.log | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); print('bench $m', d['value'], d['ms_per_step'], d['phases']['replay_and_update_ms_policy_free_policy'])"
done
done
