#!/bin/bash
# MSACL_BRANCH_LAYOUT A/B: bench lines alternating, then one kernel trace per layout with the
# update -> next sampler gap
set -o pipefail
mkdir -p gpurun_out
for m in main polyak_join side main polyak_join side; do
  MSACL_BRANCH_LAYOUT=$m timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/lay_ab.log 2>&1 || { tail -5 gpurun_out/lay_ab.log; exit 1; }
  tail -1 gpurun_out/lay_ab.log | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); print('$m', d['value'], d['ms_per_step'], d['phases']['replay_and_update_ms'])"
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for m in main polyak_join; do
  rm -rf gpurun_out/prof_$m
  MSACL_BRANCH_LAYOUT=$m timeout -k 10 600 rocprofv3 --kernel-trace -d gpurun_out/prof_$m -o bench --output-format csv -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_$m.log 2>&1 || { tail -5 gpurun_out/prof_$m.log; exit 1; }
  python3 tools/step_timeline.py "$(find gpurun_out/prof_$m -name '*kernel_trace.csv' | head -1)" gpurun_out/step_timeline_$m.txt
  head -6 gpurun_out/step_timeline_$m.txt
done
