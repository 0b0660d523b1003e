#!/bin/bash
# The policy step's stability advantage on the side stream (default) vs serial on the main stream
# (MSACL_POLICY_ADV_SIDE=0): bench lines alternating, then a kernel trace of each for the step timeline
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3; do
for v in 1 0; do
  MSACL_POLICY_ADV_SIDE=$v timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/advside_$v.log 2>&1 || { tail -5 gpurun_out/advside_$v.log; exit 1; }
  tail -1 gpurun_out/advside_$v.log | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); print('adv_side=$v', d['value'], d['ms_per_step'], d['phases']['replay_and_update_ms_policy_free_policy'])"
done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in 1 0; do
  rm -rf gpurun_out/advprof_$v
  MSACL_POLICY_ADV_SIDE=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/advprof_$v -o p --output-format csv -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/advprof_$v.log 2>&1 || { tail -5 gpurun_out/advprof_$v.log; exit 1; }
  python3 tools/step_timeline.py "$(find gpurun_out/advprof_$v -name '*kernel_trace.csv' | head -1)" gpurun_out/advside_timeline_$v.txt
  head -12 gpurun_out/advside_timeline_$v.txt | tail -2
done
