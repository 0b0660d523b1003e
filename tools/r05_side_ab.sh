#!/bin/bash
# MSACL_SIDE_BRANCH A/B (which update branch is captured first, on the side stream), alternating
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_msacl.py \
  -k "twin_stream or graph" > gpurun_out/side_tests.log 2>&1 || { tail -5 gpurun_out/side_tests.log; exit 1; }
for m in critic lyapunov critic lyapunov; do
  MSACL_SIDE_BRANCH=$m timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/side_ab.log 2>&1 || { tail -5 gpurun_out/side_ab.log; exit 1; }
  tail -1 gpurun_out/side_ab.log | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); print('$m', d['value'], d['ms_per_step'], d['phases']['replay_and_update_ms'])"
done
