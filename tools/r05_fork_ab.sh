#!/bin/bash
# MSACL_CRITIC_FORK A/B: parity tests with the fork on, then bench lines alternating
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_msacl.py \
  tests/test_gpu_msacl_bench.py tests/test_gpu_trainer.py > gpurun_out/fork_tests.log 2>&1
rc=$?; tail -2 gpurun_out/fork_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
for m in 1 0; do
  MSACL_CRITIC_FORK=$m timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/fork_ab.log 2>&1 || { tail -5 gpurun_out/fork_ab.log; exit 1; }
  tail -1 gpurun_out/fork_ab.log | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); print('fork=$m', d['value'], d['ms_per_step'], d['phases']['replay_and_update_ms'])"
done
done
