#!/bin/bash
# The sampler's window count formed inside its horizon graph (no eager copy / subtraction around
# the replay): sampler + trainer GPU tests, then a bench A/B, 3 rounds
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_trainer.py tests/test_gpu_nstep.py tests/test_gpu_fused_horizon.py tests/test_gpu_msacl_bench.py tests/test_gpu_sampling.py -m gpu -x -q --timeout 300 --timeout-method thread -rf > gpurun_out/it16_tests.log 2>&1
rc=$?; tail -3 gpurun_out/it16_tests.log; [ $rc -eq 0 ] || exit $rc
for cfg in "MSACL_SAMPLER_COUNT_IN_GRAPH=1" "MSACL_SAMPLER_COUNT_IN_GRAPH=0" "MSACL_SAMPLER_COUNT_IN_GRAPH=1" "MSACL_SAMPLER_COUNT_IN_GRAPH=0" "MSACL_SAMPLER_COUNT_IN_GRAPH=1" "MSACL_SAMPLER_COUNT_IN_GRAPH=0"; do
  env $cfg timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-4m > gpurun_out/ab_bench.log 2>&1 \
    || { tail -5 gpurun_out/ab_bench.log; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/ab_bench.log').read().strip().splitlines()[-1])
print('$cfg', d['value'], d['ms_per_step'], d['phases']['sample_ms'], d['phases']['replay_and_update_ms'])"
done
