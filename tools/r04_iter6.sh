#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_nstep.py tests/test_gpu_mlp3.py tests/test_gpu_msacl.py tests/test_gpu_msacl_bench.py tests/test_gpu_trainer.py tests/test_gpu_policy_head_rng.py -m gpu -x -q --timeout 300 --timeout-method thread -rf > gpurun_out/it6_tests.log 2>&1
rc=$?; tail -4 gpurun_out/it6_tests.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/it6_ab.txt
for r in 1 2; do
  for cfg in "MSACL_JOINT_BATCH=1" "MSACL_JOINT_BATCH=0" "MSACL_MLP3_WIDE=1" "MSACL_KERNEL_NOISE=0"; do
    env $cfg timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-4m > gpurun_out/ab_bench.log 2>&1 \
      || { tail -5 gpurun_out/ab_bench.log; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open('gpurun_out/ab_bench.log').read().strip().splitlines()[-1])
print('$cfg', d['value'], d['ms_per_step'], d['phases']['sample_ms'], d['phases']['replay_and_update_ms'])" >> gpurun_out/it6_ab.txt
  done
done
cat gpurun_out/it6_ab.txt
