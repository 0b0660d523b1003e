#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_mlp3.py tests/test_gpu_msacl.py tests/test_gpu_msacl_bench.py tests/test_gpu_trainer.py tests/test_capi.py -m gpu -x -q --timeout 300 --timeout-method thread -rf > gpurun_out/it10_tests.log 2>&1
rc=$?; tail -3 gpurun_out/it10_tests.log; [ $rc -eq 0 ] || exit $rc
for cfg in "MSACL_MLP3_SQSUM=1" "MSACL_MLP3_SQSUM=0" "MSACL_MLP3_SQSUM=1" "MSACL_MLP3_SQSUM=0"; do
  env $cfg timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-4m > gpurun_out/ab_bench.log 2>&1 \
    || { tail -5 gpurun_out/ab_bench.log; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/ab_bench.log').read().strip().splitlines()[-1])
print('$cfg', d['value'], d['ms_per_step'], d['phases']['sample_ms'], d['phases']['replay_and_update_ms'])"
done
