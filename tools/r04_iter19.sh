#!/bin/bash
# Policy step's critic forward on the one-workgroup-per-CU grid (mh_mlp3_set_row_tiles(-1) in the
# later policy iterations): tests, then a bench A/B (MSACL_POLICY_ALONE_RT 1 vs 0), 3 rounds
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_mlp3.py tests/test_gpu_msacl.py tests/test_gpu_msacl_bench.py tests/test_gpu_trainer.py -m gpu -x -q --timeout 300 --timeout-method thread -rf > gpurun_out/it19_tests.log 2>&1
rc=$?; tail -2 gpurun_out/it19_tests.log; [ $rc -eq 0 ] || exit $rc
for cfg in "MSACL_POLICY_ALONE_RT=1" "MSACL_POLICY_ALONE_RT=0" "MSACL_POLICY_ALONE_RT=1" "MSACL_POLICY_ALONE_RT=0" "MSACL_POLICY_ALONE_RT=1" "MSACL_POLICY_ALONE_RT=0"; do
  env $cfg timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-4m > gpurun_out/ab_bench.log 2>&1 \
    || { tail -5 gpurun_out/ab_bench.log; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/ab_bench.log').read().strip().splitlines()[-1])
print('$cfg', d['value'], d['ms_per_step'], d['phases']['sample_ms'], d['phases']['replay_and_update_ms'])"
done
