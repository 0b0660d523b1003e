#!/bin/bash
# GPU tests of the update's fused MLPs, then a bench A/B of the forward's row-tile rule (auto vs
# the fixed RT = 2 of before)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_mlp3.py tests/test_gpu_msacl.py tests/test_gpu_msacl_bench.py tests/test_gpu_trainer.py -m gpu -x -q --timeout 300 --timeout-method thread -rf > gpurun_out/it11_tests.log 2>&1
rc=$?; tail -3 gpurun_out/it11_tests.log; [ $rc -eq 0 ] || exit $rc
for cfg in "MH_MLP_RT=0" "MH_MLP_RT=2" "MH_MLP_RT=0" "MH_MLP_RT=2"; do
  env $cfg timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-4m > gpurun_out/ab_bench.log 2>&1 \
    || { tail -5 gpurun_out/ab_bench.log; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/ab_bench.log').read().strip().splitlines()[-1])
print('$cfg', d['value'], d['ms_per_step'], d['phases']['sample_ms'], d['phases']['replay_and_update_ms'])"
done
