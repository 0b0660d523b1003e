#!/bin/bash
# GPU tests of the update's fused MLPs, then a bench A/B of the q heads' folded weight gradients
# (mh_mlp3_backward_w3 vs the grouped head backward)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_mlp3.py tests/test_gpu_msacl.py tests/test_gpu_msacl_bench.py tests/test_gpu_trainer.py -m gpu -x -q --timeout 300 --timeout-method thread -rf > gpurun_out/it12_tests.log 2>&1
rc=$?; tail -3 gpurun_out/it12_tests.log; [ $rc -eq 0 ] || exit $rc
for cfg in "MSACL_FOLD_W3=1" "MSACL_FOLD_W3=0" "MSACL_FOLD_W3=1" "MSACL_FOLD_W3=0"; do
  env $cfg timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-4m > gpurun_out/ab_bench.log 2>&1 \
    || { tail -5 gpurun_out/ab_bench.log; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/ab_bench.log').read().strip().splitlines()[-1])
print('$cfg', d['value'], d['ms_per_step'], d['phases']['sample_ms'], d['phases']['replay_and_update_ms'])"
done
