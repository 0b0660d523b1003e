#!/bin/bash
# Bench A/B of the q heads' weight gradients folded into the chain launch, 3 rounds
set -o pipefail
mkdir -p gpurun_out
for cfg in "MSACL_FOLD_W3=1" "MSACL_FOLD_W3=0" "MSACL_FOLD_W3=1" "MSACL_FOLD_W3=0" "MSACL_FOLD_W3=1" "MSACL_FOLD_W3=0"; do
  env $cfg timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-4m > gpurun_out/ab_bench.log 2>&1 \
    || { tail -5 gpurun_out/ab_bench.log; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/ab_bench.log').read().strip().splitlines()[-1])
print('$cfg', d['value'], d['ms_per_step'], d['phases']['sample_ms'], d['phases']['replay_and_update_ms'])"
done
